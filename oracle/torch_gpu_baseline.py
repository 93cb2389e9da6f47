"""ORACLE — measurement only. The "reference single-GPU PyTorch" denominator of BASELINE.md §3:
the op-for-op restatement (oracle/restate.py) run with PyTorch-ROCm on one MI355X, fp32,
2048-ray chunks, on the same synthetic config-2 frame bench.py renders. Not a product path:
bench.py calls ``measure`` outside its timed region, as a baseline leg beside cpu_baseline.

python oracle/torch_gpu_baseline.py [--chunks N]   -> one JSON line (N = 0: the whole frame)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from animatable_nerf_amd import network, synthetic  # noqa: E402
from oracle import restate  # noqa: E402

RAY_KEYS = ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb')


def measure(sd, b, dev, reps=3, n_rays=None):
    """restate.render (Renderer.render of tpose_renderer.py:159-186, op for op) on ``dev`` over the
    first ``n_rays`` rays of the numpy batch ``b`` (all by default): one untimed pass over the same
    rays, then the median of ``reps`` device-synchronised runs.

    The untimed pass matters on ROCm: every chunk's kept-sample count n' is a new Conv1d problem
    size for MIOpen, whose first use of a size costs ~0.8 s (measured: 32 chunks 52.6 s cold, 0.16 s
    warm). The steady-state rate of the warm passes is the denominator (the most favourable reading
    of the reference); the cold pass is reported beside it."""
    R = b['ray_o'].shape[1]
    n = R if not n_rays else min(n_rays, R)
    bt = {k: torch.from_numpy(np.ascontiguousarray(v[:, :n] if k in RAY_KEYS else v)).to(dev) for k, v in b.items()}
    P = {k: torch.from_numpy(v).to(dev) for k, v in sd.items()}
    with torch.no_grad():
        t0 = time.perf_counter()
        restate.render(P, bt)
        torch.cuda.synchronize()
        cold = time.perf_counter() - t0
        print(f'[torch_gpu_baseline] cold pass {n} rays {cold:.2f} s', file=sys.stderr, flush=True)
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            restate.render(P, bt)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            print(f'[torch_gpu_baseline] {n} rays {times[-1]:.2f} s', file=sys.stderr, flush=True)
    dt = float(np.median(times))
    return {'baseline': 'reference op-for-op PyTorch-ROCm restatement (oracle/restate.py), 1 GPU, fp32, chunk 2048',
            'rays': n, 'value': n * 64 / dt, 'unit': 'ray-samples/s', 'seconds': dt, 'median_of': reps,
            'cold_pass_seconds': cold, 'torch': torch.__version__}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--chunks', type=int, default=0)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    sc = synthetic.Scene(vsize=0.025)
    ro, rd = sc.box_rays(512 * 512, seed=2)
    near, far, mask = restate.near_far(sc.bounds, ro, rd)
    b = sc.batch_arrays(ro[mask], rd[mask], near.astype(np.float32), far.astype(np.float32))
    net = network.Network()
    sd = synthetic.init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    print(json.dumps(measure(sd, b, dev, args.reps, args.chunks * 2048)))


if __name__ == '__main__':
    main()
