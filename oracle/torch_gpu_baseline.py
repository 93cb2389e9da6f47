"""ORACLE — measurement only. The "reference single-GPU PyTorch" denominator of BASELINE.md §3:
the op-for-op restatement (oracle/restate.py) run with PyTorch-ROCm on one MI355X, fp32,
2048-ray chunks, on the same synthetic config-2 frame bench.py renders. Not a product path.

python oracle/torch_gpu_baseline.py [--chunks 32]   -> one JSON line
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--chunks', type=int, default=32)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    sc = synthetic.Scene(vsize=0.025)
    ro, rd = sc.box_rays(512 * 512, seed=2)
    near, far, mask = restate.near_far(sc.bounds, ro, rd)
    b = sc.batch_arrays(ro[mask], rd[mask], near.astype(np.float32), far.astype(np.float32))
    n = min(args.chunks * 2048, b['ray_o'].shape[1])
    ray_keys = ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb')
    bt = {k: torch.from_numpy(np.ascontiguousarray(v[:, :n] if k in ray_keys else v)).to(dev) for k, v in b.items()}
    net = network.Network()
    sd = synthetic.init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    P = {k: torch.from_numpy(v).to(dev) for k, v in sd.items()}
    with torch.no_grad():
        restate.render(P, {k: (v[:, :2048] if k in ray_keys else v) for k, v in bt.items()})
        torch.cuda.synchronize()
        times = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            restate.render(P, bt)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    print(json.dumps({'baseline': 'reference op-for-op PyTorch-ROCm restatement, 1 GPU, fp32, chunk 2048',
                      'rays': n, 'value': n * 64 / dt, 'unit': 'ray-samples/s', 'seconds': dt,
                      'torch': torch.__version__}))


if __name__ == '__main__':
    main()
