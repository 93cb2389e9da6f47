"""Config 3 quality gate: PSNR after K training steps with bf16 GEMM operands vs exact fp32.

Both students start from the same weights (synthetic.init_state_dict, seed 1234) and see the same
ray batches and stratification draws; the targets are the image of a teacher network (seed 777)
rendered by the fp32 eval path on the config-2 frame, so PSNR measures how well each student learned
it. Evaluation: fp32 eval render of held-out rays (the last --eval-rays of the frame, never trained
on), A18 PSNR (lib/evaluators/if_nerf.py:15-18). The fp32 student is the reference: the fp32
training step is parity-pinned to the reference step (tests/test_gpu_train.py, golden G4).

usage: python tools/train_quality.py [--steps 300] > gpurun_out/train_quality.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from animatable_nerf_amd import config, network, synthetic  # noqa: E402
from animatable_nerf_amd.renderer import Renderer, near_far  # noqa: E402
from animatable_nerf_amd.trainer import FusedStep  # noqa: E402


def make_net(seed, dev):
    net = network.Network()
    sd = synthetic.init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()}, seed=seed)
    network.load_numpy_state(net, sd)
    return net.to(dev)


def sub(batch, idx, rgb=None):
    out = {}
    for k, v in batch.items():
        if k in ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb'):
            out[k] = v[:, idx]
        else:
            out[k] = v
    if rgb is not None:
        out['rgb'] = rgb[None]
    return out


def psnr(a, b):
    mse = torch.mean((a - b) ** 2).item()
    return -10.0 * np.log10(mse)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=300)
    ap.add_argument('--rays', type=int, default=1024)
    ap.add_argument('--eval-rays', type=int, default=16384)
    ap.add_argument('--frame-rays', type=int, default=512 * 512)
    ap.add_argument('--target', choices=('teacher', 'texture'), default='texture')
    ap.add_argument('--precisions', default='fp32,bf16,bf16_all')
    ap.add_argument('--seeds', type=int, default=1, help='batch/stratification seeds per precision (mean reported)')
    ap.add_argument('--tex-freq', type=float, nargs=2, default=(9.0, 7.0))
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    sc = synthetic.Scene(vsize=0.025)
    ro, rd = sc.box_rays(args.frame_rays, seed=2)
    nr, fr, m = near_far(torch.from_numpy(sc.bounds).to(dev), torch.from_numpy(ro).to(dev), torch.from_numpy(rd).to(dev))
    m_np = m.cpu().numpy()
    b = sc.batch_arrays(ro[m_np], rd[m_np], nr.cpu().numpy(), fr.cpu().numpy())
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()}
    R = batch['ray_o'].shape[1]
    cfg = config.defaults()
    cfg.perturb = 0
    if args.target == 'teacher':
        teacher = make_net(777, dev)
        teacher.train()
        with torch.no_grad():
            gt = Renderer(teacher, cfg).render_device(batch, bw_rows=False)['rgb_map'][0]
    else:  # a view-dependent procedural texture (PSNR in the range of real captures)
        d = batch['ray_d'][0]
        c = torch.arange(3, device=dev, dtype=torch.float32)
        fx, fy = args.tex_freq
        gt = 0.5 + 0.45 * torch.sin(fx * d[:, :1] + 11.0 * c) * torch.cos(fy * d[:, 1:2] + 7.0 * c)
    n_train = R - args.eval_rays
    ev = torch.arange(n_train, R, device=dev)
    g = torch.Generator(device=dev)
    results = {}
    precs = args.precisions.split(',')
    for prec in precs:
        runs = []
        for seed in range(args.seeds):
            tcfg = config.defaults()
            tcfg.perturb = 1
            tcfg.train_precision = prec.split('#')[0]  # 'fp32#2': a second fp32 run (run-to-run spread)
            net = make_net(1234, dev)
            net.train()
            step = FusedStep(net, tcfg)
            g.manual_seed(5 + 1000 * seed)
            losses = []
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for it in range(args.steps):
                idx = torch.randint(0, n_train, (args.rays,), device=dev, generator=g)
                t_rand = torch.rand((args.rays, 64), device=dev, generator=g)
                l3 = step.step(sub(batch, idx, gt[idx]), t_rand=t_rand)
                if it % 100 == 0 or it == args.steps - 1:
                    losses.append([it] + l3[:3].cpu().tolist())
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ecfg = config.defaults()
            ecfg.perturb = 0
            with torch.no_grad():
                out = Renderer(net, ecfg).render_device(sub(batch, ev), bw_rows=False)['rgb_map'][0]
            runs.append({'psnr': psnr(out, gt[ev]), 'ms_per_step': dt / args.steps * 1e3, 'losses': losses})
        ps = [r['psnr'] for r in runs]
        results[prec] = {'psnr': float(np.mean(ps)), 'psnr_runs': ps,
                         'ms_per_step': float(np.mean([r['ms_per_step'] for r in runs])), 'losses': runs[0]['losses']}
        print(prec, ps, results[prec]['ms_per_step'], file=sys.stderr, flush=True)
    with torch.no_grad():
        init = make_net(1234, dev)
        init.train()
        p0 = psnr(Renderer(init, cfg).render_device(sub(batch, ev), bw_rows=False)['rgb_map'][0], gt[ev])
    res = {'target': args.target, 'steps': args.steps, 'rays_per_step': args.rays, 'eval_rays': args.eval_rays,
           'psnr_init': p0}
    for prec in precs:
        res['psnr_' + prec] = results[prec]['psnr']
        res['psnr_runs_' + prec] = results[prec]['psnr_runs']
        res['ms_per_step_' + prec] = results[prec]['ms_per_step']
        if prec != 'fp32' and 'fp32' in results:
            res['delta_db_' + prec] = results[prec]['psnr'] - results['fp32']['psnr']
        res['losses_' + prec] = results[prec]['losses']
    print(json.dumps(res))


if __name__ == '__main__':
    main()
