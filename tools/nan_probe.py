"""Locate non-finite gradients in bf16_all training (tests/quality.py's config-3 protocol): for each
environment variant (ANR_* switches read per library call) and seed, run the steps and report the
first step whose gradient blob holds a non-finite value, with the tensors it is in.

    python tools/nan_probe.py [steps] [seed/seed/...] [every] [VAR=VAL[+VAR=VAL...] ...]

every: host check every that many steps (1 serialises the steps, which can hide a race between them)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from tests.quality import frame, make_net, sub  # noqa: E402
from animatable_nerf_amd import config  # noqa: E402
from animatable_nerf_amd.trainer import FusedStep  # noqa: E402


def run(dev, batch, gt, seed, steps, every=1, prec='bf16_all', rays=1024, eval_rays=16384):
    R = int(batch['ray_o'].shape[1])
    n_train = R - eval_rays
    cfg = config.subject('aninerf_313', perturb=1, train_precision=prec)
    net = make_net(cfg, 1234, dev)
    net.train()
    step = FusedStep(net, cfg)
    g = torch.Generator(device=dev)
    g.manual_seed(5 + 1000 * seed)
    for it in range(steps):
        idx = torch.randint(0, n_train, (rays,), device=dev, generator=g)
        t_rand = torch.rand((rays, 64), device=dev, generator=g)
        step.step(sub(batch, idx, gt[idx]), t_rand=t_rand)
        if (it + 1) % every and it + 1 < steps:
            continue
        bad = [i for i, v in enumerate(step.grad_views) if not bool(torch.isfinite(v).all())]
        if bad:
            return it, bad
        if not bool(torch.isfinite(step.flat).all()):
            return it, ['weights']
    return None, []


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    # runs: 'seed' (bf16_all) or 'precision:seed', in order (a run reuses the memory its predecessors freed)
    seeds = sys.argv[2].split('/') if len(sys.argv) > 2 else ['0', '2', '7']
    every = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    variants = sys.argv[4:] or ['']
    dev = torch.device('cuda:0')
    batch, gt = frame(dev)
    for var in variants:
        saved = {}
        for kv in filter(None, var.split('+')):
            k, v = kv.split('=', 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        side = os.environ.get('NAN_PROBE_STREAM') == '1'  # run the steps on a non-default torch stream
        for spec in seeds:
            prec, seed = spec.split(':') if ':' in spec else ('bf16_all', spec)
            if side:
                st = torch.cuda.Stream(dev)
                st.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(st):
                    it, bad = run(dev, batch, gt, int(seed), steps, every, prec)
                torch.cuda.current_stream(dev).wait_stream(st)
            else:
                it, bad = run(dev, batch, gt, int(seed), steps, every, prec)
            print(f'[{var or "default"}] {prec} seed {seed}: ' +
                  ('finite' if it is None else f'first non-finite at step {it}: {bad}'), flush=True)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == '__main__':
    main()
