"""Diagnose full-frame differences between the exact fp32 render kernel and the fp32 oracle run on the
GPU (tests/test_gpu_render.py test_split_precisions_fp32_level_full_frame): the worst rays, and per
sample of the worst ray the raw outputs of both, the oracle's T-pose point, sigma' and bbox margin."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from animatable_nerf_amd import config  # noqa: E402
from animatable_nerf_amd.renderer import Renderer  # noqa: E402
from oracle import restate  # noqa: E402
from tests._common import batch_np, make_net, oracle_params, scene, to_torch  # noqa: E402
from tests.test_gpu_render import _conv_mm  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    sc = scene(0.025)
    ro, rd = sc.box_rays(512 * 512, seed=2)
    b, _ = batch_np(sc, ro, rd)
    bd = to_torch(b, dev)
    restate._conv = _conv_mm
    P = {k: v.to(dev) for k, v in oracle_params().items()}
    with torch.no_grad():
        r32 = restate.render(P, bd)
    net = make_net(dev)
    net.train()
    cfg = config.defaults()
    cfg.perturb = 0
    cfg.render_precision = os.environ.get('PREC', 'fp32')
    ret = Renderer(net, cfg).render_device(bd)
    R = bd['ray_o'].shape[1]
    e = (ret['rgb_map'] - r32['rgb_map']).abs().amax(-1)[0]
    order = torch.argsort(e, descending=True)[:12]
    print('rays with rgb error > 1e-4:', int((e > 1e-4).sum()), 'of', R, flush=True)
    for ray in order.tolist():
        print(f'ray {ray} chunk {ray // 2048} rgb err {e[ray].item():.3e} acc {ret["acc_map"][0, ray].item():.4f} '
              f'vs {r32["acc_map"][0, ray].item():.4f}')
    ray = int(order[0])
    c = ray // 2048
    sub = {k: (v[:, c * 2048:(c + 1) * 2048] if k in ('ray_o', 'ray_d', 'near', 'far') else v) for k, v in bd.items()}
    tr = {}
    with torch.no_grad():
        restate.render_chunk(P, sub['ray_o'], sub['ray_d'], sub['near'], sub['far'], bd, trace=tr)
    pind = tr['pind'][0]
    kept = torch.nonzero(pind)[:, 0]
    lo, hi = bd['tbounds'][0, 0], bd['tbounds'][0, 1]
    rr = ray - c * 2048
    for s in range(64):
        gid = rr * 64 + s
        dv = ret['raw'][0, ray * 64 + s]
        ov = r32['raw'][0, ray * 64 + s]
        line = f'  s{s:2d} dev {dv.tolist()} ora {ov.tolist()}'
        j = torch.nonzero(kept == gid)
        if len(j):
            j = int(j[0, 0])
            tp = tr['tpose'][0, j]
            margin = torch.minimum(tp - lo, hi - tp).min().item()
            line += f' sigma {tr["sigma"][0, j].item():.4e} tpose {tp.tolist()} bbox margin {margin:.3e}'
        if (dv - ov).abs().max() > 1e-5:
            print(line + '  <-- differs')
    print('chunk keep equal:', torch.equal(pind.cpu(), (ret['raw'][0, c * 2048 * 64:(c + 1) * 2048 * 64, :3].abs().sum(-1) != 0).cpu()))


if __name__ == '__main__':
    main()
