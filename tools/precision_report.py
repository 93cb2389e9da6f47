"""Max |error| of each render output per render precision, against the fp32 oracle (oracle/restate.py,
the reference's arithmetic) and against an fp64 evaluation of the same network (the oracle run in float64
on the same inputs); the fp32 oracle's own error vs fp64 is listed as 'oracle_fp32'.

usage: python tools/precision_report.py > gpurun_out/precision.json   (GPU box)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from animatable_nerf_amd import config  # noqa: E402
from animatable_nerf_amd.renderer import Renderer  # noqa: E402
from oracle import restate  # noqa: E402
from tests._common import batch_np, make_net, oracle_params, rotated_batch_np, scene, to_torch  # noqa: E402

KEYS = ('rgb_map', 'acc_map', 'depth_map', 'raw', 'pbw', 'tbw')


def main():
    dev = torch.device('cuda:0')
    torch.set_num_threads(16)
    cases = {}
    sc = scene(0.025)
    ro, rd = sc.box_rays(5000, seed=21)
    cases['box_5000_fine'] = batch_np(sc, ro, rd)[0]
    cases['rotated_3000'] = rotated_batch_np()
    net = make_net(dev)
    net.train()
    out = {}
    for name, b in cases.items():
        with torch.no_grad():
            ref = restate.render(oracle_params(), to_torch(b))
            p64 = {k: v.double() for k, v in oracle_params().items()}
            b64 = {k: (v.double() if v.dtype == torch.float32 else v) for k, v in to_torch(b).items()}
            r64 = restate.render(p64, b64)
        out[f'{name}/oracle_fp32'] = {'vs_fp64': {k: float((ref[k].double() - r64[k]).abs().max()) for k in KEYS}}
        for prec in ('fp32', 'bf16x6', 'bf16x3'):
            cfg = config.defaults()
            cfg.perturb = 0
            cfg.render_precision = prec
            ret = Renderer(net, cfg).render_device(to_torch(b, dev))
            out[f'{name}/{prec}'] = {
                'vs_oracle_fp32': {k: float((ret[k].cpu() - ref[k]).abs().max()) for k in KEYS},
                'vs_fp64': {k: float((ret[k].cpu().double() - r64[k]).abs().max()) for k in KEYS}}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
