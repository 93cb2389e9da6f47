"""Max |error| of each render output vs the fp32 oracle (oracle/restate.py), per render precision.

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
        for prec in ('fp32', 'bf16x3'):
            cfg = config.defaults()
            cfg.perturb = 0
            cfg.render_precision = prec
            ret = Renderer(net, cfg).render_device(to_torch(b, dev))
            out[f'{name}/{prec}'] = {k: float((ret[k].cpu() - ref[k]).abs().max()) for k in
                                    ('rgb_map', 'acc_map', 'depth_map', 'raw', 'pbw', 'tbw')}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
