"""Config 3 quality gate as a report: PSNR after K training steps per training precision (protocol in
tests/quality.py, the same function tests/test_gpu_config3.py asserts on).

usage: python tools/train_quality.py [--steps 500] [--seeds 3] [--subject aninerf_313] > gpurun_out/train_quality.json
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.quality import train_psnr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=500)
    ap.add_argument('--seeds', type=int, default=3)
    ap.add_argument('--subject', default='aninerf_313')
    ap.add_argument('--precisions', default='fp32,bf16,bf16_all', help="'fp32#2' = a second fp32 run (run-to-run spread)")
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    precs = args.precisions.split(',')
    res = train_psnr(dev, args.subject, precs, seeds=args.seeds, steps=args.steps,
                     log=lambda m: print(m, file=sys.stderr, flush=True))
    out = {'subject': args.subject, 'steps': args.steps, 'seeds': args.seeds, 'psnr_init': res['_init']}
    for p in precs:
        out['psnr_' + p] = float(np.mean(res[p]['psnr']))
        out['psnr_runs_' + p] = res[p]['psnr']
        out['final_losses_' + p] = res[p]['losses']
        if p != 'fp32' and 'fp32' in res:
            out['delta_db_' + p] = out['psnr_' + p] - float(np.mean(res['fp32']['psnr']))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
