"""Config 3 (aninerf_313 training, bf16, 1 GPU) at its own shapes, with north_star's quality gate:
held-out PSNR after training with bf16 GEMM operands within 0.05 dB of the exact-fp32 training
(tests/quality.py describes the protocol; PSNR is lib/evaluators/if_nerf.py:15-18)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GATE_DB = 0.05   # north_star: "PSNR within 0.05 dB"
STEPS = 500
# 500-step trajectories are chaotic: split-K atomics reorder fp32 sums run to run, and single fp32 runs
# of one seed moved by up to 0.1 dB (profiles/r4n: fp32 seeds 11.843 / 11.946 / 11.942 dB). The per-seed
# PSNR spread within one precision is ~0.055 dB (round 6, profiles/round6/r7o_gpu_tests.log: fp32 seeds
# 11.806 .. 11.972), so the difference of two 8-seed means has a standard error of ~0.027 dB — too close
# to the 0.05 dB bar: that run failed with bf16 0.051 dB ABOVE fp32 (two low fp32 seeds), the code's
# weight-gradient sample ranges having changed the fp32 summation order. 16 seeds halve the variance
# (standard error ~0.019 dB, the bar at ~2.6 of it); the estimator (mean over seeds) and the bar are
# unchanged.
SEEDS = 16


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    return torch.device('cuda:0')


def test_config3_bf16_psnr_within_gate(dev):
    from .quality import train_psnr
    res = train_psnr(dev, 'aninerf_313', ('fp32', 'bf16', 'bf16_all'), seeds=SEEDS, steps=STEPS, log=print)
    p32 = float(np.mean(res['fp32']['psnr']))
    # training must actually learn the target (the gate is meaningless on an untrained image)
    assert p32 > res['_init'] + 3.0, (p32, res['_init'])
    for prec in ('bf16', 'bf16_all'):
        p = float(np.mean(res[prec]['psnr']))
        print(f'{prec}: {p:.4f} dB vs fp32 {p32:.4f} dB (delta {p - p32:+.4f}); runs {res[prec]["psnr"]}')
        assert abs(p - p32) <= GATE_DB, (prec, p, p32, res[prec]['psnr'], res['fp32']['psnr'])
