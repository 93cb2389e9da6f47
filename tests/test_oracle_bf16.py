"""CPU check of the bf16-emulating oracle mode (restate.bf16_products, config 3's training precisions):
on G4's batch each policy moves the gradients away from the fp32 oracle by the amount bf16 operands
should (so the GPU bound of tests/test_gpu_train_bf16.py resolves the precision), and leaves the
losses at fp32 level."""
from .test_gpu_train_bf16 import _emulated


def test_emulation_separates_policies():
    """The emulation itself: each bf16 policy is 1e-3..5e-2 (relative L2) away from the fp32 oracle
    for the blend-weight and NeRF tensors, so the 2e-3 device bound above resolves the precision."""
    _, g32 = _emulated('fp32')
    for policy in ('bf16', 'bf16_all'):
        _, gb = _emulated(policy)
        worst = max((gb[k] - g32[k]).norm().item() / max(g32[k].norm().item(), 1e-30) for k in g32)
        assert 5e-3 <= worst <= 5e-2, (policy, worst)
    l32, _ = _emulated('fp32')
    for policy in ('bf16', 'bf16_all'):
        lb, _ = _emulated(policy)
        assert ((lb - l32).abs() / l32.abs()).max().item() <= 1e-3, policy
