"""Network plugin with the reference's parameter layout (tpose_nerf_network.py:11-38, 218-315).

The modules exist to own the parameters under the exact state_dict names and shapes of the
reference, so ``load_network(strict=True)`` reads a reference ``latest.pth`` and the trainer's
per-parameter optimizer groups line up. The computation never runs through these modules: the
renderer hands the parameter pointers to the HIP library (``animatable_nerf_amd.renderer``).
"""
import torch
import torch.nn as nn

from . import config as _config


def _mlp(input_ch, W=256, D=8, skips=(4,)):
    return nn.ModuleList([nn.Conv1d(input_ch, W, 1)] +
                         [nn.Conv1d(W + input_ch if i in skips else W, W, 1) for i in range(D - 1)])


class TPoseHuman(nn.Module):
    """Canonical NeRF (tpose_nerf_network.py:218-239)."""

    def __init__(self, num_train_frame):
        super().__init__()
        self.nf_latent = nn.Embedding(num_train_frame, 128)
        self.actvn = nn.ReLU()
        self.skips = [4]
        self.pts_linears = _mlp(63)
        self.alpha_fc = nn.Conv1d(256, 1, 1)
        self.feature_fc = nn.Conv1d(256, 256, 1)
        self.latent_fc = nn.Conv1d(384, 256, 1)
        self.view_fc = nn.Conv1d(283, 128, 1)
        self.rgb_fc = nn.Conv1d(128, 3, 1)


class BackwardBlendWeight(nn.Module):
    """Novel-pose blend-weight field (tpose_nerf_network.py:278-294)."""

    def __init__(self, num_eval_frame):
        super().__init__()
        self.bw_latent = nn.Embedding(num_eval_frame, 128)
        self.actvn = nn.ReLU()
        self.skips = [4]
        self.bw_linears = _mlp(191)
        self.bw_fc = nn.Conv1d(256, 24, 1)


class Network(nn.Module):
    """tpose_nerf_network.Network: tpose_human + bw_latent/bw_linears/bw_fc (+ novel_pose_bw)."""

    TENSOR_ORDER_LEN = 46

    def __init__(self, cfg=None):
        super().__init__()
        cfg = cfg if cfg is not None else _config.cfg
        self.num_train_frame = int(cfg.num_train_frame)
        self.tpose_human = TPoseHuman(self.num_train_frame)
        self.bw_latent = nn.Embedding(self.num_train_frame + 1, 128)
        self.actvn = nn.ReLU()
        self.skips = [4]
        self.bw_linears = _mlp(191)
        self.bw_fc = nn.Conv1d(256, 24, 1)
        if cfg.get('aninerf_animation', False):
            self.novel_pose_bw = BackwardBlendWeight(int(cfg.num_eval_frame))

    def core_tensors(self):
        """The 46 tensors of the C-ABI order (include/aninerf.h), i.e. the reference state_dict
        order of everything except ``novel_pose_bw``."""
        ts = [t for k, t in self.named_parameters() if not k.startswith('novel_pose_bw.')]
        assert len(ts) == self.TENSOR_ORDER_LEN, len(ts)
        return ts

    def novel_tensors(self):
        """The 19 novel_pose_bw tensors (state_dict order) or [] (include/aninerf.h)."""
        if not hasattr(self, 'novel_pose_bw'):
            return []
        ts = [t for _, t in self.novel_pose_bw.named_parameters()]
        assert len(ts) == 19, len(ts)
        return ts

    def forward(self, *args, **kwargs):
        raise RuntimeError('Network is a parameter container on this backend; call '
                           'Renderer(net).render(batch) (tpose_renderer.py:159) instead')


def load_numpy_state(net, sd):
    """Load a {name: ndarray} state dict (e.g. synthetic.init_state_dict) strictly."""
    net.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()}, strict=True)
    return net
