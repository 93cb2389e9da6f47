"""Network plugin with the reference's parameter layout (tpose_nerf_network.py:11-38, 218-315).

The modules own the parameters under the exact state_dict names and shapes of the reference, so
``load_network(strict=True)`` reads a reference ``latest.pth`` and the trainer's per-parameter
optimizer groups line up. Every computation runs on the HIP library, through the same entry points
the renderers use:

* ``Network.forward(wpts, viewdir, dists, batch)`` -> {'raw', 'pbw', 'tbw'} (:139-215), the call a
  reference renderer makes per chunk (tpose_renderer.py:95): ``anr_network_fwd`` (fused kernel) in
  evaluation, ``anr_network_train_fwd/bwd`` (an autograd Function) when training;
* ``get_alpha`` / ``calculate_alpha(wpts, batch)`` (:105-137): ``anr_alpha_points`` over the call;
* ``calculate_neural_blend_weights(pts, smpl_bw, latent_index)`` (:55-77), ``novel_pose_bw(...)``
  (:304-315) and ``tpose_human.calculate_alpha(nf_pts)`` (:241-250): ``anr_blend_weights`` /
  ``anr_canonical_alpha`` (forward only).
Built with no cfg (the reference's ``make_network``), it reads the reference's global
``lib.config.cfg`` when that is loaded (``config.active``).
"""
import torch
import torch.nn as nn

from . import config as _config


def _mlp(input_ch, W=256, D=8, skips=(4,)):
    return nn.ModuleList([nn.Conv1d(input_ch, W, 1)] +
                         [nn.Conv1d(W + input_ch if i in skips else W, W, 1) for i in range(D - 1)])


def _owner(module):
    net = module.__dict__.get('_anr_owner')
    net = net() if net is not None else None
    if net is None:
        raise RuntimeError(f'{type(module).__name__} is evaluated through its Network (it has none)')
    return net


class TPoseHuman(nn.Module):
    """Canonical NeRF (tpose_nerf_network.py:218-239)."""

    def calculate_alpha(self, nf_pts):
        """TPoseHuman.calculate_alpha (:241-250): canonical points (1,n,3) -> raw alpha (1,1,n)."""
        return _owner(self)._device().canonical_alpha(nf_pts)

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

    def forward(self, ppts, smpl_bw, latent_index):
        """BackwardBlendWeight.forward (:304-315): (1,n,3), (1,24,n), index -> bw (1,24,n)."""
        return _owner(self)._device().blend_weights(ppts, smpl_bw, latent_index, field=1)

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
        cfg = cfg if cfg is not None else _config.active()
        self.__dict__['_anr_cfg'] = cfg
        self.num_train_frame = int(cfg.num_train_frame)
        self.tpose_human = TPoseHuman(self.num_train_frame)
        self.bw_latent = nn.Embedding(self.num_train_frame + 1, 128)
        self.actvn = nn.ReLU()
        self.skips = [4]
        self.bw_linears = _mlp(191)
        self.bw_fc = nn.Conv1d(256, 24, 1)
        if cfg.get('aninerf_animation', False):
            self.novel_pose_bw = BackwardBlendWeight(int(cfg.num_eval_frame))
        self._bind()

    def _bind(self):
        import weakref
        for m in (self.tpose_human, getattr(self, 'novel_pose_bw', None)):
            if m is not None:
                m.__dict__['_anr_owner'] = weakref.ref(self)

    def __getstate__(self):
        # the device renderers hold this instance: a copy (deepcopy, pickle) builds its own
        state = dict(super().__getstate__())
        state.pop('_anr_renderer', None)
        state.pop('_anr_mesh', None)
        return state

    def __setstate__(self, state):
        super().__setstate__(state)
        self._bind()

    def _device(self):
        """the device renderer that evaluates this network's calls (built on first use)"""
        r = self.__dict__.get('_anr_renderer')
        if r is None:
            from .renderer import Renderer
            r = Renderer(self, self.__dict__['_anr_cfg'])
            self.__dict__['_anr_renderer'] = r
        return r

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

    def forward(self, wpts, viewdir, dists, batch):
        """tpose_nerf_network.py:139-215: one reference network call over n free samples -> {'pbw' (1,m,24),
        'tbw' (1,m,24), 'raw' (1,n,4)}; differentiable w.r.t. the parameters when training."""
        return self._device().network_forward(wpts, viewdir, dists, batch)

    def calculate_alpha(self, wpts, batch):
        """tpose_nerf_network.py:105-137 (``get_alpha``): raw alpha (n) of world points, 0 where the pbw
        prefilter (pnorm < 0.1 plus the argmin over the call) drops them. Forward only."""
        from .renderer_mesh import MESH_NORM_TH, Renderer as MeshRenderer  # noqa: F401
        r = self.__dict__.get('_anr_mesh')
        if r is None:
            r = MeshRenderer(self, self.__dict__['_anr_cfg'])
            self.__dict__['_anr_mesh'] = r
        n = int(wpts.reshape(-1, 3).shape[0])
        return r.alpha_points(wpts, batch, chunk_pts=max(64, (n + 63) // 64 * 64))

    get_alpha = calculate_alpha

    def calculate_neural_blend_weights(self, pose_pts, smpl_bw, latent_index):
        """tpose_nerf_network.py:55-77: (1,n,3), (1,24,n), index tensor -> bw (1,24,n). Forward only."""
        return self._device().blend_weights(pose_pts, smpl_bw, latent_index, field=0)


def load_numpy_state(net, sd):
    """Load a {name: ndarray} state dict (e.g. synthetic.init_state_dict) strictly."""
    net.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()}, strict=True)
    return net
