"""Animation-stage trainer plugin (lib/train/trainers/aninerf_animation_trainer.py, SURVEY.md §8(f)
row 2): fits ``net.novel_pose_bw`` to the frozen blend-weight field on novel poses.

* ``NetworkWrapper(net)`` — the reference wrapper: ``forward(batch) -> (ret, loss, scalar_stats,
  image_stats)`` with ``scalar_stats = {bw_loss0, bw_loss1, loss}``. The sampling points are drawn
  like the reference (``torch.rand`` on the CPU, :143-160); one ``anr_anim_step`` call computes both
  paths' losses AND the novel_pose_bw gradients, which an autograd Function hands to
  ``loss.backward()``, so the reference ``Trainer.train`` loop runs unchanged. Every other parameter
  is frozen (``requires_grad = False``, :24-29). ``ret`` is empty: the reference's ``pbw0`` rows feed
  nothing downstream (the trainer only logs the scalar stats).
* ``AnimationStep(net)`` — the native loop: novel_pose_bw parameters, gradients and Adam moments in
  flat HBM blobs; ``step(batch)`` = ``anr_anim_step`` + [RCCL mean all-reduce] + ``anr_adam``.
"""
import ctypes

import torch

from . import _lib
from . import config as _config
from .parallel import allreduce_mean_, broadcast_
from .renderer import Renderer, _f32

N_POINTS = 1024 * 64  # get_sampling_points (aninerf_animation_trainer.py:153)


def sample_unit(n=N_POINTS, generator=None):
    """The three torch.rand([1, n]) draws of get_sampling_points, stacked -> (1, n, 3) on the CPU."""
    vals = [torch.rand([1, n], generator=generator) for _ in range(3)]
    return torch.stack(vals, dim=2)


def points_in(bounds, vals):
    """(max - min)[:, None] * vals + min[:, None] (:157-159), on the bounds' device."""
    lo, hi = bounds[:, 0], bounds[:, 1]
    return (hi - lo)[:, None] * vals.to(bounds.device) + lo[:, None]


class _Anim:
    """Device tensors + C structs of one anr_anim_step call."""

    def __init__(self, renderer, batch, wvals, tvals):
        cfg = renderer.cfg
        self.dev = dev = renderer.device()
        keys = ('A', 'R', 'Th', 'pbw', 'pbounds', 'tbw', 'tbounds', 'wbounds')
        fr = {k: _f32(batch[k], dev) for k in keys}
        self.fr = fr
        self.wpts = points_in(fr['wbounds'], wvals).reshape(-1, 3).contiguous()
        self.tpts = points_in(fr['tbounds'], tvals).reshape(-1, 3).contiguous()
        self.bli = batch['bw_latent_index'].to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        li = batch.get('latent_index', batch['bw_latent_index'])
        self.li = li.to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        f = _lib.Frame()
        f.A, f.R, f.Th = fr['A'].data_ptr(), fr['R'].data_ptr(), fr['Th'].data_ptr()
        f.pbw, f.pbounds = fr['pbw'].data_ptr(), fr['pbounds'].data_ptr()
        f.tbw, f.tbounds = fr['tbw'].data_ptr(), fr['tbounds'].data_ptr()
        for i in range(3):
            f.pbw_dims[i] = fr['pbw'].shape[1 + i]
            f.tbw_dims[i] = fr['tbw'].shape[1 + i]
        f.latent_index, f.bw_latent_index = self.li.data_ptr(), self.bli.data_ptr()
        self.frame = f
        o = _lib.RenderOpts()
        o.n_samples, o.chunk = 64, 2048
        o.norm_th = float(cfg.norm_th)
        o.train_th = float(cfg.train_th)
        prec = cfg.get('train_precision', 'fp32')
        precs = {'fp32': _lib.FP32, 'bf16': _lib.BF16, 'bf16_all': _lib.BF16_ALL}
        if prec not in precs:
            raise ValueError(f"train_precision must be one of {sorted(precs)}, got {prec!r}")
        o.precision = precs[prec]
        self.opts = o


def anim_step(renderer, batch, grads, loss3, wvals, tvals):
    """One anr_anim_step: accumulates the 19 novel_pose_bw gradients into ``grads`` and writes the
    (loss, bw_loss0, bw_loss1) triple into ``loss3`` (device, no sync)."""
    lib = renderer.lib
    p = renderer.params(pack=False)
    if not renderer.net.novel_tensors():
        raise RuntimeError('animation stage needs net.novel_pose_bw (cfg.aninerf_animation = True)')
    c = _Anim(renderer, batch, wvals, tvals)
    n0, n1 = c.wpts.shape[0], c.tpts.shape[0]
    nbytes = lib.anr_anim_workspace_bytes(max(n0, n1))
    ws = renderer._workspace('_anws', nbytes, c.dev)
    gp = (ctypes.c_void_p * _lib.NUM_NOVEL_TENSORS)(*[g.data_ptr() for g in grads])
    _lib.check(lib.anr_anim_step(ctypes.byref(p), gp, ctypes.byref(c.frame), _lib.ptr(c.wpts), n0, _lib.ptr(c.tpts),
                                 n1, ctypes.byref(c.opts), _lib.ptr(loss3), _lib.ptr(ws), nbytes,
                                 _lib.stream_ptr(c.dev)), 'anr_anim_step')
    return c


class _AnimLoss(torch.autograd.Function):
    """forward = anr_anim_step (loss + gradients in one pass); backward hands out the gradients."""

    @staticmethod
    def forward(ctx, renderer, batch, wvals, tvals, *novel):
        grads = [torch.zeros_like(t) for t in novel]
        loss3 = torch.zeros(3, device=novel[0].device)
        anim_step(renderer, batch, grads, loss3, wvals, tvals)
        ctx.grads = grads
        return loss3[0], loss3[1], loss3[2]

    @staticmethod
    def backward(ctx, d_loss, d_l0, d_l1):
        # loss = l0 + l1 is the only differentiated output in the reference (loss.backward())
        return (None, None, None, None, *[g * d_loss for g in ctx.grads])


class NetworkWrapper(torch.nn.Module):
    """aninerf_animation_trainer.NetworkWrapper (:11-60)."""

    def __init__(self, net, cfg=None):
        super().__init__()
        self.net = net
        self.renderer = Renderer(net, cfg)
        for prm in self.net.parameters():
            prm.requires_grad = False
        for prm in self.net.novel_pose_bw.parameters():
            prm.requires_grad = True

    def forward(self, batch, wvals=None, tvals=None):
        wvals = sample_unit() if wvals is None else wvals
        tvals = sample_unit() if tvals is None else tvals
        loss, l0, l1 = _AnimLoss.apply(self.renderer, batch, wvals, tvals, *self.net.novel_tensors())
        scalar_stats = {'bw_loss0': l0, 'bw_loss1': l1, 'loss': loss}
        return {}, loss, scalar_stats, {}


class AnimationStep:
    """Native animation-stage step: ``step(batch)`` = anr_anim_step + [all-reduce] + clip + Adam on
    the novel_pose_bw blob (optimizer.py:12-27 groups, trainer.py:64-68 clip_grad_value_(40))."""

    def __init__(self, net, cfg=None, lr=None, clip=40.0, betas=(0.9, 0.999), eps=1e-8, group=None):
        self.cfg = cfg if cfg is not None else _config.active()
        self.net = net
        self.renderer = Renderer(net, self.cfg)
        self.lib = self.renderer.lib
        self.lr = float(self.cfg.train.lr if lr is None else lr)
        self.wd = float(self.cfg.train.weight_decay)
        self.clip, self.betas, self.eps, self.group = clip, betas, eps, group
        ps = net.novel_tensors()
        if not ps:
            raise RuntimeError('animation stage needs net.novel_pose_bw (cfg.aninerf_animation = True)')
        dev = ps[0].device
        n = sum(p.numel() for p in ps)
        self.flat = torch.empty(n, device=dev)
        self.grad = torch.zeros(n, device=dev)
        self.m = torch.zeros(n, device=dev)
        self.v = torch.zeros(n, device=dev)
        self.grad_views = []
        off = 0
        for p in ps:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            self.grad_views.append(self.grad[off:off + k].view_as(p))
            off += k
        self.n, self.t = n, 0
        self.loss3 = torch.zeros(3, device=dev)
        broadcast_(self.flat, 0, group)  # DDP semantics: start every replica from rank 0's weights

    def step(self, batch, wvals=None, tvals=None, lr=None):
        wvals = sample_unit() if wvals is None else wvals
        tvals = sample_unit() if tvals is None else tvals
        self.grad.zero_()
        anim_step(self.renderer, batch, self.grad_views, self.loss3, wvals, tvals)
        allreduce_mean_(self.grad, self.group)
        self.t += 1
        _lib.check(self.lib.anr_adam(_lib.ptr(self.flat), _lib.ptr(self.grad), _lib.ptr(self.m), _lib.ptr(self.v),
                                     self.n, float(self.lr if lr is None else lr), self.betas[0], self.betas[1],
                                     self.eps, self.wd, self.t, self.clip, _lib.stream_ptr(self.flat.device)),
                   'anr_adam')
        self.net._anr_weights_epoch = getattr(self.net, '_anr_weights_epoch', 0) + 1
        return self.loss3
