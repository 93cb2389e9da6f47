"""Trainer plugin for the sdf_pdf network (config 5): ``lib/train/trainers/tpose_trainer.py:11-73``
(the trainer ``configs/sdf_pdf/anisdf_pdf_s9p.yaml:13-14`` selects) with ``crit.sdf_mask_crit``
(``crit.py:5-19``), on the HIP library's fused training step ``anr_sdf_train_step``.

The reference differentiates through ``gradients = d sdf / d x`` (create_graph) and the
``observed_gradients`` of the deformed SDF: second-order terms that the device step evaluates
forward-over-reverse (anr_sdf_train.hip). One call returns the losses AND every parameter gradient:

* ``NetworkWrapper(net)`` — ``forward(batch) -> (ret, loss, scalar_stats, image_stats)`` with the
  reference's stats keys (offset_loss, grad_loss, ograd_loss when present, mask_loss, img_loss,
  loss); ``loss.backward()`` hands the precomputed gradients to the parameters (an autograd
  Function), so the reference ``Trainer.train`` loop (clip_grad_value_, Adam) runs unchanged.
  ``batch['iter_step']`` sets the mask-loss alpha schedule, as in the reference.
* ``SdfStep(net)`` — the native loop: the 63 tensors (1,432,510 floats) and their gradients in flat
  HBM blobs with the loss floats (LOSS_KEYS) in the gradient blob's tail, so one RCCL mean all-reduce carries
  gradients and losses (DDP semantics, trainer.py:13-18); then clip + Adam (``anr_adam``).
"""
import ctypes

import torch

from . import _lib
from . import config as _config
from .parallel import GradBuckets, broadcast_, is_dist
from .renderer_sdf import Renderer

COLOUR_TENSORS = (28, 44)  # color_network.* (colour latent, lin0..lin4 g / v / bias): final first
LOSS_KEYS = ('loss', 'offset_loss', 'grad_loss', 'ograd_loss', 'mask_loss', 'img_loss', 'n_observed', 'msk_len',
             'n_kept', 'reserved')
NLOSS = len(LOSS_KEYS)


def train_precision(cfg):
    """cfg.sdf_train_precision (anr_render_opts.precision of anr_sdf_train_step): 'fp32' exact fp32 MFMA
    layer GEMMs; 'bf16x3' the forward / input-gradient products as split-bf16 tiles and the weight
    gradients on the split-bf16 slab kernel (lo*bh + hi*bl + hi*bh, fp32 accumulation), held to the
    same tolerances by tests/test_gpu_sdf_train.py."""
    prec = cfg.get('sdf_train_precision', 'fp32')
    precs = {'fp32': _lib.FP32, 'bf16x3': _lib.BF16X3}
    if prec not in precs:
        raise ValueError(f"sdf_train_precision must be one of {sorted(precs)}, got {prec!r}")
    return precs[prec]


def sdf_train_step(renderer, batch, grads, loss8, t_rand=None, iter_step=None, hooks=None):
    """One anr_sdf_train_step: ACCUMULATES the gradients of the 63 tensors into ``grads`` (list,
    state_dict order) and writes the NLOSS loss floats into ``loss8`` (device, no host sync of its own).
    Returns {'rgb_map', 'acc_map', 'depth_map'} and widens ``batch['tbounds']`` in place.
    ``hooks`` (_lib.SdfTrainHooks or None): the event / host callback of anr_sdf_train_step_hooked once
    the colour net's gradients (tensors COLOUR_TENSORS) are final."""
    lib = renderer.lib
    c = renderer.prepare(batch, t_rand)
    dev, R, rays, o = c['dev'], c['R'], c['rays'], c['opts']
    o.precision = train_precision(renderer.cfg)
    rgb = torch.empty((1, R, 3), device=dev)
    acc = torch.empty((1, R), device=dev)
    depth = torch.empty((1, R), device=dev)
    tb_out = torch.empty((2, 3), device=dev)
    out = _lib.SdfRenderOut(rgb.data_ptr(), acc.data_ptr(), depth.data_ptr(), None, None, tb_out.data_ptr())
    gt = batch['rgb'].to(device=dev, dtype=torch.float32).contiguous()
    mask = batch.get('mask_at_box')
    mask = None if mask is None else mask.to(device=dev).reshape(-1).to(torch.uint8).contiguous()
    it = int(batch.get('iter_step', 0) if iter_step is None else iter_step)
    nbytes = lib.anr_sdf_train_workspace_bytes(R, ctypes.byref(o))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    gp = (ctypes.c_void_p * _lib.NUM_SDF_TENSORS)(*[None if g is None else g.data_ptr() for g in grads])
    _lib.check(lib.anr_sdf_train_step_hooked(ctypes.byref(c['p']), gp, ctypes.byref(c['frame']),
                                             *[_lib.ptr(rays[k]) for k in ('ray_o', 'ray_d', 'near', 'far')], R,
                                             ctypes.byref(o), _lib.ptr(gt), _lib.ptr(mask), it, ctypes.byref(out),
                                             _lib.ptr(loss8), None if hooks is None else ctypes.byref(hooks),
                                             _lib.ptr(ws), nbytes, _lib.stream_ptr(dev)),
               'anr_sdf_train_step')
    with torch.no_grad():
        batch['tbounds'].copy_(tb_out.view_as(batch['tbounds']))
    return {'rgb_map': rgb, 'acc_map': acc, 'depth_map': depth}


class _SdfLoss(torch.autograd.Function):
    """forward = anr_sdf_train_step (losses + gradients in one pass); backward hands out the gradients
    (the loss is the only differentiated output in the reference: loss.backward())."""

    @staticmethod
    def forward(ctx, renderer, batch, t_rand, *params):
        grads = [torch.zeros_like(t) for t in params]
        loss8 = torch.zeros(NLOSS, device=params[0].device)
        renderer.last_ret = sdf_train_step(renderer, batch, grads, loss8, t_rand)
        ctx.grads = grads
        return tuple(loss8[k] for k in range(6)) + (loss8[6:].detach().clone(),)

    @staticmethod
    def backward(ctx, d_loss, *_):
        return (None, None, None, *[g * d_loss for g in ctx.grads])


class NetworkWrapper(torch.nn.Module):
    """tpose_trainer.NetworkWrapper (:11-73) over the sdf_pdf network."""

    def __init__(self, net, cfg=None):
        super().__init__()
        self.net = net
        self.renderer = Renderer(net, cfg)

    def forward(self, batch, t_rand=None):
        outs = _SdfLoss.apply(self.renderer, batch, t_rand, *self.net.tensors())
        loss, offset, grad, ograd, mask, img, counts = outs
        stats = {'offset_loss': offset, 'grad_loss': grad}
        if int(counts[0]) > 0:  # the reference's ret has 'observed_gradients' only then
            stats['ograd_loss'] = ograd
        stats.update({'mask_loss': mask, 'img_loss': img, 'loss': loss})
        return self.renderer.last_ret, loss, stats, {}


class SdfStep:
    """Native sdf_pdf training step: ``step(batch)`` = anr_sdf_train_step + [RCCL mean all-reduce of
    the gradient blob with the losses in its tail] + clip_grad_value_(40) + Adam (optimizer.py:12-27,
    trainer.py:64-68). Returns the device loss vector (LOSS_KEYS order): with N > 1 ranks every entry
    is the MEAN over the ranks, the count entries too (n_observed, msk_len, n_kept are then per-rank
    averages, not totals: multiply by the world size for the job's counts).

    The all-reduce runs in buckets as DDP's reducer does (trainer.py:13-18): bucket 0, the colour
    net's gradients, leaves on the side stream as soon as the library records them final (after the
    colour backward, ~1/5 of the blob) while the SDF / residual / observed-gradient backward still
    runs; the rest (SDF net, beta, residual net, losses) follows the step."""

    def __init__(self, net, cfg=None, lr=None, clip=40.0, betas=(0.9, 0.999), eps=1e-8, group=None):
        self.cfg = cfg if cfg is not None else _config.active()
        self.net = net
        self.renderer = Renderer(net, self.cfg)
        self.lib = self.renderer.lib
        self.lr = float(self.cfg.train.lr if lr is None else lr)
        self.wd = float(self.cfg.train.weight_decay)
        self.clip, self.betas, self.eps, self.group = clip, betas, eps, group
        ps = net.tensors()
        dev = ps[0].device
        n = sum(p.numel() for p in ps)
        self.flat = torch.empty(n, device=dev)
        self.grad = torch.zeros(n + NLOSS, device=dev)
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
        self.loss8 = self.grad[n:n + NLOSS]
        offs = [0]
        for p in ps:
            offs.append(offs[-1] + p.numel())
        c0, c1 = offs[COLOUR_TENSORS[0]], offs[COLOUR_TENSORS[1]]
        self.buckets = GradBuckets(self.grad, [(c0, c1), (0, c0), (c1, n + NLOSS)], group)
        self.colour_ready = None
        self._hooks = None
        if dev.type == 'cuda':
            self.colour_ready = torch.cuda.Event()
            self.colour_ready.record()  # creates the underlying hipEvent (re-recorded by the library)
            self._ready_cb = _lib.READY_FN(self._colour_ready_hook)  # kept alive with the step
            self._hooks = _lib.SdfTrainHooks(colour_grads_ready=self.colour_ready.cuda_event,
                                             colour_ready=self._ready_cb)
        self.iter_step = 0
        broadcast_(self.flat, 0, group)  # DDP semantics: every replica starts from rank 0's weights

    def _colour_ready_hook(self, user, event, stream):
        """anr_sdf_train_hooks.colour_ready: called by the library mid-step, right after it recorded
        self.colour_ready; bucket 0's collective is issued on the side stream behind that event and runs
        beside the rest of the backward."""
        try:
            self.buckets.reduce(0, self.colour_ready)
            self._issued = True
            return 0
        except Exception:  # pragma: no cover - surfaced as the call's error
            import traceback
            traceback.print_exc()
            return 1

    def step(self, batch, t_rand=None, lr=None):
        self.grad.zero_()
        it = int(batch.get('iter_step', self.iter_step))
        self._issued = False
        sdf_train_step(self.renderer, batch, self.grad_views, self.loss8, t_rand, iter_step=it,
                       hooks=self._hooks if is_dist() else None)
        if not self._issued:  # CPU blob / one rank / the hook not reached (no kept sample)
            self.buckets.reduce(0)
        self.buckets.reduce(1)
        self.buckets.reduce(2)
        self.buckets.wait()
        self.t += 1
        self.iter_step += 1
        _lib.check(self.lib.anr_adam(_lib.ptr(self.flat), _lib.ptr(self.grad), _lib.ptr(self.m), _lib.ptr(self.v),
                                     self.n, float(self.lr if lr is None else lr), self.betas[0], self.betas[1],
                                     self.eps, self.wd, self.t, self.clip, _lib.stream_ptr(self.flat.device)),
                   'anr_adam')
        return self.loss8
