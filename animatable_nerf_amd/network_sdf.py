"""sdf_pdf network plugin (config 5) with the reference parameter layout
(``lib/networks/bw_deform/anisdf_pdf_network.py:13-36, 253-269, 340-520``).

Like ``network.Network`` the modules own the parameters under the reference state_dict names,
shapes and order (so ``load_network(strict=True)`` reads a reference ``latest.pth``); the render runs
in the HIP library (``renderer_sdf.Renderer``), and ``Network.forward(wpts, viewdir, dists, batch)`` --
the per-chunk call of a reference ``tpose_renderer`` -- runs there too. Weight-normed layers keep the ``weight_g`` /
``weight_v`` pair of ``nn.utils.weight_norm``; the effective weight ``v * (g / |v|_row)`` is formed
on the device per render call.
"""
import torch
import torch.nn as nn

from . import config as _config


class WNLinear(nn.Module):
    """``nn.utils.weight_norm(nn.Linear(i, o))``: parameters bias, weight_g (o,1), weight_v (o,i)."""

    def __init__(self, i, o):
        super().__init__()
        self.bias = nn.Parameter(torch.zeros(o))
        self.weight_g = nn.Parameter(torch.ones(o, 1))
        self.weight_v = nn.Parameter(torch.zeros(o, i))


class SDFNetwork(nn.Module):
    """anisdf_pdf_network.py:340-453: gamma_6 (39) -> 8 x 256 softplus(beta 100), lin3 out 217,
    skip [x, gamma]/sqrt(2) into lin4, lin8 -> 1 + 256. Callable like the reference module
    (``sdf_network(x, batch)``, ``.sdf``, ``.gradient``) on the HIP library through the owning Network
    (the device call needs the whole parameter set; exact fp32 products, no autograd)."""
    DIMS = [(39, 256), (256, 256), (256, 256), (256, 217), (256, 256), (256, 256), (256, 256), (256, 256),
            (256, 257)]

    def __init__(self):
        super().__init__()
        for l, (i, o) in enumerate(self.DIMS):
            setattr(self, f'lin{l}', WNLinear(i, o))

    def __getstate__(self):
        state = dict(super().__getstate__())
        state.pop('_anr_owner', None)  # re-linked by the owning Network's __setstate__
        return state

    def _owner(self):
        own = self.__dict__.get('_anr_owner')
        net = own() if own is not None else None
        if net is None:
            raise RuntimeError('SDFNetwork: not part of a network_sdf.Network (the device call needs its parameters)')
        return net

    def forward(self, inputs, batch):
        """(n,3) points -> (n,257) [sdf || feature vector] (:421-437)"""
        from . import _lib
        return self._owner()._device().points(inputs, batch, _lib.SDFP_NETWORK)

    def sdf(self, x, batch):
        return self.forward(x, batch)[:, :1]

    def gradient(self, x, batch):
        """d sdf / d x -> (n,1,3) (:441-451)"""
        from . import _lib
        g, _ = self._owner()._device().points(x, batch, _lib.SDFP_GRADIENT)
        return g.unsqueeze(1)


class BetaNetwork(nn.Module):
    def __init__(self):
        super().__init__()
        self.register_parameter('beta', nn.Parameter(torch.tensor(0.1)))


class ColorNetwork(nn.Module):
    """anisdf_pdf_network.py:468-520 (mode 'idr'): 289 -> 256 -> 256 -> 256 || latent 128 -> 256 -> 3."""

    def __init__(self, num_latent_code):
        super().__init__()
        self.color_latent = nn.Embedding(num_latent_code, 128)
        for l, (i, o) in enumerate([(289, 256), (256, 256), (256, 256), (384, 256), (256, 3)]):
            setattr(self, f'lin{l}', WNLinear(i, o))


class TPoseHuman(nn.Module):
    def __init__(self, num_latent_code):
        super().__init__()
        self.sdf_network = SDFNetwork()
        self.beta_network = BetaNetwork()
        self.color_network = ColorNetwork(num_latent_code)


class Network(nn.Module):
    """anisdf_pdf_network.Network: tpose_human + resd_latent + resd_linears (135 -> 8 x 256, skip
    391 at 5) + resd_fc."""

    TENSOR_ORDER_LEN = 63

    def __init__(self, cfg=None):
        super().__init__()
        cfg = cfg if cfg is not None else _config.active()
        self.__dict__['_anr_cfg'] = cfg
        nlc = int(cfg.get('num_latent_code', -1))
        if nlc < 0:
            nlc = int(cfg.num_train_frame)  # config.py:144-145
        self.tpose_human = TPoseHuman(nlc)
        self.resd_latent = nn.Embedding(nlc, 128)
        self.actvn = nn.ReLU()
        self.skips = [4]
        self.resd_linears = nn.ModuleList([nn.Conv1d(135, 256, 1)] + [
            nn.Conv1d(256 + 135 if i in self.skips else 256, 256, 1) for i in range(7)])
        self.resd_fc = nn.Conv1d(256, 3, 1)
        self.resd_fc.bias.data.fill_(0)
        import weakref
        self.tpose_human.sdf_network.__dict__['_anr_owner'] = weakref.ref(self)

    def tensors(self):
        """The 63 tensors of the C-ABI order (include/aninerf.h ``anr_sdf_params``) = state_dict order."""
        ts = [t for _, t in self.named_parameters()]
        assert len(ts) == self.TENSOR_ORDER_LEN, len(ts)
        return ts

    def __getstate__(self):
        state = dict(super().__getstate__())
        state.pop('_anr_renderer', None)  # a copy builds its own device renderer
        return state

    def __setstate__(self, state):
        super().__setstate__(state)
        import weakref
        self.tpose_human.sdf_network.__dict__['_anr_owner'] = weakref.ref(self)

    def _device(self):
        r = self.__dict__.get('_anr_renderer')
        if r is None:
            from .renderer_sdf import Renderer
            r = Renderer(self, self.__dict__['_anr_cfg'])
            self.__dict__['_anr_renderer'] = r
        return r

    # ---- helper methods a reference renderer calls (sdf_mesh_renderer.py:16-110) ---------------------
    def gradient_of_deformed_sdf(self, x, batch):
        """:140-154: x (1,n,3) big-pose points -> (gradients (1,n,3) of sdf(x + resd(x)) w.r.t. x, sdf (1,n,1))"""
        from . import _lib
        g, sdf = self._device().points(x.reshape(-1, 3), batch, _lib.SDFP_DEFORMED_GRADIENT)
        return g[None], sdf[None]

    def calculate_bigpose_smpl_bw(self, bigpose, input_bw):
        """:109-112 = pts_sample_blend_weights(bigpose, input_bw['tbw'], input_bw['tbounds']) -> (1,25,n)"""
        from . import _lib
        r = self._device()
        dev = r.device()
        pts = bigpose.to(device=dev, dtype=torch.float32).reshape(-1, 3).contiguous()
        vol = input_bw['tbw'].to(device=dev, dtype=torch.float32).contiguous()  # (1, X, Y, Z, C)
        bounds = input_bw['tbounds'].to(device=dev, dtype=torch.float32).reshape(2, 3).contiguous()
        X, Y, Z, C = (int(v) for v in vol.shape[1:])
        n = pts.shape[0]
        out = torch.empty((C, n), device=dev)
        _lib.check(r.lib.anr_sample_volume(_lib.ptr(vol), X, Y, Z, C, _lib.ptr(bounds), _lib.ptr(pts), n, _lib.ptr(out),
                                           _lib.stream_ptr(dev)), 'anr_sample_volume')
        return out[None]

    def get_sdf(self, wpts, batch):
        """:226-257: sdf (n,1) of world points (10 where the KNN prefilter drops them: pnorm >= 0.1 except the
        call's argmin) — the eval network call's sdf output; batch['tbounds'] is left as it was."""
        tb = batch['tbounds'].clone()
        n = wpts.reshape(-1, 3).shape[0]
        with torch.no_grad():
            z = torch.zeros((n, 3), device=wpts.device, dtype=torch.float32)
            ret = self._device().network_forward(wpts.reshape(-1, 3), z, torch.zeros(n, device=wpts.device), batch)
            batch['tbounds'].copy_(tb)
        return ret['sdf'].reshape(-1, 1)

    def forward(self, wpts, viewdir, dists, batch):
        """anisdf_pdf_network.py:156-224: one reference network call over n free samples (the call
        tpose_renderer.py:95 makes per chunk) -> {'raw' (1,n,4), 'sdf' (1,n,1), 'resd' (1,n',3), 'gradients'
        (1,n',3)} (+ 'observed_gradients' under autograd); widens batch['tbounds'] in place. On the HIP
        library (renderer_sdf.Renderer.network_forward); differentiable w.r.t. the parameters when training."""
        return self._device().network_forward(wpts, viewdir, dists, batch)
