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
    skip [x, gamma]/sqrt(2) into lin4, lin8 -> 1 + 256."""
    DIMS = [(39, 256), (256, 256), (256, 256), (256, 217), (256, 256), (256, 256), (256, 256), (256, 256),
            (256, 257)]

    def __init__(self):
        super().__init__()
        for l, (i, o) in enumerate(self.DIMS):
            setattr(self, f'lin{l}', WNLinear(i, o))


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

    def tensors(self):
        """The 63 tensors of the C-ABI order (include/aninerf.h ``anr_sdf_params``) = state_dict order."""
        ts = [t for _, t in self.named_parameters()]
        assert len(ts) == self.TENSOR_ORDER_LEN, len(ts)
        return ts

    def __getstate__(self):
        state = dict(super().__getstate__())
        state.pop('_anr_renderer', None)  # a copy builds its own device renderer
        return state

    def _device(self):
        r = self.__dict__.get('_anr_renderer')
        if r is None:
            from .renderer_sdf import Renderer
            r = Renderer(self, self.__dict__['_anr_cfg'])
            self.__dict__['_anr_renderer'] = r
        return r

    def forward(self, wpts, viewdir, dists, batch):
        """anisdf_pdf_network.py:156-224: one reference network call over n free samples (the call
        tpose_renderer.py:95 makes per chunk) -> {'raw' (1,n,4), 'sdf' (1,n,1), 'resd' (1,n',3), 'gradients'
        (1,n',3)} (+ 'observed_gradients' under autograd); widens batch['tbounds'] in place. On the HIP
        library (renderer_sdf.Renderer.network_forward); differentiable w.r.t. the parameters when training."""
        return self._device().network_forward(wpts, viewdir, dists, batch)
