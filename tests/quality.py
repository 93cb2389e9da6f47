"""Config 3 quality gate (test infrastructure; used by tests/test_gpu_config3.py and tools/train_quality.py).

north_star: config 3 (aninerf_313 training, bf16) must reach a PSNR within 0.05 dB of the fp32
training. Every precision starts from the same weights (synthetic.init_state_dict, seed 1234) and sees
the same ray batches and stratification draws per seed; the target is a view-dependent procedural
texture over a 512 x 512 box-ray frame (H = W = 1024 at ratio 0.5, configs/aninerf_313.yaml:23-25).
After K FusedStep iterations (tpose_trainer losses, clip 40, Adam) the held-out rays (the last
``eval_rays`` of the frame, never trained on) are rendered by the fp32 eval path and scored with the
A18 formula (lib/evaluators/if_nerf.py:15-18, ``oracle.restate.psnr``: numpy mean of the squared error,
-10 log(mse) / log(10)).
"""
import numpy as np
import torch

from animatable_nerf_amd import config, network, synthetic
from animatable_nerf_amd.renderer import Renderer, near_far
from animatable_nerf_amd.trainer import FusedStep

RAY_KEYS = ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb')


def make_net(cfg, seed, dev):
    net = network.Network(cfg)
    sd = synthetic.init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()}, seed=seed)
    network.load_numpy_state(net, sd)
    return net.to(dev)


def sub(batch, idx, rgb=None):
    out = {k: (v[:, idx] if k in RAY_KEYS else v) for k, v in batch.items()}
    if rgb is not None:
        out['rgb'] = rgb[None]
    return out


def frame(dev, frame_rays=512 * 512, latent_index=7, tex_freq=(9.0, 7.0)):
    """(batch of the frame's in-box rays on ``dev``, target rgb (R, 3))"""
    sc = synthetic.Scene(vsize=0.025)
    ro, rd = sc.box_rays(frame_rays, seed=2)
    nr, fr, m = near_far(torch.from_numpy(sc.bounds).to(dev), torch.from_numpy(ro).to(dev), torch.from_numpy(rd).to(dev))
    m_np = m.cpu().numpy()
    b = sc.batch_arrays(ro[m_np], rd[m_np], nr.cpu().numpy(), fr.cpu().numpy(), latent_index=latent_index)
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()}
    d = batch['ray_d'][0]
    c = torch.arange(3, device=dev, dtype=torch.float32)
    fx, fy = tex_freq
    gt = 0.5 + 0.45 * torch.sin(fx * d[:, :1] + 11.0 * c) * torch.cos(fy * d[:, 1:2] + 7.0 * c)
    return batch, gt


def psnr(pred, gt):
    """lib/evaluators/if_nerf.py:15-18 on host float32 arrays."""
    from oracle import restate
    return float(restate.psnr(pred.detach().cpu().numpy(), gt.detach().cpu().numpy()))


def train_psnr(dev, subject='aninerf_313', precisions=('fp32', 'bf16', 'bf16_all'), seeds=3, steps=500, rays=1024,
               eval_rays=16384, frame_rays=512 * 512, init_seed=1234, log=None):
    """-> {precision: {'psnr': [per seed], 'losses': [...]}, '_init': psnr of the initial weights}"""
    batch, gt = frame(dev, frame_rays)
    R = int(batch['ray_o'].shape[1])
    n_train = R - eval_rays
    ev = torch.arange(n_train, R, device=dev)
    ecfg = config.subject(subject, perturb=0)
    out = {}
    g = torch.Generator(device=dev)
    for prec in precisions:
        res = {'psnr': [], 'losses': []}
        for seed in range(seeds):
            cfg = config.subject(subject, perturb=1, train_precision=prec.split('#')[0])
            net = make_net(cfg, init_seed, dev)
            net.train()
            step = FusedStep(net, cfg)
            g.manual_seed(5 + 1000 * seed)
            for it in range(steps):
                idx = torch.randint(0, n_train, (rays,), device=dev, generator=g)
                t_rand = torch.rand((rays, 64), device=dev, generator=g)
                l3 = step.step(sub(batch, idx, gt[idx]), t_rand=t_rand)
            res['losses'].append(l3[:3].cpu().tolist())
            with torch.no_grad():
                pred = Renderer(net, ecfg).render_device(sub(batch, ev), bw_rows=False)['rgb_map'][0]
            res['psnr'].append(psnr(pred, gt[ev]))
            if log is not None:
                log(f'{prec} seed {seed}: psnr {res["psnr"][-1]:.4f} loss {res["losses"][-1]}')
        out[prec] = res
    with torch.no_grad():
        init = make_net(ecfg, init_seed, dev)
        init.train()
        out['_init'] = psnr(Renderer(init, ecfg).render_device(sub(batch, ev), bw_rows=False)['rgb_map'][0], gt[ev])
    return out
