"""ORACLE — test infrastructure only. CPU (PyTorch-CPU) restatement of the reference sdf_pdf
variant's render path (config 5), op for op.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker. The product path never calls it.

Parity pin: checked against fixtures from the real reference (``oracle/gen_goldens.py --sdf`` ->
``tests/golden/g6_sdf_tiny.npz``, ``g7_sdf_chunks.npz``), with one exception: pytorch3d
``knn_points`` (v0.4.0 per ``INSTALL.md:28-33``) is neither vendored nor installed, so the reference
run uses ``knn_points`` below as its stub. **Parity at the KNN boundary is therefore unpinned**:
``knn_points`` restates pytorch3d's published CPU algorithm (exact squared L2 accumulated x, y, z
without FMA; a bounded max-heap with a strict ``<`` test, which keeps the K lexicographically
smallest (dist², index) pairs, returned ascending).

Weights: flat ``P`` dict with the reference state_dict names (``anisdf_pdf_network.py``).
Citations are into /root/reference.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import restate

CHUNK = restate.CHUNK


# --------------------------------------------------------------------------------------------
# B1: KNN blend weights -- sample_utils.py:309-348 (pytorch3d knn_points restated)
# --------------------------------------------------------------------------------------------
def knn_points(src, ref, K=5, block=2048):
    """-> (dists² (1,n,K) f32 ascending, idx (1,n,K) int64); ties broken by the lower index."""
    assert src.shape[0] == 1 and ref.shape[0] == 1
    s = src[0].float()
    r = ref[0].float()
    V = r.shape[0]
    d_out, i_out = [], []
    ar = torch.arange(V, dtype=torch.int64, device=s.device)
    for b in range(0, s.shape[0], block):
        p = s[b:b + block]
        dx = p[:, None, 0] - r[None, :, 0]
        dy = p[:, None, 1] - r[None, :, 1]
        dz = p[:, None, 2] - r[None, :, 2]
        d2 = (dx * dx + dy * dy) + dz * dz                      # (m, V) fp32, no contraction
        key = d2.view(torch.int32).to(torch.int64) * (1 << 20) + ar[None]  # d2 >= 0: bits are monotone
        k = torch.topk(key, K, dim=1, largest=False, sorted=True).values
        idx = k & ((1 << 20) - 1)
        d_out.append(torch.gather(d2, 1, idx))
        i_out.append(idx)
    return torch.cat(d_out)[None], torch.cat(i_out)[None]


def sample_blend_closest_points(src, ref, values, K=5, exp=1e-8):
    """sample_utils.py:323-348 -> blended weights (1,n,24), weighted distance (1,n,1)."""
    n_batch, n_points, _ = src.shape
    d2, vert_ids = knn_points(src, ref, K)
    d2 = d2.to(src.dtype)  # the neighbour search is fp32 (pytorch3d); an fp64 run blends in fp64
    dists = d2.sqrt()                                          # guard_knn_points :309-311
    values = values.view(-1, values.shape[-1])
    disp = 1 / (dists + exp)
    weights = disp / disp.sum(dim=-1, keepdim=True)
    dists = torch.einsum('ijk, ijk -> ij', dists, weights)
    sampled = torch.einsum('ijkl, ijk -> ijl', values[vert_ids], weights)
    return sampled.view(n_batch, n_points, -1), dists.view(n_batch, n_points, 1)


# --------------------------------------------------------------------------------------------
# B2: LBS pose -> T -> big pose, points and directions -- blend_utils.py:19-116
# --------------------------------------------------------------------------------------------
def _blend_A(bw, A):
    nb = bw.shape[0]
    return torch.bmm(bw.permute(0, 2, 1), A.view(nb, 24, -1)).view(nb, -1, 4, 4)


def world_dirs_to_pose_dirs(wdirs, R):
    return torch.matmul(wdirs, R)


def pose_dirs_to_tpose_dirs(ddirs, bw, A):
    Ab = _blend_A(bw, A)
    R_inv = torch.inverse(Ab[..., :3, :3])
    return torch.sum(R_inv * ddirs[:, :, None], dim=3)


def tpose_points_to_pose_points(pts, bw, A):
    Ab = _blend_A(bw, A)
    R = Ab[..., :3, :3]
    pts = torch.sum(R * pts[:, :, None], dim=3)
    return pts + Ab[..., :3, 3]


def tpose_dirs_to_pose_dirs(ddirs, bw, A):
    Ab = _blend_A(bw, A)
    return torch.sum(Ab[..., :3, :3] * ddirs[:, :, None], dim=3)


# --------------------------------------------------------------------------------------------
# B3: residual deformation MLP -- anisdf_pdf_network.py:49-73
# --------------------------------------------------------------------------------------------
def residual_deformation(P, x, poses):
    pts = restate.embed(x, 10).transpose(1, 2)                 # (1,63,n)
    lat = poses[..., None].expand(*poses.shape, pts.size(2))   # (1,72,n)
    feat = torch.cat((pts, lat), dim=1)
    net = feat
    for i in range(8):
        net = F.relu(restate._conv(P, f'resd_linears.{i}', net))
        if i == 4:
            net = torch.cat((feat, net), dim=1)
    resd = restate._conv(P, 'resd_fc', net).transpose(1, 2)
    return 0.05 * torch.tanh(resd)


# --------------------------------------------------------------------------------------------
# B4 / B5 / B6: SDF network, Laplace density, colour network -- anisdf_pdf_network.py:253-549
# --------------------------------------------------------------------------------------------
def _wn_linear(P, name, x):
    """nn.utils.weight_norm(nn.Linear): W = _weight_norm(v, g, dim 0)."""
    w = torch._weight_norm(P[name + '.weight_v'], P[name + '.weight_g'], 0)
    return F.linear(x, w, P[name + '.bias'])


def sdf_network(P, x):
    """SDFNetwork.forward :433-449: gamma_6, 9 weight-normed layers, Softplus(beta=100), skip at 4."""
    inputs = restate.embed(x, 6)
    h = inputs
    for l in range(9):
        if l == 4:
            h = torch.cat([h, inputs], 1) / np.sqrt(2)
        h = _wn_linear(P, f'tpose_human.sdf_network.lin{l}', h)
        if l < 8:
            h = F.softplus(h, beta=100)
    return torch.cat([h[:, :1] / 1, h[:, 1:]], dim=-1)


def sdf_to_alpha(sdf, beta):
    """TPoseHuman.sdf_to_alpha :271-286 (Laplace CDF density)."""
    x = -sdf
    ind0 = x <= 0
    val0 = 1 / beta * (0.5 * torch.exp(x[ind0] / beta))
    ind1 = x > 0
    val1 = 1 / beta * (1 - 0.5 * torch.exp(-x[ind1] / beta))
    val = torch.zeros_like(sdf)
    val[ind0] = val0
    val[ind1] = val1
    return val


def color_network(P, points, normals, view_dirs, feature, latent_index):
    """ColorNetwork.forward :522-549 (mode 'idr', squeeze_out)."""
    view_dirs = restate.embed(view_dirs, 4)
    x = torch.cat([points, view_dirs, normals, feature], dim=-1)
    pre = 'tpose_human.color_network.'
    net = F.relu(_wn_linear(P, pre + 'lin0', x))
    net = F.relu(_wn_linear(P, pre + 'lin1', net))
    net = F.relu(_wn_linear(P, pre + 'lin2', net))
    lat = F.embedding(latent_index, P[pre + 'color_latent.weight'])
    lat = lat.expand(net.size(0), lat.size(1))
    net = F.relu(_wn_linear(P, pre + 'lin3', torch.cat((net, lat), dim=1)))
    return torch.sigmoid(_wn_linear(P, pre + 'lin4', net))


def tpose_human(P, wpts, viewdir, batch):
    """TPoseHuman.forward :288-338 -> raw (n',4), sdf (n',1), gradients (n',3), feature (n',256)."""
    wpts = wpts.detach().requires_grad_()
    with torch.enable_grad():
        out = sdf_network(P, wpts)
        sdf = out[:, :1]
    feature = out[:, 1:]
    gradients = torch.autograd.grad(sdf, wpts, torch.ones_like(sdf), create_graph=False, retain_graph=True)[0]
    wpts = wpts.detach()
    beta = P['tpose_human.beta_network.beta'].clamp(1e-9, 1e6)
    alpha = sdf_to_alpha(sdf, beta)
    alpha = 1. - torch.exp(-F.relu(alpha[:, 0]) * 0.005)
    rgb = color_network(P, wpts, gradients, viewdir, feature, batch['latent_index'])
    raw = torch.cat((rgb, alpha[:, None]), dim=1)
    return {'raw': raw.detach(), 'sdf': sdf.detach(), 'gradients': gradients.detach(), 'feature': feature.detach()}


# --------------------------------------------------------------------------------------------
# Network.forward (eval) -- anisdf_pdf_network.py:156-223
# --------------------------------------------------------------------------------------------
def network_forward(P, wpts, viewdir, dists, batch, norm_th=0.1, trace=None):
    """-> {'raw' (1,n,4), 'sdf' (1,n,1), 'resd' (1,n',3), 'gradients' (1,n',3)}.

    NB ``batch['tbounds']`` is widened by 0.05 IN PLACE on every call (:203-205), exactly like the
    reference: chunk c of one render sees the bounds widened c+1 times.
    """
    wpts = wpts[None]
    pose_pts = restate.world_to_pose(wpts, batch['R'], batch['Th'])
    viewdir = viewdir[None]
    pose_dirs = world_dirs_to_pose_dirs(viewdir, batch['R'])
    with torch.no_grad():
        pbw, pnorm = sample_blend_closest_points(pose_pts, batch['pvertices'], batch['weights'])
        pnorm = pnorm[..., 0]
        pind = pnorm < norm_th
        pind[torch.arange(len(pnorm)), pnorm.argmin(dim=1)] = True
        pose_pts = pose_pts[pind][None]
        viewdir = viewdir[pind][None]
        pose_dirs = pose_dirs[pind][None]
    # pose_points_to_tpose_points :75-107 (tpose_viewdir True)
    pbw, _ = sample_blend_closest_points(pose_pts, batch['pvertices'], batch['weights'])
    pbw = pbw.permute(0, 2, 1)
    init_tpose = restate.lbs_to_tpose(pose_pts, pbw, batch['A'])
    init_bigpose = tpose_points_to_pose_points(init_tpose, pbw, batch['big_A'])
    resd = residual_deformation(P, init_bigpose, batch['poses'])
    tpose = init_bigpose + resd
    init_tdirs = pose_dirs_to_tpose_dirs(pose_dirs, pbw, batch['A'])
    tpose_dirs = tpose_dirs_to_pose_dirs(init_tdirs, pbw, batch['big_A'])
    tpose = tpose[0]
    viewdir = tpose_dirs[0]
    ret = tpose_human(P, tpose, viewdir, batch)
    tbounds = batch['tbounds'][0]
    tbounds[0] -= 0.05
    tbounds[1] += 0.05
    inside = tpose > tbounds[:1]
    inside = inside * (tpose < tbounds[1:])
    outside = torch.sum(inside, dim=1) != 3
    ret['raw'][outside] = 0
    n_batch, n_point = wpts.shape[:2]
    raw = torch.zeros([n_batch, n_point, 4]).to(wpts)
    raw[pind] = ret['raw']
    sdf = 10 * torch.ones([n_batch, n_point, 1]).to(wpts)
    sdf[pind] = ret['sdf']
    if trace is not None:
        trace.update(pnorm=pnorm, pind=pind, pbw=pbw, init_bigpose=init_bigpose, resd=resd, tpose=tpose,
                     tpose_dirs=viewdir, sdf_c=ret['sdf'], feature=ret['feature'], raw_c=ret['raw'],
                     tbounds=tbounds.clone())
    return {'raw': raw, 'sdf': sdf, 'resd': resd.detach(), 'gradients': ret['gradients'][None]}


def get_intersection_mask(sdf, z_vals):
    """nerf_net_utils.py:78-88."""
    sign = torch.sign(sdf[..., :-1] * sdf[..., 1:])
    ind = torch.min(sign * torch.arange(sign.size(2)).flip([0]).to(sign), dim=2)[1]
    sign = sign.min(dim=2)[0]
    return sign == -1, ind


def render_chunk(P, ray_o, ray_d, near, far, occ, batch, t_rand=None, n_samples=64, trace=None):
    """get_pixel_value with the sdf keys, tpose_renderer.py:71-157."""
    pts, z = restate.sample_points(ray_o, ray_d, near, far, n_samples, t_rand)
    nb, npix, ns = pts.shape[:3]
    wpts = pts.view(nb * npix * ns, -1)
    vd = ray_d[:, :, None].repeat(1, 1, ns, 1).contiguous().view(nb * npix * ns, -1)
    dists = z[..., 1:] - z[..., :-1]
    dists = torch.cat([dists, dists[..., -1:]], dim=2).view(nb * npix * ns)
    ret = network_forward(P, wpts, vd, dists, batch, trace=trace)
    raw = ret['raw'].reshape(-1, ns, 4)
    zf = z.view(-1, ns)
    rgb_map, acc, depth, w = restate.raw2outputs(raw, zf)
    out = {'raw': raw.view(nb, -1, 4), 'sdf': ret['sdf'], 'resd': ret['resd'], 'gradients': ret['gradients'],
           'rgb_map': rgb_map.view(nb, npix, -1), 'acc_map': acc.view(nb, npix), 'depth_map': depth.view(nb, npix)}
    sdf = ret['sdf'].view(nb, npix, ns)
    min_sdf = sdf.min(dim=2)[0]
    free_sdf = min_sdf[occ == 0]
    free_label = torch.zeros_like(free_sdf)
    imask, _ = get_intersection_mask(sdf, zf.view(nb, npix, ns))
    ind = (imask == False) * (occ == 1)  # noqa: E712
    s = min_sdf[ind]
    out['msk_sdf'] = torch.cat([s, free_sdf]).view(nb, -1)
    out['msk_label'] = torch.cat([torch.ones_like(s), free_label]).view(nb, -1)
    if trace is not None:
        trace.update(z=z, weights=w)
    return out


def render(P, batch, t_rand=None, n_samples=64, chunk=CHUNK, trace=None):
    """Renderer.render (tpose_renderer.py:159-186) over an sdf_pdf network (mutates batch['tbounds'])."""
    R = batch['ray_o'].shape[1]
    outs = []
    for i in range(0, R, chunk):
        tr = None if t_rand is None else t_rand[None, i:i + chunk]
        outs.append(render_chunk(P, batch['ray_o'][:, i:i + chunk], batch['ray_d'][:, i:i + chunk],
                                 batch['near'][:, i:i + chunk], batch['far'][:, i:i + chunk],
                                 batch['occupancy'][:, i:i + chunk], batch, t_rand=tr, n_samples=n_samples,
                                 trace=trace))
    return {k: torch.cat([o[k] for o in outs], dim=1) for k in outs[0]}


# --------------------------------------------------------------------------------------------
# Training (config 5's 8-GPU leg): tpose_trainer.NetworkWrapper over the sdf_pdf
# network -- Network.forward in training mode (anisdf_pdf_network.py:156-224: create_graph input
# gradients, observed_gradients :140-154 / :194-199), the renderer's msk_sdf lists
# (tpose_renderer.py:134-152) and the loss terms of tpose_trainer.py:21-73 + crit.sdf_mask_crit
# (crit.py:5-19). Differentiable w.r.t. every tensor of P (autograd, second order where the
# reference's is).
# --------------------------------------------------------------------------------------------
def tpose_human_train(P, wpts, viewdir, batch):
    """TPoseHuman.forward :288-345 under autograd: gradients with create_graph (the eikonal loss and
    the colour net's normals differentiate through them); the colour net sees detached points."""
    if not wpts.requires_grad:
        wpts = wpts.requires_grad_()
    with torch.enable_grad():
        out = sdf_network(P, wpts)
        sdf = out[:, :1]
    feature = out[:, 1:]
    gradients = torch.autograd.grad(sdf, wpts, torch.ones_like(sdf), create_graph=True, retain_graph=True,
                                    only_inputs=True)[0]
    wpts = wpts.detach()
    beta = P['tpose_human.beta_network.beta'].clamp(1e-9, 1e6)
    alpha = sdf_to_alpha(sdf, beta)
    alpha = 1. - torch.exp(-F.relu(alpha[:, 0]) * 0.005)
    rgb = color_network(P, wpts, gradients, viewdir, feature, batch['latent_index'])
    raw = torch.cat((rgb, alpha[:, None]), dim=1)
    return {'raw': raw, 'sdf': sdf, 'gradients': gradients}


def gradient_of_deformed_sdf(P, x, batch):
    """Network.gradient_of_deformed_sdf :140-154: d sdf(x + resd(x)) / d x, create_graph."""
    x = x.requires_grad_(True)
    with torch.enable_grad():
        resd = residual_deformation(P, x, batch['poses'])
        tpose = (x + resd)[0]
        y = sdf_network(P, tpose)[:, :1]
    g = torch.autograd.grad(y, x, torch.ones_like(y), create_graph=True, retain_graph=True, only_inputs=True)[0]
    return g, y[None]


def network_forward_train(P, wpts, viewdir, dists, batch, norm_th=0.1):
    """Network.forward :156-224 with grad enabled -> raw, sdf (full), resd, gradients
    (+ observed_gradients when a kept sample has |sdf| < 0.02). Widens batch['tbounds'] in place."""
    wpts = wpts[None]
    pose_pts = restate.world_to_pose(wpts, batch['R'], batch['Th'])
    viewdir = viewdir[None]
    pose_dirs = world_dirs_to_pose_dirs(viewdir, batch['R'])
    with torch.no_grad():
        pbw, pnorm = sample_blend_closest_points(pose_pts, batch['pvertices'], batch['weights'])
        pnorm = pnorm[..., 0]
        pind = pnorm < norm_th
        pind[torch.arange(len(pnorm)), pnorm.argmin(dim=1)] = True
        pose_pts = pose_pts[pind][None]
        viewdir = viewdir[pind][None]
        pose_dirs = pose_dirs[pind][None]
    pbw, _ = sample_blend_closest_points(pose_pts, batch['pvertices'], batch['weights'])
    pbw = pbw.permute(0, 2, 1)
    init_tpose = restate.lbs_to_tpose(pose_pts, pbw, batch['A'])
    init_bigpose = tpose_points_to_pose_points(init_tpose, pbw, batch['big_A'])
    resd = residual_deformation(P, init_bigpose, batch['poses'])
    tpose = init_bigpose + resd
    init_tdirs = pose_dirs_to_tpose_dirs(pose_dirs, pbw, batch['A'])
    tpose_dirs = tpose_dirs_to_pose_dirs(init_tdirs, pbw, batch['big_A'])
    tpose = tpose[0]
    ret = tpose_human_train(P, tpose, tpose_dirs[0], batch)
    ind = ret['sdf'][:, 0].detach().abs() < 0.02
    init_bigpose = init_bigpose[0][ind][None].detach().clone()
    if ret['raw'].requires_grad and ind.sum() != 0:
        og, _ = gradient_of_deformed_sdf(P, init_bigpose, batch)
        ret['observed_gradients'] = og
    tbounds = batch['tbounds'][0]
    tbounds[0] -= 0.05
    tbounds[1] += 0.05
    inside = tpose > tbounds[:1]
    inside = inside * (tpose < tbounds[1:])
    outside = torch.sum(inside, dim=1) != 3
    ret['raw'][outside] = 0
    n_batch, n_point = wpts.shape[:2]
    raw = torch.zeros([n_batch, n_point, 4]).to(wpts)
    raw[pind] = ret['raw']
    sdf = 10 * torch.ones([n_batch, n_point, 1]).to(wpts)
    sdf[pind] = ret['sdf']
    ret.update({'raw': raw, 'sdf': sdf, 'resd': resd, 'gradients': ret['gradients'][None]})
    return ret


def render_chunk_train(P, ray_o, ray_d, near, far, occ, batch, t_rand=None, n_samples=64):
    """get_pixel_value (tpose_renderer.py:71-157) over network_forward_train."""
    pts, z = restate.sample_points(ray_o, ray_d, near, far, n_samples, t_rand)
    nb, npix, ns = pts.shape[:3]
    wpts = pts.view(nb * npix * ns, -1)
    vd = ray_d[:, :, None].repeat(1, 1, ns, 1).contiguous().view(nb * npix * ns, -1)
    dists = z[..., 1:] - z[..., :-1]
    dists = torch.cat([dists, dists[..., -1:]], dim=2).view(nb * npix * ns)
    ret = network_forward_train(P, wpts, vd, dists, batch)
    raw = ret['raw'].reshape(-1, ns, 4)
    zf = z.view(-1, ns)
    rgb_map, acc, depth, w = restate.raw2outputs(raw, zf)
    out = {k: v for k, v in ret.items() if k in ('resd', 'gradients', 'observed_gradients')}
    out.update({'raw': raw.view(nb, -1, 4), 'sdf': ret['sdf'], 'rgb_map': rgb_map.view(nb, npix, -1),
                'acc_map': acc.view(nb, npix), 'depth_map': depth.view(nb, npix)})
    sdf = ret['sdf'].view(nb, npix, ns)
    min_sdf = sdf.min(dim=2)[0]
    free_sdf = min_sdf[occ == 0]
    free_label = torch.zeros_like(free_sdf)
    with torch.no_grad():
        imask, _ = get_intersection_mask(sdf, zf.view(nb, npix, ns))
    ind = (imask == False) * (occ == 1)  # noqa: E712
    s = min_sdf[ind]
    out['msk_sdf'] = torch.cat([s, free_sdf]).view(nb, -1)
    out['msk_label'] = torch.cat([torch.ones_like(s), free_label]).view(nb, -1)
    return out


def render_train(P, batch, t_rand=None, n_samples=64, chunk=CHUNK):
    """Renderer.render under autograd (mutates batch['tbounds'])."""
    R = batch['ray_o'].shape[1]
    outs = []
    for i in range(0, R, chunk):
        tr = None if t_rand is None else t_rand[None, i:i + chunk]
        outs.append(render_chunk_train(P, batch['ray_o'][:, i:i + chunk], batch['ray_d'][:, i:i + chunk],
                                       batch['near'][:, i:i + chunk], batch['far'][:, i:i + chunk],
                                       batch['occupancy'][:, i:i + chunk], batch, t_rand=tr, n_samples=n_samples))
    keys = outs[0].keys()
    return {k: torch.cat([o[k] for o in outs], dim=1) for k in keys}


def mask_alpha(iter_step):
    """crit.sdf_mask_crit's schedule (crit.py:9-14): 50, doubled past each milestone."""
    alpha = 50
    for m in (10000, 20000, 30000, 40000, 50000):
        if iter_step > m:
            alpha = alpha * 2
    return alpha


def loss_terms(ret, batch):
    """tpose_trainer.NetworkWrapper.forward :21-73 for the sdf_pdf keys -> (loss, scalar_stats)."""
    stats = {}
    loss = 0
    offset_loss = torch.norm(ret['resd'], dim=2).mean()
    stats['offset_loss'] = offset_loss
    loss += 0.01 * offset_loss
    grad_loss = ((torch.norm(ret['gradients'], dim=2) - 1.0) ** 2).mean()
    stats['grad_loss'] = grad_loss
    loss += 0.01 * grad_loss
    if 'observed_gradients' in ret:
        ograd_loss = ((torch.norm(ret['observed_gradients'], dim=2) - 1.0) ** 2).mean()
        stats['ograd_loss'] = ograd_loss
        loss += 0.01 * ograd_loss
    alpha = mask_alpha(int(batch['iter_step']))
    mask_loss = F.binary_cross_entropy_with_logits(-alpha * ret['msk_sdf'], ret['msk_label']) / alpha
    stats['mask_loss'] = mask_loss
    loss += mask_loss
    mask = batch['mask_at_box']
    img_loss = torch.mean((ret['rgb_map'][mask] - batch['rgb'][mask]) ** 2)
    stats['img_loss'] = img_loss
    loss += img_loss
    stats['loss'] = loss
    return loss, stats
