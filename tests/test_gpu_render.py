"""GPU parity: the HIP render path (through the C-ABI) against the reference goldens and the
oracle, plus size-independent properties at the full config-2 size.

Tolerances (BASELINE.json north_star): ray hit mask, sample keep mask and near/far bit-exact;
rendered rgb / acc / depth / raw and blend-weight rows within 1e-4 absolute (fp32).
"""
import numpy as np
import pytest
import torch

from oracle import restate

from ._common import batch_np, golden, make_net, oracle_params, scene, to_torch

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    return torch.device('cuda:0')


@pytest.fixture(scope='module', params=['fp32', 'bf16x3', 'bf16x6'])
def renderer(dev, request):
    """Every render precision is held to the same fp32 tolerance (north_star): exact fp32 MFMA, the
    hi/lo-split bf16 MFMA (include/aninerf.h ANR_BF16X3) and the hi/mid/lo-split bf16x6 MFMA
    (ANR_BF16X6, fp32-level products)."""
    from animatable_nerf_amd.renderer import Renderer
    net = make_net(dev)
    net.train()  # run.py evaluates in train() mode with perturb = 0
    from animatable_nerf_amd import config
    cfg = config.defaults()
    cfg.perturb = 0
    cfg.render_precision = request.param
    return Renderer(net, cfg)


def _keep(raw):
    return (raw[0, :, :3].abs().sum(-1) != 0)


def test_near_far_bit_exact(dev):
    from animatable_nerf_amd.renderer import near_far
    g = golden('g3_hits')
    nr, fr, m = near_far(torch.from_numpy(g['bounds']).to(dev), torch.from_numpy(g['ray_o']).to(dev),
                         torch.from_numpy(g['ray_d']).to(dev))
    assert np.array_equal(m.cpu().numpy(), g['mask'])
    assert np.array_equal(nr.cpu().numpy(), g['near'])
    assert np.array_equal(fr.cpu().numpy(), g['far'])


def test_g1_render_matches_reference(renderer, dev):
    g = golden('g1_tiny')
    sc = scene(0.05)
    ro, rd = sc.box_rays(64, seed=2)
    b, _ = batch_np(sc, ro, rd)
    ret = renderer.render_device(to_torch(b, dev))
    ret = {k: v.cpu() for k, v in ret.items()}
    assert torch.equal(_keep(ret['raw']), torch.from_numpy(g['out_raw'][0, :, :3].sum(-1) != 0))
    for k in ('rgb_map', 'acc_map', 'depth_map', 'raw'):
        err = (ret[k] - torch.from_numpy(g['out_' + k])).abs().max().item()
        assert err <= TOL, (k, err)
    assert ret['pbw'].shape == g['out_pbw'].shape
    assert (ret['pbw'] - torch.from_numpy(g['out_pbw'])).abs().max().item() <= TOL
    assert (ret['tbw'] - torch.from_numpy(g['out_tbw'])).abs().max().item() <= TOL


def test_g2_chunk_semantics(renderer, dev):
    g = golden('g2_chunks')
    sc = scene(0.05)
    b, _ = batch_np(sc, g['ray_o'], g['ray_d'])
    ret = renderer.render_device(to_torch(b, dev))
    keep = _keep(ret['raw']).cpu().numpy()
    assert np.array_equal(np.packbits(keep), g['keep_bits'])
    for k in ('rgb_map', 'acc_map', 'depth_map'):
        err = np.abs(ret[k].cpu().numpy() - g['out_' + k]).max()
        assert err <= TOL, (k, err)
    kept_alpha = ret['raw'][0, :, 3].cpu().numpy()[keep]
    assert np.abs(kept_alpha - g['kept_alpha']).max() <= TOL
    assert ret['pbw'].shape[1] == int(g['bw_rows'])
    idx = torch.from_numpy(g['bw_sample_idx']).to(dev)
    assert np.abs(ret['pbw'][0, idx].cpu().numpy() - g['pbw_sample']).max() <= TOL
    assert np.abs(ret['tbw'][0, idx].cpu().numpy() - g['tbw_sample']).max() <= TOL
    assert keep.reshape(-1, 64)[4096:].sum() == 1  # forced per-chunk argmin in the grazing chunk


def test_perturbed_sampling_matches_oracle(renderer, dev):
    """training-mode stratified z with a given t_rand (tpose_renderer.py:29-36), G4 rays"""
    g = golden('g4_train')
    sc = scene(0.05)
    b, _ = batch_np(sc, g['ray_o'], g['ray_d'])
    t_rand = torch.from_numpy(g['t_rand'])
    with torch.no_grad():
        ref = restate.render(oracle_params(), to_torch(b), t_rand=t_rand)
    ret = renderer.render_device(to_torch(b, dev), t_rand=t_rand.to(dev))
    assert torch.equal(_keep(ret['raw']).cpu(), _keep(ref['raw']))
    for k in ('rgb_map', 'acc_map', 'depth_map', 'raw'):
        err = (ret[k].cpu() - ref[k]).abs().max().item()
        assert err <= TOL, (k, err)


def test_multichunk_vs_oracle_fine_volume(renderer, dev):
    """5000 rays over 3 chunks on the 0.025 m volume (the bench scene)."""
    sc = scene(0.025)
    ro, rd = sc.box_rays(5000, seed=21)
    b, _ = batch_np(sc, ro, rd)
    with torch.no_grad():
        ref = restate.render(oracle_params(), to_torch(b))
    ret = renderer.render_device(to_torch(b, dev))
    assert torch.equal(_keep(ret['raw']).cpu(), _keep(ref['raw']))
    for k in ('rgb_map', 'acc_map', 'depth_map', 'raw'):
        err = (ret[k].cpu() - ref[k]).abs().max().item()
        assert err <= TOL, (k, err)
    assert ret['pbw'].shape == ref['pbw'].shape
    assert (ret['pbw'].cpu() - ref['pbw']).abs().max().item() <= TOL
    assert (ret['tbw'].cpu() - ref['tbw']).abs().max().item() <= TOL


def test_rotated_frame_vs_oracle(renderer, dev):
    """Non-identity R / Th (blend_utils.py:6-16 as torch's FMA-chain matmul): keep mask bit-exact,
    outputs within 1e-4 over 2 chunks."""
    from ._common import rotated_batch_np
    b = rotated_batch_np()
    with torch.no_grad():
        ref = restate.render(oracle_params(), to_torch(b))
    ret = renderer.render_device(to_torch(b, dev))
    assert torch.equal(_keep(ret['raw']).cpu(), _keep(ref['raw']))
    for k in ('rgb_map', 'acc_map', 'depth_map', 'raw', 'pbw', 'tbw'):
        assert ret[k].shape == ref[k].shape, k
        err = (ret[k].cpu() - ref[k]).abs().max().item()
        assert err <= TOL, (k, err)


def test_full_frame_properties(renderer, dev):
    """config 2 size (512x512 box rays): invariants that hold at any size."""
    sc = scene(0.025)
    ro, rd = sc.box_rays(512 * 512, seed=2)
    b, mask = batch_np(sc, ro, rd)
    assert mask.sum() >= 262140
    bt = to_torch(b, dev)
    r1 = renderer.render_device(bt)
    r2 = renderer.render_device(bt)
    for k in r1:  # deterministic
        assert torch.equal(r1[k], r2[k]), k
    raw = r1['raw'][0]
    keep = _keep(r1['raw'])
    assert torch.all(raw[~keep] == 0)
    frac = keep.float().mean().item()
    assert 0.25 < frac < 0.5, frac
    assert torch.all((r1['acc_map'] >= 0) & (r1['acc_map'] <= 1 + 1e-6))
    assert torch.all((r1['rgb_map'] >= 0) & (r1['rgb_map'] <= 1 + 1e-6))
    n_kept, m = renderer.last_counts
    assert n_kept == int(keep.sum().item())
    assert m == r1['pbw'].shape[1] and 0 < m <= n_kept
    s = torch.softmax(torch.zeros(1), 0)  # noqa: F841
    assert torch.allclose(r1['pbw'].sum(-1), torch.ones_like(r1['pbw'].sum(-1)), atol=1e-5)
    # a spot-check chunk against the oracle (chunk 60 of 128)
    i0 = 60 * 2048
    sub = {k: (v[:, i0:i0 + 2048] if k in ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb') else v)
           for k, v in b.items()}
    with torch.no_grad():
        ref = restate.render(oracle_params(), to_torch(sub))
    for k in ('rgb_map', 'acc_map', 'depth_map'):
        err = (r1[k][:, i0:i0 + 2048].cpu() - ref[k]).abs().max().item()
        assert err <= TOL, (k, err)


@pytest.mark.parametrize('precision', ['fp32', 'bf16x3', 'bf16x6'])
def test_novel_pose_render_matches_reference(dev, precision):
    """A19: cfg.test_novel_pose renders with novel_pose_bw + bw_latent_index (golden G5)."""
    from animatable_nerf_amd.renderer import Renderer
    from ._common import make_net_novel, novel_batch_np, novel_cfg
    g = golden('g5_novel_pose')
    net = make_net_novel(dev)
    net.train()
    ncfg = novel_cfg()
    ncfg.render_precision = precision
    r = Renderer(net, ncfg)
    ret = r.render_device(to_torch(novel_batch_np(), dev))
    ret = {k: v.cpu() for k, v in ret.items()}
    assert torch.equal(_keep(ret['raw']), torch.from_numpy(g['out_raw'][0, :, :3].sum(-1) != 0))
    for k in ('rgb_map', 'acc_map', 'depth_map', 'raw', 'pbw', 'tbw'):
        assert ret[k].shape == g['out_' + k].shape, k
        err = (ret[k] - torch.from_numpy(g['out_' + k])).abs().max().item()
        assert err <= TOL, (k, err)
    # the same network without the flag renders the training-pose path (different weights)
    cfg = novel_cfg()
    cfg.test_novel_pose = False
    cfg.render_precision = precision
    r2 = Renderer(net, cfg)
    ret2 = r2.render_device(to_torch(novel_batch_np(), dev))
    assert (ret2['rgb_map'].cpu() - ret['rgb_map']).abs().max().item() > 1e-3


def test_mmsk_visibility_filter_matches_reference(renderer, dev):
    """(f) tpose_renderer_mmsk: golden G9 (64 rays; 2 chunks, the second with no visible sample)."""
    from animatable_nerf_amd.renderer_mmsk import Renderer as MRenderer
    from ._common import mmsk_batch_np
    g = golden('g9_mmsk')
    r = MRenderer(renderer.net, renderer.cfg)
    sc = scene(0.05)
    ro, rd = sc.box_rays(64, seed=2)
    b, _ = mmsk_batch_np(ro, rd)
    ret = r.render(to_torch(b, dev))
    for k in ('rgb_map', 'acc_map', 'depth_map'):
        err = (ret[k] - torch.from_numpy(g['tiny_' + k])).abs().max().item()
        assert err <= TOL, (k, err)
    b, _ = mmsk_batch_np(g['chunks_ray_o'], g['chunks_ray_d'])
    ret = r.render_device(to_torch(b, dev), bw_rows=False)
    keep = _keep(ret['raw']).cpu().numpy()
    vis = np.unpackbits(g['chunks_inside_bits'])[:keep.size].astype(bool)
    assert not keep[~vis].any()  # kept samples are visible ones
    assert not keep[2048 * 64:].any()  # the chunk with no visible sample keeps nothing
    for k in ('rgb_map', 'acc_map', 'depth_map'):
        err = (ret[k].cpu() - torch.from_numpy(g['chunks_' + k])).abs().max().item()
        assert err <= TOL, (k, err)
    # the visibility-filtered keep set equals the oracle's
    tr = {}
    with torch.no_grad():
        restate.render_mmsk(oracle_params(), to_torch(b), trace=tr)
    ref_raw = torch.cat(tr['raw'], dim=1)
    assert torch.equal(_keep(ret['raw']).cpu(), _keep(ref_raw))


def test_render_overlapped_host_copy_equals_device_render(renderer, dev):
    """Renderer.render (the drop-in call, outputs on the host) renders a frame of >= 8 chunks in
    parts of whole chunks and copies each part to page-locked memory while the next renders: every
    output, the alpha_ind rows included, equals the one-call device render moved to the host."""
    sc = scene(0.025)
    ro, rd = sc.box_rays(9 * 2048 + 777, seed=4)
    b, _ = batch_np(sc, ro, rd)
    bt = to_torch(b, dev)
    full = renderer.render_device(bt)
    ref = {k: v.cpu() for k, v in full.items()}
    with torch.no_grad():  # as run.py evaluates (network in train() mode, perturb 0)
        got = renderer.render(bt)
    assert renderer.last_counts[1] == ref['pbw'].shape[1]
    for k in ('rgb_map', 'acc_map', 'depth_map', 'raw', 'pbw', 'tbw'):
        assert not got[k].is_cuda, k
        assert got[k].shape == ref[k].shape, (k, got[k].shape, ref[k].shape)
        assert torch.equal(got[k], ref[k]), k
    with torch.no_grad():
        again = renderer.render(bt)  # a second call does not overwrite the first call's outputs
    assert again['raw'].data_ptr() != got['raw'].data_ptr()
    assert torch.equal(got['raw'], ref['raw'])
    # the second call sizes the alpha_ind row buffers from the first's count (rows placed as parts
    # finish); a too-small estimate moves the placed rows into exact-size buffers, a far too large one
    # (a bigger frame's) is trimmed to exact size, and an estimate for another ray count is not used
    R = int(bt['ray_o'].shape[1])
    m = int(ref['pbw'].shape[1])
    for est in (None, (R, 1), (R, 40 * m + 100000), (R + 1, 1)):
        if est is not None:
            renderer._rows_est = est
        with torch.no_grad():
            again = renderer.render(bt)
        for k in ('rgb_map', 'acc_map', 'depth_map', 'raw', 'pbw', 'tbw'):
            assert got[k].shape == again[k].shape and torch.equal(again[k], ref[k]), (k, est)
        assert again['pbw'].is_contiguous() and again['pbw'].is_pinned()
        # no capacity-sized host allocation behind the returned rows
        assert again['pbw'].untyped_storage().nbytes() <= (2 * m + 4096 + 64) * 24 * 4 * 1.2, est
    # after render() (the frame in parts on two workspaces) the per-workspace queries refuse
    with pytest.raises(RuntimeError):
        renderer.row_ids(R)
    renderer.render_device(bt)
    assert renderer.row_ids(R).shape[0] == m


@pytest.mark.parametrize('world', [3, 8])
def test_frame_shards_equal_whole_frame(renderer, dev, world):
    """§8(e): one frame split over `world` ranks by whole chunks (parallel.shard_batch, as
    render_sharded does per rank), each shard rendered on its own: concatenated in rank order the
    rgb/acc/depth/raw equal the unsplit render bit for bit (per-chunk argmin/argmax and per-sample
    arithmetic do not depend on the split). The all-gather itself: tests/test_distributed.py."""
    from animatable_nerf_amd import parallel
    sc = scene(0.025)
    ro, rd = sc.box_rays(9 * 2048 + 777, seed=4)
    b, _ = batch_np(sc, ro, rd)
    bt = to_torch(b, dev)
    full = renderer.render_device(bt, bw_rows=False)
    parts = []
    for r in range(world):
        sub, (s, e) = parallel.shard_batch(bt, r, world)
        if e > s:
            parts.append(renderer.render_device(sub, bw_rows=False))
    for k in ('rgb_map', 'acc_map', 'depth_map', 'raw'):
        cat = torch.cat([p[k] for p in parts], dim=1)
        assert torch.equal(cat, full[k]), k


@pytest.mark.parametrize('split', ['bf16x6', 'bf16x3'])
def test_split_precisions_are_fp32_level(dev, split):
    """Against an fp64 evaluation of the same network (oracle/restate.py run in float64 on the same
    fp32 inputs), each split-bf16 render is as close as the reference's own fp32 arithmetic (the fp32
    oracle) and the exact fp32 MFMA kernel are — every output's max error within 1.5x the larger of
    those two (5000 rays, 3 chunks, fine volume). Measured (profiles/r3_precision_fp64.json): all
    four agree to within ~5 %: the shared fp32 inputs, sampling and blending set the error, not the
    MLP products (bf16x6 ~2^-23, bf16x3 ~2^-16 relative per product)."""
    from animatable_nerf_amd import config
    from animatable_nerf_amd.renderer import Renderer
    torch.set_num_threads(16)
    sc = scene(0.025)
    ro, rd = sc.box_rays(5000, seed=21)
    b, _ = batch_np(sc, ro, rd)
    with torch.no_grad():
        r32 = restate.render(oracle_params(), to_torch(b))
        p64 = {k: v.double() for k, v in oracle_params().items()}
        b64 = {k: (v.double() if v.dtype == torch.float32 else v) for k, v in to_torch(b).items()}
        r64 = restate.render(p64, b64)
    assert torch.equal(_keep(r32['raw']), _keep(r64['raw']))  # same samples, same rows
    net = make_net(dev)
    net.train()
    got = {}
    for prec in ('fp32', split):
        cfg = config.defaults()
        cfg.perturb = 0
        cfg.render_precision = prec
        ret = Renderer(net, cfg).render_device(to_torch(b, dev))
        got[prec] = {k: float((ret[k].cpu().double() - r64[k]).abs().max())
                     for k in ('rgb_map', 'acc_map', 'depth_map', 'raw', 'pbw', 'tbw')}
    ref_err = {k: float((r32[k].double() - r64[k]).abs().max()) for k in got['fp32']}
    for k, e in got[split].items():
        bar = 1.5 * max(ref_err[k], got['fp32'][k])
        assert e <= bar, (k, e, ref_err[k], got['fp32'][k])


def _conv_mm(P, name, x):
    """oracle/restate.py's Conv1d(k=1) as one GEMM (einsum -> rocBLAS): the same products and fp32 /
    fp64 accumulation, without MIOpen's per-shape kernel builds on a fresh box (the fp64 convolutions
    alone ran past the test's time limit)"""
    return torch.einsum('oc,bcn->bon', P[name + '.weight'][:, :, 0], x) + P[name + '.bias'][None, :, None]


class _RowTrace:
    """Wraps restate.network_forward during an oracle render and records, per reference chunk, the sample
    ids (frame order) of the alpha_ind rows and the pre-activation sigma' of every kept sample."""

    def __init__(self, fn, n_samples):
        self.fn, self.base, self.ids = fn, 0, []
        self.sig = torch.zeros(n_samples, dtype=torch.float64)
        self.margin = torch.full((n_samples,), float('inf'), dtype=torch.float64)

    def __call__(self, P, wpts, viewdir, dists, batch, trace=None, **kw):
        t = {}
        ret = self.fn(P, wpts, viewdir, dists, batch, trace=t, **kw)
        kept = torch.nonzero(t['pind'][0])[:, 0] + self.base
        self.ids.append(kept[t['alpha_ind'][0]])
        self.sig = self.sig.to(kept.device)
        self.margin = self.margin.to(kept.device)
        self.sig[kept] = t['sigma'][0].detach().double()
        # signed distance of the T-pose point to the nearest face of the strict bbox test (negative outside;
        # tpose_nerf_network.py:186-189)
        tp = t['tpose'][0].detach().double()
        lo, hi = batch['tbounds'][0, 0].double(), batch['tbounds'][0, 1].double()
        self.margin[kept] = torch.minimum(tp - lo, hi - tp).amin(-1)
        self.base += wpts.shape[0]
        return ret

    def row_ids(self):
        return torch.cat(self.ids)


def _match_rows(ids_a, ids_b):
    """positions (ia, ib) of the sample ids both row lists hold (each list strictly increasing), and the
    ids only one of them holds"""
    common, ia, ib = np.intersect1d(ids_a.cpu().numpy(), ids_b.cpu().numpy(), assume_unique=True, return_indices=True)
    only = np.setxor1d(ids_a.cpu().numpy(), ids_b.cpu().numpy(), assume_unique=True)
    return torch.from_numpy(ia), torch.from_numpy(ib), torch.from_numpy(only)


def test_split_precisions_fp32_level_full_frame(dev, monkeypatch):
    """A whole config-2 frame (512 x 512 box rays of the bench's scene, 128 chunks): the fp64 and fp32
    oracle evaluations run with PyTorch-ROCm on the GPU (oracle/restate.py on device tensors, its 1x1
    convolutions as GEMMs), the three device precisions are rendered from the same batch.

    * The device keep mask equals the fp32 oracle's (the reference's arithmetic) in every precision.
    * The exact fp32 kernel (the bench's value) is held to the north_star bar against the fp32 oracle
      over the WHOLE frame: rgb / acc / depth / raw within 1e-4 on every ray and sample, pbw / tbw within
      1e-4 on every alpha_ind row, rows matched by sample id (anr_render_row_ids); the alpha_ind row SET
      may differ only at samples whose sigma' is within 1e-4 of train_th (a threshold tie, not an error).
    * Against the fp64 evaluation (which may keep a few boundary samples differently: pnorm against
      norm_th), errors are taken over the rays whose 64 keep decisions agree in both oracle runs, rows
      matched by sample over the ids all runs share. bf16x6 (fp32-level products) must be within 1.5x the
      larger of the reference's own fp32 error and the exact kernel's; bf16x3 (~2^-16 relative products,
      not fp32-level by construction) is held to the 1e-4 bar on rgb / acc vs the fp64 evaluation."""
    from animatable_nerf_amd import config
    from animatable_nerf_amd.renderer import Renderer
    sc = scene(0.025)
    ro, rd = sc.box_rays(512 * 512, seed=2)
    b, _ = batch_np(sc, ro, rd)
    bd = to_torch(b, dev)
    N = int(bd['ray_o'].shape[1]) * 64
    monkeypatch.setattr(restate, '_conv', _conv_mm)
    fwd = restate.network_forward
    with torch.no_grad():
        p32 = {k: v.to(dev) for k, v in oracle_params().items()}
        t32 = _RowTrace(fwd, N)
        monkeypatch.setattr(restate, 'network_forward', t32)
        r32 = restate.render(p32, bd)
        p64 = {k: v.double() for k, v in p32.items()}
        b64 = {k: (v.double() if v.dtype == torch.float32 else v) for k, v in bd.items()}
        t64 = _RowTrace(fwd, N)
        monkeypatch.setattr(restate, 'network_forward', t64)
        r64 = restate.render(p64, b64)
        monkeypatch.setattr(restate, 'network_forward', fwd)
    ids32, ids64 = t32.row_ids(), t64.row_ids()
    assert ids32.numel() == r32['pbw'].shape[1] and ids64.numel() == r64['pbw'].shape[1]
    k32, k64 = _keep(r32['raw']), _keep(r64['raw'])
    R = k32.numel() // 64
    # rays whose 64 keep decisions agree in both oracle runs and hold no bbox-face tie (see below)
    ray_ok = (k32 == k64).view(R, 64).all(1) & ~((t32.margin.abs() < 1e-6) | (t64.margin.abs() < 1e-6)).view(R, 64).any(1)
    assert ray_ok.float().mean().item() > 0.99, ray_ok.float().mean().item()
    both = (k32 & k64 & ray_ok.repeat_interleave(64))

    def errs(out, ids):
        """max |out - fp64| per key over the agreeing rays / samples and the rows all runs share"""
        e = {}
        for k in ('rgb_map', 'acc_map', 'depth_map'):
            e[k] = float((out[k][0][ray_ok].double() - r64[k][0][ray_ok]).abs().max())
        e['raw'] = float((out['raw'][0][both].double() - r64['raw'][0][both]).abs().max())
        ia, ib, _ = _match_rows(ids, ids64)
        ok = both.cpu()[ids64.cpu()[ib]]  # rows of samples both oracle runs keep on agreeing rays
        assert ok.float().mean().item() > 0.99
        for k in ('pbw', 'tbw'):
            e[k] = float((out[k][0][ia[ok].to(dev)].double() - r64[k][0][ib[ok].to(dev)]).abs().max())
        return e
    ref_err = errs(r32, ids32)
    net = make_net(dev)
    net.train()
    got = {}
    for prec in ('fp32', 'bf16x6', 'bf16x3'):
        cfg = config.defaults()
        cfg.perturb = 0
        cfg.render_precision = prec
        rnd = Renderer(net, cfg)
        ret = rnd.render_device(bd)
        assert torch.equal(_keep(ret['raw']), k32), prec
        ids = rnd.row_ids(R)
        assert ids.numel() == ret['pbw'].shape[1]
        assert bool((ids[1:] > ids[:-1]).all()), prec  # rows in frame order
        if prec == 'fp32':  # the exact kernel against the reference's own arithmetic, whole frame
            # Threshold ties: a kept sample whose T-pose point lies within 1e-6 of a bbox face (the LBS
            # inverse's rounding differs between the adjugate here and torch's LU inverse, ~1e-7) may be
            # masked by one and not the other (measured: one sample of the 16.8 M, margin 4.5e-8). Such
            # samples and their rays are counted and excluded from the 1e-4 bound, which every other ray /
            # sample / row of the frame must meet.
            tie = t32.margin.abs() < 1e-6
            tie_ray = tie.view(R, 64).any(1)
            assert int(tie_ray.sum()) <= max(4, R // 10000), int(tie_ray.sum())
            for k in ('rgb_map', 'acc_map', 'depth_map'):
                err = float((ret[k][0][~tie_ray] - r32[k][0][~tie_ray]).abs().max())
                assert err <= 1e-4, (k, err)
            err = float((ret['raw'][0][~tie] - r32['raw'][0][~tie]).abs().max())
            assert err <= 1e-4, ('raw', err)
            ia, ib, only = _match_rows(ids, ids32)
            assert only.numel() <= max(8, ids32.numel() // 10000), only.numel()
            if only.numel():  # a row-set difference only at a tie: sigma' at train_th = 0, or a bbox tie
                od = only.to(dev)
                assert bool(((t32.sig[od].abs() <= 1e-4) | tie[od]).all()), (only, t32.sig[od], t32.margin[od])
            row_ok = ~tie[ids32[ib.to(dev)]]
            for k in ('pbw', 'tbw'):
                err = float((ret[k][0][ia.to(dev)][row_ok] - r32[k][0][ib.to(dev)][row_ok]).abs().max())
                assert err <= 1e-4, (k, err)
        got[prec] = errs(ret, ids)
        del ret
    del r32
    print({p: got[p] for p in got}, ref_err)
    for k in ref_err:
        bar = 1.5 * max(ref_err[k], got['fp32'][k])
        assert got['bf16x6'][k] <= bar, (k, got['bf16x6'][k], ref_err[k], got['fp32'][k])
    for k in ('rgb_map', 'acc_map'):
        assert got['bf16x3'][k] <= 1e-4, (k, got['bf16x3'][k])
