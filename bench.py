#!/usr/bin/env python
"""Headline benchmark: BASELINE.json metric on config 2 (aninerf_s9p full 512x512 render, fp32,
novel-view eval) through the drop-in renderer (HIP C-ABI).

step    = one full-frame render of 512x512 box rays x 64 samples (262,142 rays hit the box),
          inputs resident in HBM, outputs (rgb/acc/depth/raw + pbw/tbw rows) left in HBM
          (Renderer.render_device). ``render_s`` reports the drop-in Renderer.render(batch) with its
          eval D2H of every output (tpose_renderer.py:154-155) beside it.
N GPUs  = one process per GPU (torch.distributed.run, or ``--gpus N`` spawns them itself), each
          rendering its own frame (rays seed 2 + rank): frames are independent, so no collective on
          the data path ("scaling": "weak"); the timed region is bracketed by barriers and the max
          over ranks is reported.
precision: the headline is config 2's fp32: the exact-fp32-MFMA fused kernel k_mlp. The split-bf16
          kernel k_mlp_b16 (every layer as hi/lo bf16 pieces, 3 MFMA products per MAC, fp32
          accumulation; outputs held to the same 1e-4 fp32 tolerance by the parity tests) is timed in
          the same run and reported under ``bf16x3_split`` with its own roofline.
roofline: the fused network kernel dominates; its per-launch time is measured with hipEvents on the
          render stream (anr_profile_*). k_mlp: SURVEY.md §8(d)'s 2,312,192 credited FLOP per kept
          sample against the 157.3 TF fp32 MFMA peak (the 3,044,352 FLOP it executes, T-pose BW MLP
          included and the colour head folded, beside it). k_mlp_b16: the bf16 MFMA FLOP it executes against the 2.5 PF dense bf16
          peak, credited figure beside it. traffic: HBM bytes per launch from the committed PMC passes
          (profiles/pmc_latest.json, per kernel).
baselines (rank 0 at N=1, outside the timed region): cpu_baseline = the oracle (op-for-op PyTorch-CPU
          restatement) on the first 16 chunks of the frame with every host thread this job may use;
          torch_gpu_baseline = the same restatement with PyTorch-ROCm on this GPU over the whole frame
          (BASELINE.md §3's denominator of the 30x target) -> vs_baseline.
"""
import argparse
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

FLOP_PER_KEPT = 2_312_192          # render credit (BW pose + NeRF, latent folded)
MAC_BW, MAC_NERF = 497_152, 658_944  # per kept sample, latent folded
# the render kernels' NeRF with the folded colour head (anr_layers.h ANR_L_HEAD): trunk 491,008 +
# alpha_fc 256 + (Wv_f Wl_f Wf || Wv_d) 128 x 283 + rgb_fc 384
MAC_NERF_FOLDED = 491_008 + 256 + 128 * 283 + 384
# executed per kept sample: pose-space BW + T-pose BW (the tbw rows are render outputs) + folded NeRF
FLOP_PER_KEPT_EXECUTED = 2 * (2 * MAC_BW + MAC_NERF_FOLDED)
PEAK_FP32_MFMA_TFLOPS = 157.3      # MI355X_MICROARCH.md, Peak FP32 (matrix)
PEAK_BF16_MFMA_TFLOPS = 2500.0     # MI355X_MICROARCH.md, BF16 dense (no sparsity)
METRIC = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'BASELINE.json')))['metric']


def max_over_ranks(x, dev, world):
    """max of a host float over ranks (the timed region's max, bench contract)"""
    if world == 1:
        return float(x)
    on_cpu = dist.get_backend() == 'gloo'
    t = torch.tensor([float(x)], dtype=torch.float64, device='cpu' if on_cpu else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--rays', type=int, default=512 * 512)
    ap.add_argument('--cpu-rays', type=int, default=16 * 2048)
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--mode', choices=('render', 'train', 'sdf', 'sdf-train', 'mesh', 'anim'), default='render',
                    help='render: config 2 (headline); train: config 3/4 training step (1024 rays/GPU); '
                         'sdf: config 5 sdf_pdf full-frame render; sdf-train: config 5 training step '
                         '(1024 rays/GPU, second-order losses, RCCL all-reduce); mesh: aninerf mesh extraction '
                         '(get_alpha on the 5 mm voxel grid + marching cubes); anim: animation-stage '
                         'training step (2 x 65,536 points, novel_pose_bw)')
    ap.add_argument('--voxel', type=float, default=0.005, help='mesh mode: cfg.voxel_size (aninerf_s9p.yaml:95)')
    ap.add_argument('--sdf-cpu-rays', type=int, default=2048)
    ap.add_argument('--sdf-precision', choices=('fp32', 'bf16x6', 'bf16x3'), default='bf16x6',
                    help='sdf mode value: bf16x6 = the four fused launches with hi/mid/lo split products, fp32-level '
                         '(every output as close to an fp64 evaluation as the reference\'s fp32 arithmetic, '
                         'tests/test_gpu_sdf.py test_sdf_split_precisions_are_fp32_level); fp32 = exact fp32 MFMA layer '
                         'GEMMs; bf16x3 = hi/lo split (the 1e-4 parity bars, not fp32-level); the other two are timed '
                         'beside it unless --no-exact')
    ap.add_argument('--no-exact', action='store_true', help='skip timing the other render precision')
    ap.add_argument('--no-side', action='store_true',
                    help='render mode: skip the side legs (train_step / sdf_render / sdf_train_step keys)')
    ap.add_argument('--no-host-render', action='store_true',
                    help='skip the render_s leg (Renderer.render with the D2H): PMC passes then see full-frame launches only')
    ap.add_argument('--torch-rays', type=int, default=16 * 2048,
                    help='rays of the frame the PyTorch-ROCm denominator renders (cold pass ~0.8 s per chunk)')
    ap.add_argument('--no-torch-baseline', action='store_true',
                    help='skip the PyTorch-ROCm restatement denominator (vs_baseline)')
    ap.add_argument('--shard-frame', action='store_true',
                    help='render: split ONE frame over the ranks by whole chunks and all-gather rgb/acc/depth '
                         '(strong scaling, parallel.render_sharded) instead of one frame per GPU')
    ap.add_argument('--render-precision', choices=('fp32', 'bf16x3', 'bf16x6'), default='fp32',
                    help='fp32: exact fp32 MFMA; bf16x3: T-pose BW MLP + NeRF as hi/lo-split bf16 MFMA '
                         '(outputs within the 1e-4 fp32 tolerance, tests/test_gpu_render.py)')
    ap.add_argument('--train-rays', type=int, default=1024)
    ap.add_argument('--sdf-train-precision', choices=('fp32', 'bf16x3'), default='fp32',
                    help='sdf-train: layer GEMM products (cfg.sdf_train_precision): exact fp32 MFMA, or split-bf16 '
                         '(fp32-level, tests/test_gpu_sdf_train.py tolerances)')
    ap.add_argument('--subject', choices=('aninerf_313', 'aninerf_s9p'), default=None,
                    help='train mode network shapes (config.SUBJECTS): default aninerf_313 at N=1 (config 3), '
                         'aninerf_s9p at N>1 (config 4)')
    ap.add_argument('--precision', choices=('fp32', 'bf16', 'bf16_all'), default='bf16_all',
                    help='training GEMM operand precision (config 3 is bf16: bf16_all = every GEMM on bf16 operands; '
                         'bf16 = the pose-space blend-weight MLP kept at fp32 level; both hold the config-3 PSNR gate, '
                         'tests/test_gpu_config3.py; fp32 = exact reference arithmetic)')
    return ap.parse_args()


def host_threads():
    """CPU threads the baseline legs may use on this host: os.cpu_count(), limited by the process's
    affinity mask and by a cgroup CPU quota when one is set (on a shared GPU box the quota is the
    job's share of the node; running more threads than that only time-slices them)."""
    n = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = n
    quota = None
    try:
        q, period = open('/sys/fs/cgroup/cpu.max').read().split()
        if q != 'max':
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = ''
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    omp = None
    try:
        omp = int(os.environ['OMP_NUM_THREADS'])
    except (KeyError, ValueError):
        pass
    threads = min(x for x in (n, aff, quota, omp) if x)
    return threads, {'nproc': n, 'affinity': aff, 'cgroup_cpu_quota': quota, 'OMP_NUM_THREADS': omp,
                     'cpu_model': model}


def progress(msg):
    """one line per finished leg on stderr (the GPU box kills a command that is silent for 3 min)"""
    import sys
    print(f'[bench {time.strftime("%H:%M:%S")}] {msg}', file=sys.stderr, flush=True)


def render_roofline(prec, n_kept, kernel_ms):
    """roofline of the fused network kernel of one render precision: k_mlp (exact fp32 MFMA) is
    priced on SURVEY.md §8(d)'s credited 2,312,192 FLOP per kept sample against the fp32 MFMA peak;
    k_mlp_b16 (split bf16, 3 products per MAC) on the bf16 MFMA FLOP it executes against the dense
    bf16 peak, with the credited figure beside it."""
    split = prec in ('bf16x3', 'bf16x6')
    prods = 6 if prec == 'bf16x6' else 3
    kernel = {'bf16x3': 'k_mlp_b16', 'bf16x6': 'k_mlp_x6'}.get(prec, 'k_mlp')
    t = kernel_ms * 1e-3
    credited = n_kept * FLOP_PER_KEPT / t / 1e12
    if split:
        flop_exec = 2 * prods * (2 * MAC_BW + MAC_NERF_FOLDED)
        executed = n_kept * flop_exec / t / 1e12
        r = {'bound': 'mfma', 'kernel': kernel, 'achieved': executed, 'peak': PEAK_BF16_MFMA_TFLOPS,
             'unit': 'TFLOP/s', 'frac': executed / PEAK_BF16_MFMA_TFLOPS, 'traffic': None,
             'flop_per_kept': flop_exec, 'flop_basis': f'executed bf16 MFMA FLOP ({prods} products per MAC)',
             'achieved_credited': credited, 'frac_credited_vs_bf16_peak': credited / PEAK_BF16_MFMA_TFLOPS,
             'flop_per_kept_credited': FLOP_PER_KEPT}
    else:
        executed = n_kept * FLOP_PER_KEPT_EXECUTED / t / 1e12
        r = {'bound': 'mfma', 'kernel': kernel, 'achieved': credited, 'peak': PEAK_FP32_MFMA_TFLOPS,
             'unit': 'TFLOP/s', 'frac': credited / PEAK_FP32_MFMA_TFLOPS, 'traffic': None,
             'flop_per_kept': FLOP_PER_KEPT, 'flop_basis': 'SURVEY.md §8(d) credit (BW pose + NeRF, latent folded)',
             'achieved_executed': executed, 'frac_executed': executed / PEAK_FP32_MFMA_TFLOPS,
             'flop_per_kept_executed': FLOP_PER_KEPT_EXECUTED}
    r['kernel_ms'] = kernel_ms
    r['kept_samples_per_launch'] = n_kept
    pmc = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'pmc_latest.json')
    if os.path.exists(pmc):
        t = json.load(open(pmc)).get(kernel)
        if t:
            r['traffic'] = t['bytes_per_launch']
            r['traffic_source'] = t['source'] + '; ' + t['correction']
    return r


def launch_workers(args):
    """``python bench.py --gpus N`` without a launcher: one process per GPU, spawned before this
    process touches the GPU, rendezvous on 127.0.0.1 (the torch.distributed.run contract)."""
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + sys.argv, env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def main():
    args = parse()
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        raise SystemExit(launch_workers(args))
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    if world != args.gpus:
        raise SystemExit(f'bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks')
    # rehearsal knobs for the N > 1 path on a one-GPU box or a CPU host (never set by the driver):
    # ANR_BENCH_BACKEND=gloo, ANR_BENCH_ONE_DEVICE=1 maps every rank to cuda:0, ANR_BENCH_DRYRUN=1
    # runs the launch / rendezvous / timing / max-over-ranks logic with no GPU work at all
    backend = os.environ.get('ANR_BENCH_BACKEND', 'nccl')
    if os.environ.get('ANR_BENCH_DRYRUN') == '1':
        return dry_run(args, rank, world)
    if os.environ.get('ANR_BENCH_ONE_DEVICE') == '1':
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)

    from animatable_nerf_amd import _lib, config, network, parallel, synthetic
    from animatable_nerf_amd.renderer import Renderer, near_far
    if args.mode == 'train':
        return bench_train(args, rank, world, dev)
    if args.mode == 'sdf':
        return bench_sdf(args, rank, world, dev)
    if args.mode == 'mesh':
        return bench_mesh(args, rank, world, dev)
    if args.mode == 'anim':
        return bench_anim(args, rank, world, dev)
    if args.mode == 'sdf-train':
        return bench_sdf_train(args, rank, world, dev)

    sc = synthetic.Scene(vsize=0.025)
    ro, rd = sc.box_rays(args.rays, seed=2 if args.shard_frame else 2 + rank)
    nr, fr, m = near_far(torch.from_numpy(sc.bounds).to(dev), torch.from_numpy(ro).to(dev),
                         torch.from_numpy(rd).to(dev))
    m_np = m.cpu().numpy()
    b = sc.batch_arrays(ro[m_np], rd[m_np], nr.cpu().numpy(), fr.cpu().numpy())
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()}
    R = int(batch['ray_o'].shape[1])

    net = network.Network()
    sd = synthetic.init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    network.load_numpy_state(net, sd)
    net = net.to(dev)
    net.train()  # run.py evaluates in train() mode with perturb = 0
    lib = _lib.load()
    frames = 1 if args.shard_frame else world  # frames rendered per timed step, all ranks together
    s0, s1 = parallel.shard_chunks(R, rank, world) if args.shard_frame else (0, R)
    R_local = max(1, s1 - s0)  # this rank's rays (n_kept, kernel_ms are this rank's)

    def make_renderer(precision):
        cfg = config.defaults()
        cfg.perturb = 0
        cfg.render_precision = precision
        return Renderer(net, cfg)

    def timed(precision):
        renderer = make_renderer(precision)
        render = (lambda: parallel.render_sharded(renderer, batch)) if args.shard_frame else \
            (lambda: renderer.render_device(batch))
        for _ in range(args.warmup):
            out = render()
        torch.cuda.synchronize()
        lib.anr_profile_enable(1)
        lib.anr_profile_read(None, None)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = render()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        mlp_ms, launches, mhz = profile_read(lib)
        counts = renderer.counts(R_local) if args.shard_frame else renderer.last_counts
        timed.clock_mhz = mhz
        return out, max_over_ranks(dt, dev, world), mlp_ms / max(1, launches), counts

    prec = args.render_precision
    out, dt_max, kernel_ms, (n_kept, m_rows) = timed(prec)
    clocks = {prec: timed.clock_mhz}
    progress(f'{prec}: {dt_max / args.steps * 1e3:.2f} ms/frame, kernel {kernel_ms:.2f} ms, clock {timed.clock_mhz:.0f} MHz')
    value = R * 64 * args.steps * frames / dt_max
    result = {
        'metric': METRIC, 'value': value, 'unit': 'ray-samples/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt_max / args.steps * 1e3, 'higher_is_better': True,
        'scaling': 'strong' if args.shard_frame else 'weak', 'vs_baseline': None,
        'dtype': {'fp32': 'fp32', 'bf16x6': 'bf16 MFMA operands (hi/mid/lo split, 6 products per MAC), fp32 accumulate'}.get(
            prec, 'bf16 MFMA operands (hi/lo split, 3 products per MAC), fp32 accumulate'),
        'data': 'synthetic',
        'config': {'workload': 'aninerf_s9p full 512x512 render (config 2: fp32, novel-view eval, perturb=0)',
                   'render_precision': prec,
                   'rays_per_gpu': R, 'samples_per_ray': 64, 'chunk': 2048,
                   'kept_fraction': n_kept / (R_local * 64), 'alpha_ind_rows': m_rows,
                   'timed_call': 'Renderer.render_device (outputs left in HBM); render_s below adds the D2H',
                   'parallelism': (f'frame-split{world} (whole 2048-ray chunks per rank, rgb/acc/depth '
                                   'all-gathered over RCCL)') if args.shard_frame else
                                  f'replicas{world} (one frame per GPU)'},
        'roofline': dict(render_roofline(prec, n_kept, kernel_ms), clock_mhz=clocks[prec]),
    }
    if not args.no_exact:
        notes = {
            'bf16x3': ('bf16x3_split', 'same frame, every MLP layer as hi/lo-split bf16 MFMA (outputs held to the '
                       'same 1e-4 fp32 tolerance by tests/test_gpu_render.py)'),
            'bf16x6': ('bf16x6_fp32_level', 'same frame, every MLP layer as hi/mid/lo-split bf16 MFMA, 6 products '
                       'per multiply-add, fp32 accumulation: fp32-level products (each output as close to an fp64 '
                       'evaluation as the reference\'s fp32 arithmetic, tests/test_gpu_render.py '
                       'test_split_precisions_are_fp32_level)'),
            'fp32': ('fp32_exact', 'exact fp32 MFMA')}
        for other in [p for p in ('fp32', 'bf16x6', 'bf16x3') if p != prec]:
            o2, dt2, kms2, (nk2, _) = timed(other)
            progress(f'{other}: {dt2 / args.steps * 1e3:.2f} ms/frame, kernel {kms2:.2f} ms, clock {timed.clock_mhz:.0f} MHz')
            key, note = notes[other]
            result[key] = {
                'value': R * 64 * args.steps * frames / dt2, 'ms_per_step': dt2 / args.steps * 1e3,
                'render_precision': other, 'note': note,
                'roofline': dict(render_roofline(other, nk2, kms2), clock_mhz=timed.clock_mhz)}
            del o2
    if not args.shard_frame and not args.no_host_render:
        # the drop-in call as run.py:63-69 makes it: Renderer.render(batch) with the eval D2H of every
        # output (tpose_renderer.py:154-155) inside the measured time
        renderer = make_renderer(prec)
        with torch.no_grad():
            renderer.render(batch)
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                host = renderer.render(batch)
                ts.append(time.perf_counter() - t0)
        rs = float(np.median(ts))
        progress(f'Renderer.render with D2H: {rs * 1e3:.2f} ms')
        result['render_s'] = {'seconds': rs, 'value': R * 64 / rs, 'unit': 'ray-samples/s',
                              'call': 'Renderer.render(batch): fused render + .cpu() of rgb/acc/depth/raw/pbw/tbw '
                                      '(%.0f MB to the host; the frame in %d parts of whole chunks, each copied to '
                                      'page-locked memory while the next renders)' % (
                                          sum(v.numel() * v.element_size() for v in host.values()) / 1e6,
                                          renderer.HOST_PARTS),
                              'median_of': 3}
        del host
    if not args.no_side:
        result.update(side_legs(args, rank, world, dev))
    if rank == 0 and world == 1 and not args.no_cpu:
        result['cpu_baseline'], result['psnr_vs_fp32_oracle'] = cpu_baseline(sd, b, out, args.cpu_rays)
        progress(f"cpu_baseline: {result['cpu_baseline']['value']:.4g} ray-samples/s, "
                 f"{result['cpu_baseline']['cores']} threads")
    if rank == 0 and world == 1 and not args.no_torch_baseline:
        tg = torch_gpu_baseline(sd, b, dev, args.torch_rays)
        progress(f"torch_gpu_baseline: {tg['value']:.4g} ray-samples/s")
        result['torch_gpu_baseline'] = tg
        result['vs_baseline'] = value / tg['value']
        result['vs_baseline_denominator'] = ('BASELINE.md §3 GPU denominator: the reference op-for-op PyTorch-ROCm '
                                             'restatement on this GPU, same frame (torch_gpu_baseline)')
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def profile_read(lib):
    """(summed ms, launches, median in-kernel clock MHz) of the profiled fused launches since the last
    read (anr_profile_read_clock), and profiling off"""
    from animatable_nerf_amd import _lib
    ms, n, mhz = _lib.ctypes.c_double(0), _lib.ctypes.c_int(0), _lib.ctypes.c_double(0)
    _lib.check(lib.anr_profile_read_clock(_lib.ctypes.byref(ms), _lib.ctypes.byref(n), _lib.ctypes.byref(mhz)),
               'anr_profile_read_clock')
    lib.anr_profile_enable(0)
    return ms.value, n.value, mhz.value


def side_legs(args, rank, world, dev):
    """Configs 3-5 timed inside the default run (so the driver's own bench call measures them too):
    'train_step' (config 3 at N = 1, config 4 at N > 1: the training iteration with its RCCL gradient
    all-reduce), and at N = 1 'sdf_render' (config 5's network, bf16x6 fp32-level render of a 512x512
    frame, exact fp32 beside it) and 'sdf_train_step' (config 5's training iteration, exact fp32); at
    every N 'mesh_extract' (aninerf mesh extraction, 5 mm grid) and 'anim_step' (animation stage). Each
    is the full --mode leg at a short step count; its JSON line is returned instead of printed."""
    import copy
    out = {}

    def leg(fn, key, **over):
        a = copy.copy(args)
        a.no_cpu = True
        for k, v in over.items():
            setattr(a, k, v)
        t0 = time.perf_counter()
        r = fn(a, rank, world, dev, emit=False)
        keep = ('value', 'unit', 'ms_per_step', 'steps', 'warmup', 'dtype', 'config', 'roofline', 'scaling',
                'host_issue_ms_per_step', 'loss_last_step', 'fp32_exact', 'bf16x3_split', 'metric')
        out[key] = {k: r[k] for k in keep if k in r}
        out[key]['leg_wall_s'] = time.perf_counter() - t0
        progress(f"side leg {key}: {r['ms_per_step']:.3f} ms/step")
    leg(bench_train, 'train_step', steps=50, warmup=10)  # ~1 ms steps: 50 amortise the first step's host issue
    if world == 1:
        leg(bench_sdf, 'sdf_render', steps=3, warmup=1, no_exact=False, sdf_exact_only=True)
        leg(bench_sdf_train, 'sdf_train_step', steps=20, warmup=3)
    # SURVEY §8(f) rows in the driver's line too: mesh extraction of one frame (5 mm grid) and the
    # animation-stage training step (aninerf_animation_trainer.py)
    leg(bench_mesh, 'mesh_extract', steps=2, warmup=1)
    leg(bench_anim, 'anim_step', steps=10, warmup=3)
    return out


def dry_run(args, rank, world):
    """ANR_BENCH_DRYRUN=1: the N-process contract without GPU work (CPU rehearsal of --gpus N):
    gloo rendezvous, barriers around K empty steps, max over ranks, one JSON line from rank 0."""
    if world > 1:
        dist.init_process_group('gloo')
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if world > 1:
            dist.barrier()
    dt = max_over_ranks(time.perf_counter() - t0, None, world)
    if rank == 0:
        print(json.dumps({'metric': METRIC, 'value': None, 'unit': 'ray-samples/s', 'n_gpus': world,
                          'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': dt / max(1, args.steps) * 1e3,
                          'dry_run': True, 'ranks_seen': world}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def torch_gpu_baseline(sd, b, dev, n_rays, reps=3):
    """BASELINE.md §3's GPU denominator, outside the timed region: the op-for-op PyTorch restatement
    of the reference (oracle/restate.py) with PyTorch-ROCm on this GPU, fp32, 2048-ray chunks, over
    the first ``n_rays`` rays of the same frame: one untimed pass (MIOpen meets every chunk's Conv1d
    size for the first time), then the median of ``reps`` warm passes."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import torch_gpu_baseline as tgb
    r = tgb.measure(sd, b, dev, reps, n_rays)
    r['sample'] = f'first {r["rays"]} rays ({r["rays"] // 2048} reference chunks) of the config-2 frame'
    return r


FLOP_PER_KEPT_TRAIN = 9_919_488  # 3 x 2 x (2 x 497,152 + 658,944)


def bench_train(args, rank, world, dev, emit=True):
    """Configs 3/4: one training iteration (trainer.py:50-68) per step on 1,024 rays per GPU:
    forward + losses + backward (anr_train_step) + RCCL mean all-reduce of the 5.3 MB gradient blob
    (N > 1) + clip + Adam (anr_adam). Weak scaling: every rank trains on its own ray batch, which is
    the reference's DDP semantics (one image per rank, samplers.py:75-131)."""
    from animatable_nerf_amd import config, network, synthetic
    from animatable_nerf_amd.renderer import near_far
    from animatable_nerf_amd.trainer import FusedStep
    sc = synthetic.Scene(vsize=0.025)
    batches = []
    nb = max(1, min(8, args.steps + args.warmup))
    for j in range(nb):
        ro, rd = sc.box_rays(args.train_rays * 2, seed=1000 + 97 * rank + j)
        nr, fr, m = near_far(torch.from_numpy(sc.bounds).to(dev), torch.from_numpy(ro).to(dev),
                             torch.from_numpy(rd).to(dev))
        m_np = m.cpu().numpy()
        rgb = np.random.default_rng(j + 31 * rank).random((len(ro), 3)).astype(np.float32)
        b = sc.batch_arrays(ro[m_np][:args.train_rays], rd[m_np][:args.train_rays],
                            nr.cpu().numpy()[:args.train_rays], fr.cpu().numpy()[:args.train_rays],
                            rgb=rgb[m_np][:args.train_rays])
        batches.append({k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()})
    subject = args.subject or ('aninerf_313' if world == 1 else 'aninerf_s9p')
    cfg = config.subject(subject, perturb=1, train_precision=args.precision)
    net = network.Network(cfg)
    sd = synthetic.init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    network.load_numpy_state(net, sd)
    net = net.to(dev)
    net.train()
    step = FusedStep(net, cfg)
    for j in range(args.warmup):
        step.step(batches[j % nb])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0  # host time inside step() (issue only: nothing in a step waits on the device)
    for j in range(args.steps):
        th = time.perf_counter()
        step.step(batches[(args.warmup + j) % nb])
        host += time.perf_counter() - th
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_max = max_over_ranks(dt, dev, world)
    # the in-kernel shader clock (anr_profile_read_clock: entry / exit stamps of the fused chain launches)
    # over 3 more steps profiled after the timed ones, so events and stamps stay out of the timed region
    step.lib.anr_profile_enable(1)
    step.lib.anr_profile_read(None, None)
    for j in range(3):
        step.step(batches[j % nb])
    torch.cuda.synchronize()
    chain_ms, n_chain, mhz = profile_read(step.lib)
    R = int(batches[0]['ray_o'].shape[1])
    loss = step.loss3.cpu().tolist()
    # kept samples of the last step (host read inside anr_train_step)
    from animatable_nerf_amd import _lib as L  # noqa: F401
    n_kept = step.renderer._counts(step.renderer._tws, R)[0]
    achieved = n_kept * FLOP_PER_KEPT_TRAIN * args.steps / dt_max / 1e12
    peak = PEAK_FP32_MFMA_TFLOPS if args.precision == 'fp32' else PEAK_BF16_MFMA_TFLOPS
    result = {
        'metric': 'training ray-samples/s (1024 rays x 64 samples per GPU per step), aninerf training step',
        'value': R * 64 * args.steps * world / dt_max, 'unit': 'ray-samples/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt_max / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': None, 'dtype': args.precision, 'data': 'synthetic',
        'config': {'workload': f'{subject} training step (config {3 if world == 1 else 4}: 1024 rays/GPU, perturb 1, Adam)',
                   'subject': subject, 'num_train_frame': int(cfg.num_train_frame),
                   'precision': f'{args.precision} GEMM operands, fp32 accumulation / master weights / Adam',
                   'rays_per_gpu': R, 'kept_samples_last_step': n_kept,
                   'parallelism': f'dp{world} (RCCL mean all-reduce of the flat gradient blob)'},
        'roofline': {'bound': 'mfma', 'kernel': 'whole step', 'achieved': achieved, 'peak': peak,
                     'unit': 'TFLOP/s', 'frac': achieved / peak, 'traffic': None,
                     'flop_per_kept': FLOP_PER_KEPT_TRAIN,
                     'clock_mhz': mhz if n_chain else None,
                     'clock_source': 'median over workgroups of the fused chain launches (anr_tchain.hip), '
                                     '3 profiled steps after the timed ones',
                     'chain_launch_ms_per_step': chain_ms / 3 if n_chain else None},
        'loss_last_step': loss[:3],
        'host_issue_ms_per_step': host / args.steps * 1e3,
    }
    if not emit:
        return result
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


# sdf_pdf per kept sample, exact from the layer shapes (anisdf_pdf_network.py): residual MLP 528,640 MAC
# + SDF forward 524,544 + its input gradient 459,008 (lin8 row 0, lin7..lin1, lin0 to gamma) + colour 304,128
FLOP_PER_KEPT_SDF = 2 * (528_640 + 524_544 + 459_008 + 304_128)


def bench_sdf(args, rank, world, dev, emit=True):
    """Config 5 (sdf_pdf) geometry at the config-2 size: a 512x512 box-ray frame per GPU through
    renderer_sdf.Renderer.render_device (anr_sdf_render_fwd); replicas, no collective."""
    from animatable_nerf_amd import config, network, network_sdf, synthetic
    from animatable_nerf_amd.renderer import near_far
    from animatable_nerf_amd.renderer_sdf import Renderer
    sc = synthetic.PdfScene(vsize=0.05)
    ro, rd = sc.box_rays(args.rays, seed=2 + rank)
    nr, fr, m = near_far(torch.from_numpy(sc.pbounds).to(dev), torch.from_numpy(ro).to(dev),
                         torch.from_numpy(rd).to(dev))
    m_np = m.cpu().numpy()
    b = sc.batch_arrays(ro[m_np], rd[m_np], nr.cpu().numpy(), fr.cpu().numpy(), latent_index=7)
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()}
    tb0 = batch['tbounds'].clone()
    R = int(batch['ray_o'].shape[1])
    cfg = config.subject('anisdf_pdf_s9p', perturb=0, render_precision=args.sdf_precision)
    net = network_sdf.Network(cfg)
    sd = synthetic.init_state_dict_sdf({k: tuple(v.shape) for k, v in net.state_dict().items()})
    network.load_numpy_state(net, sd)
    net = net.to(dev)
    net.train()

    from animatable_nerf_amd import _lib
    lib = _lib.load()

    def timed(prec, steps, warmup):
        c = config.subject('anisdf_pdf_s9p', perturb=0, render_precision=prec)
        r = Renderer(net, c)
        for _ in range(warmup):
            batch['tbounds'].copy_(tb0)
            o = r.render_device(batch)
        torch.cuda.synchronize()
        lib.anr_profile_enable(1)
        lib.anr_profile_read(None, None)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            batch['tbounds'].copy_(tb0)
            o = r.render_device(batch)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        ms, n, mhz = profile_read(lib)  # the fused network launches (split precisions; k_lgemm in exact fp32)
        timed.net = {'network_launch_ms_per_frame': ms / steps, 'network_launches_per_frame': n / steps,
                     'clock_mhz': mhz if n else None}
        return o, max_over_ranks(dt, dev, world), r.last_counts[0]

    def sdf_roofline(prec, n_kept, dt_step):
        prods = {'fp32': 1, 'bf16x6': 6, 'bf16x3': 3}[prec]
        flop_exec = FLOP_PER_KEPT_SDF * prods
        peak = PEAK_FP32_MFMA_TFLOPS if prec == 'fp32' else PEAK_BF16_MFMA_TFLOPS
        achieved = n_kept * flop_exec / dt_step / 1e12
        r = {'bound': 'mfma', 'kernel': 'whole render (the network launches dominate)', 'achieved': achieved,
             'peak': peak, 'unit': 'TFLOP/s', 'frac': achieved / peak, 'traffic': None,
             'flop_per_kept': FLOP_PER_KEPT_SDF, 'flop_per_kept_executed': flop_exec,
             'achieved_credited': n_kept * FLOP_PER_KEPT_SDF / dt_step / 1e12}
        r.update(timed.net)
        if prec == 'fp32':  # the profiled launches are the exact path's k_lgemm layer GEMMs, not the whole network
            r['lgemm_launch_ms_per_frame'] = r.pop('network_launch_ms_per_frame')
            r['lgemm_launches_per_frame'] = r.pop('network_launches_per_frame')
        elif timed.net['network_launches_per_frame']:
            # the four fused network launches alone (k_resd / k_sdfnet / k_sdfgrad / k_color)
            r['network_frac'] = achieved * dt_step * 1e3 / timed.net['network_launch_ms_per_frame'] / peak
        return r

    prec = args.sdf_precision
    out, dt_max, n_kept = timed(prec, args.steps, args.warmup)
    progress(f'sdf {prec}: {dt_max / args.steps * 1e3:.2f} ms/frame, clock {timed.net["clock_mhz"]}')
    dtypes = {'fp32': 'fp32', 'bf16x6': 'bf16 MFMA operands (hi/mid/lo split, 6 products per MAC: fp32-level), fp32 accumulate',
              'bf16x3': 'bf16 MFMA operands (hi/lo split, 3 products per MAC), fp32 accumulate'}
    result = {
        'metric': 'ray-samples/sec (512x512 rays x 64 samples), sdf_pdf render', 'value': R * 64 * args.steps * world / dt_max,
        'unit': 'ray-samples/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': dt_max / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': dtypes[prec], 'data': 'synthetic',
        'config': {'workload': 'sdf_pdf (config 5 network) full 512x512 box-ray render, eval; outputs held to the '
                               'fp32 tolerances of tests/test_gpu_sdf.py in every render precision',
                   'render_precision': prec,
                   'rays_per_gpu': R, 'kept_fraction': n_kept / (R * 64), 'parallelism': f'replicas{world}'},
        'roofline': sdf_roofline(prec, n_kept, dt_max / args.steps),
    }
    if not args.no_exact:
        names = {'fp32': 'fp32_exact', 'bf16x6': 'bf16x6_fp32_level', 'bf16x3': 'bf16x3_split'}
        others = ['fp32'] if getattr(args, 'sdf_exact_only', False) else ['fp32', 'bf16x6', 'bf16x3']
        for other in [q for q in others if q != prec]:
            k = max(1, min(args.steps, 3 if other == 'fp32' else args.steps))
            o2, dt2, nk2 = timed(other, k, 1)
            progress(f'sdf {other}: {dt2 / k * 1e3:.2f} ms/frame')
            result[names[other]] = {'value': R * 64 * k * world / dt2, 'ms_per_step': dt2 / k * 1e3, 'steps': k,
                                    'render_precision': other, 'dtype': dtypes[other],
                                    'roofline': sdf_roofline(other, nk2, dt2 / k)}
            del o2
    if rank == 0 and world == 1 and not args.no_cpu:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from oracle import restate_sdf
        threads, host = host_threads()
        torch.set_num_threads(threads)
        n = min(args.sdf_cpu_rays, R)
        sub = {k: torch.from_numpy(np.ascontiguousarray(
            v[:, :n] if k in ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb') else v).copy())
            for k, v in b.items()}
        P = {k: torch.from_numpy(v) for k, v in sd.items()}
        with torch.no_grad():
            t1 = time.perf_counter()
            ref = restate_sdf.render(P, sub)
            dtc = time.perf_counter() - t1
        result['cpu_baseline'] = {'value': n * 64 / dtc, 'unit': 'ray-samples/s', 'cores': threads, 'kind': 'port',
                                  'sample': f'first {n} rays of the frame, oracle/restate_sdf.py, {dtc:.1f} s'}
        from oracle import restate
        result['psnr_vs_fp32_oracle'] = float(restate.psnr(out['rgb_map'][0, :n].cpu().numpy(), ref['rgb_map'][0].numpy()))
    if not emit:
        return result
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


# sdf_pdf training, MAC per kept sample executed by anr_sdf_train_step (exact fp32 MFMA): forward (residual
# 528,640 + SDF 524,544 + its input gradient 459,008 + colour 304,128), colour backward (dW + dX 2 x 304,128),
# SDF tangent pass 524,544, stacked SDF reverse (dX over 2n rows + dW of both halves: 4 x 524,544), residual
# backward (dW + dX 2 x 528,640); the observed-gradient rows (|sdf| < 0.02) add their own passes on top
MAC_SDF_TRAIN = (528_640 + 524_544 + 459_008 + 304_128) + 2 * 304_128 + 524_544 + 4 * 524_544 + 2 * 528_640


def bench_sdf_train(args, rank, world, dev, emit=True):
    """Config 5's training leg: one tpose_trainer step of the sdf_pdf network per GPU on 1,024 rays
    (N_rand, perturb 1): anr_sdf_train_step (forward, second-order losses, every gradient) + RCCL mean
    all-reduce of the 1,432,510-float gradient blob with the losses in its tail (N > 1) + clip + Adam.
    Weak scaling: every rank trains on its own batch (DDP semantics)."""
    from animatable_nerf_amd import config, network, network_sdf, synthetic
    from animatable_nerf_amd.renderer import near_far
    from animatable_nerf_amd.trainer_sdf import LOSS_KEYS, SdfStep
    sc = synthetic.PdfScene(vsize=0.05)
    batches = []
    nb = max(1, min(4, args.steps + args.warmup))
    for j in range(nb):
        ro, rd = sc.box_rays(args.train_rays * 2, seed=2000 + 97 * rank + j)
        nr, fr, m = near_far(torch.from_numpy(sc.pbounds).to(dev), torch.from_numpy(ro).to(dev),
                             torch.from_numpy(rd).to(dev))
        m_np = m.cpu().numpy()
        rgb = np.random.default_rng(j + 31 * rank).random((len(ro), 3)).astype(np.float32)
        b = sc.batch_arrays(ro[m_np][:args.train_rays], rd[m_np][:args.train_rays],
                            nr.cpu().numpy()[:args.train_rays], fr.cpu().numpy()[:args.train_rays], latent_index=7,
                            rgb=rgb[m_np][:args.train_rays])
        bt = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()}
        bt['iter_step'] = 12000
        batches.append(bt)
    tb0 = [b['tbounds'].clone() for b in batches]
    cfg = config.subject('anisdf_pdf_s9p', perturb=1, sdf_train_precision=args.sdf_train_precision)
    net = network_sdf.Network(cfg)
    sd = synthetic.init_state_dict_sdf({k: tuple(v.shape) for k, v in net.state_dict().items()})
    network.load_numpy_state(net, sd)
    net = net.to(dev)
    net.train()
    step = SdfStep(net, cfg)

    def one(j):
        k = j % nb
        batches[k]['tbounds'].copy_(tb0[k])
        return step.step(batches[k])
    for j in range(args.warmup):
        one(j)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(args.steps):
        l8 = one(args.warmup + j)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt_max = max_over_ranks(time.perf_counter() - t0, dev, world)
    # in-kernel clock of the step's k_lgemm layer products (exact fp32 F32 kernels), 2 profiled steps after
    # the timed ones
    step.lib.anr_profile_enable(1)
    step.lib.anr_profile_read(None, None)
    for j in range(2):
        one(j)
    torch.cuda.synchronize()
    lg_ms, n_lg, mhz = profile_read(step.lib)
    R = int(batches[0]['ray_o'].shape[1])
    losses = dict(zip(LOSS_KEYS, l8.cpu().tolist()))  # rank means (the losses ride in the all-reduced blob)
    n_kept = losses['n_kept']
    achieved = n_kept * 2 * MAC_SDF_TRAIN / (dt_max / args.steps) / 1e12
    # split-bf16: three bf16 MFMA products per multiply-add, priced against the bf16 dense peak / 3
    peak = PEAK_FP32_MFMA_TFLOPS if args.sdf_train_precision == 'fp32' else PEAK_BF16_MFMA_TFLOPS / 3
    result = {
        'metric': 'sdf_pdf training ray-samples/s (1024 rays x 64 samples per GPU per step)',
        'value': R * 64 * args.steps * world / dt_max, 'unit': 'ray-samples/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt_max / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': None, 'data': 'synthetic',
        'dtype': 'fp32' if args.sdf_train_precision == 'fp32' else
                 'bf16 MFMA operands (hi/lo split, 3 products per MAC) on the parts tests/test_gpu_sdf_train.py '
                 'allows, exact fp32 on the rest; fp32 accumulation',
        'config': {'workload': 'sdf_pdf training step (config 5: tpose_trainer losses incl. eikonal, observed '
                               'gradients, msk_sdf BCE, image MSE; Adam)', 'rays_per_gpu': R,
                   'sdf_train_precision': args.sdf_train_precision,
                   'parallelism': f'dp{world} (RCCL mean all-reduce of the 1,432,510-float gradient blob + losses)'},
        'roofline': {'bound': 'mfma', 'kernel': 'whole step (layer GEMMs dominate)', 'achieved': achieved,
                     'peak': peak, 'unit': 'TFLOP/s', 'frac': achieved / peak,
                     'traffic': None, 'flop_per_kept_executed_main_path': 2 * MAC_SDF_TRAIN,
                     'kept_samples_per_step': n_kept,
                     'clock_mhz': mhz if n_lg else None,
                     'clock_source': 'median over workgroups of the k_lgemm layer products, 2 profiled steps '
                                     'after the timed ones',
                     'lgemm_launches_per_step': n_lg / 2, 'lgemm_ms_per_step': lg_ms / 2},
        'losses_last_step_rank_mean': losses,
    }
    if not emit:
        return result
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


# get_alpha per kept point, latent folded: pose-space BW MLP 497,152 MAC + NeRF trunk and alpha_fc
# (63*256 + 6*256*256 + 319*256 + 256 = 491,264 MAC)
MAC_NERF_TRUNK = 491_264
FLOP_PER_KEPT_ALPHA = 2 * (MAC_BW + MAC_NERF_TRUNK)


def bench_mesh(args, rank, world, dev, emit=True):
    """Mesh extraction (aninerf_mesh_renderer.py:26-63) of one frame per GPU at the reference's
    voxel size (5 mm): get_alpha over every grid voxel (`inside` all ones: an upper bound of the
    masked grid the dataset produces), the density volume, device marching cubes. Replicas."""
    from animatable_nerf_amd import config, network, synthetic
    from animatable_nerf_amd.renderer_mesh import Renderer, marching_cubes
    b = synthetic.mesh_scene(voxel=args.voxel, inside_frac=1.01)
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()}
    net = network.Network()
    sd = synthetic.init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    network.load_numpy_state(net, sd)
    net = net.to(dev)
    cfg = config.load_cfg(opts=['vis_posed_mesh', 'True', 'render_precision', args.render_precision])
    renderer = Renderer(net, cfg)
    inside = batch['inside'][0].bool()
    wpts = batch['pts'][0][inside].contiguous()
    n = int(wpts.shape[0])
    iso = 2.95  # raw alpha of the synthetic weights sits near the alpha_fc bias (3); cfg.mesh_th = 5 is empty

    def once():
        alpha = renderer.alpha_points(wpts, batch)
        cube = torch.zeros(tuple(inside.shape), device=dev)
        cube[inside] = alpha
        return cube

    for _ in range(args.warmup):
        cube = once()
        marching_cubes(cube, iso)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps)]
    t0 = time.perf_counter()
    for j in range(args.steps):
        ev[2 * j].record()
        alpha = renderer.alpha_points(wpts, batch)
        ev[2 * j + 1].record()
        cube = torch.zeros(tuple(inside.shape), device=dev)
        cube[inside] = alpha
        verts, tris = marching_cubes(cube, iso)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_max = max_over_ranks(dt, dev, world)
    alpha_ms = sum(ev[2 * j].elapsed_time(ev[2 * j + 1]) for j in range(args.steps)) / args.steps
    n_kept = int(renderer._aws[:4].view(torch.int32).item())  # anr_alpha_counts: kept points
    split = args.render_precision in ('bf16x3', 'bf16x6')
    prods = 6 if args.render_precision == 'bf16x6' else 3
    flop_exec = prods * FLOP_PER_KEPT_ALPHA if split else FLOP_PER_KEPT_ALPHA
    peak = PEAK_BF16_MFMA_TFLOPS if split else PEAK_FP32_MFMA_TFLOPS
    achieved = n_kept * flop_exec / (alpha_ms * 1e-3) / 1e12
    t1 = time.perf_counter()
    verts, tris = marching_cubes(cube, iso)
    torch.cuda.synchronize()
    mc_ms = (time.perf_counter() - t1) * 1e3
    result = {
        'metric': 'mesh grid points/s (get_alpha + marching cubes), aninerf_s9p mesh extraction',
        'value': n * args.steps * world / dt_max, 'unit': 'points/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt_max / args.steps * 1e3, 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None,
        'dtype': (f'bf16 MFMA operands ({"hi/mid/lo" if prods == 6 else "hi/lo"} split), fp32 accumulate'
                  if split else 'fp32'), 'data': 'synthetic',
        'config': {'workload': f'mesh extraction, {args.voxel * 1000:g} mm voxel grid over wbounds, inside = all voxels',
                   'grid': list(inside.shape), 'points': n, 'kept_fraction': n_kept / n, 'iso': iso,
                   'vertices': int(verts.shape[0]), 'triangles': int(tris.shape[0]),
                   'alpha_ms': alpha_ms, 'marching_cubes_ms': mc_ms, 'parallelism': f'replicas{world}'},
        'roofline': {'bound': 'mfma', 'kernel': 'anr_alpha_points (k_alpha%s dominates)' % (
                     {'bf16x3': '_b16', 'bf16x6': '_x6'}.get(args.render_precision, '')),
                     'achieved': achieved, 'peak': peak, 'unit': 'TFLOP/s', 'frac': achieved / peak, 'traffic': None,
                     'flop_per_kept_executed': flop_exec, 'flop_per_kept_credited': FLOP_PER_KEPT_ALPHA},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from oracle import restate
        threads, host = host_threads()
        torch.set_num_threads(threads)
        m = min(16 * 2048 * 64, n)  # 16 reference chunks, ~10 s on 16 host threads
        P = {k: torch.from_numpy(v) for k, v in sd.items()}
        cb = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in b.items() if k not in ('pts', 'inside')}
        sub = wpts[:m].cpu()
        with torch.no_grad():
            t2 = time.perf_counter()
            ref = restate.mesh_alpha(P, sub, cb)
            dtc = time.perf_counter() - t2
        result['cpu_baseline'] = {'value': m / dtc, 'unit': 'points/s', 'cores': threads, 'kind': 'port',
                                  'sample': f'first {m} grid points ({m // (2048 * 64)} reference chunks), oracle/restate.py '
                                            f'mesh_alpha (get_alpha only), {dtc:.1f} s'}
        result['alpha_max_abs_err_vs_oracle'] = float((alpha[:m].cpu() - ref).abs().max())
    if not emit:
        return result
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_anim(args, rank, world, dev, emit=True):
    """Animation stage (aninerf_animation_trainer.py): one step = 65,536 observation-space + 65,536
    canonical points (get_sampling_points), forward + backward of both paths (anr_anim_step), RCCL
    mean all-reduce of the novel_pose_bw gradient blob (N > 1), clip + Adam. Weak scaling."""
    from animatable_nerf_amd import config, network, synthetic
    from animatable_nerf_amd.trainer_anim import AnimationStep, sample_unit
    cfg = config.defaults()
    cfg.aninerf_animation = True
    cfg.train_precision = args.precision
    b = synthetic.mesh_scene(voxel=0.1)
    b['bw_latent_index'] = np.array([7])
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items() if k not in ('pts', 'inside')}
    net = network.Network(cfg)
    sd = synthetic.init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    network.load_numpy_state(net, sd)
    net = net.to(dev)
    st = AnimationStep(net, cfg)
    gen = torch.Generator().manual_seed(rank)
    draws = [(sample_unit(generator=gen), sample_unit(generator=gen)) for _ in range(4)]
    for j in range(args.warmup):
        st.step(batch, *draws[j % 4])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for j in range(args.steps):
        st.step(batch, *draws[j % 4])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt_max = max_over_ranks(time.perf_counter() - t0, dev, world)
    pts = 2 * 65536
    result = {
        'metric': 'animation-stage points/s (2 x 65,536 sampled points per step, novel_pose_bw training)',
        'value': pts * args.steps * world / dt_max, 'unit': 'points/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt_max / args.steps * 1e3, 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': args.precision, 'data': 'synthetic',
        'config': {'workload': 'aninerf animation stage step (forward + backward of both paths, Adam)',
                   'points_per_step': pts, 'parallelism': f'dp{world} (RCCL mean all-reduce of the novel_pose_bw blob)'},
        'roofline': None, 'loss_last_step': st.loss3.cpu().tolist(),
    }
    if not emit:
        return result
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(sd, b, out, n_rays):
    """Oracle (PyTorch-CPU restatement) on a bounded sample of the same frame; PSNR of the HIP
    image against it over that sample (A18 formula)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import restate
    threads, host = host_threads()
    torch.set_num_threads(threads)
    P = {k: torch.from_numpy(v) for k, v in sd.items()}
    n_rays = min(n_rays, b['ray_o'].shape[1])
    sub = {k: torch.from_numpy(np.ascontiguousarray(
        v[:, :n_rays] if k in ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb') else v))
        for k, v in b.items()}
    warm = {k: (v[:, :2048] if k in ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb') else v)
            for k, v in sub.items()}
    with torch.no_grad():
        restate.render(P, warm)
        t0 = time.perf_counter()
        ref = restate.render(P, sub)
        dt = time.perf_counter() - t0
    rgb = out['rgb_map'][0, :n_rays].cpu().numpy()
    psnr = float(restate.psnr(rgb, ref['rgb_map'][0].numpy()))
    cpu = {'value': n_rays * 64 / dt, 'unit': 'ray-samples/s', 'cores': threads, 'kind': 'port',
           'sample': f'first {n_rays} rays ({n_rays // 2048} reference chunks) of the config-2 frame, '
                     f'oracle/restate.py, torch CPU {threads} threads, {dt:.1f} s', 'host': host}
    return cpu, psnr


if __name__ == '__main__':
    main()
