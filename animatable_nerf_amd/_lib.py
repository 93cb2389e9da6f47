"""ctypes binding of the C-ABI library ``libaninerf_hip.so`` (include/aninerf.h).

The library is built in-tree by ``make`` (``__graft_entry__.build()``). Loading it is mandatory:
there is no CPU or PyTorch fallback for the render path, a missing or stale library raises.
``torch`` is imported first so the HIP runtime torch ships (same SONAME ``libamdhip64.so.7``)
is the one the library binds to — one runtime, one set of streams.
"""
import ctypes
import os

import torch  # noqa: F401  (must be loaded before the library, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libaninerf_hip.so')
# kernel experiments (tools/): an alternative build of the same C-ABI, e.g. with other -D options
if os.environ.get('ANR_LIB_PATH'):
    LIB_PATH = os.environ['ANR_LIB_PATH']
NUM_TENSORS = 46
NUM_NOVEL_TENSORS = 19
NUM_SDF_TENSORS = 63

EXPORTS = ('anr_near_far', 'anr_params_packed_bytes', 'anr_params_pack', 'anr_render_workspace_bytes',
           'anr_render_fwd', 'anr_render_counts', 'anr_render_bw_rows', 'anr_render_row_ids', 'anr_profile_enable', 'anr_profile_read', 'anr_profile_read_clock',
           'anr_train_workspace_bytes', 'anr_train_fwd', 'anr_train_bwd', 'anr_train_step', 'anr_adam',
           'anr_camera_rays_workspace_bytes', 'anr_camera_rays', 'anr_sdf_render_workspace_bytes', 'anr_sdf_render_fwd', 'anr_sdf_render_counts', 'anr_sdf_render_rows',
           'anr_alpha_workspace_bytes', 'anr_alpha_points', 'anr_alpha_counts', 'anr_mc_workspace_bytes',
           'anr_mc_count', 'anr_mc_emit', 'anr_anim_workspace_bytes', 'anr_anim_step',
           'anr_train_ray_workspace_bytes', 'anr_train_ray_lists', 'anr_train_ray_gather',
           'anr_network_workspace_bytes', 'anr_network_fwd', 'anr_network_counts', 'anr_network_bw_rows',
           'anr_network_train_workspace_bytes', 'anr_network_train_fwd', 'anr_network_train_bwd',
           'anr_points_workspace_bytes', 'anr_blend_weights', 'anr_canonical_alpha', 'anr_train_step_hooked',
           'anr_sdf_train_workspace_bytes', 'anr_sdf_train_step', 'anr_sdf_train_step_hooked', 'anr_sdf_render_knn',
           'anr_sdf_network_workspace_bytes', 'anr_sdf_network_fwd', 'anr_sdf_network_counts', 'anr_sdf_network_rows',
           'anr_sdf_network_train_workspace_bytes', 'anr_sdf_network_train_fwd', 'anr_sdf_network_train_counts',
           'anr_sdf_network_train_rows', 'anr_sdf_network_train_bwd', 'anr_sdf_points_workspace_bytes', 'anr_sdf_points',
           'anr_sample_volume', 'anr_knn_blend_workspace_bytes', 'anr_knn_blend', 'anr_sdf_mesh_pose',
           'anr_last_error', 'anr_version')

c_float_p = ctypes.c_void_p


class Params(ctypes.Structure):
    _fields_ = [('t', ctypes.c_void_p * NUM_TENSORS), ('num_train_frame', ctypes.c_int),
                ('packed', ctypes.c_void_p), ('novel', ctypes.c_void_p * NUM_NOVEL_TENSORS)]


class Frame(ctypes.Structure):
    _fields_ = [('A', ctypes.c_void_p), ('R', ctypes.c_void_p), ('Th', ctypes.c_void_p),
                ('pbw', ctypes.c_void_p), ('pbw_dims', ctypes.c_int * 3), ('pbounds', ctypes.c_void_p),
                ('tbw', ctypes.c_void_p), ('tbw_dims', ctypes.c_int * 3), ('tbounds', ctypes.c_void_p),
                ('latent_index', ctypes.c_void_p), ('bw_latent_index', ctypes.c_void_p),
                ('n_views', ctypes.c_int), ('Ks', ctypes.c_void_p), ('RT', ctypes.c_void_p), ('msks', ctypes.c_void_p),
                ('img_h', ctypes.c_int), ('img_w', ctypes.c_int)]


class RenderOpts(ctypes.Structure):
    _fields_ = [('n_samples', ctypes.c_int), ('chunk', ctypes.c_int), ('norm_th', ctypes.c_float),
                ('train_th', ctypes.c_float), ('t_rand', ctypes.c_void_p), ('novel_pose', ctypes.c_int),
                ('precision', ctypes.c_int)]


FP32, BF16, BF16_ALL, BF16X3, BF16X6 = 0, 1, 2, 3, 4  # anr_render_opts.precision


class RenderOut(ctypes.Structure):
    _fields_ = [('rgb_map', ctypes.c_void_p), ('acc_map', ctypes.c_void_p), ('depth_map', ctypes.c_void_p),
                ('raw', ctypes.c_void_p)]


class Samples(ctypes.Structure):
    _fields_ = [('wpts', ctypes.c_void_p), ('viewdir', ctypes.c_void_p), ('dists', ctypes.c_void_p),
                ('n_pts', ctypes.c_int)]


REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)
SDFP_NETWORK, SDFP_GRADIENT, SDFP_DEFORMED_GRADIENT = 0, 1, 2  # anr_sdf_points modes
REDUCE_MIN_U64, REDUCE_MAX_U64, REDUCE_SUM_F32 = 0, 1, 2  # anr_train_hooks.reduce ops


class TrainHooks(ctypes.Structure):
    """anr_train_hooks (ANR_TRAIN_HOOKS_VERSION 2): struct_size is filled in by the constructor."""
    _fields_ = [('struct_size', ctypes.c_size_t), ('nerf_grads_ready', ctypes.c_void_p), ('ray_offset', ctypes.c_int),
                ('reduce', REDUCE_FN), ('reduce_user', ctypes.c_void_p)]

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(TrainHooks), *args, **kw)


READY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)


class SdfTrainHooks(ctypes.Structure):
    """anr_sdf_train_hooks: struct_size is filled in by the constructor."""
    _fields_ = [('struct_size', ctypes.c_size_t), ('colour_grads_ready', ctypes.c_void_p), ('colour_ready', READY_FN),
                ('user', ctypes.c_void_p)]

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(SdfTrainHooks), *args, **kw)


class AlphaOpts(ctypes.Structure):
    _fields_ = [('chunk_pts', ctypes.c_int), ('norm_th', ctypes.c_float), ('novel_pose', ctypes.c_int),
                ('precision', ctypes.c_int)]


class SdfParams(ctypes.Structure):
    _fields_ = [('t', ctypes.c_void_p * NUM_SDF_TENSORS)]


class SdfFrame(ctypes.Structure):
    _fields_ = [('A', ctypes.c_void_p), ('big_A', ctypes.c_void_p), ('R', ctypes.c_void_p), ('Th', ctypes.c_void_p),
                ('poses', ctypes.c_void_p), ('pvertices', ctypes.c_void_p), ('weights', ctypes.c_void_p),
                ('n_verts', ctypes.c_int), ('tbounds', ctypes.c_void_p), ('latent_index', ctypes.c_void_p),
                ('occupancy', ctypes.c_void_p), ('n_views', ctypes.c_int), ('Ks', ctypes.c_void_p),
                ('RT', ctypes.c_void_p), ('msks', ctypes.c_void_p), ('img_h', ctypes.c_int), ('img_w', ctypes.c_int)]


class SdfRenderOut(ctypes.Structure):
    _fields_ = [('rgb_map', ctypes.c_void_p), ('acc_map', ctypes.c_void_p), ('depth_map', ctypes.c_void_p),
                ('raw', ctypes.c_void_p), ('sdf', ctypes.c_void_p), ('tbounds_out', ctypes.c_void_p)]


_lib = None


def load():
    """Load (once) and return the library; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f'{LIB_PATH} not built: run `make` (or __graft_entry__.build()) first; '
                           'the HIP path has no fallback')
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    lib.anr_near_far.argtypes = [P, P, ctypes.c_int, P, P, P, P, P]
    lib.anr_params_packed_bytes.restype = ctypes.c_size_t
    lib.anr_params_pack.argtypes = [ctypes.POINTER(Params), P, P]
    lib.anr_render_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_render_workspace_bytes.argtypes = [ctypes.c_int, ctypes.POINTER(RenderOpts), ctypes.POINTER(Frame)]
    lib.anr_render_fwd.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(Frame), P, P, P, P, ctypes.c_int,
                                   ctypes.POINTER(RenderOpts), ctypes.POINTER(RenderOut), P, ctypes.c_size_t, P]
    lib.anr_render_counts.restype = P
    lib.anr_render_counts.argtypes = [P, ctypes.c_int]
    lib.anr_render_bw_rows.argtypes = [P, ctypes.c_int, P, P, P]
    lib.anr_render_row_ids.argtypes = [P, ctypes.c_int, P, P]
    lib.anr_train_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_train_workspace_bytes.argtypes = [ctypes.c_int, ctypes.POINTER(RenderOpts), ctypes.POINTER(Frame)]
    lib.anr_train_fwd.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(Frame), P, P, P, P, ctypes.c_int,
                                  ctypes.POINTER(RenderOpts), ctypes.POINTER(RenderOut), P, ctypes.c_size_t, P]
    lib.anr_train_bwd.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p * NUM_TENSORS, ctypes.POINTER(Frame), P, P, P, P,
                                  ctypes.c_int, ctypes.POINTER(RenderOpts), P, P, P, P, ctypes.c_size_t, P]
    lib.anr_train_step.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p * NUM_TENSORS, ctypes.POINTER(Frame), P, P, P,
                                   P, ctypes.c_int, ctypes.POINTER(RenderOpts), P, P, ctypes.POINTER(RenderOut), P, P,
                                   ctypes.c_size_t, P]
    lib.anr_train_step_hooked.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p * NUM_TENSORS, ctypes.POINTER(Frame), P,
                                          P, P, P, ctypes.c_int, ctypes.POINTER(RenderOpts), P, P,
                                          ctypes.POINTER(RenderOut), P, ctypes.POINTER(TrainHooks), P, ctypes.c_size_t, P]
    lib.anr_adam.argtypes = [P, P, P, P, ctypes.c_long, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                             ctypes.c_float, ctypes.c_int, ctypes.c_float, P]
    lib.anr_sdf_render_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_sdf_render_workspace_bytes.argtypes = [ctypes.c_int, ctypes.POINTER(RenderOpts)]
    lib.anr_sdf_render_fwd.argtypes = [ctypes.POINTER(SdfParams), ctypes.POINTER(SdfFrame), P, P, P, P, ctypes.c_int,
                                       ctypes.POINTER(RenderOpts), ctypes.POINTER(SdfRenderOut), P, ctypes.c_size_t, P]
    lib.anr_sdf_render_counts.restype = P
    lib.anr_sdf_render_counts.argtypes = [P, ctypes.c_int, ctypes.POINTER(RenderOpts)]
    lib.anr_sdf_render_knn.restype = P
    lib.anr_sdf_render_knn.argtypes = [P, ctypes.c_int, ctypes.POINTER(RenderOpts)]
    lib.anr_sdf_render_rows.argtypes = [P, ctypes.c_int, ctypes.POINTER(RenderOpts), P, P, P, P, P]
    lib.anr_sdf_train_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_sdf_train_workspace_bytes.argtypes = [ctypes.c_int, ctypes.POINTER(RenderOpts)]
    lib.anr_sdf_train_step.argtypes = [ctypes.POINTER(SdfParams), ctypes.c_void_p * NUM_SDF_TENSORS,
                                       ctypes.POINTER(SdfFrame), P, P, P, P, ctypes.c_int, ctypes.POINTER(RenderOpts),
                                       P, P, ctypes.c_int, ctypes.POINTER(SdfRenderOut), P, P, ctypes.c_size_t, P]
    lib.anr_sdf_train_step_hooked.argtypes = [ctypes.POINTER(SdfParams), ctypes.c_void_p * NUM_SDF_TENSORS,
                                              ctypes.POINTER(SdfFrame), P, P, P, P, ctypes.c_int,
                                              ctypes.POINTER(RenderOpts), P, P, ctypes.c_int,
                                              ctypes.POINTER(SdfRenderOut), P, ctypes.POINTER(SdfTrainHooks), P,
                                              ctypes.c_size_t, P]
    SP, SF, SS = ctypes.POINTER(SdfParams), ctypes.POINTER(SdfFrame), ctypes.POINTER(Samples)
    lib.anr_sdf_network_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_sdf_network_workspace_bytes.argtypes = [ctypes.c_int, ctypes.POINTER(RenderOpts)]
    lib.anr_sdf_network_fwd.argtypes = [SP, SF, SS, ctypes.POINTER(RenderOpts), P, P, P, P, ctypes.c_size_t, P]
    lib.anr_sdf_network_counts.restype = P
    lib.anr_sdf_network_counts.argtypes = [P, ctypes.c_int]
    lib.anr_sdf_network_rows.argtypes = [P, ctypes.c_int, P, P, P]
    lib.anr_sdf_network_train_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_sdf_network_train_workspace_bytes.argtypes = [ctypes.c_int]
    lib.anr_sdf_network_train_fwd.argtypes = [SP, SF, SS, ctypes.POINTER(RenderOpts), P, P, P, P, ctypes.c_size_t, P]
    lib.anr_sdf_network_train_counts.restype = P
    lib.anr_sdf_network_train_counts.argtypes = [P, ctypes.c_int]
    lib.anr_sdf_network_train_rows.argtypes = [P, ctypes.c_int, P, P, P, P]
    lib.anr_sdf_network_train_bwd.argtypes = [SP, ctypes.c_void_p * NUM_SDF_TENSORS, SF, SS, ctypes.POINTER(RenderOpts),
                                              P, P, P, P, P, P, ctypes.c_size_t, P]
    lib.anr_sdf_points_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_sdf_points_workspace_bytes.argtypes = [ctypes.c_int]
    lib.anr_sdf_points.argtypes = [SP, SF, P, ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_size_t, P]
    lib.anr_sample_volume.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int, P, P]
    lib.anr_knn_blend_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_knn_blend_workspace_bytes.argtypes = [ctypes.c_int]
    lib.anr_knn_blend.argtypes = [P, P, ctypes.c_int, P, ctypes.c_int, ctypes.c_float, P, P, P, ctypes.c_size_t, P]
    lib.anr_sdf_mesh_pose.argtypes = [P, P, ctypes.c_int, P, P, P, P, P, P]
    lib.anr_camera_rays_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_camera_rays_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    D = ctypes.POINTER(ctypes.c_double)
    lib.anr_camera_rays.argtypes = [ctypes.c_int, ctypes.c_int, D, D, D, D, ctypes.c_int, P, P, P, P, P, P, P, P, P,
                                    ctypes.c_size_t, P]
    lib.anr_train_ray_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_train_ray_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.anr_train_ray_lists.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, P, ctypes.c_size_t, P]
    lib.anr_train_ray_gather.argtypes = [ctypes.c_int, ctypes.c_int, D, D, D, D, ctypes.c_int, P, P, P, ctypes.c_int,
                                         P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         P, P, P, P, P, P, P, P]
    lib.anr_alpha_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_alpha_workspace_bytes.argtypes = [ctypes.c_long, ctypes.POINTER(AlphaOpts), ctypes.POINTER(Frame)]
    lib.anr_alpha_points.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(Frame), P, ctypes.c_long,
                                     ctypes.POINTER(AlphaOpts), P, P, ctypes.c_size_t, P]
    lib.anr_alpha_counts.restype = P
    lib.anr_alpha_counts.argtypes = [P]
    lib.anr_mc_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_mc_workspace_bytes.argtypes = [ctypes.c_int] * 4
    lib.anr_mc_count.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, P, P,
                                 ctypes.c_size_t, P]
    lib.anr_mc_emit.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, P, P, P,
                                ctypes.c_size_t, P]
    lib.anr_anim_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_anim_workspace_bytes.argtypes = [ctypes.c_int]
    lib.anr_anim_step.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p * NUM_NOVEL_TENSORS, ctypes.POINTER(Frame), P,
                                  ctypes.c_int, P, ctypes.c_int, ctypes.POINTER(RenderOpts), P, P, ctypes.c_size_t, P]
    S, PP, PF, PO = ctypes.POINTER(Samples), ctypes.POINTER(Params), ctypes.POINTER(Frame), ctypes.POINTER(RenderOpts)
    for name in ('anr_network_workspace_bytes', 'anr_network_train_workspace_bytes'):
        getattr(lib, name).restype = ctypes.c_size_t
        getattr(lib, name).argtypes = [ctypes.c_int, PO, PF]
    lib.anr_network_fwd.argtypes = [PP, PF, S, PO, P, P, ctypes.c_size_t, P]
    lib.anr_network_train_fwd.argtypes = [PP, PF, S, PO, P, P, ctypes.c_size_t, P]
    lib.anr_network_train_bwd.argtypes = [PP, ctypes.c_void_p * NUM_TENSORS, PF, S, PO, P, P, P, P, ctypes.c_size_t, P]
    lib.anr_network_counts.restype = P
    lib.anr_network_counts.argtypes = [P, ctypes.c_int]
    lib.anr_network_bw_rows.argtypes = [P, ctypes.c_int, P, P, P]
    lib.anr_points_workspace_bytes.restype = ctypes.c_size_t
    lib.anr_points_workspace_bytes.argtypes = [ctypes.c_int]
    lib.anr_blend_weights.argtypes = [PP, ctypes.c_int, P, P, ctypes.c_int, P, ctypes.c_int, P, P, ctypes.c_size_t, P]
    lib.anr_canonical_alpha.argtypes = [PP, P, ctypes.c_int, P, P, ctypes.c_size_t, P]
    lib.anr_profile_enable.argtypes = [ctypes.c_int]
    lib.anr_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
    lib.anr_profile_read_clock.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_double)]
    lib.anr_last_error.restype = ctypes.c_char_p
    for name in EXPORTS:
        getattr(lib, name)
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = _lib.anr_last_error().decode() if _lib is not None else ''
        raise RuntimeError(f'{what} failed (code {rc}): {msg}')


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
