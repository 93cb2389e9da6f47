"""CPU: the C-ABI library loads and exports every symbol include/aninerf.h declares; host-side
contracts (sizes, argument validation) without compute calls."""
import ctypes
import os
import re

import pytest

from animatable_nerf_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'aninerf.h')


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r'\b(anr_[a-z_0-9]+)\s*\(', src)))


def test_header_matches_binding_list():
    assert set(declared_symbols()) == set(_lib.EXPORTS)


@pytest.fixture(scope='module')
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail('libaninerf_hip.so is not built (run `make` / __graft_entry__.build())')
    return _lib.load()


def test_library_exports_every_declared_symbol(lib):
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_version_and_sizes(lib):
    assert lib.anr_version() == 2
    assert _lib.TrainHooks().struct_size == ctypes.sizeof(_lib.TrainHooks) == 40
    # 19 weight layers + view/rgb heads, fp32 weight image + padded biases
    # + 9 novel_pose_bw layers (same image as the 9 BW layers)
    # + alpha_fc alone (layer 30, the mesh path's density program): 64 k-steps x 1 KiB, 16 biases
    # + the folded colour head (layer 31: 72 k-steps x 3 chunks x 1 KiB, 9 x 16 biases from the per-frame fold)
    fp32 = 4_767_744 + 2_031_616 + 65_536 + 221_184 + 4 * (4_800 + 2_080 + 16 + 144)  # fp32 image + biases
    # bf16x3 image: per layer ceil(in/32) k-steps x out-blocks x 2 KiB (hi + lo fragments)
    ks_ob = [(2, 16), (8, 16), (8, 16), (8, 16), (8, 16), (10, 16), (8, 16), (8, 16), (8, 2),
             (2, 16), (8, 16), (8, 16), (8, 16), (8, 16), (10, 16), (8, 16), (8, 16), (8, 17), (8, 16), (9, 8), (4, 1)]
    # + novel copy, alpha, the folded colour head (layer 31: 9 k-steps x 9 out-blocks)
    b16 = (sum(k * o for k, o in ks_ob) + sum(k * o for k, o in ks_ob[:9]) + 8 * 1 + 9 * 9) * 2048
    # bf16x6 image (render precision bf16x6): every layer 0..31 as hi/mid/lo fragments, 3 KiB per (k-step, out-block)
    x6 = (sum(k * o for k, o in ks_ob) + sum(k * o for k, o in ks_ob[:9]) + 8 * 1 + 9 * 9) * 3072
    base16 = (fp32 + 255) // 256 * 256
    end_x6 = (base16 + b16 + 255) // 256 * 256 + x6
    # head region: H (129 x 283), P (128 x 128), q (128) f32, then fp64 scratch G (128 x 256) and u (256)
    head = (end_x6 + 255) // 256 * 256
    scratch = (head + 4 * (129 * 283 + 128 * 128 + 128) + 255) // 256 * 256
    assert lib.anr_params_packed_bytes() == scratch + 8 * (128 * 256 + 256)


def test_workspace_grows_with_rays(lib):
    o = _lib.RenderOpts(64, 2048, 0.05, 0.0, None)
    f = _lib.Frame()
    for i, d in enumerate((25, 73, 17)):
        f.pbw_dims[i] = d
        f.tbw_dims[i] = d
    a = lib.anr_render_workspace_bytes(1024, ctypes.byref(o), ctypes.byref(f))
    b = lib.anr_render_workspace_bytes(262144, ctypes.byref(o), ctypes.byref(f))
    assert 0 < a < b
    assert b < 8 * 2 ** 30  # fits comfortably in 288 GB HBM


def test_argument_errors_do_not_launch(lib):
    # NULL arguments are rejected before any HIP call (no GPU needed)
    rc = lib.anr_render_fwd(None, None, None, None, None, None, 0, None, None, None, 0, None)
    assert rc == 2
    assert b'NULL' in lib.anr_last_error()
    o = _lib.RenderOpts(32, 2048, 0.05, 0.0, None)
    p = _lib.Params()
    f = _lib.Frame()
    out = _lib.RenderOut()
    rc = lib.anr_render_fwd(ctypes.byref(p), ctypes.byref(f), None, None, None, None, 10, ctypes.byref(o),
                            ctypes.byref(out), ctypes.c_void_p(1), 0, None)
    assert rc == 2 and b'N_samples' in lib.anr_last_error()
    assert lib.anr_near_far(None, None, -1, None, None, None, None, None) == 2
