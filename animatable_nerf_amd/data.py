"""Eval-split ray pipeline on the device: ``get_rays`` /
``get_rays_within_bounds`` of ``lib/utils/if_nerf/if_nerf_data_utils.py:64-89, 310-339`` through
``anr_camera_rays`` (include/aninerf.h). The 3x3 inverse of K and the camera origin -R^T T are
formed with numpy on the host exactly as the reference does; the per-pixel rays, the box test and
the ordered hit list run on the GPU, so a full-resolution render needs no host ray generation.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def _camera(K, R, T):
    K = np.asarray(K)
    R = np.asarray(R)
    T = np.asarray(T)
    fp64 = K.dtype == np.float64 or R.dtype == np.float64 or T.dtype == np.float64
    Kinv = np.linalg.inv(K)                  # if_nerf_data_utils.py:81
    origin = -np.dot(R.T, T).ravel()         # :76
    as_d = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1))
    return as_d(Kinv), as_d(R), as_d(T), as_d(origin), fp64


def get_rays_within_bounds(H, W, K, R, T, bounds, device='cuda'):
    """-> ray_o (n,3), ray_d (n,3), near (n,), far (n,), mask_at_box (H,W) bool, coord (n,2) int32,
    all on ``device`` (the reference returns numpy arrays of the same values)."""
    lib = _lib.load()
    dev = torch.device(device)
    Kinv, Rd, Td, o, fp64 = _camera(K, R, T)
    P = H * W
    b = torch.as_tensor(np.asarray(bounds, dtype=np.float32).reshape(2, 3)).to(dev)
    ray_o = torch.empty((P, 3), device=dev)
    ray_d = torch.empty((P, 3), device=dev)
    near = torch.empty(P, device=dev)
    far = torch.empty(P, device=dev)
    coord = torch.empty((P, 2), dtype=torch.int32, device=dev)
    mask = torch.empty(P, dtype=torch.uint8, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    ws_bytes = lib.anr_camera_rays_workspace_bytes(H, W)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    _lib.check(lib.anr_camera_rays(H, W, dp(Kinv), dp(Rd), dp(Td), dp(o), 1 if fp64 else 0, _lib.ptr(b),
                                   _lib.ptr(ray_o), _lib.ptr(ray_d), _lib.ptr(near), _lib.ptr(far), _lib.ptr(coord),
                                   _lib.ptr(mask), _lib.ptr(count), _lib.ptr(ws), ws_bytes, _lib.stream_ptr(dev)),
               'anr_camera_rays')
    n = int(count.item())
    return ray_o[:n], ray_d[:n], near[:n], far[:n], mask.view(H, W).bool(), coord[:n]
