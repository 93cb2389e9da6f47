"""Probe: library fp32 GEMM rate (torch -> hipBLASLt / rocBLAS) at the training / sdf layer shapes,
to size what a better exact-fp32 layer GEMM could reach. Not part of the product path."""
import time

import torch

torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device('cuda:0')
for M, N, K, what in ((36864, 256, 256, 'fwd'), (73728, 256, 256, 'fwd 2n'), (524288, 256, 256, 'sdf batch'),
                      (256, 256, 36864, 'wgrad')):
    if what == 'wgrad':
        A = torch.randn(K, M, device=dev).t()  # dY^T: m-contiguous
        B = torch.randn(K, N, device=dev)
    else:
        A = torch.randn(M, K, device=dev)
        B = torch.randn(N, K, device=dev).t()
    for _ in range(3):
        C = A @ B
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        C = A @ B
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f'{what:10s} M={M} N={N} K={K}: {dt * 1e6:8.1f} us  {2 * M * N * K / dt / 1e12:6.1f} TFLOP/s', flush=True)
