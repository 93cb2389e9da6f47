// anr_resd_b16.hip — the sdf_pdf render's fused MLP launches (split-bf16, render precision
// ANR_BF16X3), one per batch each, on the render kernel's machinery (anr_mlp_body.h): activations in
// registers, hi/lo-split bf16 weights streamed through the LDS ring.
//   k_resd_b16    residual deformation MLP (anisdf_pdf_network.py:49-73), program V = 3
//   k_sdfnet_b16  SDF network forward (anisdf_pdf_network.py:421-437), program V = 5
//   k_sdfgrad_b16 its input gradient d sdf / d x (anisdf_pdf_network.py:302-311), program V = 7
//   k_color_b16   colour network (anisdf_pdf_network.py:516-545), program V = 6
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_resd_b16(MlpArgs a) { resd_body(a); }
__global__ __launch_bounds__(512) void k_sdfnet_b16(MlpArgs a) { sdfnet_body(a); }
__global__ __launch_bounds__(512) void k_sdfgrad_b16(MlpArgs a) { sdfgrad_body(a); }
__global__ __launch_bounds__(512) void k_color_b16(MlpArgs a) { color_body(a); }

int launch_color(const MlpArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k_color_b16, hipFuncAttributeMaxDynamicSharedMemorySize,
                            mlp_lds_bytes<true>()) != hipSuccess)
      return -1;
    attr = true;
  }
  if (a.n_rows <= 0) return 0;
  const int ntiles = (a.n_rows + 127) / 128;
  hipLaunchKernelGGL(k_color_b16, dim3(grid < ntiles ? grid : ntiles), dim3(512), mlp_lds_bytes<true>(), s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_sdfgrad(const MlpArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k_sdfgrad_b16, hipFuncAttributeMaxDynamicSharedMemorySize,
                            mlp_lds_bytes<true>()) != hipSuccess)
      return -1;
    attr = true;
  }
  if (a.n_rows <= 0) return 0;
  const int ntiles = (a.n_rows + 127) / 128;
  hipLaunchKernelGGL(k_sdfgrad_b16, dim3(grid < ntiles ? grid : ntiles), dim3(512), mlp_lds_bytes<true>(), s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_sdfnet(const MlpArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k_sdfnet_b16, hipFuncAttributeMaxDynamicSharedMemorySize,
                            mlp_lds_bytes<true>()) != hipSuccess)
      return -1;
    attr = true;
  }
  if (a.n_rows <= 0) return 0;
  const int ntiles = (a.n_rows + 127) / 128;
  hipLaunchKernelGGL(k_sdfnet_b16, dim3(grid < ntiles ? grid : ntiles), dim3(512), mlp_lds_bytes<true>(), s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_resd(const MlpArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k_resd_b16, hipFuncAttributeMaxDynamicSharedMemorySize, mlp_lds_bytes<true>()) !=
        hipSuccess)
      return -1;
    attr = true;
  }
  if (a.n_rows <= 0) return 0;
  const int ntiles = (a.n_rows + 127) / 128;
  hipLaunchKernelGGL(k_resd_b16, dim3(grid < ntiles ? grid : ntiles), dim3(512), mlp_lds_bytes<true>(), s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace anr
