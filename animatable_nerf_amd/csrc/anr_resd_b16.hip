// anr_resd_b16.hip — k_resd_b16: the sdf_pdf residual deformation MLP (anisdf_pdf_network.py:49-73)
// as one fused launch per batch, the render kernel's machinery (anr_mlp_body.h program V = 3):
// activations in registers, hi/lo-split bf16 weights streamed through the LDS ring.
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_resd_b16(MlpArgs a) { resd_body(a); }

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
