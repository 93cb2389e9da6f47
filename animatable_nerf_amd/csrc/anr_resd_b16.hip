// anr_resd_b16.hip — the sdf_pdf render's fused MLP launches, one per batch each, on the render
// kernel's machinery (anr_mlp_body.h): activations in registers, split-bf16 weights streamed through
// the LDS ring. Render precision ANR_BF16X3 (hi/lo, 3 products per multiply-add):
//   k_resd_b16    residual deformation MLP (anisdf_pdf_network.py:49-73), program V = 3
//   k_sdfnet_b16  SDF network forward (anisdf_pdf_network.py:421-437), program V = 5
//   k_sdfgrad_b16 its input gradient d sdf / d x (anisdf_pdf_network.py:302-311), program V = 7
//   k_color_b16   colour network (anisdf_pdf_network.py:516-545), program V = 6
// and ANR_BF16X6 (hi/mid/lo, 6 products, fp32-level; anr_resd_x6.hip): k_*_x6, programs V + 10.
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_resd_b16(MlpArgs a) { ANR_STAMPED(resd_body<false>(a);); }
__global__ __launch_bounds__(512) void k_sdfnet_b16(MlpArgs a) { ANR_STAMPED(sdfnet_body<false>(a);); }
__global__ __launch_bounds__(512) void k_sdfgrad_b16(MlpArgs a) { ANR_STAMPED(sdfgrad_body<false>(a);); }
__global__ __launch_bounds__(512) void k_color_b16(MlpArgs a) { ANR_STAMPED(color_body<false>(a);); }

namespace {
// one persistent launch of a fused sdf program over the batch's rows (grid <= one workgroup per tile)
int launch_prog(const void* kernel, bool& attr, const MlpArgs& a, int grid, hipStream_t s) {
  if (!attr) {
    if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, mlp_lds_bytes<true>()) != hipSuccess)
      return -1;
    attr = true;
  }
  if (a.n_rows <= 0) return 0;
  const int ntiles = (a.n_rows + 127) / 128;
  MlpArgs args = a;
  const int g = grid < ntiles ? grid : ntiles;
  ProfSlot* ps = prof_begin(s, g);  // the sdf leg's network time and clock (anr_profile_*)
  args.clk = ps ? ps->clk : nullptr;
  void* kargs[] = {&args};
  if (hipLaunchKernel(kernel, dim3(g), dim3(512), kargs, mlp_lds_bytes<true>(), s) != hipSuccess) return -1;
  if (hipGetLastError() != hipSuccess) return -1;
  return prof_end(ps, s) == 0 ? 0 : -1;
}
bool attr_b16[4], attr_x6[4];
}  // namespace

int launch_resd(const MlpArgs& a, int grid, hipStream_t s, bool x6) {
  return x6 ? launch_prog((const void*)k_resd_x6, attr_x6[0], a, grid, s)
            : launch_prog((const void*)k_resd_b16, attr_b16[0], a, grid, s);
}
int launch_sdfnet(const MlpArgs& a, int grid, hipStream_t s, bool x6) {
  return x6 ? launch_prog((const void*)k_sdfnet_x6, attr_x6[1], a, grid, s)
            : launch_prog((const void*)k_sdfnet_b16, attr_b16[1], a, grid, s);
}
int launch_sdfgrad(const MlpArgs& a, int grid, hipStream_t s, bool x6) {
  return x6 ? launch_prog((const void*)k_sdfgrad_x6, attr_x6[2], a, grid, s)
            : launch_prog((const void*)k_sdfgrad_b16, attr_b16[2], a, grid, s);
}
int launch_color(const MlpArgs& a, int grid, hipStream_t s, bool x6) {
  return x6 ? launch_prog((const void*)k_color_x6, attr_x6[3], a, grid, s)
            : launch_prog((const void*)k_color_b16, attr_b16[3], a, grid, s);
}

}  // namespace anr
