// anr_resd_x6.hip — the sdf_pdf render's fused MLP programs in render precision ANR_BF16X6 (every
// weight and activation as hi/mid/lo bf16, six MFMA products per multiply-add with fp32 accumulation:
// fp32-level products; softplus and its backward factor at libm accuracy): programs 13, 15, 17, 16 =
// the bf16x3 programs 3, 5, 7, 6 of anr_resd_b16.hip (own TU: the two instantiation sets build in
// parallel). Launched through anr_resd_b16.hip's launch_* (x6 = true).
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_resd_x6(MlpArgs a) { ANR_STAMPED(resd_body<true>(a);); }
__global__ __launch_bounds__(512) void k_sdfnet_x6(MlpArgs a) { ANR_STAMPED(sdfnet_body<true>(a);); }
__global__ __launch_bounds__(512) void k_sdfgrad_x6(MlpArgs a) { ANR_STAMPED(sdfgrad_body<true>(a);); }
__global__ __launch_bounds__(512) void k_color_x6(MlpArgs a) { ANR_STAMPED(color_body<true>(a);); }

}  // namespace anr
