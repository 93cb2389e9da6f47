// anr_alpha_x6.hip — k_alpha_x6: the density program (mesh path get_alpha) with every layer in bf16x6
// (render precision ANR_BF16X6: fp32-level products on the bf16 MFMA pipe; anr_mlp_body.h V = 8).
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_alpha_x6(MlpArgs a) { ANR_STAMPED(alpha_body<true, 8>(a);); }

}  // namespace anr
