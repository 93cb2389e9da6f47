// anr_alpha_b16.hip — k_alpha_b16: the density program (mesh path get_alpha) with the NeRF trunk and
// alpha_fc (and the pose pass, like k_mlp_b16) in hi/lo-split bf16 MFMA (ANR_BF16X3; anr_mlp_body.h).
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_alpha_b16(MlpArgs a) { ANR_STAMPED(alpha_body<true>(a);); }

}  // namespace anr
