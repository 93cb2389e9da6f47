// anr_mlp_b16.hip — k_mlp_b16: the fused network kernel with the T-pose BW MLP and the NeRF in
// hi/lo-split bf16 MFMA (render precision ANR_BF16X3; anr_mlp_body.h, anr_layers.h).
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_mlp_b16(MlpArgs a) { ANR_STAMPED(mlp_body<true>(a);); }

}  // namespace anr
