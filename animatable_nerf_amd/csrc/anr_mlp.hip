// anr_mlp.hip — k_mlp: the fused network kernel with exact fp32 MFMA everywhere (anr_mlp_body.h).
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_mlp(MlpArgs a) { ANR_STAMPED(mlp_body<false>(a);); }

}  // namespace anr
