// anr_alpha.hip — k_alpha: the density program of the fused network kernel (mesh path get_alpha,
// anr_mlp_body.h alpha_body), exact fp32 MFMA.
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_alpha(MlpArgs a) { ANR_STAMPED(alpha_body<false>(a);); }

}  // namespace anr
