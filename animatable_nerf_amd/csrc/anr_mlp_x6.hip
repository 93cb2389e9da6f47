// anr_mlp_x6.hip — k_mlp_x6: the fused render kernel with every MLP layer in bf16x6 (render precision
// ANR_BF16X6): weights and activations split into hi + mid + lo bf16 (24 bits, the fp32 mantissa),
// six MFMA products per multiply-add (the dropped mid*lo, lo*mid, lo*lo terms are <= ~2^-23 of the
// product), fp32 accumulation — fp32-level products on the bf16 MFMA pipe (anr_mlp_body.h V = 4).
#include "anr_mlp_body.h"

namespace anr {

__global__ __launch_bounds__(512) void k_mlp_x6(MlpArgs a) { ANR_STAMPED(mlp_body<true, 4>(a);); }

}  // namespace anr
