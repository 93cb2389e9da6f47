// anr_tchain.hip — fused forward chains of the bf16 training executor (training precisions bf16 /
// bf16_all, A17): one launch runs a whole MLP of tpose_nerf_network.py over the kept samples, the
// activations chained in registers from layer to layer instead of round-tripping through HBM between
// one row-GEMM launch per layer (anr_tgemm.hip k_rgemm).
//
//   program BW (the blend-weight MLP, :55-77; pose pass with latent li + 1, T-pose pass with latent 0):
//     gamma(x) -> 8 x 256 ReLU (skip [gamma, h4] into layer 5; latents folded into the layer-0/5
//     biases) -> bw_fc (24 logits)
//   program NF (TPoseHuman.calculate_alpha_rgb, :252-275): gamma(x_T) -> 8 x 256 ReLU (skip into
//     layer 5) -> feature_fc || alpha_fc -> latent_fc (latent folded) -> view_fc [latent, gamma(dir)]
//     ReLU -> rgb_fc
//
// Arithmetic is the layer-wise bf16 path's: bf16 (RNE) weights and activations, fp32 accumulation,
// bias, ReLU, then RNE to bf16 for the stored rows AND for the next layer's operand (the values the
// layer-wise path reads back), so the backward sees the same activations.
//
// Layout: workgroup = 7 compute waves x 16 samples (a 112-sample tile, TC_TR) + 1 producer wave,
// persistent over tiles (below, before tc_body). v_mfma_f32_16x16x32_bf16 with the weights as the A
// operand (16 output neurons x 32 inputs) and the samples as B: the C fragment of out-blocks 2s, 2s+1 is
// the B fragment of the next layer's k-step s when the packed weight columns follow the same neuron
// order (tc_nrn: lane h of a sample holds neurons 32s + 8h + 0..7, one 16-B row store per k-step pair),
// so activations never leave registers. Memory segments (gamma rows, gamma(dir) rows) are read straight
// into B fragments in natural column order. Weights stream through an LDS ring of slices (one 32-input
// k-step of all of a layer's out-blocks, <= 20 KiB; 8 slots BW, 6 NeRF, 7 backward) by LDS-DMA that the
// producer wave alone issues and waits for (counted vmcnt), one barrier per slice; biases sit in an LDS
// table filled once per launch. Each layer's outputs are stored once (bf16 rows for the backward's
// masks and weight gradients; fp32 heads) while the next layer's MFMAs run.
#include <type_traits>

#include "anr_common.h"
#include "anr_kernels.h"
#include "anr_train.h"

namespace anr {

namespace {

typedef __bf16 tc_bf16x8 __attribute__((ext_vector_type(8)));

template <int B, int E, typename F>
__device__ __forceinline__ void tc_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    tc_for<B + 1, E>(f);
  }
}

// one layer of a chain program
struct TcL {
  int ob;          // output blocks of 16 neurons
  int kmem;        // k-steps (32 inputs) from a memory segment (rows), 0 = none
  int kprev;       // k-steps from the previous layer's outputs (registers)
  int mem_first;   // the memory segment's k-steps come first (weight-image and MFMA order)
  int relu;
  int out;         // TC_BF16 / TC_F32 rows, TC_FA (feature bf16 || alpha fp32), TC_SPLIT (blocks 0..15 bf16 rows,
                   // the rest fp32 aux rows), TC_AUX (every block fp32 aux rows)
  int mem2;        // the memory segment is the second memory operand
  int mask;        // backward: multiply by the ReLU mask (H > 0) of the forward's activations, read from the
                   // mask bits the forward chain wrote (TcArgs::bits), LDS-DMA'd with the layer's first slice
  int aux_add;     // TC_SPLIT / TC_AUX: add into the aux rows (else store)
};
enum { TC_BF16 = 0, TC_F32 = 1, TC_FA = 2, TC_SPLIT = 3, TC_AUX = 4 };

// forward programs: 0 the blend-weight MLP, 1 the NeRF with its heads
constexpr TcL kProgBW[9] = {
    {16, 2, 0, 1, 1, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0},
    {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {16, 2, 8, 1, 1, TC_BF16, 0, 0, 0},
    {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {2, 0, 8, 0, 0, TC_F32, 0, 0, 0}};
constexpr TcL kProgNF[12] = {
    {16, 2, 0, 1, 1, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0},
    {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {16, 2, 8, 1, 1, TC_BF16, 0, 0, 0},
    {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 1, TC_BF16, 0, 0, 0}, {17, 0, 8, 0, 0, TC_FA, 0, 0, 0},
    {16, 0, 8, 0, 0, TC_BF16, 0, 0, 0}, {8, 1, 8, 0, 1, TC_F32, 1, 0, 0}, {1, 0, 4, 0, 0, TC_F32, 0, 0, 0}};
// input-gradient programs (transposed weights, no bias): 2 the blend-weight MLP from the logit gradient
// (bw_fc, layers 7..0; layer 5 also the gamma gradient, stored; layer 0 adds its gamma gradient);
// 3 the NeRF from d rgb (rgb_fc with the View ReLU mask, view_fc to the latent input, latent_fc,
// feature_fc || alpha_fc with d alpha, layers 7..0 as in 2)
constexpr TcL kProgBWB[9] = {
    {16, 1, 0, 1, 0, TC_BF16, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0},
    {20, 0, 8, 0, 0, TC_SPLIT, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0},
    {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0}, {4, 0, 8, 0, 0, TC_AUX, 0, 0, 1}};
constexpr TcL kProgNFB[12] = {
    {8, 1, 0, 1, 0, TC_F32, 0, 1, 0},   {16, 0, 4, 0, 0, TC_BF16, 0, 0, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 0, 0},
    {16, 1, 8, 0, 0, TC_BF16, 1, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0},
    {20, 0, 8, 0, 0, TC_SPLIT, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0},
    {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0}, {16, 0, 8, 0, 0, TC_BF16, 0, 1, 0}, {4, 0, 8, 0, 0, TC_AUX, 0, 0, 1}};

template <int P>
__host__ __device__ constexpr int tc_nl() { return (P == 0 || P == 2) ? 9 : 12; }
template <int P>
__host__ __device__ constexpr TcL tc_layer(int l) {
  return P == 0 ? kProgBW[l] : P == 1 ? kProgNF[l] : P == 2 ? kProgBWB[l] : kProgNFB[l];
}
template <int P>
__host__ __device__ constexpr bool tc_bwd() { return P >= 2; }
// k-steps of the programs' memory operands (loaded once per tile): gamma 2 (forward), the logit / rgb
// gradient 1 (backward); the second operand (gamma(dir), d alpha) 1
template <int P>
__host__ __device__ constexpr int tc_ks(int l) { return tc_layer<P>(l).kmem + tc_layer<P>(l).kprev; }
// first slice of layer l, total slices
template <int P>
__host__ __device__ constexpr int tc_slice0(int l) {
  int q = 0;
  for (int i = 0; i < l; ++i) q += tc_ks<P>(i);
  return q;
}
template <int P>
__host__ __device__ constexpr int tc_nslices() { return tc_slice0<P>(tc_nl<P>()); }
// layer of slice q
template <int P>
__host__ __device__ constexpr int tc_layer_of(int q) {
  int l = 0;
  while (l + 1 < tc_nl<P>() && tc_slice0<P>(l + 1) <= q) ++l;
  return l;
}
// KiB offset of slice q in the program's weight image, and its out-blocks
template <int P>
__host__ __device__ constexpr int tc_slice_kb(int q) {
  int kb = 0;
  for (int i = 0; i < q; ++i) kb += tc_layer<P>(tc_layer_of<P>(i)).ob;
  return kb;
}
template <int P>
__host__ __device__ constexpr int tc_image_kb() { return tc_slice_kb<P>(tc_nslices<P>()); }
template <int P>
__host__ __device__ constexpr int tc_obmax() { return P == 0 ? 16 : P == 1 ? 17 : 20; }
template <int P>
__host__ __device__ constexpr int tc_memk() { return tc_bwd<P>() ? 1 : 2; }
// LDS-DMA pieces (1 KiB) every wave issues per slice (pieces past a slice's out-blocks repeat its last)
template <int P>
__host__ __device__ constexpr int tc_pieces() { return (tc_obmax<P>() + 7) / 8; }
// ring slots: a slice certified at the middle of the slice before it was issued NB - 2 slices earlier,
// so NB - 2 slices of MFMA work cover the L2 latency of the weight stream (4 slots: 1.5 us per slice
// measured on a 195-tile BW pass, latency-bound; 8 / 7 fill what the LDS holds)
#ifndef TC_NB_BW
#define TC_NB_BW 8
#endif
#ifndef TC_NB_NF
#define TC_NB_NF 6
#endif
#ifndef TC_NB_BWD
#define TC_NB_BWD 7
#endif
template <int P>
__host__ __device__ constexpr int tc_nb() { return tc_bwd<P>() ? TC_NB_BWD : P == 0 ? TC_NB_BW : TC_NB_NF; }
// mask slots (backward): the 128 x 256-bit ReLU mask of a layer's outputs for the tile (4 KiB)
constexpr int TC_MS = 4;
// bias table: per layer ob x 16 floats (forward programs)
template <int P>
__host__ __device__ constexpr int tc_bias_off(int l) {
  int o = 0;
  if (!tc_bwd<P>())
    for (int i = 0; i < l; ++i) o += tc_layer<P>(i).ob * 16;
  return o;
}
template <int P>
__host__ __device__ constexpr int tc_ring_off() { return (tc_bias_off<P>(tc_nl<P>()) * 4 + 255) / 256 * 256; }
template <int P>
__host__ __device__ constexpr int tc_mask_off() { return tc_ring_off<P>() + tc_nb<P>() * tc_obmax<P>() * 1024; }
template <int P>
__host__ __device__ constexpr int tc_lds_bytes() { return tc_mask_off<P>() + (tc_bwd<P>() ? TC_MS * 4096 : 0); }
// the masked layer whose mask travels with slice q (its first), or -1; a layer's mask slot
template <int P>
__host__ __device__ constexpr int tc_mask_layer(int q) {
  for (int l = 0; l < tc_nl<P>(); ++l)
    if (tc_layer<P>(l).mask && tc_slice0<P>(l) == q) return l;
  return -1;
}
template <int P>
__host__ __device__ constexpr int tc_mslot(int l) {
  int k = 0;
  for (int i = 0; i < l; ++i) k += tc_layer<P>(i).mask ? 1 : 0;
  return k % TC_MS;
}
// vector-memory operations the producer wave issues with slice q: the out-blocks' pieces, plus four
// mask pieces with the first slice of a masked layer
template <int P>
__host__ __device__ constexpr int tc_ops(int q) {
  return tc_layer<P>(tc_layer_of<P>(q)).ob + (tc_mask_layer<P>(q) >= 0 ? 4 : 0);
}
// a mask slot is refilled only after the layer that read it finished its epilogue and passed a barrier:
// the next mask to the same slot is issued at mid(q0 - NB + 1), which must come at or after the first
// slice of the layer that follows the reader
template <int P>
__host__ __device__ constexpr bool tc_masks_ok() {
  for (int l = 0; l < tc_nl<P>(); ++l) {
    if (!tc_layer<P>(l).mask) continue;
    int seen = 0;
    for (int l2 = l + 1; l2 < tc_nl<P>(); ++l2) {
      if (!tc_layer<P>(l2).mask) continue;
      if (++seen == TC_MS) {
        const int at = tc_slice0<P>(l2) - tc_nb<P>() + 1;
        if (at < tc_slice0<P>(l + 1)) return false;
        break;
      }
    }
    if (tc_slice0<P>(l) > tc_nb<P>() - 2 && tc_slice0<P>(l) - tc_nb<P>() + 1 < 0) return false;
  }
  return true;
}
static_assert(tc_nslices<0>() == 68 && tc_nslices<1>() == 89 && tc_nslices<2>() == 65 && tc_nslices<3>() == 86,
              "chain program slice counts");
static_assert(tc_lds_bytes<0>() <= 160 * 1024 && tc_lds_bytes<1>() <= 160 * 1024 && tc_lds_bytes<2>() <= 160 * 1024 &&
                  tc_lds_bytes<3>() <= 160 * 1024,
              "LDS");
static_assert(tc_masks_ok<2>() && tc_masks_ok<3>(), "mask slot reuse");

// input column of MFMA k slot (8 h + j) of a k-step s that reads the previous layer's registers
// output neuron of row m of out-block o: blocks 2s, 2s + 1 hold neurons 32 s + 8 (m >> 2) + {0..3} and
// + {4..7}, so C lane l of the pair holds the 8 consecutive neurons 32 s + 8 (l >> 4) + j — one 16-B
// row store, and in natural order the B fragment (k slot 8 (l >> 4) + j) of the next layer's k-step s
__host__ __device__ constexpr int tc_nrn(int o, int m) { return 32 * (o >> 1) + 8 * (m >> 2) + 4 * (o & 1) + (m & 3); }

__device__ __forceinline__ unsigned short tc_bf(float f) {  // RNE (the layer-wise path's rounding)
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

typedef __bf16 tc_bf16x2 __attribute__((ext_vector_type(2)));
typedef float tc_f32x2 __attribute__((ext_vector_type(2)));
typedef short tc_s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short tc_u16x2 __attribute__((ext_vector_type(2)));
// two fp32 -> packed bf16 (v_cvt_pk_bf16_f32, RNE: tc_bf's rounding), x in the low half
__device__ __forceinline__ uint32_t tc_cvt2(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((tc_f32x2){x, y}, tc_bf16x2));
}
// ReLU of two packed bf16 (v_pk_max_i16 with 0: negative values and -0 have the sign bit)
__device__ __forceinline__ uint32_t tc_pk_relu(uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(tc_s16x2, w), (tc_s16x2){0, 0}));
}
// (half != 0) per half of a ReLU'd word: bits 0 and 16
__device__ __forceinline__ uint32_t tc_nz01(uint32_t w) {
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(w), "v"(0x00010001u));  // (an inline 1 feeds the low half only)
  return r;
}
// 16 such words -> 32 mask bits: word k's halves at bits k and 16 + k (shift-or tree, 15 instructions)
__device__ __forceinline__ uint32_t tc_tree(const uint32_t* t) {
  uint32_t a[8], b[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = t[k] | (t[k + 8] << 8);
#pragma unroll
  for (int k = 0; k < 4; ++k) b[k] = a[k] | (a[k + 4] << 4);
  const uint32_t c0 = b[0] | (b[2] << 2), c1 = b[1] | (b[3] << 2);
  return c0 | (c1 << 1);
}
// bits 0 and 16 of f -> a 0xffff / 0 mask per half
__device__ __forceinline__ uint32_t tc_expand(uint32_t f) {
  const tc_u16x2 e = __builtin_bit_cast(tc_u16x2, f & 0x00010001u);
  return __builtin_bit_cast(uint32_t, (tc_u16x2){0, 0} - e);
}

template <int N>
__device__ __forceinline__ void tc_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt out of range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// ---- weight images -------------------------------------------------------------------------
// fragment layout per slice: [out-block][lane 64][8 bf16]; lane l holds A[m = l & 15][k = 8 (l >> 4) + j]
// = W[16 o + m][column of k slot], RNE bf16, 0 past the layer's outputs / a segment's columns
__global__ void k_tc_pack(TcPackArgs a) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.total) return;
  int l = 0;
  while (l + 1 < a.nl && e >= a.L[l + 1].start) ++l;
  const TcPackLayer& L = a.L[l];
  const long loc = e - L.start;
  const int j = (int)(loc & 7), lane = (int)((loc >> 3) & 63);
  const long fr = loc >> 9;  // fragment index = t * ob + o
  const int o = (int)(fr % L.ob), t = (int)(fr / L.ob);
  const int m = tc_nrn(o, lane & 15), h = lane >> 4;
  float v = 0.f;
  const bool mem = L.mem_first ? t < L.kmem : t >= L.kprev;
  const int s = mem ? (L.mem_first ? t : t - L.kprev) : (L.mem_first ? t - L.kmem : t);
  // input index of this k slot (natural order: memory operands and the previous layer's registers alike)
  const int c = 32 * s + 8 * h + j;
  if (c < (mem ? L.kmem_cols : L.kprev_cols)) {
    if (!L.trans) {
      const int col = (mem ? L.cmem : L.cprev) + c;
      if (m < L.n1) v = L.W[(long)m * L.in_ch + col];
      else if (m - L.n1 < L.n2) v = L.W2[(long)(m - L.n1) * L.in_ch2 + col];
    } else {
      // transposed (input gradient): out neuron m = forward input column (groups A, B), k = forward output c
      int col = -1;
      if (m < L.oa) col = L.oc0 + m;
      else if (m >= L.ob_b0 && m - L.ob_b0 < L.nb) col = L.oc1 + (m - L.ob_b0);
      if (col >= 0) v = mem ? L.W2[(long)c * L.in_ch2 + col] : L.W[(long)c * L.in_ch + col];
    }
  }
  a.out[e] = tc_bf(v);
}

// ---- the chain kernel ------------------------------------------------------------------------
// Workgroup = 7 compute waves (16 samples each: a 112-sample tile) + 1 producer wave that issues every
// LDS-DMA of the ring and alone waits on vmcnt for it. A wave's vmcnt also counts its global stores
// (gfx9 has no separate store counter) and stores may complete out of order with loads, so a compute
// wave that both stored its rows and waited for its DMA pieces waited for its stores too: the
// epilogue stores cost a store round trip at every certify after them (probe: the BW pass 61 us with
// stores, 34 us without, the same 61 with the stores L2-resident). The producer stores nothing.
constexpr int TC_CW = 7;
constexpr int TC_TR = 16 * TC_CW;

struct TcRing {
  unsigned char* lds;  // ring base
  unsigned char* mlds; // mask slots (backward programs)
  const unsigned char* img;
  const TcArgs* a;
  int lane, tile;
  // (producer) issue slice Q into its ring slot: its out-blocks' 1-KiB pieces, and with the first
  // slice of a masked layer the 4 KiB of the layer's mask bits for this tile's rows (+ 16 rows past)
  template <int P, int Q>
  __device__ __forceinline__ void issue() {
    if constexpr (Q < tc_nslices<P>()) {
      constexpr int ob = tc_layer<P>(tc_layer_of<P>(Q)).ob;
      constexpr int kb = tc_slice_kb<P>(Q);
      const unsigned dst = (unsigned)(uintptr_t)(lds + (Q % tc_nb<P>()) * tc_obmax<P>() * 1024);
      const unsigned char* w = img;
      asm volatile("" : "+s"(w));
#pragma unroll
      for (int piece = 0; piece < ob; ++piece) {
        const unsigned m0 = dst + piece * 1024;
        const unsigned char* sbase = w + (size_t)(kb + piece) * 1024;
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(lane * 16), "s"(sbase), "s"(m0)
                     : "memory");
      }
      constexpr int ml = tc_mask_layer<P>(Q);
      if constexpr (ml >= 0) {
#pragma unroll
        for (int piece = 0; piece < 4; ++piece) {
          const unsigned m0 = (unsigned)(uintptr_t)(mlds + tc_mslot<P>(ml) * 4096 + piece * 1024);
          const unsigned char* sbase = (const unsigned char*)a->bits[ml] + (size_t)tile * (TC_TR * 32) + piece * 1024;
          asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(lane * 16), "s"(sbase),
                       "s"(m0)
                       : "memory");
        }
      }
    }
  }
  // slice Q certified at mid(Q - 1) (or the prologue): the producer waits until only the operations
  // of the slices issued after it are outstanding (loads complete in order; a count past the counter's
  // 63 waits for more, which is safe), then every wave meets at the barrier
  template <int P, int Q>
  __device__ __forceinline__ void certify(bool producer) {
    // issued so far: the prologue's slices 0 .. NB-2, then one per mid(): mid(Q - 2) issued Q + NB - 3
    constexpr int last = tc_nslices<P>() - 1;
    constexpr int issued0 = Q == 0 ? tc_nb<P>() - 2 : Q + tc_nb<P>() - 3;
    constexpr int issued = issued0 < last ? issued0 : last;
    constexpr int after = [] {
      int n = 0;
      for (int x = Q + 1; x <= issued; ++x) n += tc_ops<P>(x);
      return n < 63 ? n : 63;
    }();
    if (producer) tc_wait_vmcnt<after>();
    __syncthreads();
  }
  template <int P, int Q>
  __device__ __forceinline__ const unsigned char* slot() const {
    return lds + (Q % tc_nb<P>()) * tc_obmax<P>() * 1024;
  }
};

template <int P>
__device__ __forceinline__ void tc_body(const TcArgs& a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 4, pl = lane & 15;
  float* sb = (float*)smem;
  unsigned char* ring = smem + tc_ring_off<P>();
  unsigned char* mring = smem + tc_mask_off<P>();
  // bias table (forward programs; zero past each layer's outputs; feature||alpha's row 256 = alpha_fc's bias)
  if constexpr (!tc_bwd<P>()) {
    tc_for<0, tc_nl<P>()>([&](auto lc) {
      constexpr int l = decltype(lc)::value;
      constexpr int n = tc_layer<P>(l).ob * 16;
      for (int i = tid; i < n; i += 512) {  // in out-block row order: row i % 16 of block i / 16
        const int nr = tc_nrn(i >> 4, i & 15);
        float v = 0.f;
        if (nr < a.nout[l]) v = a.bias[l][nr];
        else if (tc_layer<P>(l).out == TC_FA && nr == 256) v = a.bias2[0];
        sb[tc_bias_off<P>(l) + i] = v;
      }
    });
  }
  const int M = *a.M_dev;
  const int ntiles = (M + TC_TR - 1) / TC_TR;
  if ((int)blockIdx.x >= ntiles) return;  // uniform per workgroup
  TcRing rg{ring, mring, a.img, &a, lane, 0};
  if (wave == TC_CW) {
    // the producer: the same barriers as the compute waves (prologue, one per slice, tile end)
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      rg.tile = __builtin_amdgcn_readfirstlane(tile);
      tc_for<0, tc_nb<P>() - 1>([&](auto qc) { rg.template issue<P, decltype(qc)::value>(); });
      rg.template certify<P, 0>(true);
      tc_for<0, tc_nslices<P>() - 1>([&](auto qc) {
        constexpr int Q = decltype(qc)::value;
        rg.template certify<P, Q + 1>(true);
        rg.template issue<P, Q + tc_nb<P>() - 1>();
      });
      __syncthreads();
    }
    return;
  }
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row = tile * TC_TR + wave * 16 + pl;
    const bool valid = row < M;
    const int rr = valid ? row : M - 1;
    // memory B fragments (bf16 or fp32 rows, rounded RNE to bf16 as the layer-wise path rounds its
    // operands); columns past the segment read as 0 and are not loaded (rows may be narrower than 32)
    auto load_mem = [&](const void* base, int ld, int cols, int f32, int s) {
      tc_bf16x8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 32 * s + 8 * h + j;
        unsigned short u = 0;
        if (c < cols) u = f32 ? tc_bf(((const float*)base)[(size_t)rr * ld + c]) : ((const unsigned short*)base)[(size_t)rr * ld + c];
        b[j] = __builtin_bit_cast(__bf16, u);
      }
      return b;
    };
    tc_bf16x8 gm[2], gv = {};
    tc_for<0, tc_memk<P>()>([&](auto sc) { gm[decltype(sc)::value] = load_mem(a.mem, a.ld_mem, a.kmem_cols, a.mem_f32, decltype(sc)::value); });
    if constexpr (P == 1 || P == 3) gv = load_mem(a.mem2, a.ld_mem2, a.kmem2_cols, a.mem2_f32, 0);
    // ring prologue (the producer's): slice 0 certified
    rg.template certify<P, 0>(false);
    tc_bf16x8 bprev[8];
    f32x4 acc[20];
    tc_for<0, tc_nl<P>()>([&](auto lc) {
      constexpr int l = decltype(lc)::value;
      constexpr TcL L = tc_layer<P>(l);
      constexpr int KS = L.kmem + L.kprev;
      constexpr int Q0 = tc_slice0<P>(l);
      constexpr int NMB = L.mask ? (L.out == TC_SPLIT ? 16 : L.ob) : 0;  // masked out-blocks
      tc_for<0, L.ob>([&](auto oc) {
        constexpr int o = decltype(oc)::value;
        if constexpr (tc_bwd<P>()) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
        else acc[o] = *(const f32x4*)(sb + tc_bias_off<P>(l) + 16 * o + 4 * h);
      });
      tc_for<0, KS>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        constexpr int Q = Q0 + t;
        constexpr bool mem = L.mem_first ? t < L.kmem : t >= L.kprev;
        constexpr int s = mem ? (L.mem_first ? t : t - L.kprev) : (L.mem_first ? t - L.kmem : t);
        tc_bf16x8 b;
        if constexpr (mem && L.mem2) b = gv;
        else if constexpr (mem) b = gm[s];
        else b = bprev[s];
        const unsigned char* buf = rg.template slot<P, Q>();
        constexpr int PF = 3;
        tc_bf16x8 fa[PF + 1];
        tc_for<0, PF>([&](auto pc) {
          constexpr int o = decltype(pc)::value;
          if constexpr (o < L.ob) fa[o] = *(const tc_bf16x8*)(buf + o * 1024 + lane * 16);
        });
        tc_for<0, L.ob>([&](auto oc) {
          constexpr int o = decltype(oc)::value;
          if constexpr (o + PF < L.ob) fa[(o + PF) % (PF + 1)] = *(const tc_bf16x8*)(buf + (o + PF) * 1024 + lane * 16);
          __builtin_amdgcn_sched_barrier(0);
          acc[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[o % (PF + 1)], b, acc[o], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          // halfway through the slice: certify the next slice, refill the slot of the previous one
          if constexpr (o == (L.ob - 1) / 2) {
            if constexpr (Q + 1 < tc_nslices<P>()) rg.template certify<P, Q + 1>(false);
          }
        });
      });
      // epilogue: RNE to bf16 (v_cvt_pk_bf16_f32) for the stored rows and the next layer's operand, then
      // ReLU on the packed words (forward; max with 0 as int16 = ReLU, and ReLU commutes with RNE) or the
      // ReLU-derivative mask (backward); fp32 heads / gamma gradients from the fp32 accumulators
      if constexpr (L.out == TC_BF16 || L.out == TC_FA || L.out == TC_SPLIT) {
        // word 4 s + j: neurons 32 s + 8 h + 2 j + {0, 1} (tc_nrn; the 4 words of s: one row store, one B fragment)
        uint32_t wd[32];
        tc_for<0, 8>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          wd[4 * s + 0] = tc_cvt2(acc[2 * s][0], acc[2 * s][1]);
          wd[4 * s + 1] = tc_cvt2(acc[2 * s][2], acc[2 * s][3]);
          wd[4 * s + 2] = tc_cvt2(acc[2 * s + 1][0], acc[2 * s + 1][1]);
          wd[4 * s + 3] = tc_cvt2(acc[2 * s + 1][2], acc[2 * s + 1][3]);
        });
        if constexpr (L.relu) {
#pragma unroll
          for (int i = 0; i < 32; ++i) wd[i] = tc_pk_relu(wd[i]);
          // the mask bits of the stored rows for the backward chains (bf16 value > 0, the layer-wise
          // backward's test of the bf16 row)
          if constexpr (!tc_bwd<P>()) {
            if (a.bits[l] && valid) {
              uint32_t t[32];
#pragma unroll
              for (int i = 0; i < 32; ++i) t[i] = tc_nz01(wd[i]);
              *(uint2*)((unsigned char*)a.bits[l] + ((size_t)row * 4 + h) * 8) = make_uint2(tc_tree(t), tc_tree(t + 16));
            }
          }
        }
        if constexpr (NMB > 0) {
          const uint2 F = *(const uint2*)(mring + tc_mslot<P>(l) * 4096 + ((wave * 16 + pl) * 4 + h) * 8);
#pragma unroll
          for (int i = 0; i < 32; ++i) wd[i] &= tc_expand((i < 16 ? F.x : F.y) >> (i & 15));
        }
        unsigned short* orow = (unsigned short*)a.out[l] + (size_t)row * a.ldo[l];
        tc_for<0, 8>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          if (valid) {
            *(uint4*)(orow + 32 * s + 8 * h) = make_uint4(wd[4 * s], wd[4 * s + 1], wd[4 * s + 2], wd[4 * s + 3]);
          }
          bprev[s] = __builtin_bit_cast(tc_bf16x8, make_uint4(wd[4 * s], wd[4 * s + 1], wd[4 * s + 2], wd[4 * s + 3]));
        });
        if constexpr (L.out == TC_FA) {
          if (valid && h == 0) a.out2[row] = acc[16][0];  // alpha_fc (row 256 of the stacked layer)
        }
      } else if constexpr (L.out == TC_F32) {
        // fp32 rows (heads; view_fc's ReLU rows; d view): ReLU / mask in fp32, mask bits from the fp32
        // value (the layer-wise path masks d view by View > 0)
        constexpr int NW = L.ob * 2;  // packed words, as above
        if constexpr (L.relu) {
          tc_for<0, L.ob>([&](auto oc) {
            constexpr int o = decltype(oc)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[o][r] = fmaxf(acc[o][r], 0.0f);
          });
          if constexpr (!tc_bwd<P>()) {
            if (a.bits[l] && valid) {
              uint32_t t[32] = {};
              tc_for<0, L.ob>([&](auto oc) {
                constexpr int o = decltype(oc)::value;
                constexpr int i0 = 4 * (o >> 1) + 2 * (o & 1);
                t[i0] = (acc[o][0] > 0.f ? 1u : 0u) | (acc[o][1] > 0.f ? 0x10000u : 0u);
                t[i0 + 1] = (acc[o][2] > 0.f ? 1u : 0u) | (acc[o][3] > 0.f ? 0x10000u : 0u);
              });
              *(uint2*)((unsigned char*)a.bits[l] + ((size_t)row * 4 + h) * 8) =
                  make_uint2(tc_tree(t), NW > 16 ? tc_tree(t + 16) : 0u);
            }
          }
        }
        if constexpr (NMB > 0) {
          const uint2 F = *(const uint2*)(mring + tc_mslot<P>(l) * 4096 + ((wave * 16 + pl) * 4 + h) * 8);
          tc_for<0, L.ob>([&](auto oc) {
            constexpr int o = decltype(oc)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i = 4 * (o >> 1) + 2 * (o & 1) + (r >> 1);
              const uint32_t f = (i < 16 ? F.x : F.y) >> ((i & 15) + 16 * (r & 1));
              acc[o][r] = (f & 1u) ? acc[o][r] : 0.0f;
            }
          });
        }
        float* orow = (float*)a.out[l] + (size_t)row * a.ldo[l];
        const int nout = a.nout[l];
        tc_for<0, L.ob>([&](auto oc) {
          constexpr int o = decltype(oc)::value;
          const int c = 32 * (o >> 1) + 8 * h + 4 * (o & 1);
          if (valid) {
            if (c + 4 <= nout) {
              *(f32x4*)(orow + c) = acc[o];
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (c + r < nout) orow[c + r] = acc[o][r];
            }
          }
        });
        // the next layer's operand (view_fc -> rgb_fc: 128 ReLU outputs; d view -> view_fc^T)
        if constexpr (l + 1 < tc_nl<P>()) {
          tc_for<0, L.ob / 2>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            bprev[s] = __builtin_bit_cast(
                tc_bf16x8, make_uint4(tc_cvt2(acc[2 * s][0], acc[2 * s][1]), tc_cvt2(acc[2 * s][2], acc[2 * s][3]),
                                      tc_cvt2(acc[2 * s + 1][0], acc[2 * s + 1][1]), tc_cvt2(acc[2 * s + 1][2], acc[2 * s + 1][3])));
          });
        }
      }
      if constexpr (L.out == TC_SPLIT || L.out == TC_AUX) {
        // the gamma gradient (fp32 rows, aux_cols columns at ld_aux): out-blocks past the hidden part
        constexpr int O0 = L.out == TC_SPLIT ? 16 : 0;
        if (a.aux && valid) {
          float* arow = a.aux + (size_t)row * a.ld_aux;
          tc_for<O0, L.ob>([&](auto oc) {
            constexpr int o = decltype(oc)::value;
            const int c = 32 * ((o - O0) >> 1) + 8 * h + 4 * (o & 1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (c + r < a.aux_cols) {
                if (L.aux_add || a.aux_acc) arow[c + r] += acc[o][r];
                else arow[c + r] = acc[o][r];
              }
            }
          });
        }
      }
    });
    __syncthreads();  // every wave is done with the ring before the next tile's prologue refills it
  }
}

// (entry / exit clock stamps of thread 0 when profiling: anr_profile_read_clock's in-kernel clock)
__global__ __launch_bounds__(512) void k_tchain_bw(TcArgs a) { ANR_STAMPED(tc_body<0>(a)); }
__global__ __launch_bounds__(512) void k_tchain_nf(TcArgs a) { ANR_STAMPED(tc_body<1>(a)); }
__global__ __launch_bounds__(512) void k_tchain_bwb(TcArgs a) { ANR_STAMPED(tc_body<2>(a)); }
__global__ __launch_bounds__(512) void k_tchain_nfb(TcArgs a) { ANR_STAMPED(tc_body<3>(a)); }

}  // namespace

size_t tchain_image_bytes(int prog) {
  const int kb = prog == 0 ? tc_image_kb<0>() : prog == 1 ? tc_image_kb<1>() : prog == 2 ? tc_image_kb<2>() : tc_image_kb<3>();
  return (size_t)kb * 1024;
}

template <int P>
static void tc_fill(TcPackArgs& a, long& e) {
  for (int l = 0; l < tc_nl<P>(); ++l) {
    const TcL L = tc_layer<P>(l);
    a.L[l].start = e;
    a.L[l].ob = L.ob;
    a.L[l].kmem = L.kmem;
    a.L[l].kprev = L.kprev;
    a.L[l].mem_first = L.mem_first;
    a.L[l].trans = tc_bwd<P>() ? 1 : 0;
    e += (long)(L.kmem + L.kprev) * L.ob * 512;
  }
  a.nl = tc_nl<P>();
}

// pack one program's image: layers' weight sources in TcPackLayer (start / ob / k-steps filled here)
int tchain_pack(int prog, TcPackArgs a, void* dst, hipStream_t s) {
  long e = 0;
  if (prog == 0) tc_fill<0>(a, e);
  else if (prog == 1) tc_fill<1>(a, e);
  else if (prog == 2) tc_fill<2>(a, e);
  else tc_fill<3>(a, e);
  a.total = e;
  a.out = (unsigned short*)dst;
  if ((size_t)e * 2 != tchain_image_bytes(prog)) return -1;
  hipLaunchKernelGGL(k_tc_pack, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int tchain_run(int prog, const TcArgs& a, int cap, int cus, hipStream_t s) {
  static bool attr[4] = {false, false, false, false};
  const void* k = prog == 0 ? (const void*)k_tchain_bw : prog == 1 ? (const void*)k_tchain_nf
                  : prog == 2 ? (const void*)k_tchain_bwb : (const void*)k_tchain_nfb;
  const int lds = prog == 0 ? tc_lds_bytes<0>() : prog == 1 ? tc_lds_bytes<1>() : prog == 2 ? tc_lds_bytes<2>() : tc_lds_bytes<3>();
  if (!attr[prog]) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return -1;
    attr[prog] = true;
  }
  const int tiles = (cap + TC_TR - 1) / TC_TR;
  const int grid = tiles < cus ? tiles : cus;
  if (grid <= 0) return 0;
  TcArgs args = a;
  ProfSlot* ps = prof_begin(s, grid);
  args.clk = ps ? ps->clk : nullptr;
  void* kargs[] = {&args};
  if (hipLaunchKernel(k, dim3(grid), dim3(512), kargs, lds, s) != hipSuccess) return -1;
  if (prof_end(ps, s) != 0) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace anr
