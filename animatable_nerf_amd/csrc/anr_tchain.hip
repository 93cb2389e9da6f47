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
// Layout: workgroup = 8 waves x 16 samples (a 128-sample tile), persistent over tiles. v_mfma_f32_16x16x32_bf16
// with the weights as the A operand (16 output neurons x 32 inputs) and the samples as B: the C
// layout of out-blocks 2s, 2s+1 (lane l: neurons 32s + 4(l>>4) + r and 32s + 16 + 4(l>>4) + r of sample
// l & 15) is the B fragment of the next layer's k-step s when the packed weight columns follow the same
// order (tc_perm), so activations never leave registers. Memory segments (gamma rows, gamma(dir) rows)
// are read straight into B fragments in natural column order. Weights stream through a 4-slot LDS ring
// of slices (one 32-input k-step of all of a layer's out-blocks, <= 17 KiB) by LDS-DMA, one barrier per
// slice with counted vmcnt waits (the render kernel's scheme, anr_mlp_body.h Pipe); biases sit in an LDS
// table filled once per launch. Each layer's outputs are stored once (bf16 rows for the backward's
// masks and weight gradients; fp32 heads) while the next layer's MFMAs run.
#include <type_traits>

#include "anr_common.h"
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
  int kmem;        // k-steps (32 inputs) from a memory segment (bf16 rows), 0 = none
  int kprev;       // k-steps from the previous layer's outputs (registers)
  int mem_first;   // the memory segment's k-steps come first (weight-image and MFMA order)
  int relu;
  int out;         // TC_BF16 rows, TC_F32 rows, TC_FA (feature bf16 || alpha fp32)
  int mem2;        // the memory segment is the second memory operand (gamma(dir))
};
enum { TC_BF16 = 0, TC_F32 = 1, TC_FA = 2 };

constexpr TcL kProgBW[9] = {
    {16, 2, 0, 1, 1, TC_BF16, 0}, {16, 0, 8, 0, 1, TC_BF16, 0}, {16, 0, 8, 0, 1, TC_BF16, 0},
    {16, 0, 8, 0, 1, TC_BF16, 0}, {16, 0, 8, 0, 1, TC_BF16, 0}, {16, 2, 8, 1, 1, TC_BF16, 0},
    {16, 0, 8, 0, 1, TC_BF16, 0}, {16, 0, 8, 0, 1, TC_BF16, 0}, {2, 0, 8, 0, 0, TC_F32, 0}};
constexpr TcL kProgNF[12] = {
    {16, 2, 0, 1, 1, TC_BF16, 0}, {16, 0, 8, 0, 1, TC_BF16, 0}, {16, 0, 8, 0, 1, TC_BF16, 0},
    {16, 0, 8, 0, 1, TC_BF16, 0}, {16, 0, 8, 0, 1, TC_BF16, 0}, {16, 2, 8, 1, 1, TC_BF16, 0},
    {16, 0, 8, 0, 1, TC_BF16, 0}, {16, 0, 8, 0, 1, TC_BF16, 0}, {17, 0, 8, 0, 0, TC_FA, 0},
    {16, 0, 8, 0, 0, TC_BF16, 0}, {8, 1, 8, 0, 1, TC_F32, 1}, {1, 0, 4, 0, 0, TC_F32, 0}};

template <int P>
__host__ __device__ constexpr int tc_nl() { return P == 0 ? 9 : 12; }
template <int P>
__host__ __device__ constexpr TcL tc_layer(int l) { return P == 0 ? kProgBW[l] : kProgNF[l]; }
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
__host__ __device__ constexpr int tc_obmax() { return P == 0 ? 16 : 17; }
// LDS-DMA pieces (1 KiB) every wave issues per slice (pieces past a slice's out-blocks repeat its last)
template <int P>
__host__ __device__ constexpr int tc_pieces() { return (tc_obmax<P>() + 7) / 8; }
constexpr int TC_NB = 4;  // ring slots
// bias table: per layer ob x 16 floats
template <int P>
__host__ __device__ constexpr int tc_bias_off(int l) {
  int o = 0;
  for (int i = 0; i < l; ++i) o += tc_layer<P>(i).ob * 16;
  return o;
}
template <int P>
__host__ __device__ constexpr int tc_lds_bytes() {
  return (tc_bias_off<P>(tc_nl<P>()) * 4 + 255) / 256 * 256 + TC_NB * tc_obmax<P>() * 1024;
}
static_assert(tc_nslices<0>() == 68 && tc_nslices<1>() == 89, "chain program slice counts");
static_assert(tc_lds_bytes<1>() <= 160 * 1024, "LDS");

// input column of MFMA k slot (8 h + j) of a k-step s that reads the previous layer's registers
__host__ __device__ constexpr int tc_perm(int s, int h, int j) { return 32 * s + (j < 4 ? 4 * h + j : 16 + 4 * h + (j - 4)); }

__device__ __forceinline__ unsigned short tc_bf(float f) {  // RNE (the layer-wise path's rounding)
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
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
  const int m = 16 * o + (lane & 15), h = lane >> 4;
  float v = 0.f;
  const bool mem = L.mem_first ? t < L.kmem : t >= L.kprev;
  if (mem) {
    const int s = L.mem_first ? t : t - L.kprev;
    const int c = 32 * s + 8 * h + j;
    if (c < L.kmem_cols) {
      if (m < L.n1) v = L.W[(long)m * L.in_ch + L.cmem + c];
      else if (m - L.n1 < L.n2) v = L.W2[(long)(m - L.n1) * L.in_ch2 + L.cmem + c];
    }
  } else {
    const int s = L.mem_first ? t - L.kmem : t;
    const int c = tc_perm(s, h, j);
    if (c < L.kprev_cols) {
      if (m < L.n1) v = L.W[(long)m * L.in_ch + L.cprev + c];
      else if (m - L.n1 < L.n2) v = L.W2[(long)(m - L.n1) * L.in_ch2 + L.cprev + c];
    }
  }
  a.out[e] = tc_bf(v);
}

// ---- the chain kernel ------------------------------------------------------------------------
struct TcRing {
  unsigned char* lds;  // ring base
  const unsigned char* img;
  int wave, lane;
  // issue slice Q into its ring slot (every wave exactly tc_pieces<P>() 1-KiB pieces)
  template <int P, int Q>
  __device__ __forceinline__ void issue() {
    if constexpr (Q < tc_nslices<P>()) {
      constexpr int ob = tc_layer<P>(tc_layer_of<P>(Q)).ob;
      constexpr int kb = tc_slice_kb<P>(Q);
      const unsigned dst = (unsigned)(uintptr_t)(lds + (Q % TC_NB) * tc_obmax<P>() * 1024);
      const unsigned char* w = img;
      asm volatile("" : "+s"(w));
#pragma unroll
      for (int i = 0; i < tc_pieces<P>(); ++i) {
        int piece = wave + 8 * i;
        piece = piece < ob ? piece : ob - 1;
        const unsigned m0 = dst + piece * 1024;
        const unsigned char* sbase = w + (size_t)(kb + piece) * 1024;
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(lane * 16), "s"(sbase), "s"(m0)
                     : "memory");
      }
    }
  }
  // slices issued after slice Q by the time slice Q is certified at mid(Q - 1) (or the prologue)
  template <int P, int Q>
  __device__ __forceinline__ void certify() {
    // issued so far: the prologue's slices 0 .. NB-2, then one per mid(): mid(Q - 2) issued Q + NB - 3
    constexpr int last = tc_nslices<P>() - 1;
    constexpr int issued0 = Q == 0 ? TC_NB - 2 : Q + TC_NB - 3;
    constexpr int issued = issued0 < last ? issued0 : last;
    constexpr int after = issued - Q;
    tc_wait_vmcnt<tc_pieces<P>() * (after > 0 ? after : 0)>();
    __syncthreads();
  }
  template <int P, int Q>
  __device__ __forceinline__ const unsigned char* slot() const {
    return lds + (Q % TC_NB) * tc_obmax<P>() * 1024;
  }
};

template <int P>
__device__ __forceinline__ void tc_body(const TcArgs& a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 4, pl = lane & 15;
  float* sb = (float*)smem;
  unsigned char* ring = smem + (tc_bias_off<P>(tc_nl<P>()) * 4 + 255) / 256 * 256;
  // bias table (zero past each layer's outputs; the FA layer's out-block 16 row 0 = alpha_fc's bias)
  tc_for<0, tc_nl<P>()>([&](auto lc) {
    constexpr int l = decltype(lc)::value;
    constexpr int n = tc_layer<P>(l).ob * 16;
    for (int i = tid; i < n; i += 512) {
      float v = 0.f;
      if (i < a.nout[l]) v = a.bias[l][i];
      else if (tc_layer<P>(l).out == TC_FA && i == 256) v = a.bias2[0];
      sb[tc_bias_off<P>(l) + i] = v;
    }
  });
  const int M = *a.M_dev;
  const int ntiles = (M + 127) / 128;
  if ((int)blockIdx.x >= ntiles) return;  // uniform per workgroup
  TcRing rg{ring, a.img, wave, lane};
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row = tile * 128 + wave * 16 + pl;
    const bool valid = row < M;
    const int rr = valid ? row : M - 1;
    // memory B fragments: gamma (2 k-steps), gamma(dir) (1 k-step, program NF); columns past the
    // segment read as 0 (the rows' padding is not assumed to be finite)
    tc_bf16x8 gm[2], gv = {};
    {
      tc_for<0, 2>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        const uint4 u = *(const uint4*)(a.mem + (size_t)rr * a.ld_mem + 32 * s + 8 * h);
        tc_bf16x8 b = __builtin_bit_cast(tc_bf16x8, u);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (32 * s + 8 * h + j >= a.kmem_cols) b[j] = (__bf16)0.0f;
        gm[s] = b;
      });
      if constexpr (P == 1) {
        const uint4 u = *(const uint4*)(a.mem2 + (size_t)rr * a.ld_mem2 + 8 * h);
        gv = __builtin_bit_cast(tc_bf16x8, u);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (8 * h + j >= a.kmem2_cols) gv[j] = (__bf16)0.0f;
      }
    }
    // ring prologue: slices 0 .. NB-2, slice 0 certified
    tc_for<0, TC_NB - 1>([&](auto qc) { rg.template issue<P, decltype(qc)::value>(); });
    rg.template certify<P, 0>();
    tc_bf16x8 bprev[8];
    f32x4 acc[17];
    tc_for<0, tc_nl<P>()>([&](auto lc) {
      constexpr int l = decltype(lc)::value;
      constexpr TcL L = tc_layer<P>(l);
      constexpr int KS = L.kmem + L.kprev;
      constexpr int Q0 = tc_slice0<P>(l);
      tc_for<0, L.ob>([&](auto oc) {
        constexpr int o = decltype(oc)::value;
        acc[o] = *(const f32x4*)(sb + tc_bias_off<P>(l) + 16 * o + 4 * h);
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
            if constexpr (Q + 1 < tc_nslices<P>()) {
              rg.template certify<P, Q + 1>();
              rg.template issue<P, Q + TC_NB - 1>();
            }
          }
        });
      });
      // epilogue: ReLU, RNE to bf16 for the stored rows and the next layer's operand; fp32 heads
      if constexpr (L.relu) {
        tc_for<0, L.ob>([&](auto oc) {
          constexpr int o = decltype(oc)::value;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[o][r] = fmaxf(acc[o][r], 0.0f);
        });
      }
      if constexpr (L.out == TC_BF16 || L.out == TC_FA) {
        unsigned short* orow = (unsigned short*)a.out[l] + (size_t)row * a.ldo[l];
        tc_for<0, 8>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          unsigned short u[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            u[r] = tc_bf(acc[2 * s][r]);
            u[4 + r] = tc_bf(acc[2 * s + 1][r]);
          }
          const uint2 lo = make_uint2(u[0] | ((uint32_t)u[1] << 16), u[2] | ((uint32_t)u[3] << 16));
          const uint2 hi = make_uint2(u[4] | ((uint32_t)u[5] << 16), u[6] | ((uint32_t)u[7] << 16));
          if (valid) {
            *(uint2*)(orow + 32 * s + 4 * h) = lo;
            *(uint2*)(orow + 32 * s + 16 + 4 * h) = hi;
          }
          bprev[s] = __builtin_bit_cast(tc_bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
        });
        if constexpr (L.out == TC_FA) {
          if (valid && h == 0) a.out2[row] = acc[16][0];  // alpha_fc (row 256 of the stacked layer)
        }
      } else {
        // fp32 rows: columns [0, nout) at ld
        float* orow = (float*)a.out[l] + (size_t)row * a.ldo[l];
        const int nout = a.nout[l];
        tc_for<0, L.ob>([&](auto oc) {
          constexpr int o = decltype(oc)::value;
          const int c = 16 * o + 4 * h;
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
        // the next layer's operand (view_fc -> rgb_fc: 128 ReLU outputs in 4 k-steps)
        if constexpr (l + 1 < tc_nl<P>()) {
          tc_for<0, L.ob / 2>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            unsigned short u[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              u[r] = tc_bf(acc[2 * s][r]);
              u[4 + r] = tc_bf(acc[2 * s + 1][r]);
            }
            bprev[s] = __builtin_bit_cast(tc_bf16x8, make_uint4(u[0] | ((uint32_t)u[1] << 16), u[2] | ((uint32_t)u[3] << 16),
                                                                u[4] | ((uint32_t)u[5] << 16), u[6] | ((uint32_t)u[7] << 16)));
          });
        }
      }
    });
    __syncthreads();  // every wave is done with the ring before the next tile's prologue refills it
  }
}

__global__ __launch_bounds__(512) void k_tchain_bw(TcArgs a) { tc_body<0>(a); }
__global__ __launch_bounds__(512) void k_tchain_nf(TcArgs a) { tc_body<1>(a); }

}  // namespace

size_t tchain_image_bytes(int prog) { return (size_t)(prog == 0 ? tc_image_kb<0>() : tc_image_kb<1>()) * 1024; }

// pack one program's image: layers' weight sources in TcPackLayer (start / ob / k-steps filled here)
int tchain_pack(int prog, TcPackArgs a, void* dst, hipStream_t s) {
  long e = 0;
  const int nl = prog == 0 ? tc_nl<0>() : tc_nl<1>();
  for (int l = 0; l < nl; ++l) {
    const TcL L = prog == 0 ? tc_layer<0>(l) : tc_layer<1>(l);
    a.L[l].start = e;
    a.L[l].ob = L.ob;
    a.L[l].kmem = L.kmem;
    a.L[l].kprev = L.kprev;
    a.L[l].mem_first = L.mem_first;
    e += (long)(L.kmem + L.kprev) * L.ob * 512;
  }
  a.nl = nl;
  a.total = e;
  a.out = (unsigned short*)dst;
  if ((size_t)e * 2 != tchain_image_bytes(prog)) return -1;
  hipLaunchKernelGGL(k_tc_pack, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int tchain_run(int prog, const TcArgs& a, int cap, int cus, hipStream_t s) {
  static bool attr[2] = {false, false};
  const void* k = prog == 0 ? (const void*)k_tchain_bw : (const void*)k_tchain_nf;
  const int lds = prog == 0 ? tc_lds_bytes<0>() : tc_lds_bytes<1>();
  if (!attr[prog]) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return -1;
    attr[prog] = true;
  }
  const int tiles = (cap + 127) / 128;
  const int grid = tiles < cus ? tiles : cus;
  if (grid <= 0) return 0;
  TcArgs args = a;
  void* kargs[] = {&args};
  if (hipLaunchKernel(k, dim3(grid), dim3(512), kargs, lds, s) != hipSuccess) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace anr
