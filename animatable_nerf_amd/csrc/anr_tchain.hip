// anr_tchain.hip — one launch per MLP for the forward of the training executor (precision bf16 with
// bf16 storage, configs 3/4): the T-pose blend-weight MLP (9 layers) and the canonical NeRF (8 trunk
// layers + alpha / feature / latent / view / rgb heads) each run as one chain of layers per 128-row
// tile, instead of one row-GEMM launch per layer.
//
// A workgroup (8 waves = 2 row groups x 4 column groups of 64, as k_rgemm) owns 128 rows for the
// whole chain. The layer's output tile (<= 256 columns, bf16) stays in LDS as the next layer's A
// operand; every layer's activation is still written to HBM once (bf16, the backward reads it), so
// per layer what leaves the chip is that write, and what comes in is only the weights: one stream of
// 64-deep bf16 weight chunks (32 KiB, LDS-DMA into a 2-slot ring) that runs across layer boundaries,
// so the next layer's first chunk is in flight during this layer's epilogue. gamma inputs (<= 64
// bf16 columns: gamma(x_T), gamma(dir)) are loaded into LDS once. Products: bf16 MFMA with fp32
// accumulation exactly as k_rgemm's (the same operand rounding), so the chain computes what the
// per-layer launches computed.
#include "anr_common.h"
#include "anr_train.h"

namespace anr {

constexpr int TC_BM = 128, TC_WAVES = 8, TC_KC = 64;
constexpr int TC_SLAB = TC_BM * TC_KC * 2;            // one 64-deep bf16 slab of 128 rows: 16 KiB
constexpr int TC_ACT = 4 * TC_SLAB;                   // activation tile, 256 columns: 64 KiB
constexpr int TC_B = 256 * TC_KC * 2;                 // weight chunk: 256 rows x 64 k: 32 KiB
constexpr int TC_NS = 2;                              // ring slots
constexpr int TC_OFF_G0 = TC_ACT, TC_OFF_G1 = TC_ACT + TC_SLAB, TC_OFF_RING = TC_ACT + 2 * TC_SLAB;
constexpr int TC_LDS = TC_OFF_RING + TC_NS * TC_B;    // 160 KiB
constexpr int TC_OPS = TC_B / 1024 / TC_WAVES;        // 1-KiB DMA pieces per wave per chunk
static_assert(TC_LDS <= 160 * 1024, "LDS");

typedef __bf16 tcbf8 __attribute__((ext_vector_type(8)));

// XOR swizzle of a 128-B row's 16-B groups: the 16-lane groups of a ds_read_b128 fragment read
// (rows r..r+15, one or two k groups) land on distinct bank slots
__device__ __forceinline__ int tc_sw(int r) { return r & 7; }

template <int N>
__device__ __forceinline__ void tc_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void tc_dma(const void* src, unsigned m0) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory");
}

__device__ __forceinline__ unsigned short tc_bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

// chunk q of the chain's stream -> (layer, segment, k offset)
__device__ __forceinline__ void tc_locate(const ChainArgs& a, int q, int& l, int& s, int& kk) {
  for (l = 0; l < a.nl; ++l)
    for (s = 0; s < a.L[l].nseg; ++s) {
      const int n = (a.L[l].K[s] + TC_KC - 1) / TC_KC;
      if (q < n) {
        kk = q * TC_KC;
        return;
      }
      q -= n;
    }
  l = s = kk = 0;  // not reached for q < total
}

// 128 rows x 64 bf16 columns of a gamma matrix (row stride ld) into an LDS slab, swizzled as the
// activation slabs (two 1-KiB pieces per wave)
__device__ __forceinline__ void tc_load_gamma(const unsigned short* G, long ld, int m0, int M, unsigned dst, int w,
                                              int lane) {
#pragma unroll
  for (int i = 0; i < TC_SLAB / 1024 / TC_WAVES; ++i) {
    const int p = w + TC_WAVES * i;
    const int r = 8 * p + lane / 8;
    const int gr = min(m0 + r, M - 1);
    const int ch = (lane % 8) ^ tc_sw(r);
    tc_dma(G + (long)gr * ld + ch * 8, dst + p * 1024);
  }
}

__global__ __launch_bounds__(TC_WAVES * 64) void k_chain(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int M = a.M_dev ? *a.M_dev : a.M;
  const int m0 = blockIdx.x * TC_BM;
  if (m0 >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned base = (unsigned)(uintptr_t)lds;
  // gamma tiles first (drained before the weight stream starts, so its vmcnt bookkeeping is exact)
  if (a.G0) tc_load_gamma(a.G0, a.ldg0, m0, M, base + TC_OFF_G0, w, lane);
  if (a.G1) tc_load_gamma(a.G1, a.ldg1, m0, M, base + TC_OFF_G1, w, lane);
  tc_wait<0>();
  int Q = 0;
  for (int l = 0; l < a.nl; ++l)
    for (int s = 0; s < a.L[l].nseg; ++s) Q += (a.L[l].K[s] + TC_KC - 1) / TC_KC;
  auto issue = [&](int q) {
    int l, s, kk;
    tc_locate(a, q, l, s, kk);
    const ChainLayer& L = a.L[l];
    const unsigned short* B = L.B[s];
    const long ldb = L.ldb[s];
    const int bcol = L.bcol[s], brows = L.brows[s];
    const unsigned slot = base + TC_OFF_RING + (q % TC_NS) * TC_B;
#pragma unroll
    for (int i = 0; i < TC_OPS; ++i) {
      const int p = w + TC_WAVES * i;
      const int r = 8 * p + lane / 8;
      const int br = min(r, brows - 1);
      const int ch = (lane % 8) ^ tc_sw(r);
      tc_dma(B + (long)br * ldb + bcol + kk + ch * 8, slot + p * 1024);
    }
  };
  for (int q = 0; q < (Q < TC_NS ? Q : TC_NS); ++q) issue(q);
  __syncthreads();  // gamma tiles visible to every wave

  const int wr = (w >> 2) * 64;  // this wave's 64 rows of the tile
  const int wc = (w & 3) * 64;   // and 64 output columns
  int q = 0;
  for (int l = 0; l < a.nl; ++l) {
    const ChainLayer& L = a.L[l];
    const int N = L.N;
    const bool active = wc < N;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < L.nseg; ++s) {
      const int K = L.K[s];
      const int src = L.src[s];
      for (int kk = 0; kk < K; kk += TC_KC, ++q) {
        const int later = (Q < q + TC_NS ? Q : q + TC_NS) - q - 1;
        if (later >= 1) tc_wait<TC_OPS>();
        else tc_wait<0>();
        __builtin_amdgcn_s_barrier();
        const unsigned char* sA = lds + (src == 0 ? (kk / TC_KC) * TC_SLAB : src == 1 ? TC_OFF_G0 : TC_OFF_G1);
        const unsigned char* sB = lds + TC_OFF_RING + (q % TC_NS) * TC_B;
        if (active) {
#pragma unroll
          for (int ks = 0; ks < TC_KC / 32; ++ks) {
            tcbf8 af[4], bfr[4];
            const int kc = 4 * ks + (lane >> 4);  // 8-element k group of this lane
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = wr + 16 * i + (lane & 15);
              af[i] = *(const tcbf8*)(sA + r * (TC_KC * 2) + ((kc ^ tc_sw(r)) * 16));
              if (kk + TC_KC > K) {  // the segment's last, partial chunk: columns past K read as zero
#pragma unroll
                for (int e = 0; e < 8; ++e) af[i][e] = (kk + 8 * kc + e < K) ? af[i][e] : (__bf16)0.0f;
              }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = wc + 16 * j + (lane & 15);
              bfr[j] = *(const tcbf8*)(sB + r * (TC_KC * 2) + ((kc ^ tc_sw(r)) * 16));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
          }
        }
        // every wave is past this slot's (and the activation slab's) reads before it is refilled
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (q + TC_NS < Q) issue(q + TC_NS);
      }
    }
    // epilogue: lane holds C[wr + 16 i + (l & 15)][wc + 16 j + 4 (l >> 4) + r], r = 0..3
    if (active) {
      f32x4 bj[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = wc + 16 * j + 4 * (lane >> 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) bj[j][r] = (L.bias && n + r < N) ? L.bias[n + r] : 0.f;
      }
      unsigned short* O16 = (unsigned short*)L.out;
      float* O32 = (float*)L.out;
      const bool vec = L.out && (N % 4 == 0) && (L.ldo % 4 == 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rl = wr + 16 * i + (lane & 15);  // row in the tile
          const int m = m0 + rl;
          const int n = wc + 16 * j + 4 * (lane >> 4);
          f32x4 v = acc[i][j] + bj[j];
          if (L.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          const unsigned short h0 = tc_bf(v[0]), h1 = tc_bf(v[1]), h2 = tc_bf(v[2]), h3 = tc_bf(v[3]);
          acc[i][j] = v;  // kept for the LDS write below
          if (L.out && m < M && n < N) {
            if (L.out_bf16) {
              if (vec) {
                *(uint2*)(O16 + (long)m * L.ldo + n) =
                    make_uint2((uint32_t)h0 | ((uint32_t)h1 << 16), (uint32_t)h2 | ((uint32_t)h3 << 16));
              } else {
                const unsigned short hh[4] = {h0, h1, h2, h3};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                  if (n + e < N) O16[(long)m * L.ldo + n + e] = hh[e];
              }
            } else {
              if (vec) {
                *(f32x4*)(O32 + (long)m * L.ldo + n) = v;
              } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                  if (n + e < N) O32[(long)m * L.ldo + n + e] = v[e];
              }
            }
          }
        }
    }
    if (L.to_lds) {
      // every wave finished reading this layer's activation slabs (the last chunk's barrier), so the
      // output overwrites them in place: column n -> slab n / 64, 16-B group (n % 64) / 8 (swizzled)
      if (active) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int rl = wr + 16 * i + (lane & 15);
            const int n = wc + 16 * j + 4 * (lane >> 4);
            const f32x4 v = acc[i][j];
            unsigned char* dst = lds + (n / TC_KC) * TC_SLAB + rl * (TC_KC * 2) +
                                 ((((n % TC_KC) / 8) ^ tc_sw(rl)) * 16) + (n % 8) * 2;
            *(uint2*)dst = make_uint2((uint32_t)tc_bf(v[0]) | ((uint32_t)tc_bf(v[1]) << 16),
                                      (uint32_t)tc_bf(v[2]) | ((uint32_t)tc_bf(v[3]) << 16));
          }
      }
      __syncthreads();  // the next layer reads the tile
    }
  }
}

int launch_chain(const ChainArgs& a, int M_host, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_chain, hipFuncAttributeMaxDynamicSharedMemorySize, TC_LDS);
    attr = true;
  }
  if (M_host <= 0) return 0;
  hipLaunchKernelGGL(k_chain, dim3((M_host + TC_BM - 1) / TC_BM), dim3(TC_WAVES * 64), TC_LDS, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace anr
