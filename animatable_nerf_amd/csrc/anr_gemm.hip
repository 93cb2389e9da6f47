// anr_gemm.hip — strided fp32-MFMA GEMM used by the layer-wise training executor.
//
//   C[M][N] (+)= epi( sum_s A_s(m, k) * B_s(k, n) ),  A_s(m,k) = A_s[m*a_rs + k*a_cs],
//                                                     B_s(k,n) = B_s[k*b_rs + n*b_cs]
// One kernel serves the three products of a Conv1d(k=1) layer over the point batch:
//   forward  Y  = X W^T   (A = X row-major: contiguous in k;  B(k,n) = W[n][k]: contiguous in k)
//   backward dX = dY W    (A = dY row-major: contiguous in k; B(k,n) = W[k][c0+n]: contiguous in n)
//   weights  dW = dY^T X  (A(m,k) = dY[k][m]: contiguous in m; B = X row-major: contiguous in n;
//                          split-K over samples, fp32 atomics into dW)
// Up to two K segments (the skip concatenation [gamma(x), net] of layers 5 / pts_linears.5, or the
// two heads feature_fc / alpha_fc feeding one input), each padded to the K tile separately.
// Epilogue: bias, ReLU, or the ReLU mask of the forward activation (dX of a ReLU layer),
// accumulate into C.
//
// Tile 64x64x32, 256 threads = 4 waves, each a 32x32 quadrant of v_mfma_f32_16x16x4_f32 (exact fp32).
// Global -> registers with float4 loads along the contiguous dimension of each operand (template
// flags), registers -> LDS [k][m|n] after the barrier so the next tile's loads overlap the MFMAs.
#include "anr_common.h"
#include "anr_train.h"

namespace anr {

#define GBM 64
#define GBN 64
#define GBK 32
#define GLD (64 + 4)

// element (r, k) of a segment operand with r the M (or N) index; contiguous-in-k or in-r layouts
struct Tile4 {
  float v[2][4];
};

template <bool KCONTIG>
__device__ __forceinline__ void load_tile(const float* __restrict__ P, long rs, long cs, int R, int r0, int K, int k0,
                                          int tid, Tile4& t) {
  // 64 (r) x 32 (k) elements = 512 float4 groups, 2 per thread
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int q = tid + h * 256;
    int r, k;
    if (KCONTIG) {
      r = q >> 3;
      k = (q & 7) * 4;
    } else {
      k = q >> 4;
      r = (q & 15) * 4;
    }
    const int gr = r0 + r, gk = k0 + k;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (KCONTIG) {
      // 4 consecutive k of row gr
      if (gr < R) {
        const float* p = P + (long)gr * rs + (long)gk * cs;
        if (gk + 3 < K) {
          x.x = p[0]; x.y = p[1]; x.z = p[2]; x.w = p[3];
        } else {
          if (gk < K) x.x = p[0];
          if (gk + 1 < K) x.y = p[1];
          if (gk + 2 < K) x.z = p[2];
        }
      }
    } else {
      // 4 consecutive r of k-row gk
      if (gk < K) {
        const float* p = P + (long)gr * rs + (long)gk * cs;
        if (gr + 3 < R) {
          x.x = p[0]; x.y = p[rs]; x.z = p[2 * rs]; x.w = p[3 * rs];
        } else {
          if (gr < R) x.x = p[0];
          if (gr + 1 < R) x.y = p[rs];
          if (gr + 2 < R) x.z = p[2 * rs];
        }
      }
    }
    t.v[h][0] = x.x; t.v[h][1] = x.y; t.v[h][2] = x.z; t.v[h][3] = x.w;
  }
}

template <bool KCONTIG>
__device__ __forceinline__ void store_tile(float (*S)[GLD], int tid, const Tile4& t) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int q = tid + h * 256;
    if (KCONTIG) {
      const int r = q >> 3, k = (q & 7) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) S[k + e][r] = t.v[h][e];
    } else {
      const int k = q >> 4, r = (q & 15) * 4;
      *(float4*)&S[k][r] = make_float4(t.v[h][0], t.v[h][1], t.v[h][2], t.v[h][3]);
    }
  }
}

template <bool A_K, bool B_K>
__global__ __launch_bounds__(256) void k_gemm_t(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[GBK][GLD];
  __shared__ __attribute__((aligned(16))) float Bs[GBK][GLD];
  const int M = g.M_dev ? *g.M_dev : g.M;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  if (m0 >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;

  // k range of this split (split-K only with one segment)
  int kb = 0, ke = g.seg[0].K;
  if (g.ksplit > 1) {
    const int per = ((g.seg[0].K + g.ksplit - 1) / g.ksplit + GBK - 1) / GBK * GBK;
    kb = blockIdx.z * per;
    ke = min(g.seg[0].K, kb + per);
    if (kb >= ke) return;
  }

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // flattened (segment, k0) iteration
  int s = 0, k0 = kb;
  int kend = (g.ksplit > 1) ? ke : g.seg[0].K;
  Tile4 ta, tb;
  load_tile<A_K>(g.seg[0].A, g.seg[0].a_rs, g.seg[0].a_cs, M, m0, kend, k0, tid, ta);
  load_tile<B_K>(g.seg[0].B, g.seg[0].b_cs, g.seg[0].b_rs, g.N, n0, kend, k0, tid, tb);
  while (true) {
    store_tile<A_K>(As, tid, ta);
    store_tile<B_K>(Bs, tid, tb);
    __syncthreads();
    // next tile position
    int ns = s, nk = k0 + GBK;
    if (nk >= kend) {
      ns = s + 1;
      nk = 0;
    }
    const bool more = ns < g.nseg && (g.ksplit == 1 || ns == 0);
    if (more) {
      const int kend2 = (g.ksplit > 1) ? ke : g.seg[ns].K;
      load_tile<A_K>(g.seg[ns].A, g.seg[ns].a_rs, g.seg[ns].a_cs, M, m0, kend2, nk, tid, ta);
      load_tile<B_K>(g.seg[ns].B, g.seg[ns].b_cs, g.seg[ns].b_rs, g.N, n0, kend2, nk, tid, tb);
    }
#pragma unroll
    for (int ks = 0; ks < GBK; ks += 4) {
      const int kr = ks + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kr][wr + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kr][wc + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (!more) break;
    s = ns;
    k0 = nk;
    kend = (g.ksplit > 1) ? ke : g.seg[s].K;
  }
  // epilogue: lane holds C[wr + i*16 + 4*(lane>>4) + r][wc + j*16 + (lane&15)]
  const bool first_split = blockIdx.z == 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wc + j * 16 + (lane & 15);
        if (m >= M || n >= g.N) continue;
        float v = acc[i][j][r];
        float* c = g.C + (long)m * g.ldc + n;
        if (g.atomic) {
          if (g.bias && first_split) v += g.bias[n];
          atomicAdd(c, v);
          continue;
        }
        if (g.bias) v += g.bias[n];
        if (g.accumulate) v += *c;
        if (g.div_pre != 0.f) v = v / g.div_pre;
        if (g.relu) v = fmaxf(v, 0.f);
        if (g.softplus) {  // torch softplus(beta=100, threshold=20) and the factor its backward uses
          const float z = v * 100.f;
          const float e = expf(z);
          g.deriv[(long)m * g.ldd + n] = z > 20.f ? -1.f : e;
          v = z > 20.f ? v : log1pf(e) / 100.f;
        }
        if (g.spd && n < g.spd_n) {
          const float d = g.spd[(long)m * g.ldsd + n];
          if (d >= 0.f) v = v * d / (d + 1.f);
        }
        if (g.mask && !(g.mask[(long)m * g.ldm + n] > 0.f)) v = 0.f;
        if (g.div_post != 0.f) v = v / g.div_post;
        *c = v;
      }
}

// ------------------------------------------------------------------------------------------
// bf16-operand variant (training precision 'bf16', config 3): the same tiles and epilogues, the
// operands rounded to bf16 (RNE) as they are staged into LDS, v_mfma_f32_16x16x32_bf16 with fp32
// accumulation. K tile 64; LDS images [m|n][k] with k contiguous so each lane's fragment
// (8 consecutive k) is one 16-B read.
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#define BBK 64
#define BLD (64 + 8)

__device__ __forceinline__ unsigned short f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

struct Tile16 {
  float v[4][4];
};

template <bool KCONTIG>
__device__ __forceinline__ void load_tile16(const float* __restrict__ P, long rs, long cs, int R, int r0, int K, int k0,
                                            int tid, Tile16& t) {
  // 64 (r) x 64 (k) elements = 1024 groups of 4, 4 per thread
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int q = tid + h * 256;
    int r, k;
    if (KCONTIG) {
      r = q >> 4;
      k = (q & 15) * 4;
    } else {
      k = q >> 4;
      r = (q & 15) * 4;
    }
    const int gr = r0 + r, gk = k0 + k;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f;
    if (KCONTIG) {
      if (gr < R) {
        const float* p = P + (long)gr * rs + (long)gk * cs;
        if (gk + 3 < K) {
          x0 = p[0]; x1 = p[1]; x2 = p[2]; x3 = p[3];
        } else {
          if (gk < K) x0 = p[0];
          if (gk + 1 < K) x1 = p[1];
          if (gk + 2 < K) x2 = p[2];
        }
      }
    } else {
      if (gk < K) {
        const float* p = P + (long)gr * rs + (long)gk * cs;
        if (gr + 3 < R) {
          x0 = p[0]; x1 = p[rs]; x2 = p[2 * rs]; x3 = p[3 * rs];
        } else {
          if (gr < R) x0 = p[0];
          if (gr + 1 < R) x1 = p[rs];
          if (gr + 2 < R) x2 = p[2 * rs];
        }
      }
    }
    t.v[h][0] = x0; t.v[h][1] = x1; t.v[h][2] = x2; t.v[h][3] = x3;
  }
}

template <bool KCONTIG>
__device__ __forceinline__ void store_tile16(unsigned short (*S)[BLD], int tid, const Tile16& t) {
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int q = tid + h * 256;
    if (KCONTIG) {
      const int r = q >> 4, k = (q & 15) * 4;
      const uint32_t lo = (uint32_t)f2bf(t.v[h][0]) | ((uint32_t)f2bf(t.v[h][1]) << 16);
      const uint32_t hi = (uint32_t)f2bf(t.v[h][2]) | ((uint32_t)f2bf(t.v[h][3]) << 16);
      *(uint2*)&S[r][k] = make_uint2(lo, hi);
    } else {
      const int k = q >> 4, r = (q & 15) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) S[r + e][k] = f2bf(t.v[h][e]);
    }
  }
}

template <bool A_K, bool B_K>
__global__ __launch_bounds__(256) void k_gemm_b(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned short As[GBM][BLD];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[GBN][BLD];
  const int M = g.M_dev ? *g.M_dev : g.M;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  if (m0 >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  int kb = 0, ke = g.seg[0].K;
  if (g.ksplit > 1) {
    const int per = ((g.seg[0].K + g.ksplit - 1) / g.ksplit + BBK - 1) / BBK * BBK;
    kb = blockIdx.z * per;
    ke = min(g.seg[0].K, kb + per);
    if (kb >= ke) return;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int s = 0, k0 = kb;
  int kend = (g.ksplit > 1) ? ke : g.seg[0].K;
  Tile16 ta, tb;
  load_tile16<A_K>(g.seg[0].A, g.seg[0].a_rs, g.seg[0].a_cs, M, m0, kend, k0, tid, ta);
  load_tile16<B_K>(g.seg[0].B, g.seg[0].b_cs, g.seg[0].b_rs, g.N, n0, kend, k0, tid, tb);
  while (true) {
    store_tile16<A_K>(As, tid, ta);
    store_tile16<B_K>(Bs, tid, tb);
    __syncthreads();
    int ns = s, nk = k0 + BBK;
    if (nk >= kend) {
      ns = s + 1;
      nk = 0;
    }
    const bool more = ns < g.nseg && (g.ksplit == 1 || ns == 0);
    if (more) {
      const int kend2 = (g.ksplit > 1) ? ke : g.seg[ns].K;
      load_tile16<A_K>(g.seg[ns].A, g.seg[ns].a_rs, g.seg[ns].a_cs, M, m0, kend2, nk, tid, ta);
      load_tile16<B_K>(g.seg[ns].B, g.seg[ns].b_cs, g.seg[ns].b_rs, g.N, n0, kend2, nk, tid, tb);
    }
#pragma unroll
    for (int ks = 0; ks < BBK; ks += 32) {
      const int kk = ks + 8 * (lane >> 4);
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *(const bf16x8*)&As[wr + i * 16 + (lane & 15)][kk];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *(const bf16x8*)&Bs[wc + j * 16 + (lane & 15)][kk];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (!more) break;
    s = ns;
    k0 = nk;
    kend = (g.ksplit > 1) ? ke : g.seg[s].K;
  }
  const bool first_split = blockIdx.z == 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wc + j * 16 + (lane & 15);
        if (m >= M || n >= g.N) continue;
        float v = acc[i][j][r];
        float* c = g.C + (long)m * g.ldc + n;
        if (g.atomic) {
          if (g.bias && first_split) v += g.bias[n];
          atomicAdd(c, v);
          continue;
        }
        if (g.bias) v += g.bias[n];
        if (g.accumulate) v += *c;
        if (g.relu) v = fmaxf(v, 0.f);
        if (g.mask && !(g.mask[(long)m * g.ldm + n] > 0.f)) v = 0.f;
        *c = v;
      }
}

template __global__ void k_gemm_b<true, true>(GemmArgs);
template __global__ void k_gemm_b<true, false>(GemmArgs);
template __global__ void k_gemm_b<false, true>(GemmArgs);
template __global__ void k_gemm_b<false, false>(GemmArgs);

template __global__ void k_gemm_t<true, true>(GemmArgs);
template __global__ void k_gemm_t<true, false>(GemmArgs);
template __global__ void k_gemm_t<false, true>(GemmArgs);
template __global__ void k_gemm_t<false, false>(GemmArgs);

// host-side dispatch on the operand layouts
void launch_gemm(GemmArgs g, dim3 grid, hipStream_t s) {
  const bool a_k = g.seg[0].a_cs == 1;
  const bool b_k = g.seg[0].b_rs == 1;
  if (g.bf16) {  // the sdf epilogues (softplus, div) are fp32-path only
    if (a_k && b_k) hipLaunchKernelGGL((k_gemm_b<true, true>), grid, dim3(256), 0, s, g);
    else if (a_k) hipLaunchKernelGGL((k_gemm_b<true, false>), grid, dim3(256), 0, s, g);
    else if (b_k) hipLaunchKernelGGL((k_gemm_b<false, true>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((k_gemm_b<false, false>), grid, dim3(256), 0, s, g);
    return;
  }
  if (a_k && b_k) hipLaunchKernelGGL((k_gemm_t<true, true>), grid, dim3(256), 0, s, g);
  else if (a_k) hipLaunchKernelGGL((k_gemm_t<true, false>), grid, dim3(256), 0, s, g);
  else if (b_k) hipLaunchKernelGGL((k_gemm_t<false, true>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((k_gemm_t<false, false>), grid, dim3(256), 0, s, g);
}

// column sums of X[M][N] (ld) into out[N] (+=), M from device when given: bias gradients
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ X, long ld, int M, const int* M_dev, int N,
                                                float* __restrict__ out, int rows_per_block) {
  const int MM = M_dev ? *M_dev : M;
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(MM, r0 + rows_per_block);
  float s = 0.f;
  for (int m = r0 + (threadIdx.x >> 6); m < r1; m += 4)
    if (n < N) s += X[(long)m * ld + n];
  __shared__ float sh[4][64];
  sh[threadIdx.x >> 6][threadIdx.x & 63] = s;
  __syncthreads();
  if (threadIdx.x < 64 && n < N && r0 < r1)
    atomicAdd(out + n, sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x]);
}

}  // namespace anr
