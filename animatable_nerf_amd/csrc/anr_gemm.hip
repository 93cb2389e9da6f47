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
                                          int tid, Tile4& t, bool vec) {
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
        if (gk + 3 < K && vec) {
          x = *(const float4*)p;
        } else if (gk + 3 < K) {
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
        if (gr + 3 < R && vec) {
          x = *(const float4*)p;
        } else if (gr + 3 < R) {
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

// rows r = 4 (tid & 15) .. +3 of the A tile are summed by the threads sharing tid & 15: lanes l, l^16,
// l^32, l^48 of each wave, then one atomic per row and wave
__device__ __forceinline__ void rowsum_flush(const GemmArgs& g, int m0, float (&rsum)[4]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int M = g.M_dev ? *g.M_dev : g.M;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    rsum[e] += __shfl_xor(rsum[e], 16);
    rsum[e] += __shfl_xor(rsum[e], 32);
  }
  if (lane < 16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + 4 * lane + e;
      if (m < M) {
        atomicAdd(g.rowsum + m, rsum[e]);
        if (g.rowsum2) atomicAdd(g.rowsum2 + m, rsum[e]);
      }
    }
  }
}

// epilogue shared by the GEMM kernels: lane holds C[wr + i*16 + 4*(lane>>4) + r][wc + j*16 + (lane&15)]
__device__ __forceinline__ void epilogue(const GemmArgs& g, const f32x4 (&acc)[2][2], int M, int m0, int n0, int wr,
                                         int wc, int lane) {
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
          const float e = fast_exp(z);
          if (g.deriv) g.deriv[(long)m * g.ldd + n] = z > 20.f ? -1.f : e;
          v = z > 20.f ? v : fast_log1p(e) / 100.f;
        }
        if (g.spd && n < g.spd_n) {
          const float d = g.spd[(long)m * g.ldsd + n];
          if (g.spd_h) v = v * softplus_factor_h(g.spd_scale != 0.f ? d * g.spd_scale : d);
          else if (d >= 0.f) v = v * d * __builtin_amdgcn_rcpf(d + 1.f);
        }
        if (g.mask && !(g.mask[(long)m * g.ldm + n] > 0.f)) v = 0.f;
        if (g.div_post != 0.f) v = v / g.div_post;
        *c = v;
      }
}

// epilogue of the swapped product (non-atomic launches): the MFMAs take the B fragment as their A
// operand, so lane l holds C[m0 + wr + 16 i + (l & 15)][n0 + wc + 16 j + 4 (l >> 4) + r], r = 0..3 —
// four consecutive columns of one row, finished and stored as one 16-B access when every operand is
// 16-B addressable (g.vec_out). All operand loads precede the first use.
__device__ __forceinline__ void epilogue_sw(const GemmArgs& g, const f32x4 (&acc)[2][2], int M, int m0, int n0, int wr,
                                            int wc, int lane) {
  if (g.vec_out) {
    f32x4 bj[2], cv[2][2], mk[2][2], sp[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = min(n0 + wc + 16 * j + 4 * (lane >> 4), g.N - 4);
      bj[j] = g.bias ? *(const f32x4*)(g.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const long m = min(m0 + wr + 16 * i + (lane & 15), M - 1);
        const int n = min(n0 + wc + 16 * j + 4 * (lane >> 4), g.N - 4);
        if (g.accumulate) cv[i][j] = *(const f32x4*)(g.C + m * g.ldc + n);
        if (g.mask) mk[i][j] = *(const f32x4*)(g.mask + m * g.ldm + n);
        if (g.spd) sp[i][j] = *(const f32x4*)(g.spd + m * g.ldsd + n);
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = m0 + wr + 16 * i + (lane & 15);
        const int n = n0 + wc + 16 * j + 4 * (lane >> 4);
        if (m >= M || n >= g.N) continue;
        f32x4 v = acc[i][j], dv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = v[e];
          if (g.bias) x += bj[j][e];
          if (g.accumulate) x += cv[i][j][e];
          if (g.div_pre != 0.f) x = x / g.div_pre;
          if (g.relu) x = fmaxf(x, 0.f);
          if (g.softplus) {  // torch softplus(beta=100, threshold=20) and the factor its backward uses
            const float z = x * 100.f;
            const float ez = fast_exp(z);
            dv[e] = z > 20.f ? -1.f : ez;
            x = z > 20.f ? x : fast_log1p(ez) / 100.f;
          }
          if (g.spd && n + e < g.spd_n) {
            const float d = sp[i][j][e];
            if (g.spd_h) x = x * softplus_factor_h(g.spd_scale != 0.f ? d * g.spd_scale : d);
            else if (d >= 0.f) x = x * d * __builtin_amdgcn_rcpf(d + 1.f);
          }
          if (g.mask && !(mk[i][j][e] > 0.f)) x = 0.f;
          if (g.div_post != 0.f) x = x / g.div_post;
          v[e] = x;
        }
        if (g.softplus && g.deriv) *(f32x4*)(g.deriv + (long)m * g.ldd + n) = dv;
        *(f32x4*)(g.C + (long)m * g.ldc + n) = v;
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr + 16 * i + (lane & 15);
        const int n = n0 + wc + 16 * j + 4 * (lane >> 4) + r;
        if (m >= M || n >= g.N) continue;
        float v = acc[i][j][r];
        float* c = g.C + (long)m * g.ldc + n;
        if (g.bias) v += g.bias[n];
        if (g.accumulate) v += *c;
        if (g.div_pre != 0.f) v = v / g.div_pre;
        if (g.relu) v = fmaxf(v, 0.f);
        if (g.softplus) {
          const float z = v * 100.f;
          const float e = fast_exp(z);
          if (g.deriv) g.deriv[(long)m * g.ldd + n] = z > 20.f ? -1.f : e;
          v = z > 20.f ? v : fast_log1p(e) / 100.f;
        }
        if (g.spd && n < g.spd_n) {
          const float d = g.spd[(long)m * g.ldsd + n];
          if (g.spd_h) v = v * softplus_factor_h(g.spd_scale != 0.f ? d * g.spd_scale : d);
          else if (d >= 0.f) v = v * d * __builtin_amdgcn_rcpf(d + 1.f);
        }
        if (g.mask && !(g.mask[(long)m * g.ldm + n] > 0.f)) v = 0.f;
        if (g.div_post != 0.f) v = v / g.div_post;
        *c = v;
      }
}

// SW: the swapped MFMA operand order and epilogue_sw (non-atomic launches)
template <bool A_K, bool B_K, bool SW>
__global__ __launch_bounds__(256) void k_gemm_t(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[GBK][GLD];
  __shared__ __attribute__((aligned(16))) float Bs[GBK][GLD];
  const int M = g.M_dev ? *g.M_dev : g.M;
  const int K0 = g.K_dev ? *g.K_dev : g.seg[0].K;  // segment 0's depth (device: the kept-sample count)
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  if (m0 >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;

  // k range of this split (split-K only with one segment)
  int kb = 0, ke = K0;
  if (g.ksplit > 1) {
    const int per = g.kper > 0 ? g.kper : ((K0 + g.ksplit - 1) / g.ksplit + GBK - 1) / GBK * GBK;
    kb = blockIdx.z * per;
    ke = min(K0, kb + per);
    if (kb >= ke) return;
  }

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // flattened (segment, k0) iteration
  int s = 0, k0 = kb;
  int kend = (g.ksplit > 1) ? ke : K0;
  Tile4 ta, tb;
  load_tile<A_K>(g.seg[0].A, g.seg[0].a_rs, g.seg[0].a_cs, M, m0, kend, k0, tid, ta, g.a_vec[0]);
  load_tile<B_K>(g.seg[0].B, g.seg[0].b_cs, g.seg[0].b_rs, g.N, n0, kend, k0, tid, tb, g.b_vec[0]);
  float rsum[4] = {0.f, 0.f, 0.f, 0.f};
  const bool do_rsum = !A_K && g.rowsum != nullptr && blockIdx.x == 0;
  while (true) {
    if (do_rsum) {  // A(r..r+3, k) in the thread's registers (!A_K layout), out-of-range entries are 0
#pragma unroll
      for (int e = 0; e < 4; ++e) rsum[e] += ta.v[0][e] + ta.v[1][e];
    }
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
      const int kend2 = (g.ksplit > 1) ? ke : (ns ? g.seg[1].K : K0);
      load_tile<A_K>(g.seg[ns].A, g.seg[ns].a_rs, g.seg[ns].a_cs, M, m0, kend2, nk, tid, ta, g.a_vec[ns]);
      load_tile<B_K>(g.seg[ns].B, g.seg[ns].b_cs, g.seg[ns].b_rs, g.N, n0, kend2, nk, tid, tb, g.b_vec[ns]);
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
        for (int j = 0; j < 2; ++j)
          acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x4f32(b[j], a[i], acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (!more) break;
    s = ns;
    k0 = nk;
    kend = (g.ksplit > 1) ? ke : (s ? g.seg[1].K : K0);
  }
  if (do_rsum) rowsum_flush(g, m0, rsum);
  if constexpr (SW) epilogue_sw(g, acc, M, m0, n0, wr, wc, lane);
  else epilogue(g, acc, M, m0, n0, wr, wc, lane);
}

// ------------------------------------------------------------------------------------------
// bf16-operand variant (training precision 'bf16', config 3): the same tiles and epilogues, the
// operands rounded to bf16 (RNE) as they are staged into LDS, v_mfma_f32_16x16x32_bf16 with fp32
// accumulation. K tile 64; LDS images [m|n][k] with k contiguous so each lane's fragment
// (8 consecutive k) is one 16-B read.
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#define BBK 64  // K tile (measured against 128: 4.82 vs 4.97 ms per bf16 step)
#define BLD (BBK + 8)
#define BNH (BBK / 16)                    // 4-element groups per thread per 64-row operand tile
#define BKSH (BBK == 128 ? 5 : 4)         // log2(groups per k-contiguous row)

__device__ __forceinline__ unsigned short f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

struct Tile16 {
  float v[BNH][4];
};

template <bool KCONTIG>
__device__ __forceinline__ void load_tile16(const float* __restrict__ P, long rs, long cs, int R, int r0, int K, int k0,
                                            int tid, Tile16& t, bool vec) {
  // 64 (r) x 64 (k) elements = 1024 groups of 4, 4 per thread
#pragma unroll
  for (int h = 0; h < BNH; ++h) {
    const int q = tid + h * 256;
    int r, k;
    if (KCONTIG) {
      r = q >> BKSH;
      k = (q & ((1 << BKSH) - 1)) * 4;
    } else {
      k = q >> 4;
      r = (q & 15) * 4;
    }
    const int gr = r0 + r, gk = k0 + k;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f;
    if (KCONTIG) {
      if (gr < R) {
        const float* p = P + (long)gr * rs + (long)gk * cs;
        if (gk + 3 < K && vec) {
          const float4 v = *(const float4*)p;
          x0 = v.x; x1 = v.y; x2 = v.z; x3 = v.w;
        } else if (gk + 3 < K) {
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
        if (gr + 3 < R && vec) {
          const float4 v = *(const float4*)p;
          x0 = v.x; x1 = v.y; x2 = v.z; x3 = v.w;
        } else if (gr + 3 < R) {
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

// LDS images: a k-contiguous operand as [r][k] (row stride BLD), read as 16-B fragments; an
// r-contiguous one (weight gradients, dY W) as [k][r] (row stride RLD), written as it was loaded
// (8 B per 4 consecutive r) and read with the transposing ds_read_b64_tr_b16 (two per fragment).
#define RLD (64 + 4)
typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float((uint32_t)h << 16); }

// X3: also the low part lo = bf16(x - hi) into SL (x = hi + lo to ~2^-16 relative)
template <bool KCONTIG, bool X3>
__device__ __forceinline__ void store_tile16(unsigned short* S, unsigned short* SL, int tid, const Tile16& t) {
#pragma unroll
  for (int h = 0; h < BNH; ++h) {
    const int q = tid + h * 256;
    unsigned short e[4], l[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      e[c] = f2bf(t.v[h][c]);
      if (X3) l[c] = f2bf(t.v[h][c] - bf2f(e[c]));
    }
    const int off = KCONTIG ? (q >> BKSH) * BLD + (q & ((1 << BKSH) - 1)) * 4 : (q >> 4) * RLD + (q & 15) * 4;
    *(uint2*)&S[off] = make_uint2((uint32_t)e[0] | ((uint32_t)e[1] << 16), (uint32_t)e[2] | ((uint32_t)e[3] << 16));
    if (X3)
      *(uint2*)&SL[off] = make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
  }
}

// MFMA 16x16x32 operand fragment of rows rb..rb+15, k = ks + 8 (lane >> 4) .. + 7
template <bool KCONTIG>
__device__ __forceinline__ bf16x8 frag16(const unsigned short* S, int rb, int ks, int lane) {
  if (KCONTIG) return *(const bf16x8*)&S[(rb + (lane & 15)) * BLD + ks + 8 * (lane >> 4)];
  // 16-lane group g reads rows k = ks + 8g + q (q = 0..3, then 4..7), lane 4q + p supplying columns
  // rb + 4p .. +3 of row q; lane i receives column rb + i, element q = row q
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  const unsigned short* a0 = S + (ks + 8 * g + q) * RLD + rb + 4 * p;
  const v4s x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(uintptr_t)(unsigned)(uintptr_t)a0);
  const v4s x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(uintptr_t)(unsigned)(uintptr_t)(a0 + 4 * RLD));
  bf16x8 f;
  const short e[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  __builtin_memcpy(&f, e, 16);
  return f;
}

// X3 (render precision bf16x3, the sdf_pdf GEMMs): hi/lo images of both operands and three MFMAs per
// fragment pair, lo*bh + hi*bl + hi*bh, fp32 accumulation (~2^-16 relative per product).
template <bool A_K, bool B_K, bool X3, bool SW>
__global__ __launch_bounds__(256) void k_gemm_b(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned short As[(X3 ? 2 : 1) * GBM * BLD];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[(X3 ? 2 : 1) * GBN * BLD];
  unsigned short* const Al = As + GBM * BLD;
  unsigned short* const Bl = Bs + GBN * BLD;
  const int M = g.M_dev ? *g.M_dev : g.M;
  const int K0 = g.K_dev ? *g.K_dev : g.seg[0].K;  // segment 0's depth (device: the kept-sample count)
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  if (m0 >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  int kb = 0, ke = K0;
  if (g.ksplit > 1) {
    const int per = g.kper > 0 ? g.kper : ((K0 + g.ksplit - 1) / g.ksplit + BBK - 1) / BBK * BBK;
    kb = blockIdx.z * per;
    ke = min(K0, kb + per);
    if (kb >= ke) return;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int s = 0, k0 = kb;
  int kend = (g.ksplit > 1) ? ke : K0;
  Tile16 ta, tb;
  load_tile16<A_K>(g.seg[0].A, g.seg[0].a_rs, g.seg[0].a_cs, M, m0, kend, k0, tid, ta, g.a_vec[0]);
  load_tile16<B_K>(g.seg[0].B, g.seg[0].b_cs, g.seg[0].b_rs, g.N, n0, kend, k0, tid, tb, g.b_vec[0]);
  float rsum[4] = {0.f, 0.f, 0.f, 0.f};
  const bool do_rsum = !A_K && g.rowsum != nullptr && blockIdx.x == 0;
  while (true) {
    if (do_rsum) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int h = 0; h < BNH; ++h) rsum[e] += ta.v[h][e];
    }
    store_tile16<A_K, X3>(As, Al, tid, ta);
    store_tile16<B_K, X3>(Bs, Bl, tid, tb);
    __syncthreads();
    int ns = s, nk = k0 + BBK;
    if (nk >= kend) {
      ns = s + 1;
      nk = 0;
    }
    const bool more = ns < g.nseg && (g.ksplit == 1 || ns == 0);
    if (more) {
      const int kend2 = (g.ksplit > 1) ? ke : (ns ? g.seg[1].K : K0);
      load_tile16<A_K>(g.seg[ns].A, g.seg[ns].a_rs, g.seg[ns].a_cs, M, m0, kend2, nk, tid, ta, g.a_vec[ns]);
      load_tile16<B_K>(g.seg[ns].B, g.seg[ns].b_cs, g.seg[ns].b_rs, g.N, n0, kend2, nk, tid, tb, g.b_vec[ns]);
    }
#pragma unroll
    for (int ks = 0; ks < BBK; ks += 32) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = frag16<A_K>(As, wr + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = frag16<B_K>(Bs, wc + j * 16, ks, lane);
      if constexpr (X3) {
        bf16x8 al[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) al[i] = frag16<A_K>(Al, wr + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) bl[j] = frag16<B_K>(Bl, wc + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if constexpr (SW) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], al[i], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], a[i], acc[i][j], 0, 0, 0);
            } else {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], b[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bl[j], acc[i][j], 0, 0, 0);
            }
          }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (!more) break;
    s = ns;
    k0 = nk;
    kend = (g.ksplit > 1) ? ke : (s ? g.seg[1].K : K0);
  }
  if (do_rsum) rowsum_flush(g, m0, rsum);
  if constexpr (SW) epilogue_sw(g, acc, M, m0, n0, wr, wc, lane);
  else epilogue(g, acc, M, m0, n0, wr, wc, lane);
}

#define ANR_GEMM_INST(SW)                                            \
  template __global__ void k_gemm_b<true, true, false, SW>(GemmArgs);  \
  template __global__ void k_gemm_b<true, false, false, SW>(GemmArgs); \
  template __global__ void k_gemm_b<false, true, false, SW>(GemmArgs); \
  template __global__ void k_gemm_b<false, false, false, SW>(GemmArgs); \
  template __global__ void k_gemm_b<true, true, true, SW>(GemmArgs);   \
  template __global__ void k_gemm_b<true, false, true, SW>(GemmArgs);  \
  template __global__ void k_gemm_t<true, true, SW>(GemmArgs);         \
  template __global__ void k_gemm_t<true, false, SW>(GemmArgs);        \
  template __global__ void k_gemm_t<false, true, SW>(GemmArgs);        \
  template __global__ void k_gemm_t<false, false, SW>(GemmArgs);
ANR_GEMM_INST(false)
ANR_GEMM_INST(true)

template <bool SW>
static void launch_gemm_sw(const GemmArgs& g, dim3 grid, hipStream_t s, bool a_k, bool b_k) {
  if (g.x3 && a_k) {  // split-bf16 (the sdf_pdf forward and input-gradient GEMMs)
    if (b_k) hipLaunchKernelGGL((k_gemm_b<true, true, true, SW>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((k_gemm_b<true, false, true, SW>), grid, dim3(256), 0, s, g);
    return;
  }
  if (g.bf16) {
    if (a_k && b_k) hipLaunchKernelGGL((k_gemm_b<true, true, false, SW>), grid, dim3(256), 0, s, g);
    else if (a_k) hipLaunchKernelGGL((k_gemm_b<true, false, false, SW>), grid, dim3(256), 0, s, g);
    else if (b_k) hipLaunchKernelGGL((k_gemm_b<false, true, false, SW>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((k_gemm_b<false, false, false, SW>), grid, dim3(256), 0, s, g);
    return;
  }
  if (a_k && b_k) hipLaunchKernelGGL((k_gemm_t<true, true, SW>), grid, dim3(256), 0, s, g);
  else if (a_k) hipLaunchKernelGGL((k_gemm_t<true, false, SW>), grid, dim3(256), 0, s, g);
  else if (b_k) hipLaunchKernelGGL((k_gemm_t<false, true, SW>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((k_gemm_t<false, false, SW>), grid, dim3(256), 0, s, g);
}

// host-side dispatch on the operand layouts
void launch_gemm(GemmArgs g, dim3 grid, hipStream_t s) {
  // a one-row A (a_rs == a_cs == 1: the weight gradient of a 1-output layer) is contiguous both ways;
  // with row sums requested it takes the m-contiguous path, the one that computes them
  const bool a_k = g.seg[0].a_cs == 1 && !(g.rowsum && g.seg[0].a_rs == 1);
  const bool b_k = g.seg[0].b_rs == 1;
  // 16-B operand loads where every 4-group the tile reads is aligned: base aligned and the stride
  // between the groups a multiple of 4 floats (the groups run along the contiguous dimension)
  for (int i = 0; i < g.nseg; ++i) {
    const GemmSeg& q = g.seg[i];
    const long a_stride = a_k ? q.a_rs : q.a_cs, b_stride = b_k ? q.b_cs : q.b_rs;
    g.a_vec[i] = ((uintptr_t)q.A % 16 == 0) && (a_stride % 4 == 0) && (a_k || q.a_rs == 1);
    g.b_vec[i] = ((uintptr_t)q.B % 16 == 0) && (b_stride % 4 == 0) && (b_k || q.b_cs == 1);
  }
  // non-atomic launches: swapped product + vectorised epilogue where every operand is 16-B addressable
  const bool sw = !g.atomic;
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  g.vec_out = sw && g.N % 4 == 0 && g.ldc % 4 == 0 && al16(g.C) && (!g.bias || al16(g.bias)) &&
              (!g.mask || (g.ldm % 4 == 0 && al16(g.mask))) && (!g.spd || (g.ldsd % 4 == 0 && al16(g.spd))) &&
              (!g.softplus || !g.deriv || (g.ldd % 4 == 0 && al16(g.deriv)));
  if (sw) launch_gemm_sw<true>(g, grid, s, a_k, b_k);
  else launch_gemm_sw<false>(g, grid, s, a_k, b_k);
}

}  // namespace anr
