// anr_gemm.hip — strided fp32-MFMA GEMM used by the layer-wise training executor.
//
//   C[M][N] (+)= epi( sum_s A_s(m, k) * B_s(k, n) ),  A_s(m,k) = A_s[m*a_rs + k*a_cs],
//                                                     B_s(k,n) = B_s[k*b_rs + n*b_cs]
// One kernel serves the three products of a Conv1d(k=1) layer over the point batch:
//   forward  Y  = X W^T   (A = X row-major, B(k,n) = W[n][k])
//   backward dX = dY W    (A = dY row-major, B(k,n) = W[k][col0+n])
//   weights  dW = dY^T X  (A(m=n_out,k=point) = dY[k][n], B = X row-major; split-K + atomics)
// Up to two K segments (the skip concatenation [gamma(x), net] of layers 5 / pts_linears.5, or
// the two heads feature_fc / alpha_fc feeding one input). Epilogue: bias, ReLU, or the ReLU mask of
// the forward activation (dX of a ReLU layer), accumulate into C.
//
// Tile 64x64x16, 256 threads = 4 waves, each wave a 32x32 quadrant of v_mfma_f32_16x16x4_f32
// (exact fp32). M may be taken from device memory (kept-sample count) so no host sync is needed.
#include "anr_common.h"
#include "anr_train.h"

namespace anr {

#define GBM 64
#define GBN 64
#define GBK 16

__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  __shared__ float As[GBK][GBM + 4];
  __shared__ float Bs[GBK][GBN + 4];
  const int M = g.M_dev ? *g.M_dev : g.M;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  if (m0 >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  // split-K over the concatenated K of all segments
  int Ktot = 0;
  for (int s = 0; s < g.nseg; ++s) Ktot += g.seg[s].K;
  const int per = (((Ktot + g.ksplit - 1) / g.ksplit) + GBK - 1) / GBK * GBK;
  const int kb = blockIdx.z * per;
  const int ke = min(Ktot, kb + per);
  if (kb >= ke) return;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = kb; k0 < ke; k0 += GBK) {
    // stage A (64 x 16) and B (16 x 64): 4 elements per thread each
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + e * 256;
      // A: element (m = idx % 64, k = idx / 64) -> consecutive threads walk m (row-major dY^T reads)
      {
        const int mm = idx & 63, kk = idx >> 6;
        const int m = m0 + mm, k = k0 + kk;
        float v = 0.f;
        if (m < M && k < ke) {
          int kl = k, s = 0;
          while (s + 1 < g.nseg && kl >= g.seg[s].K) { kl -= g.seg[s].K; ++s; }
          v = g.seg[s].A[(long)m * g.seg[s].a_rs + (long)kl * g.seg[s].a_cs];
        }
        As[kk][mm] = v;
      }
      {
        const int nn = idx & 63, kk = idx >> 6;
        const int n = n0 + nn, k = k0 + kk;
        float v = 0.f;
        if (n < g.N && k < ke) {
          int kl = k, s = 0;
          while (s + 1 < g.nseg && kl >= g.seg[s].K) { kl -= g.seg[s].K; ++s; }
          v = g.seg[s].B[(long)kl * g.seg[s].b_rs + (long)n * g.seg[s].b_cs];
        }
        Bs[kk][nn] = v;
      }
    }
    __syncthreads();
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
        if (g.relu) v = fmaxf(v, 0.f);
        if (g.mask && !(g.mask[(long)m * g.ldm + n] > 0.f)) v = 0.f;
        *c = v;
      }
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
  if (threadIdx.x < 64 && n < N && r0 < r1) atomicAdd(out + n, sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x]);
}

}  // namespace anr
