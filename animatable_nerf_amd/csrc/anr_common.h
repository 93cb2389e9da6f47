// anr_common.h — shared device helpers for the Animatable-NeRF hot path on gfx950 (CDNA4).
//
// Everything here that feeds the sample keep-mask (linspace bits, z, world->pose, the trilinear
// volume lookup) reproduces the reference's fp32 operation order exactly and must be compiled
// without FP contraction (each TU that uses it sets `#pragma clang fp contract(off)` where needed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ANR_WAVE 64
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace anr {

// torch.linspace(start=0, end=1, steps=n) on CPU: symmetric formula (tpose_renderer.py:26)
__device__ __forceinline__ float linspace01(int i, int n) {
  const float step = 1.0f / (float)(n - 1);
  const int half = n / 2;
  return (i < half) ? fmaf(step, (float)i, 0.0f) : fmaf(-step, (float)(n - 1 - i), 1.0f);
}

// One trilinear lookup in the layout of blend_utils.py:119-149 / ATen grid_sampler_3d (CPU):
// volume memory (X,Y,Z,C) viewed as (C, D=X, H=Y, W=Z); grid = normalised (z, y, x).
struct TriCell {
  int base[8];     // voxel offsets (in voxels) of the 8 corners, -1 if out of bounds
  float w[8];      // tnw, tne, tsw, tse, bnw, bne, bsw, bse
};

__device__ __forceinline__ float grid_src(float g, int size) {
#pragma clang fp contract(off)
  float c = ((g + 1.0f) / 2.0f) * (float)(size - 1);
  return fminf((float)(size - 1), fmaxf(c, 0.0f));
}

// corner offsets and weights from the unnormalised source coordinates (ix along Z, iy along Y, iz along X)
__device__ __forceinline__ void tri_cell_src(float ix, float iy, float iz, int X, int Y, int Z, TriCell& t);

// p: point in the volume's frame; lo/hi: bounds (2,3); dims X,Y,Z.
__device__ __forceinline__ void tri_cell(const float p[3], const float lo[3], const float hi[3],
                                         int X, int Y, int Z, TriCell& t) {
#pragma clang fp contract(off)
  float g[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float ext = hi[c] - lo[c];
    float v = (p[c] - lo[c]) / ext;
    g[c] = v * 2.0f - 1.0f;
  }
  tri_cell_src(grid_src(g[2], Z), grid_src(g[1], Y), grid_src(g[0], X), X, Y, Z, t);
}

__device__ __forceinline__ void tri_cell_src(float ix, float iy, float iz, int X, int Y, int Z, TriCell& t) {
#pragma clang fp contract(off)
  const int x0 = (int)floorf(ix), y0 = (int)floorf(iy), z0 = (int)floorf(iz);
  const int x1 = x0 + 1, y1 = y0 + 1, z1 = z0 + 1;
  const float fx0 = (float)x0, fy0 = (float)y0, fz0 = (float)z0;
  const float fx1 = (float)x1, fy1 = (float)y1, fz1 = (float)z1;
  const float ax = fx1 - ix, bx = ix - fx0, ay = fy1 - iy, by = iy - fy0, az = fz1 - iz, bz = iz - fz0;
  t.w[0] = (ax * ay) * az;  t.w[1] = (bx * ay) * az;
  t.w[2] = (ax * by) * az;  t.w[3] = (bx * by) * az;
  t.w[4] = (ax * ay) * bz;  t.w[5] = (bx * ay) * bz;
  t.w[6] = (ax * by) * bz;  t.w[7] = (bx * by) * bz;
  const int xs[2] = {x0, x1}, ys[2] = {y0, y1}, zs[2] = {z0, z1};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int cx = xs[k & 1], cy = ys[(k >> 1) & 1], cz = zs[k >> 2];
    const bool ok = cx >= 0 && cx < Z && cy >= 0 && cy < Y && cz >= 0 && cz < X;
    t.base[k] = ok ? ((cz * Y + cy) * Z + cx) : -1;
  }
}

// Exact single-channel lookup (reference accumulation order, rounded after each add).
__device__ __forceinline__ float tri_channel(const float* __restrict__ vol, int C, int ch, const TriCell& t) {
#pragma clang fp contract(off)
  float acc = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (t.base[k] >= 0) acc = acc + vol[(size_t)t.base[k] * C + ch] * t.w[k];
  return acc;
}

// (x - Th) @ R  (blend_utils.py:6-16). torch's CPU matmul of a (1, n, 3) x (1, 3, 3) float32 product
// with n >= 45 (every chunk: n = rays x 64) runs a BLAS kernel whose dot is the FMA chain
// fma(d2, R2j, fma(d1, R1j, d0 * R0j)) (measured bit-exact; n < 45 takes a plain multiply-add path)
__device__ __forceinline__ void world_to_pose(const float x[3], const float* R, const float* Th, float out[3]) {
#pragma clang fp contract(off)
  const float d0 = x[0] - Th[0], d1 = x[1] - Th[1], d2 = x[2] - Th[2];
#pragma unroll
  for (int j = 0; j < 3; ++j) out[j] = fmaf(d2, R[2 * 3 + j], fmaf(d1, R[1 * 3 + j], d0 * R[0 * 3 + j]));
}

// the same product when torch's matmul takes its small path (n < 45 points, measured): separate
// multiplies, left-to-right adds. Free points (the mesh path's get_alpha) can end in such a chunk.
__device__ __forceinline__ void world_to_pose_small(const float x[3], const float* R, const float* Th, float out[3]) {
#pragma clang fp contract(off)
  const float d0 = x[0] - Th[0], d1 = x[1] - Th[1], d2 = x[2] - Th[2];
#pragma unroll
  for (int j = 0; j < 3; ++j) out[j] = (d0 * R[0 * 3 + j] + d1 * R[1 * 3 + j]) + d2 * R[2 * 3 + j];
}

// world -> pose of free point i of a call split into chunks of chunk_pts points (matmul per chunk)
__device__ __forceinline__ void world_to_pose_pt(const float* __restrict__ wpts, long i, long n_pts, int chunk_pts,
                                                 const float* R, const float* Th, float out[3]) {
  const float x[3] = {wpts[3 * i], wpts[3 * i + 1], wpts[3 * i + 2]};
  const long c0 = (i / chunk_pts) * chunk_pts;
  const long len = n_pts - c0 < chunk_pts ? n_pts - c0 : chunk_pts;
  if (len >= 45) world_to_pose(x, R, Th, out);
  else world_to_pose_small(x, R, Th, out);
}

// novel-view filter (tpose_renderer_mmsk.py:14-57): world point -> every training view (RT world ->
// camera, K), rounded half-to-even, clamped to the image, looked up in that view's mask; visible = in all
__device__ __forceinline__ bool visible_in_views(const float pts[3], int n_views, const float* __restrict__ Ks,
                                                 const float* __restrict__ RT, const uint8_t* __restrict__ msks,
                                                 int img_h, int img_w) {
  bool vis = true;
  for (int v = 0; v < n_views; ++v) {
    const float* R = RT + 12 * v;
    const float* K = Ks + 9 * v;
    float q[3], s3[3];
    for (int j = 0; j < 3; ++j) q[j] = fmaf(pts[2], R[4 * j + 2], fmaf(pts[1], R[4 * j + 1], pts[0] * R[4 * j])) + R[4 * j + 3];
    for (int j = 0; j < 3; ++j) s3[j] = fmaf(q[2], K[3 * j + 2], fmaf(q[1], K[3 * j + 1], q[0] * K[3 * j]));
    long long xi = (long long)rintf(s3[0] / s3[2]);
    long long yi = (long long)rintf(s3[1] / s3[2]);
    xi = xi < 0 ? 0 : (xi > img_w - 1 ? img_w - 1 : xi);
    yi = yi < 0 ? 0 : (yi > img_h - 1 ? img_h - 1 : yi);
    vis = vis && msks[((size_t)v * img_h + yi) * img_w + xi] != 0;
  }
  return vis;
}

// Positional-encoding feature f of gamma(x) (embedder.py:5-54): [x, sin(2^0 x), cos(2^0 x), ...]
__device__ __forceinline__ float embed_feature(const float x[3], int f, int nfreq) {
  if (f < 3) return x[f];
  const int g = f - 3;
  const int freq = g / 6;
  if (freq >= nfreq) return 0.0f;
  const int w = g - freq * 6;
  const int comp = (w >= 3) ? w - 3 : w;
  const float v = x[comp] * (float)(1 << freq);
  return (w >= 3) ? cosf(v) : sinf(v);
}

// ------------------------------------------------------------------------------------------
// A2/A3: z of sample s (perturbed when t_rand != NULL), identical ops to tpose_renderer.py:26-36
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float z_base(float nr, float fr, int i, int n) {
#pragma clang fp contract(off)
  const float t = linspace01(i, n);
  const float a = nr * (1.0f - t);
  const float b = fr * t;
  return a + b;
}

__device__ __forceinline__ float z_sample(float nr, float fr, const float* __restrict__ trow, int s, int n) {
#pragma clang fp contract(off)
  if (trow == nullptr) return z_base(nr, fr, s, n);
  float upper, lower;
  if (s < n - 1) upper = 0.5f * (z_base(nr, fr, s + 1, n) + z_base(nr, fr, s, n));
  else upper = z_base(nr, fr, n - 1, n);
  if (s > 0) lower = 0.5f * (z_base(nr, fr, s, n) + z_base(nr, fr, s - 1, n));
  else lower = z_base(nr, fr, 0, n);
  return lower + (upper - lower) * trow[s];
}

__device__ __forceinline__ void sample_point(const float* __restrict__ ray_o, const float* __restrict__ ray_d, const float* __restrict__ near_,
                             const float* __restrict__ far_, const float* __restrict__ t_rand, int ray, int s, int n,
                             float& z, float& dist, float pts[3]) {
#pragma clang fp contract(off)
  const float nr = near_[ray], fr = far_[ray];
  const float* trow = t_rand ? t_rand + (size_t)ray * n : nullptr;
  z = z_sample(nr, fr, trow, s, n);
  if (s < n - 1) dist = z_sample(nr, fr, trow, s + 1, n) - z;
  else dist = z - z_sample(nr, fr, trow, s - 1, n);
#pragma unroll
  for (int c = 0; c < 3; ++c) pts[c] = ray_o[3 * ray + c] + ray_d[3 * ray + c] * z;
}

// exclusive scan of one int per thread over a 256-thread block (sh: 4 ints of LDS); total = block sum
__device__ __forceinline__ int block_excl_scan_256(int v, int* sh, int& total) {
  // 256 threads: wave inclusive scans + wave totals in LDS
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  int base = 0;
  for (int k = 0; k < w; ++k) base += sh[k];
  total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return base + x - v;
}

// exp(z) within ~2 ulp: exact-split exponent, v_exp_f32 on the reduced argument, ldexp (the
// libm-accurate expf costs ~3x the instructions; the softplus epilogues are VALU-bound on it)
__device__ __forceinline__ float fast_exp(float z) {
  const float n = rintf(z * 1.44269502f);
  const float r = fmaf(z, 1.44269502f, -n) + z * 1.92596299e-8f;
  return ldexpf(__builtin_amdgcn_exp2f(r), (int)n);
}

// log1p(e), e >= 0, within a few ulp: a 6-term series below 1/32, else log(u) e / (u - 1) with
// u = 1 + e (Goldberg's correction of the rounding in u; u - 1 is exact)
__device__ __forceinline__ float fast_log1p(float e) {
  const float s = e * (1.f + e * (-0.5f + e * (0.333333343f + e * (-0.25f + e * (0.2f + e * -0.166666672f)))));
  const float u = 1.f + e;
  const float l = __builtin_amdgcn_logf(u) * 0.693147182f * (e * __builtin_amdgcn_rcpf(u - 1.f));
  return e < 0.03125f ? s : l;
}

// x / b for a constant b with its float reciprocal rb = RN(1 / b): the product, then one FMA residual
// correction (Markstein) — the correctly rounded quotient (as the IEEE division torch performs) in 3
// instructions instead of the ~10 of the compiler's division sequence (v_div_scale / v_div_fmas /
// v_div_fixup); ANR_EXACT_DIV=1 keeps the plain division
#ifndef ANR_EXACT_DIV
#define ANR_EXACT_DIV 0
#endif
__device__ __forceinline__ float div_const(float x, float b, float rb) {
#if ANR_EXACT_DIV
  (void)rb;
  return x / b;
#else
  const float q = x * rb;
  return __builtin_fmaf(__builtin_fmaf(-q, b, x), rb, q);
#endif
}

// softplus(beta=100, threshold=20) backward factor sigmoid(100 z) recomputed from the layer's OUTPUT
// h = softplus(z) instead of a stored exp(100 z): sigmoid(100 z) = 1 - exp(-100 h) exactly (above the
// threshold h = z and the factor rounds to 1, as torch's pass-through). One hardware exp2: the factor
// is within ~1.5e-7 ABSOLUTE of the stored-factor path's everywhere (relative precision is lost only
// where the factor itself is < ~1e-3 and its gradient contribution with it; the sdf backward is held
// to 2e-4 absolute).
__device__ __forceinline__ float softplus_factor_h(float h) {
  return 1.f - __builtin_amdgcn_exp2f(h * -144.269504f);
}

}  // namespace anr
