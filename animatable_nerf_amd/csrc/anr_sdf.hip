// anr_sdf.hip — per-sample kernels of the sdf_pdf render path (config 5).
//
//   k_sdf_front     B1 + A2-A6: z, world->pose, exact 5-NN over the posed SMPL vertices (LDS-resident),
//                   inverse-distance weights, keep ballot (pnorm < 0.1) + per-chunk argmin
//                   (anisdf_pdf_network.py:156-177, sample_utils.py:309-348)
//   k_sdf_wnorm     effective weights v * (g / |v|_row) of the 14 weight-normed layers
//   k_sdf_fold      per-frame folded biases: poses into resd_linears.0/.5, color_latent into lin3
//   k_sdf_tbtab     per-chunk tbounds after the reference's in-place widening (:203-205)
//   k_sdf_prep      B2: KNN blend, LBS pose -> T -> big pose (points and directions), gamma_10
//   k_sdf_mid       B3 tail: 0.05 tanh, tpose, gamma_6 / gamma_4 inputs of the SDF / colour nets
//   k_sdf_gtop      B4: d sdf / d h7 = softplus'(z7) * W8[0]
//   k_sdf_gamma_bwd B4: gamma_6 backward -> gradients (the normal fed to the colour net)
//   k_sdf_raw       B5/B6 tail: Laplace density, alpha with 0.005, sigmoid rgb, tbounds mask, scatter
//   k_sdf_msk_*     B7: per-ray min sdf, sign-change intersection, ordered msk_sdf / msk_label lists
// The GEMMs between them run on anr_gemm.hip (anr_sdf_capi.hip drives the sequence).
#include "anr_common.h"
#include "anr_sdf.h"

#pragma clang fp contract(off)

namespace anr {

#define SDF_MAX_VERTS 6912  // 108 cells of 64 vertices
#define SDF_CELL 64
#define SDF_MAX_CELLS (SDF_MAX_VERTS / SDF_CELL)
#define SDF_SORT_N 8192     // power-of-two key array for the in-LDS bitonic sort

typedef float pf2 __attribute__((ext_vector_type(2)));

// squared distance from p to an axis-aligned box, in the vertex formula's association
// ((dx*dx + dy*dy) + dz*dz). Each |dx| here is the rounded distance to the box face between p and
// any vertex inside, so by the monotonicity of IEEE rounding it is <= that vertex's rounded |dx|,
// and the sum is <= every in-box vertex's d^2 exactly — a bound with no margin.
__device__ __forceinline__ float box_d2(const float p[3], float4 lo, float4 hi) {
  const float dx = p[0] < lo.x ? p[0] - lo.x : (p[0] > hi.x ? p[0] - hi.x : 0.f);
  const float dy = p[1] < lo.y ? p[1] - lo.y : (p[1] > hi.y ? p[1] - hi.y : 0.f);
  const float dz = p[2] < lo.z ? p[2] - lo.z : (p[2] > hi.z ? p[2] - hi.z : 0.f);
  return (dx * dx + dy * dy) + dz * dz;
}

__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // 6 bits -> every third bit
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 6; ++b) r |= ((v >> b) & 1u) << (3 * b);
  return r;
}

// ------------------------------------------------------------------------------------------
// B1 front-end. Persistent: one 1024-thread workgroup per CU. Prologue (per workgroup, ~tens of µs):
// the posed vertices are Morton-sorted in LDS (18-bit cell code above the 13-bit vertex index,
// bitonic sort of 8192 keys) and stored in cells of 64 consecutive sorted vertices with their
// bounding boxes. Wave = ray, lane = sample. The wave visits the cells nearest its middle sample
// first (a 128-key bitonic sort across the lanes) and skips a cell when no lane's 5th-best d^2
// reaches the cell's box bound (box_d2: exact, so a skipped cell holds no vertex that could enter
// or tie). Insertion compares (d^2, index) lexicographically, so the result is the K smallest
// (d^2, index) pairs whatever the visiting order — pytorch3d knn_points' bounded max-heap result,
// bit-identical to the earlier full index-order scan. d^2 = (dx*dx + dy*dy) + dz*dz, no contraction.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_sdf_front(SdfFrontArgs a) {
  // sorted vertex pairs (2i, 2i + 1) as {x, x', y, y', z, z', idx, idx'}: two 16-B reads per pair
  __shared__ float4 sv[SDF_MAX_VERTS];
  __shared__ uint32_t keys[SDF_SORT_N];
  __shared__ float4 cbox[2 * SDF_MAX_CELLS];
  __shared__ float red[16][6];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nv = a.nv, ncell = (nv + SDF_CELL - 1) / SDF_CELL;

  // vertex bounds -> 64^3 Morton cells
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int j = tid; j < nv; j += blockDim.x)
    for (int c = 0; c < 3; ++c) {
      const float v = a.verts[3 * j + c];
      mn[c] = fminf(mn[c], v); mx[c] = fmaxf(mx[c], v);
    }
  for (int c = 0; c < 3; ++c)
    for (int off = 32; off > 0; off >>= 1) {
      mn[c] = fminf(mn[c], __shfl_xor(mn[c], off));
      mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], off));
    }
  if (lane == 0)
    for (int c = 0; c < 3; ++c) { red[wid][c] = mn[c]; red[wid][3 + c] = mx[c]; }
  __syncthreads();
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w)
    for (int c = 0; c < 3; ++c) { mn[c] = fminf(mn[c], red[w][c]); mx[c] = fmaxf(mx[c], red[w][3 + c]); }
  float sc[3];
  for (int c = 0; c < 3; ++c) sc[c] = mx[c] > mn[c] ? 63.99f / (mx[c] - mn[c]) : 0.f;
  for (int j = tid; j < SDF_SORT_N; j += blockDim.x) {
    uint32_t k = 0xffffffffu;
    if (j < nv) {
      uint32_t m = 0;
      for (int c = 0; c < 3; ++c) {
        const float f = (a.verts[3 * j + c] - mn[c]) * sc[c];
        const uint32_t q = f >= 0.f ? min((uint32_t)f, 63u) : 0u;  // NaN -> 0
        m |= spread3(q) << c;
      }
      k = (m << 13) | (uint32_t)j;
    }
    keys[j] = k;
  }
  __syncthreads();
  for (int k = 2; k <= SDF_SORT_N; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < SDF_SORT_N; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t x = keys[i], y = keys[l];
          if (((i & k) == 0) == (x > y)) { keys[i] = y; keys[l] = x; }
        }
      }
      __syncthreads();
    }
  for (int s = tid; s < ncell * SDF_CELL; s += blockDim.x) {
    const bool in = s < nv;
    const uint32_t j = in ? (keys[s] & 8191u) : 0x7fffu;
    float* q = (float*)&sv[(s >> 1) * 2] + (s & 1);
    q[0] = in ? a.verts[3 * j] : INFINITY;
    q[2] = in ? a.verts[3 * j + 1] : INFINITY;
    q[4] = in ? a.verts[3 * j + 2] : INFINITY;
    ((uint32_t*)q)[6] = j;  // index bits (a plain store: never touched by float arithmetic)
  }
  __syncthreads();
  for (int c = wid; c < ncell; c += blockDim.x >> 6) {
    const int s = c * SDF_CELL + lane;
    const float* q = (const float*)&sv[(s >> 1) * 2] + (s & 1);
    float lo[3], hi[3];
    for (int e = 0; e < 3; ++e) {
      lo[e] = s < nv ? q[2 * e] : INFINITY;
      hi[e] = s < nv ? q[2 * e] : -INFINITY;
      for (int off = 32; off > 0; off >>= 1) {
        lo[e] = fminf(lo[e], __shfl_xor(lo[e], off));
        hi[e] = fmaxf(hi[e], __shfl_xor(hi[e], off));
      }
    }
    if (lane == 0) {
      cbox[2 * c] = make_float4(lo[0], lo[1], lo[2], 0.f);
      cbox[2 * c + 1] = make_float4(hi[0], hi[1], hi[2], 0.f);
    }
  }
  __syncthreads();

  const int wpb = blockDim.x >> 6;
  for (int ray = blockIdx.x * wpb + wid; ray < a.n_rays; ray += gridDim.x * wpb) {
    float p[3];
    const long pid_ = (long)ray * 64 + lane;
    const bool valid = !a.wpts || pid_ < a.n_pts;
    bool vis = true;  // novel-view renders: the world sample projects inside every training view's mask
    if (a.wpts) {
      if (valid) world_to_pose_pt(a.wpts, pid_, a.n_pts, a.n_pts, a.R, a.Th, p);
      else p[0] = p[1] = p[2] = 0.f;
    } else {
      float z, dist, pts[3];
      sample_point(a.ray_o, a.ray_d, a.near_, a.far_, a.t_rand, ray, lane, 64, z, dist, pts);
      world_to_pose(pts, a.R, a.Th, p);
      if (a.n_views > 0) vis = visible_in_views(pts, a.n_views, a.Ks, a.RT, a.msks, a.img_h, a.img_w);
    }
    float b0 = INFINITY, b1 = INFINITY, b2 = INFINITY, b3 = INFINITY, b4 = INFINITY;
    int i0 = 0, i1 = 0, i2 = 0, i3 = 0, i4 = 0;
    auto lt = [](float d, int j, float b, int i) { return d < b || (d == b && j < i); };
    auto insert = [&](float d, int j) {
      if (lt(d, j, b4, i4)) {
        if (lt(d, j, b3, i3)) {
          b4 = b3; i4 = i3;
          if (lt(d, j, b2, i2)) {
            b3 = b2; i3 = i2;
            if (lt(d, j, b1, i1)) {
              b2 = b1; i2 = i1;
              if (lt(d, j, b0, i0)) { b1 = b0; i1 = i0; b0 = d; i0 = j; }
              else { b1 = d; i1 = j; }
            } else { b2 = d; i2 = j; }
          } else { b3 = d; i3 = j; }
        } else { b4 = d; i4 = j; }
      }
    };
    // visiting order: cells by box distance from the ray's middle sample (keys carry the cell id in
    // their low 7 bits; only the order changes, never the result)
    const float pm[3] = {__shfl(p[0], 32), __shfl(p[1], 32), __shfl(p[2], 32)};
    uint32_t ck[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = lane + 64 * r;
      ck[r] = 0xffffffffu;
      if (c < ncell) {
        const float d = box_d2(pm, cbox[2 * c], cbox[2 * c + 1]);
        ck[r] = ((d == d ? __float_as_uint(d) : 0x7f800000u) & ~127u) | (uint32_t)c;
      }
    }
#pragma unroll
    for (int k = 2; k <= 128; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        if (j == 64) {  // element l vs l + 64: both in this lane
          const uint32_t x = ck[0], y = ck[1];
          const bool up = (lane & k) == 0;  // k == 128: always ascending
          ck[0] = up ? min(x, y) : max(x, y);
          ck[1] = up ? max(x, y) : min(x, y);
        } else {
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            const int i = lane + 64 * r;
            const uint32_t o = __shfl_xor(ck[r], j);
            const bool up = (i & k) == 0, low = (i & j) == 0;
            ck[r] = (up == low) ? min(ck[r], o) : max(ck[r], o);
          }
        }
      }
    // two vertices per step on packed fp32 (v_pk_add / v_pk_mul: per-element IEEE, no contraction,
    // so each d^2 is the scalar formula's); padding vertices sit at infinity and never enter
    const pf2 P0 = {p[0], p[0]}, P1 = {p[1], p[1]}, P2 = {p[2], p[2]};
    for (int t = 0; t < ncell; ++t) {
      const uint32_t key = __builtin_amdgcn_readlane(t < 64 ? ck[0] : ck[1], t & 63);
      const int c = (int)(key & 127u);
      if (!__any(box_d2(p, cbox[2 * c], cbox[2 * c + 1]) <= b4)) continue;
      const int j0 = c * SDF_CELL;
#pragma unroll 2
      for (int j = j0; j < j0 + SDF_CELL; j += 2) {
        const float4 va = sv[j], vb = sv[j + 1];
        const pf2 dx = P0 - pf2{va.x, va.y}, dy = P1 - pf2{va.z, va.w}, dz = P2 - pf2{vb.x, vb.y};
        const pf2 d = (dx * dx + dy * dy) + dz * dz;
        if (fminf(d[0], d[1]) <= b4) {  // one test per pair: most pairs insert nothing
          insert(d[0], (int)__float_as_uint(vb.z));
          insert(d[1], (int)__float_as_uint(vb.w));
        }
      }
    }
    // sample_blend_closest_points: dists = sqrt(d^2); disp = 1 / (dists + 1e-8); torch's 5-element
    // sum order is ((((x0 + x4) + x1) + x2) + x3); weights = disp / sum; pnorm = sequential sum d*w
    const float d0 = sqrtf(b0), d1 = sqrtf(b1), d2 = sqrtf(b2), d3 = sqrtf(b3), d4 = sqrtf(b4);
    const float q0 = 1.0f / (d0 + 1e-8f), q1 = 1.0f / (d1 + 1e-8f), q2 = 1.0f / (d2 + 1e-8f);
    const float q3 = 1.0f / (d3 + 1e-8f), q4 = 1.0f / (d4 + 1e-8f);
    const float S = (((q0 + q4) + q1) + q2) + q3;
    const float w0 = q0 / S, w1 = q1 / S, w2 = q2 / S, w3 = q3 / S, w4 = q4 / S;
    const float pn = valid ? (((d0 * w0 + d1 * w1) + d2 * w2) + d3 * w3) + d4 * w4 : INFINITY;
    const size_t pid = (size_t)ray * 64 + lane;
    uint4* rec = (uint4*)(a.knn + pid * 8);
    rec[0] = make_uint4(__float_as_uint(w0), __float_as_uint(w1), __float_as_uint(w2), __float_as_uint(w3));
    rec[1] = make_uint4(__float_as_uint(w4), (uint32_t)i0 | ((uint32_t)i1 << 16), (uint32_t)i2 | ((uint32_t)i3 << 16),
                        (uint32_t)i4);
    const bool keep = vis && pn < a.norm_th;
    const uint64_t m = __ballot(keep);
    if (lane == 0) a.mask[ray] = m;
    if (!keep && valid) {
      a.raw[pid] = make_float4(0.f, 0.f, 0.f, 0.f);
      a.sdf[pid] = 10.f;
    }
    const int rc = ray % a.chunk;
    uint64_t key = valid && vis ? ((uint64_t)__float_as_uint(pn) << 32) | (uint32_t)(rc * 64 + lane) : ~0ull;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t o = __shfl_xor(key, off);
      key = o < key ? o : key;
    }
    if (lane == 0) atomicMin((unsigned long long*)&a.chunk_min[ray / a.chunk], (unsigned long long)key);
  }
}

// ------------------------------------------------------------------------------------------
// weight norm (nn.utils.weight_norm, dim 0): one block per output row of the 14 layers
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sdf_wnorm(SdfTensors T, float* wimg) {
  const float* const* t = T.t;
  int row = blockIdx.x, L = 0;
  while (L < SDF_NUM_WN - 1 && row >= wn_layer(L).out) { row -= wn_layer(L).out; ++L; }
  const WnLayer d = wn_layer(L);
  const float* v = t[d.v] + (size_t)row * d.in;
  float s = 0.f;
  for (int k = threadIdx.x; k < d.in; k += 256) s += v[k] * v[k];
  __shared__ float sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  const float scale = t[d.g][row] / sqrtf(sh[0]);
  float* o = wimg + d.off + (size_t)row * d.in;
  for (int k = threadIdx.x; k < d.in; k += 256) o[k] = v[k] * scale;
}

// fold[0:256] = resd_linears.0 bias + W0[:, 63:135] poses; fold[256:512] = same for .5;
// fold[512:768] = colour lin3 bias + W3[:, 256:384] color_latent[latent_index]
__global__ __launch_bounds__(256) void k_sdf_fold(SdfTensors T, const float* wimg, const float* poses,
                                                  const int64_t* li, float* fold) {
  const float* const* t = T.t;
  const int which = blockIdx.x, n = threadIdx.x;
  float acc;
  if (which < 2) {
    const int l = which == 0 ? 0 : 5;
    const int in_ch = which == 0 ? 135 : 391;
    const float* W = t[SDF_RLIN0 + 2 * l] + (size_t)n * in_ch;
    acc = t[SDF_RLIN0 + 2 * l + 1][n];
    for (int q = 0; q < 72; ++q) acc = fmaf(W[63 + q], poses[q], acc);
  } else {
    const WnLayer d = wn_layer(12);
    const float* W = wimg + d.off + (size_t)n * 384;
    const float* lat = t[SDF_COLOR_LAT] + (size_t)li[0] * 128;
    acc = t[d.v - 2][n];
    for (int q = 0; q < 128; ++q) acc = fmaf(W[256 + q], lat[q], acc);
  }
  fold[which * 256 + n] = acc;
}

// tbounds[0] -= 0.05; tbounds[1] += 0.05 once per chunk, in place on the batch (fp32)
// chunk_min != NULL (the visibility-filtered render): only chunks with a visible sample widen, the others
// make no network call (tpose_renderer_mmsk.py:80-83)
__global__ void k_sdf_tbtab(const float* tbounds, int nchunks, float* tbtab, float* tb_out, const uint64_t* chunk_min) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float b[6];
  for (int k = 0; k < 6; ++k) b[k] = tbounds[k];
  for (int c = 0; c < nchunks; ++c) {
    if (!chunk_min || chunk_min[c] != ~0ull)
      for (int k = 0; k < 3; ++k) { b[k] = b[k] - 0.05f; b[3 + k] = b[3 + k] + 0.05f; }
    for (int k = 0; k < 6; ++k) tbtab[c * 6 + k] = b[k];
  }
  if (tb_out)
    for (int k = 0; k < 6; ++k) tb_out[k] = b[k];
}

// ------------------------------------------------------------------------------------------
// B2: thread per kept sample
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void blend16(const float bw[24], const float* __restrict__ A, float Ab[16]) {
#pragma clang fp contract(fast)
  for (int m = 0; m < 16; ++m) Ab[m] = 0.f;
  for (int j = 0; j < 24; ++j)
    for (int m = 0; m < 16; ++m) Ab[m] += bw[j] * A[j * 16 + m];
}

__device__ __forceinline__ void inv33(const float Ab[16], float Ri[9]) {
  const float a = Ab[0], b = Ab[1], c = Ab[2], d = Ab[4], e = Ab[5], f = Ab[6], g = Ab[8], h = Ab[9], k = Ab[10];
  const float c00 = e * k - f * h, c01 = c * h - b * k, c02 = b * f - c * e;
  const float c10 = f * g - d * k, c11 = a * k - c * g, c12 = c * d - a * f;
  const float c20 = d * h - e * g, c21 = b * g - a * h, c22 = a * e - b * d;
  const float rd = 1.0f / (a * c00 + b * c10 + c * c20);
  Ri[0] = c00 * rd; Ri[1] = c01 * rd; Ri[2] = c02 * rd;
  Ri[3] = c10 * rd; Ri[4] = c11 * rd; Ri[5] = c12 * rd;
  Ri[6] = c20 * rd; Ri[7] = c21 * rd; Ri[8] = c22 * rd;
}

// the workgroup's 256 rows of a [P][W] block, written column-fastest by all threads (coalesced):
// value(row, col) from the per-row values staged in LDS by the thread-per-sample phase
template <int W, typename F>
__device__ __forceinline__ void sdf_rows_store(float* base, int i0, int cnt, F value) {
  const int rows = min(256, cnt - i0);
  for (int f = threadIdx.x; f < rows * W; f += 256) {
    const int r = f / W, c = f - r * W;
    base[(size_t)(i0 + r) * W + c] = value(r, c);
  }
}

__device__ void sdf_prep_point(const SdfPointArgs& a, int i, float (*sp)[4]);

// thread per kept sample (LBS to the big pose), then gamma_10(bigpose) rows written coalesced
__global__ __launch_bounds__(256) void k_sdf_prep(SdfPointArgs a) {
  __shared__ float sp[256][4];
  const int i0 = blockIdx.x * 256, i = i0 + threadIdx.x;
  if (i < a.cnt) sdf_prep_point(a, i, sp);
  __syncthreads();
  // gamma_10 rows for the layer-GEMM residual MLP (the fused k_resd_b16 forms them on chip: Gr NULL)
  if (a.Gr) sdf_rows_store<64>(a.Gr, i0, a.cnt, [&](int r, int c) { return c < 63 ? embed_feature(sp[r], c, 10) : 0.f; });
}

__device__ void sdf_prep_point(const SdfPointArgs& a, int i, float (*sp)[4]) {
  const int pid = a.list[a.b0 + i];
  const int ray = pid >> 6, s = pid & 63;
  float p[3], pd[3];
  if (a.wpts) {  // free samples: pose_pts / pose_dirs of the call's (n_pts, 3) products
    world_to_pose_pt(a.wpts, pid, a.n_pts, a.n_pts, a.R, a.Th, p);
    const float zero[3] = {0.f, 0.f, 0.f};
    world_to_pose_pt(a.vdir, pid, a.n_pts, a.n_pts, a.R, zero, pd);  // world_dirs_to_pose_dirs: d @ R
  } else {
    float z, dist, pts[3];
    sample_point(a.ray_o, a.ray_d, a.near_, a.far_, a.t_rand, ray, s, 64, z, dist, pts);
    world_to_pose(pts, a.R, a.Th, p);
    // world_dirs_to_pose_dirs: d @ R
    const float* d = a.ray_d + 3 * ray;
    for (int j = 0; j < 3; ++j) pd[j] = fmaf(d[2], a.R[6 + j], fmaf(d[1], a.R[3 + j], d[0] * a.R[j]));  // torch matmul (n >= 45)
  }
  const uint4* rec = (const uint4*)(a.knn + (size_t)pid * 8);
  const uint4 r0 = rec[0], r1 = rec[1];
  const float w[5] = {__uint_as_float(r0.x), __uint_as_float(r0.y), __uint_as_float(r0.z), __uint_as_float(r0.w),
                      __uint_as_float(r1.x)};
  const int idx[5] = {(int)(r1.y & 0xffff), (int)(r1.y >> 16), (int)(r1.z & 0xffff), (int)(r1.z >> 16), (int)r1.w};
  float bw[24];
  for (int l = 0; l < 24; ++l) {
    float acc = a.weights[idx[0] * 24 + l] * w[0];
    for (int k = 1; k < 5; ++k) acc = acc + a.weights[idx[k] * 24 + l] * w[k];
    bw[l] = acc;
  }
  float Ab[16], Bb[16], Ri[9];
  blend16(bw, a.A, Ab);
  blend16(bw, a.bigA, Bb);
  inv33(Ab, Ri);
  const float y[3] = {p[0] - Ab[3], p[1] - Ab[7], p[2] - Ab[11]};
  float tp[3], td[3], bp[3], bd[3];
  for (int r = 0; r < 3; ++r) {
    tp[r] = (Ri[3 * r] * y[0] + Ri[3 * r + 1] * y[1]) + Ri[3 * r + 2] * y[2];
    td[r] = (Ri[3 * r] * pd[0] + Ri[3 * r + 1] * pd[1]) + Ri[3 * r + 2] * pd[2];
  }
  for (int r = 0; r < 3; ++r) {
    bp[r] = ((Bb[4 * r] * tp[0] + Bb[4 * r + 1] * tp[1]) + Bb[4 * r + 2] * tp[2]) + Bb[4 * r + 3];
    bd[r] = (Bb[4 * r] * td[0] + Bb[4 * r + 1] * td[1]) + Bb[4 * r + 2] * td[2];
  }
  float* pt = a.ptb + (size_t)i * 8;
  pt[0] = bp[0]; pt[1] = bp[1]; pt[2] = bp[2];
  pt[3] = bd[0]; pt[4] = bd[1]; pt[5] = bd[2];
  sp[threadIdx.x][0] = bp[0]; sp[threadIdx.x][1] = bp[1]; sp[threadIdx.x][2] = bp[2];
}

// sample_blend_closest_points of free points (anr_knn_blend): the front-end's KNN records (k_sdf_front
// with R = I, Th = 0) -> inside = pnorm < norm_th (no forced argmin: the mesh path's filter,
// sdf_mesh_renderer.py:58-60) and the blended weights in k_sdf_prep's summation order
__global__ __launch_bounds__(256) void k_knn_blend_out(const uint32_t* __restrict__ knn, const uint64_t* __restrict__ mask,
                                                       const float* __restrict__ weights, int n, float* bw,
                                                       uint8_t* inside) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (inside) inside[i] = (uint8_t)((mask[i >> 6] >> (i & 63)) & 1ull);
  if (!bw) return;
  const uint4* rec = (const uint4*)(knn + (size_t)i * 8);
  const uint4 r0 = rec[0], r1 = rec[1];
  const float w[5] = {__uint_as_float(r0.x), __uint_as_float(r0.y), __uint_as_float(r0.z), __uint_as_float(r0.w),
                      __uint_as_float(r1.x)};
  const int idx[5] = {(int)(r1.y & 0xffff), (int)(r1.y >> 16), (int)(r1.z & 0xffff), (int)(r1.z >> 16), (int)r1.w};
  for (int l = 0; l < 24; ++l) {
    float acc = weights[idx[0] * 24 + l] * w[0];
    for (int k = 1; k < 5; ++k) acc = acc + weights[idx[k] * 24 + l] * w[k];
    bw[(size_t)i * 24 + l] = acc;
  }
}

// the sdf mesh path's posed vertices (sdf_mesh_renderer.py:96-101): big pose -> T pose (inverse LBS with
// big_A), -> pose (LBS with A), -> world (x R^T + Th); blend weights bw (n, 24)
__global__ __launch_bounds__(256) void k_mesh_pose(const float* __restrict__ pts, const float* __restrict__ bw, int n,
                                                   const float* __restrict__ bigA, const float* __restrict__ A,
                                                   const float* __restrict__ R, const float* __restrict__ Th, float* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float w[24];
  for (int l = 0; l < 24; ++l) w[l] = bw[(size_t)i * 24 + l];
  float Bb[16], Ab[16], Ri[9];
  blend16(w, bigA, Bb);
  blend16(w, A, Ab);
  inv33(Bb, Ri);
  const float y[3] = {pts[3 * i] - Bb[3], pts[3 * i + 1] - Bb[7], pts[3 * i + 2] - Bb[11]};
  float tp[3], pp[3];
  for (int r = 0; r < 3; ++r) tp[r] = (Ri[3 * r] * y[0] + Ri[3 * r + 1] * y[1]) + Ri[3 * r + 2] * y[2];
  for (int r = 0; r < 3; ++r) pp[r] = ((Ab[4 * r] * tp[0] + Ab[4 * r + 1] * tp[1]) + Ab[4 * r + 2] * tp[2]) + Ab[4 * r + 3];
  for (int r = 0; r < 3; ++r)  // pose_points_to_world_points: pts @ R^T + Th
    out[(size_t)i * 3 + r] = ((pp[0] * R[3 * r] + pp[1] * R[3 * r + 1]) + pp[2] * R[3 * r + 2]) + Th[r];
}

// resd = 0.05 tanh(y); tpose = bigpose + resd; gamma_6(tpose) -> Xs0 and X4[:, 217:] / sqrt(2);
// colour input [tpose, gamma_4(bigdir), gradient (k_sdf_gamma_bwd)]. Thread per sample for tpose,
// then the rows are written column-fastest by the whole workgroup.
__global__ __launch_bounds__(256) void k_sdf_mid(SdfPointArgs a) {
  __shared__ float sp[256][8];
  const int i0 = blockIdx.x * 256, i = i0 + threadIdx.x;
  if (i < a.cnt) {
    const float* pt = a.ptb + (size_t)i * 8;
    const float* y = a.Yr + (size_t)i * 4;
    for (int r = 0; r < 3; ++r) {
      const float rs = 0.05f * tanhf(y[r]);
      a.resd_rows[(size_t)(a.b0 + i) * 3 + r] = rs;
      sp[threadIdx.x][r] = pt[r] + rs;
      sp[threadIdx.x][4 + r] = pt[3 + r];
    }
  }
  __syncthreads();
  const float sqrt2 = 1.41421356237309515f;
  const int rows = min(256, a.cnt - i0);
  if (!a.skip_sdf_in) {
    sdf_rows_store<40>(a.Xs0, i0, a.cnt, [&](int r, int c) { return c < 39 ? embed_feature(sp[r], c, 6) : 0.f; });
    for (int f = threadIdx.x; f < rows * 39; f += 256) {
      const int r = f / 39, c = f - r * 39;
      a.X4[(size_t)(i0 + r) * 256 + 217 + c] = embed_feature(sp[r], c, 6) / sqrt2;
    }
  }
  // C0: tpose (0..2), gamma_4(bigdir) (3..29); 30..32 (gradient) belong to k_sdf_gamma_bwd
  for (int f = threadIdx.x; f < rows * 40; f += 256) {
    const int r = f / 40, c = f - r * 40;
    if (c >= 30 && c < 33) continue;
    a.C0[(size_t)(i0 + r) * 40 + c] = c < 3 ? sp[r][c] : c < 30 ? embed_feature(sp[r] + 4, c - 3, 4) : 0.f;
  }
}

// d sdf / d z7 = softplus_backward(W8[0], z7)
__global__ __launch_bounds__(256) void k_sdf_gtop(SdfPointArgs a) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)a.cnt * 256) return;
  const int k = (int)(e & 255);
  const float g = a.wimg[wn_layer(8).off + k];
  const float d = a.D7[e];
  a.G7[e] = a.d7_h ? g * softplus_factor_h(d) : d >= 0.f ? g * d / (d + 1.f) : g;
}

// gamma_6 backward: x.grad = g_x + sum_f f*(g_sin cos(f x)) + f*(g_cos * -sin(f x)). The two input
// gradients (lin4's gamma columns, lin0's input) are summed into LDS by coalesced row reads first.
__global__ __launch_bounds__(256) void k_sdf_gamma_bwd(SdfPointArgs a) {
  __shared__ float gs_[256][40];
  const int i0 = blockIdx.x * 256, i = i0 + threadIdx.x;
  const int rows = min(256, a.cnt - i0);
  for (int f = threadIdx.x; f < rows * 39; f += 256) {
    const int r = f / 39, c = f - r * 39;
    gs_[r][c] = a.Gc[(size_t)(i0 + r) * 256 + 217 + c] + a.gB[(size_t)(i0 + r) * 40 + c];
  }
  __syncthreads();
  if (i >= a.cnt) return;
  const float* g = gs_[threadIdx.x];
  const float* c = a.C0 + (size_t)i * 40;
  const float tp[3] = {c[0], c[1], c[2]};
  float gr[3];
  for (int r = 0; r < 3; ++r) gr[r] = g[r];
  for (int f = 0; f < 6; ++f) {
    const float fr = (float)(1 << f);
    for (int r = 0; r < 3; ++r) {
      const float v = tp[r] * fr;
      const float gs = g[3 + 6 * f + r];
      const float gc = g[6 + 6 * f + r];
      gr[r] = gr[r] + (gs * cosf(v)) * fr;
      gr[r] = gr[r] + (gc * -sinf(v)) * fr;
    }
  }
  float* cc = a.C0 + (size_t)i * 40;
  for (int r = 0; r < 3; ++r) {
    cc[30 + r] = gr[r];
    a.grad_rows[(size_t)(a.b0 + i) * 3 + r] = gr[r];
  }
}

// sdf_to_alpha (Laplace CDF, beta clamped) -> 1 - exp(-relu(s) * 0.005); rgb = sigmoid; tbounds mask
__global__ __launch_bounds__(256) void k_sdf_raw(SdfPointArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.cnt) return;
  const int pid = a.list[a.b0 + i];
  const int ray = pid >> 6;
  const float sdf = a.Y8[(size_t)i * 264];
  const float beta = fminf(fmaxf(a.beta, 1e-9f), 1e6f);
  const float x = -sdf;
  const float ib = 1.0f / beta;
  const float sig = x <= 0.f ? ib * (0.5f * expf(x / beta)) : ib * (1.0f - 0.5f * expf(-x / beta));
  const float alpha = 1.0f - expf(-fmaxf(sig, 0.f) * 0.005f);
  const float* yc = a.Yc + (size_t)i * 4;
  float4 raw = make_float4(1.0f / (1.0f + expf(-yc[0])), 1.0f / (1.0f + expf(-yc[1])), 1.0f / (1.0f + expf(-yc[2])),
                           alpha);
  const float* tb = a.tbtab + (size_t)(ray / a.chunk) * 6;
  const float* c = a.C0 + (size_t)i * 40;
  bool inside = true;
  for (int r = 0; r < 3; ++r) inside = inside && c[r] > tb[r] && c[r] < tb[3 + r];
  if (!inside) raw = make_float4(0.f, 0.f, 0.f, 0.f);
  a.raw[pid] = raw;
  a.sdf[pid] = sdf;
}

// ------------------------------------------------------------------------------------------
// B7 msk_sdf (tpose_renderer.py:134-152): wave per ray for min / sign change, then per-chunk lists
// [min_sdf where no intersection and occ == 1] ++ [min_sdf where occ == 0], chunks concatenated
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sdf_msk_rays(SdfMskArgs a) {
  const int lane = threadIdx.x & 63;
  const int ray = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= a.n_rays) return;
  const float s = a.sdf[(size_t)ray * 64 + lane];
  const float nx = __shfl_down(s, 1);
  float mn = s;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mn = fminf(mn, __shfl_xor(mn, off));
  const float prod = s * nx;
  const bool neg = lane < 63 && prod < 0.f;  // sign(...).min() == -1
  const bool inter = __ballot(neg) != 0ull;
  if (lane == 0) {
    const uint8_t o = a.occ[ray];
    a.min_sdf[ray] = mn;
    a.flags[ray] = (uint8_t)(((!inter && o == 1) ? 1 : 0) | (o == 0 ? 2 : 0));
  }
}

__device__ __forceinline__ int block_scan_1024(int v, int* sh, int& total) {
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
  total = 0;
  for (int k = 0; k < 16; ++k) {
    if (k < w) base += sh[k];
    total += sh[k];
  }
  __syncthreads();
  return base + x - v;
}

// block per chunk (1024 threads, 2 rays each): list lengths
__global__ __launch_bounds__(1024) void k_sdf_msk_count(SdfMskArgs a) {
  __shared__ int sh[16];
  const int r0 = blockIdx.x * a.chunk;
  const int r1 = min(a.n_rays, r0 + a.chunk);
  int cnt = 0;
  for (int r = r0 + threadIdx.x; r < r1; r += 1024) {
    const uint8_t f = a.flags[r];
    cnt += (f & 1) + ((f >> 1) & 1);
  }
  int total;
  block_scan_1024(cnt, sh, total);
  if (threadIdx.x == 0) a.chunk_cnt[blockIdx.x] = total;
}

// chunk_cnt now holds exclusive chunk offsets; write the two ordered lists of each chunk
__global__ __launch_bounds__(1024) void k_sdf_msk_write(SdfMskArgs a) {
  __shared__ int sh[16];
  const int r0 = blockIdx.x * a.chunk;
  const int r1 = min(a.n_rays, r0 + a.chunk);
  const int base = a.chunk_cnt[blockIdx.x];
  int n_ind_total = 0;
  // pass 1: the "ind" list (rays in order), pass 2: the "free" list
  for (int pass = 0; pass < 2; ++pass) {
    int carry = 0;
    for (int r = r0; r < r1; r += 1024) {
      const int rr = r + threadIdx.x;
      const int f = rr < r1 ? ((a.flags[rr] >> pass) & 1) : 0;
      int tot;
      const int ex = block_scan_1024(f, sh, tot);
      if (f) {
        const int pos = base + (pass ? n_ind_total : 0) + carry + ex;
        a.msk_sdf[pos] = a.min_sdf[rr];
        a.msk_label[pos] = pass ? 0.f : 1.f;
      }
      carry += tot;
    }
    if (pass == 0) n_ind_total = carry;
  }
}

}  // namespace anr
