// anr_rays.hip — ray-side kernels of the render path (HBM-bound integer / fp32 work, no MFMA).
//
//   k_near_far      A14  ray/box slab test in fp64 (if_nerf_data_utils.py:156-196), bit-exact
//   k_frontend      A2-A6 z sampling, world->pose, channel-24 trilinear lookup, keep ballot,
//                   per-chunk argmin (tpose_renderer.py:14-39, tpose_nerf_network.py:143-157)
//   k_count/k_scan/k_compact   ordered compaction of kept samples (no host sync)
//   k_chunk_argmax / k_flag*   alpha_ind rows (tpose_nerf_network.py:192-196)
//   k_composite     A12 raw2outputs (nerf_net_utils.py:6-36), one wave per ray, wave product-scan
//
// One wave per ray everywhere a ray is touched: lane = sample (N_samples == 64 == wave width),
// so every per-ray access is one coalesced 256-B (or 1-KiB for float4 raw) wave instruction.
#include <type_traits>

#include "anr_common.h"
#include "anr_kernels.h"

#pragma clang fp contract(off)

namespace anr {

// ------------------------------------------------------------------------------------------
// A14 near/far, fp64, numpy operation order; eps 1e-6, padding 0.01; hit <=> exactly 2 planes.
// ------------------------------------------------------------------------------------------
// T = float: test-split rays (cast to float32 before get_near_far, :330-333); T = double: the
// train split, where get_near_far sees get_rays' float64 arrays (:256-262), |d| included.
template <typename T>
__device__ __forceinline__ void near_far_one(const T ro[3], const T rd[3], const float* __restrict__ bounds,
                                             uint8_t& hit_out, float& near_out, float& far_out) {
  double b[2][3];
  for (int c = 0; c < 3; ++c) {
    b[0][c] = (double)bounds[c] + (-0.01);
    b[1][c] = (double)bounds[3 + c] + 0.01;
  }
  const double o[3] = {(double)ro[0], (double)ro[1], (double)ro[2]};
  const double d[3] = {(double)rd[0], (double)rd[1], (double)rd[2]};
  const double eps = 1e-6;
  int hits = 0;
  double pin[2][3] = {{0, 0, 0}, {0, 0, 0}};
  for (int k = 0; k < 6; ++k) {  // order: min_x, min_y, min_z, max_x, max_y, max_z
    const int side = k / 3, ax = k % 3;
    const double t = (b[side][ax] - o[ax]) / d[ax];
    double p[3];
    for (int c = 0; c < 3; ++c) p[c] = t * d[c] + o[c];
    const bool in = (p[0] >= (b[0][0] - eps)) & (p[0] <= (b[1][0] + eps)) & (p[1] >= (b[0][1] - eps)) &
                    (p[1] <= (b[1][1] + eps)) & (p[2] >= (b[0][2] - eps)) & (p[2] <= (b[1][2] + eps));
    if (in) {
      if (hits < 2)
        for (int c = 0; c < 3; ++c) pin[hits][c] = p[c];
      ++hits;
    }
  }
  hit_out = hits == 2 ? 1 : 0;
  // np.linalg.norm(axis=1): sqrt((x0*x0 + x1*x1) + x2*x2); ray_d is float32 in the test split,
  // so |d| is evaluated in float32 and promoted at the division (if_nerf_data_utils.py:189-191)
  double nd;
  if constexpr (std::is_same<T, float>::value) nd = (double)sqrtf((rd[0] * rd[0] + rd[1] * rd[1]) + rd[2] * rd[2]);
  else nd = sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
  double dd[2];
  for (int h = 0; h < 2; ++h) {
    const double e0 = pin[h][0] - o[0], e1 = pin[h][1] - o[1], e2 = pin[h][2] - o[2];
    dd[h] = sqrt((e0 * e0 + e1 * e1) + e2 * e2) / nd;
  }
  near_out = (float)fmin(dd[0], dd[1]);
  far_out = (float)fmax(dd[0], dd[1]);
}

__global__ void k_near_far(const float* __restrict__ ray_o, const float* __restrict__ ray_d, int n,
                           const float* __restrict__ bounds, uint8_t* __restrict__ mask,
                           float* __restrict__ near_, float* __restrict__ far_) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float ro[3] = {ray_o[3 * i], ray_o[3 * i + 1], ray_o[3 * i + 2]};
  const float rd[3] = {ray_d[3 * i], ray_d[3 * i + 1], ray_d[3 * i + 2]};
  near_far_one<float>(ro, rd, bounds, mask[i], near_[i], far_[i]);
}

// ------------------------------------------------------------------------------------------
// (f) eval-split ray pipeline: get_rays (if_nerf_data_utils.py:64-89) per pixel + A14, then ordered
// compaction of the hits (get_rays_within_bounds :310-339). Arithmetic follows what numpy's np.dot
// does in the reference run: a sequential FMA chain for float64 cameras (dgemm kernel), separate
// multiply/add for float32 ones; |d| as sqrt((x*x + y*y) + z*z). Kinv and the origin -R^T T are
// computed by the caller with numpy exactly as the reference does.
// ------------------------------------------------------------------------------------------
// get_rays for pixel (r, c): d32 = the float32 direction the caller sees; for a float64 camera also
// d64 = the float64 direction before the cast (the train split tests the box with it)
__device__ __forceinline__ void cam_ray(const CamArgs& a, int r, int c, float d32[3], double d64[3]) {
  if (a.fp64) {
    const double xy[3] = {(double)c, (double)r, 1.0};
    double pc[3], q[3], pw[3], d[3];
    for (int j = 0; j < 3; ++j) pc[j] = fma(xy[2], a.Kinv[3 * j + 2], fma(xy[1], a.Kinv[3 * j + 1], xy[0] * a.Kinv[3 * j]));
    for (int k = 0; k < 3; ++k) q[k] = pc[k] - a.T[k];
    for (int j = 0; j < 3; ++j) pw[j] = fma(q[2], a.R[6 + j], fma(q[1], a.R[3 + j], q[0] * a.R[j]));
    for (int k = 0; k < 3; ++k) d[k] = pw[k] - a.o[k];
    const double n = sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
    for (int k = 0; k < 3; ++k) {
      d64[k] = d[k] / n;
      d32[k] = (float)d64[k];
    }
  } else {
    const float xy[3] = {(float)c, (float)r, 1.0f};
    float kinv[9], R[9], T[3], o[3], pc[3], q[3], pw[3], d[3];
    for (int k = 0; k < 9; ++k) { kinv[k] = (float)a.Kinv[k]; R[k] = (float)a.R[k]; }
    for (int k = 0; k < 3; ++k) { T[k] = (float)a.T[k]; o[k] = (float)a.o[k]; }
    for (int j = 0; j < 3; ++j) pc[j] = (xy[0] * kinv[3 * j] + xy[1] * kinv[3 * j + 1]) + xy[2] * kinv[3 * j + 2];
    for (int k = 0; k < 3; ++k) q[k] = pc[k] - T[k];
    for (int j = 0; j < 3; ++j) pw[j] = (q[0] * R[j] + q[1] * R[3 + j]) + q[2] * R[6 + j];
    for (int k = 0; k < 3; ++k) d[k] = pw[k] - o[k];
    const float n = sqrtf((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
    for (int k = 0; k < 3; ++k) {
      d32[k] = d[k] / n;
      d64[k] = (double)d32[k];
    }
  }
}

__global__ void k_cam_rays(CamArgs a) {
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= a.H * a.W) return;
  const int r = pix / a.W, c = pix - r * a.W;
  float d32[3];
  double d64[3];
  cam_ray(a, r, c, d32, d64);
  const float o32[3] = {(float)a.o[0], (float)a.o[1], (float)a.o[2]};
  for (int k = 0; k < 3; ++k) {
    a.all_o[3 * (size_t)pix + k] = o32[k];
    a.all_d[3 * (size_t)pix + k] = d32[k];
  }
  if (a.bounds) near_far_one<float>(o32, d32, a.bounds, a.mask[pix], a.all_near[pix], a.all_far[pix]);
}

// ordered compaction of the hit pixels: per-256-pixel counts, k_scan_blocks, scatter

__global__ __launch_bounds__(256) void k_cam_count(CamArgs a) {
  __shared__ int sh[4];
  const int pix = blockIdx.x * 256 + threadIdx.x;
  const int v = pix < a.H * a.W ? (int)a.mask[pix] : 0;
  int total;
  block_excl_scan_256(v, sh, total);
  if (threadIdx.x == 0) a.block_sum[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_cam_scatter(CamArgs a) {
  __shared__ int sh[4];
  const int pix = blockIdx.x * 256 + threadIdx.x;
  const int v = pix < a.H * a.W ? (int)a.mask[pix] : 0;
  int total;
  const int ex = block_excl_scan_256(v, sh, total);
  if (v) {
    const int pos = a.block_sum[blockIdx.x] + ex;
    for (int k = 0; k < 3; ++k) {
      a.ray_o[3 * (size_t)pos + k] = a.all_o[3 * (size_t)pix + k];
      a.ray_d[3 * (size_t)pos + k] = a.all_d[3 * (size_t)pix + k];
    }
    a.near_[pos] = a.all_near[pix];
    a.far_[pos] = a.all_far[pix];
    a.coord[2 * (size_t)pos] = pix / a.W;
    a.coord[2 * (size_t)pos + 1] = pix % a.W;
  }
}

// ------------------------------------------------------------------------------------------
// (f) train-split ray sampler: sample_ray_h36m(split='train') (if_nerf_data_utils.py:198-283).
// The pixel lists np.argwhere(msk == 1), (msk == 13) and (bound_mask == 1) (:238-249), row-major
// like argwhere, with msk = msk * bound_mask (u8, wrapping) and bound_mask[msk == 100] = 0
// (:230-231); the random draws into them stay on the host (np.random, so the stream of draws is
// the reference's), then k_trl_gather turns one round of draws into rays.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void trl_flags(const TrainRayArgs& a, int pix, int f[3]) {
  const int P = a.cam.H * a.cam.W;
  f[0] = f[1] = f[2] = 0;
  if (pix >= P) return;
  const uint8_t bm = a.bound_mask[pix];
  const uint8_t m = (uint8_t)(a.msk[pix] * bm);
  f[0] = m == 1;
  f[1] = m == 13;
  f[2] = bm == 1 && m != 100;
}

__global__ __launch_bounds__(256) void k_trl_count(TrainRayArgs a) {
  __shared__ int sh[4];
  int f[3];
  trl_flags(a, blockIdx.x * 256 + threadIdx.x, f);
  const int nb = gridDim.x;
  for (int k = 0; k < 3; ++k) {
    int total;
    block_excl_scan_256(f[k], sh, total);
    if (threadIdx.x == 0) a.block_sum[k * nb + blockIdx.x] = total;
  }
}

__global__ __launch_bounds__(256) void k_trl_scatter(TrainRayArgs a) {
  __shared__ int sh[4];
  const int pix = blockIdx.x * 256 + threadIdx.x;
  int f[3];
  trl_flags(a, pix, f);
  const int nb = gridDim.x;
  const size_t P = (size_t)a.cam.H * a.cam.W;
  for (int k = 0; k < 3; ++k) {
    int total;
    const int ex = block_excl_scan_256(f[k], sh, total);
    if (f[k]) a.lists[k * P + a.block_sum[k * nb + blockIdx.x] + ex] = pix;
  }
}

// One round of the sampling loop (:236-271): draws[i] indexes list 0 for i < n_seg[0], list 1 for
// the next n_seg[1], list 2 for the rest (the reference's concatenation order). Per draw: get_rays
// at the pixel, get_near_far on get_rays' arrays (float64 for a float64 camera), rgb = img (zero
// outside the bound mask when mask_bkgd, :228); the hits are appended in draw order at *n_out.
// One 1024-thread workgroup (a round draws at most nrays).
__global__ __launch_bounds__(1024) void k_trl_gather(TrainRayArgs a) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) base = *a.n_out;
  __syncthreads();
  const size_t P = (size_t)a.cam.H * a.cam.W;
  const int n = a.n_seg[0] + a.n_seg[1] + a.n_seg[2];
  for (int i0 = 0; i0 < n; i0 += 1024) {
    const int i = i0 + threadIdx.x;
    int hit = 0, pix = 0;
    float d32[3] = {0.f, 0.f, 0.f}, nr = 0.f, fr = 0.f;
    if (i < n) {
      const int seg = i < a.n_seg[0] ? 0 : (i < a.n_seg[0] + a.n_seg[1] ? 1 : 2);
      pix = a.lists[seg * P + a.draws[i]];
      const int r = pix / a.cam.W, c = pix - r * a.cam.W;
      double d64[3];
      cam_ray(a.cam, r, c, d32, d64);
      uint8_t h;
      if (a.cam.fp64) {
        near_far_one<double>(a.cam.o, d64, a.cam.bounds, h, nr, fr);
      } else {
        const float o32[3] = {(float)a.cam.o[0], (float)a.cam.o[1], (float)a.cam.o[2]};
        near_far_one<float>(o32, d32, a.cam.bounds, h, nr, fr);
      }
      hit = h;
    }
    // block-wide exclusive scan of the hit flags (16 waves)
    const uint64_t bal = __ballot(hit);
    const int before = __popcll(bal & ((1ull << lane) - 1));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = base, tot = 0;
    for (int k = 0; k < 16; ++k) {
      if (k < w) off += wsum[k];
      tot += wsum[k];
    }
    const int pos = off + before;
    if (hit && pos < a.cap) {
      for (int k = 0; k < 3; ++k) {
        a.ray_o[3 * (size_t)pos + k] = (float)a.cam.o[k];
        a.ray_d[3 * (size_t)pos + k] = d32[k];
        a.rgb[3 * (size_t)pos + k] = (a.mask_bkgd && a.bound_mask[pix] != 1) ? 0.0f : a.img[3 * (size_t)pix + k];
      }
      a.near_[pos] = nr;
      a.far_[pos] = fr;
      a.coord[2 * (size_t)pos] = pix / a.cam.W;
      a.coord[2 * (size_t)pos + 1] = pix % a.cam.W;
    }
    __syncthreads();
    if (threadIdx.x == 0) base += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *a.n_out = base;
}

// ------------------------------------------------------------------------------------------
// A4-A6 front-end: one wave per ray, lane = sample.
// ------------------------------------------------------------------------------------------
// One wave per ray (lane = sample), 16 rays per 1024-thread block. The prefilter lookup reads the
// compact channel-24 copy of pbw (4 B per voxel, k_prep): the 8 corners of a sample share lines
// and the whole array stays L2-resident. Per-chunk argmin keys are reduced inside the block first
// (one atomic per chunk present in the block instead of one per ray).
__global__ __launch_bounds__(1024) void k_frontend(FrontArgs a) {
  __shared__ uint64_t skey[16];
  __shared__ int schunk[16];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int ray = blockIdx.x * 16 + w;
  const bool live = ray < a.n_rays;
  uint64_t key = ~0ull;
  if (live) {
    float z, dist, pts[3], pose[3];
    sample_point(a.ray_o, a.ray_d, a.near_, a.far_, a.t_rand, ray, lane, 64, z, dist, pts);
    world_to_pose(pts, a.R, a.Th, pose);
    float lo[3], hi[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = a.pbounds[c]; hi[c] = a.pbounds[3 + c]; }
    TriCell cell;
    tri_cell(pose, lo, hi, a.X, a.Y, a.Z, cell);
    const float pn = a.pn24 ? tri_channel(a.pn24, 1, 0, cell) : tri_channel(a.pbw, 25, 24, cell);
    // novel-view filter (tpose_renderer_mmsk.py:14-57): world point -> every training view, rounded
    // half-to-even, clamped, looked up in its mask; the network then sees only visible samples, so
    // the per-chunk argmin runs over them (a chunk with none keeps nothing)
    const bool vis = visible_in_views(pts, a.n_views, a.Ks, a.RT, a.msks, a.img_h, a.img_w);
    const bool keep = vis && pn < a.norm_th;
    const uint64_t m = __ballot(keep);
    if (lane == 0) a.mask[ray] = m;
    if (a.raw != nullptr && !keep) a.raw[(size_t)ray * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    // per-chunk argmin of pnorm over the visible samples (first index on ties):
    // key = bits(pn) << 32 | index-in-chunk
    const int rc = (ray + a.ray_offset) % a.chunk;
    key = vis ? (((uint64_t)__float_as_uint(pn) << 32) | (uint32_t)(rc * 64 + lane)) : ~0ull;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t o = __shfl_xor(key, off);
      key = o < key ? o : key;
    }
  }
  if (lane == 0) {
    skey[w] = key;
    schunk[w] = live ? ray / a.chunk : -1;
  }
  __syncthreads();
  // one thread per run of equal chunk ids: min over the run, one atomic
  if (threadIdx.x < 16) {
    const int c = schunk[threadIdx.x];
    if (c >= 0 && (threadIdx.x == 0 || schunk[threadIdx.x - 1] != c)) {
      uint64_t k = skey[threadIdx.x];
      for (int j = threadIdx.x + 1; j < 16 && schunk[j] == c; ++j) k = skey[j] < k ? skey[j] : k;
      if (k != ~0ull) atomicMin((unsigned long long*)&a.chunk_min[c], (unsigned long long)k);
    }
  }
}

// (f) mesh path: the prefilter of get_alpha over free points (tpose_nerf_network.py:105-116):
// pnorm < norm_th (0.1 there) plus the argmin of pnorm over each batchify chunk
// (aninerf_mesh_renderer.py:14-23, 2048 x 64 points). One wave per 64 consecutive points, so the
// keep ballots, per-chunk argmin keys and ordered compaction are the render path's, unchanged.
__global__ __launch_bounds__(256) void k_frontend_pts(FrontArgs a) {
  const int lane = threadIdx.x & 63;
  const int grp = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (grp >= a.n_rays) return;
  const long i = (long)grp * 64 + lane;
  const bool valid = i < a.n_pts;
  float pn = 0.0f;
  if (valid) {
    float pose[3], lo[3], hi[3];
    world_to_pose_pt(a.wpts, i, a.n_pts, a.chunk_pts, a.R, a.Th, pose);
#pragma unroll
    for (int c = 0; c < 3; ++c) { lo[c] = a.pbounds[c]; hi[c] = a.pbounds[3 + c]; }
    TriCell cell;
    tri_cell(pose, lo, hi, a.X, a.Y, a.Z, cell);
    pn = tri_channel(a.pbw, 25, 24, cell);
  }
  const bool keep = valid && pn < a.norm_th;
  const uint64_t m = __ballot(keep);
  if (lane == 0) a.mask[grp] = m;
  if (a.raw != nullptr && !keep) a.raw[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int rc = grp % a.chunk;
  uint64_t key = valid ? (((uint64_t)__float_as_uint(pn) << 32) | (uint32_t)(rc * 64 + lane)) : ~0ull;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(key, off);
    key = o < key ? o : key;
  }
  if (lane == 0) atomicMin((unsigned long long*)&a.chunk_min[grp / a.chunk], (unsigned long long)key);
}

// ------------------------------------------------------------------------------------------
// ordered compaction of kept samples: count (+ forced argmin bit), scan, write
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_count(CompactArgs a) {
  __shared__ int sh[4];
  const int ray = blockIdx.x * 256 + threadIdx.x;
  int cnt = 0;
  if (ray < a.n_rays) {
    uint64_t m = a.mask[ray];
    const int c = ray / a.chunk;
    const uint64_t key = a.chunk_min[c];
    const uint32_t idx = (uint32_t)(key & 0xffffffffu);
    if ((int)(idx >> 6) == (ray + a.ray_offset) % a.chunk) m |= 1ull << (idx & 63);
    a.mask[ray] = m;
    cnt = __popcll(m);
  }
  int total;
  const int ex = block_excl_scan_256(cnt, sh, total);
  if (ray < a.n_rays) a.ray_off[ray] = ex;
  if (threadIdx.x == 0) a.block_sum[blockIdx.x] = total;
}

// single-block scan of block sums (any count), writes exclusive offsets in place and the total
__global__ __launch_bounds__(1024) void k_scan_blocks(int* __restrict__ sums, int nb, int* __restrict__ total_out) {
  __shared__ int sh[16];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + threadIdx.x;
    const int v = i < nb ? sums[i] : 0;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int pre = 0;
    for (int k = 0; k < w; ++k) pre += sh[k];
    int tot = 0;
    for (int k = 0; k < 16; ++k) tot += sh[k];
    if (i < nb) sums[i] = carry + pre + x - v;
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total_out = carry;
}

// wave per ray: global exclusive offset, then kept lanes write their point id in order
__global__ __launch_bounds__(256) void k_compact(CompactArgs a) {
  const int lane = threadIdx.x & 63;
  const int ray = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= a.n_rays) return;
  const uint64_t m = a.mask[ray];
  const int off = a.block_sum[ray / 256] + a.ray_off[ray];
  if ((m >> lane) & 1ull) {
    const int pos = off + __popcll(m & ((1ull << lane) - 1ull));
    a.list[pos] = ray * 64 + lane;
  }
  // ray_off[ray] is read and rewritten only by this wave: local offset -> global offset
  if (lane == 0) a.ray_off[ray] = off;
  if (ray == a.n_rays - 1 && lane == 0) a.ray_off[a.n_rays] = off + __popcll(m);
}

// R <= 1024: the three passes above in one workgroup (a ray per thread for the count and the scan, then
// a wave per ray for the ordered writes, as k_compact); same mask, ray_off (global, with ray_off[R] =
// the total), list and total as k_count + k_scan_blocks + k_compact
__global__ __launch_bounds__(1024) void k_compact1(CompactArgs a, int* __restrict__ total_out) {
  __shared__ int sh[16];
  __shared__ uint64_t sm[1024];
  __shared__ int so[1024];
  const int ray = threadIdx.x;
  const int lane = ray & 63, w = ray >> 6;
  uint64_t m = 0;
  if (ray < a.n_rays) {
    m = a.mask[ray];
    const uint64_t key = a.chunk_min[ray / a.chunk];
    const uint32_t idx = (uint32_t)(key & 0xffffffffu);
    if ((int)(idx >> 6) == (ray + a.ray_offset) % a.chunk) m |= 1ull << (idx & 63);
    a.mask[ray] = m;
  }
  const int cnt = __popcll(m);
  int x = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int v = sh[k];
    pre += k < w ? v : 0;
    tot += v;
  }
  const int off = pre + x - cnt;
  sm[ray] = m;
  so[ray] = off;
  if (ray < a.n_rays) a.ray_off[ray] = off;
  if (ray == 0) {
    a.ray_off[a.n_rays] = tot;
    *total_out = tot;
  }
  __syncthreads();
  for (int r = w; r < a.n_rays; r += 16) {
    const uint64_t mr = sm[r];
    if ((mr >> lane) & 1ull) a.list[so[r] + __popcll(mr & ((1ull << lane) - 1ull))] = r * 64 + lane;
  }
}

// ------------------------------------------------------------------------------------------
// alpha_ind (tpose_nerf_network.py:186-196): sigma' > train_th, plus per-chunk argmax(sigma')
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ordered_bits(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// grid (nchunks, splits); each block reduces a slice of the chunk's compact range
__global__ __launch_bounds__(256) void k_chunk_argmax(AlphaArgs a) {
  const int c = blockIdx.x;
  const int r0 = c * a.chunk;
  const int r1 = min(a.n_rays, r0 + a.chunk);
  const int s0 = a.ray_off[r0], s1 = a.ray_off[r1];
  uint64_t best = 0;
  for (int i = s0 + blockIdx.y * 256 + threadIdx.x; i < s1; i += gridDim.y * 256) {
    const int pid = a.list[i];
    const uint32_t g = (uint32_t)((((pid >> 6) + a.ray_offset) % a.chunk) * 64 + (pid & 63));
    const uint64_t key = ((uint64_t)ordered_bits(a.sigma[i]) << 32) | (uint32_t)(~g);
    best = key > best ? key : best;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(best, off);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & 63) == 0 && best != 0) atomicMax((unsigned long long*)&a.chunk_max[c], (unsigned long long)best);
}

// flags -> per-block counts (1024 items per block)
__global__ __launch_bounds__(256) void k_flag_count(AlphaArgs a) {
  __shared__ int sh[4];
  const int n = *a.n_kept;
  int cnt = 0;
  for (int k = 0; k < 4; ++k) {
    const int i = blockIdx.x * 1024 + k * 256 + threadIdx.x;
    if (i < n) {
      bool f = a.sigma[i] > a.train_th;
      a.flags[i] = f ? 1 : 0;
      cnt += f;
    }
  }
  int total;
  block_excl_scan_256(cnt, sh, total);
  if (threadIdx.x == 0) a.block_sum[blockIdx.x] = total;
}

// forced argmax rows: one thread per chunk, fixes flag + block count
__global__ void k_flag_force(AlphaArgs a, int nchunks) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const uint64_t key = a.chunk_max[c];
  const int r0 = c * a.chunk;
  const int r1 = min(a.n_rays, r0 + a.chunk);
  const int s0 = a.ray_off[r0], s1 = a.ray_off[r1];
  if (s1 <= s0 || key == 0) return;
  // the winning sample's index within the chunk -> this call's ray (another rank's under a ray split)
  const uint32_t g = ~(uint32_t)(key & 0xffffffffu);
  const int ray = r0 + (int)(g >> 6) - (r0 + a.ray_offset) % a.chunk;
  if (ray < r0 || ray >= r1) return;
  const int lane = (int)(g & 63u);
  const uint64_t m = a.mask[ray];
  if (!((m >> lane) & 1ull)) return;
  const int i = a.ray_off[ray] + __popcll(m & ((1ull << lane) - 1ull));
  if (a.flags[i] == 0) {
    a.flags[i] = 1;
    atomicAdd(&a.block_sum[i / 1024], 1);
  }
}

__global__ __launch_bounds__(256) void k_flag_scatter(AlphaArgs a) {
  __shared__ int sh[4];
  const int n = *a.n_kept;
  int base = a.block_sum[blockIdx.x];
  for (int k = 0; k < 4; ++k) {
    const int i = blockIdx.x * 1024 + k * 256 + threadIdx.x;
    const int f = (i < n) ? a.flags[i] : 0;
    int total;
    const int ex = block_excl_scan_256(f, sh, total);
    if (i < n) a.out_row[i] = f ? base + ex : -1;
    base += total;
  }
}

// one chunk of <= 64 blocks of 1024 compact samples (a training batch): k_chunk_argmax + k_flag_count +
// k_flag_force + k_scan_blocks + k_flag_scatter as two launches. Count: each block counts its
// sigma' > train_th and folds its argmax key into chunk_max[0]. Scatter: each block takes its base from
// the earlier blocks' counts (<= 63 loads), decodes the chunk's argmax sample as k_flag_force and adds
// it where it was not flagged already; the last block writes the total (counts[1]).
__global__ __launch_bounds__(256) void k_alpha_count1(AlphaArgs a) {
  __shared__ int sh[4];
  const int n = *a.n_kept;
  int cnt = 0;
  uint64_t best = 0;
  for (int k = 0; k < 4; ++k) {
    const int i = blockIdx.x * 1024 + k * 256 + threadIdx.x;
    if (i < n) {
      const float sg = a.sigma[i];
      cnt += sg > a.train_th;
      const int pid = a.list[i];
      const uint32_t g = (uint32_t)((((pid >> 6) + a.ray_offset) % a.chunk) * 64 + (pid & 63));
      const uint64_t key = ((uint64_t)ordered_bits(sg) << 32) | (uint32_t)(~g);
      best = key > best ? key : best;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(best, off);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & 63) == 0 && best != 0) atomicMax((unsigned long long*)&a.chunk_max[0], (unsigned long long)best);
  int total;
  block_excl_scan_256(cnt, sh, total);
  if (threadIdx.x == 0) a.block_sum[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_alpha_scatter1(AlphaArgs a, int* __restrict__ total_out) {
  __shared__ int sh[4];
  __shared__ int s_base, s_force;
  const int n = *a.n_kept;
  if (threadIdx.x < 64) {  // wave 0: the earlier blocks' counts, and the forced sample
    int v = (int)threadIdx.x < (int)blockIdx.x ? a.block_sum[threadIdx.x] : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (threadIdx.x == 0) {
      int i_f = -1;
      const uint64_t key = a.chunk_max[0];
      const int r1 = min(a.n_rays, a.chunk);
      if (key != 0 && a.ray_off[r1] > a.ray_off[0]) {
        const uint32_t g = ~(uint32_t)(key & 0xffffffffu);
        const int ray = (int)(g >> 6) - a.ray_offset % a.chunk;
        if (ray >= 0 && ray < r1) {
          const int lane = (int)(g & 63u);
          const uint64_t m = a.mask[ray];
          if ((m >> lane) & 1ull) i_f = a.ray_off[ray] + __popcll(m & ((1ull << lane) - 1ull));
        }
      }
      if (i_f >= 0 && a.sigma[i_f] > a.train_th) i_f = -1;  // flagged anyway
      s_force = i_f;
      s_base = v + (i_f >= 0 && i_f < (int)blockIdx.x * 1024 ? 1 : 0);
    }
  }
  __syncthreads();
  int base = s_base;
  const int i_f = s_force;
  for (int k = 0; k < 4; ++k) {
    const int i = blockIdx.x * 1024 + k * 256 + threadIdx.x;
    const int f = i < n ? (a.sigma[i] > a.train_th || i == i_f) : 0;
    int total;
    const int ex = block_excl_scan_256(f, sh, total);
    if (i < n) a.out_row[i] = f ? base + ex : -1;
    base += total;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *total_out = base;
}

__global__ __launch_bounds__(256) void k_gather_rows(const int* __restrict__ out_row, const int* __restrict__ n_kept,
                                                     const float4* __restrict__ pbw_rows, const float4* __restrict__ tbw_rows,
                                                     float4* __restrict__ pbw, float4* __restrict__ tbw) {
  // 6 float4 per 24-float row; thread per float4
  const int n = *n_kept;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int i = e / 6, j = e - i * 6;
  if (i >= n) return;
  const int r = out_row[i];
  if (r < 0) return;
  pbw[(size_t)r * 6 + j] = pbw_rows[(size_t)i * 6 + j];
  tbw[(size_t)r * 6 + j] = tbw_rows[(size_t)i * 6 + j];
}

// pts_sample_blend_weights of free points (anr_sample_volume): thread per (point, channel), out (C, n)
__global__ __launch_bounds__(256) void k_sample_volume(const float* __restrict__ vol, int X, int Y, int Z, int C,
                                                       const float* __restrict__ bounds, const float* __restrict__ pts,
                                                       int n, float* __restrict__ out) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)n * C) return;
  const int i = (int)(e / C), ch = (int)(e - (long)i * C);
  const float p[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
  const float lo[3] = {bounds[0], bounds[1], bounds[2]}, hi[3] = {bounds[3], bounds[4], bounds[5]};
  TriCell t;
  tri_cell(p, lo, hi, X, Y, Z, t);
  out[(size_t)ch * n + i] = tri_channel(vol, C, ch, t);
}

// sample id (ray * 64 + sample) of every alpha_ind output row: the row order of k_gather_rows
__global__ __launch_bounds__(256) void k_row_ids(const int* __restrict__ out_row, const int* __restrict__ n_kept,
                                                 const int* __restrict__ list, int* __restrict__ ids) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= *n_kept) return;
  const int r = out_row[i];
  if (r >= 0) ids[r] = list[i];
}

// ------------------------------------------------------------------------------------------
// A12 compositing: wave per ray; exclusive product scan of (1 - alpha + 1e-10) across lanes
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_composite(CompositeArgs a) {
  const int lane = threadIdx.x & 63;
  const int ray = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= a.n_rays) return;
  const float4 r = a.raw[(size_t)ray * 64 + lane];
  const float nr = a.near_[ray], fr = a.far_[ray];
  const float* trow = a.t_rand ? a.t_rand + (size_t)ray * 64 : nullptr;
  const float z = z_sample(nr, fr, trow, lane, 64);
  const float p = (1.0f - r.w) + 1e-10f;
  float incl = p;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float y = __shfl_up(incl, off);
    if (lane >= off) incl = incl * y;
  }
  float T = __shfl_up(incl, 1);
  if (lane == 0) T = 1.0f;
  const float w = r.w * T;
  float s0 = w * r.x, s1 = w * r.y, s2 = w * r.z, sd = w * z, sa = w;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off);
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
    sd += __shfl_xor(sd, off);
    sa += __shfl_xor(sa, off);
  }
  if (a.weights) a.weights[(size_t)ray * 64 + lane] = w;
  if (lane == 0) {
    a.rgb[3 * ray] = s0;
    a.rgb[3 * ray + 1] = s1;
    a.rgb[3 * ray + 2] = s2;
    a.depth[ray] = sd;
    a.acc[ray] = sa;
  }
}

}  // namespace anr
