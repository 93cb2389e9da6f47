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
#include "anr_common.h"
#include "anr_kernels.h"

#pragma clang fp contract(off)

namespace anr {

// ------------------------------------------------------------------------------------------
// A14 near/far, fp64, numpy operation order; eps 1e-6, padding 0.01; hit <=> exactly 2 planes.
// ------------------------------------------------------------------------------------------
__global__ void k_near_far(const float* __restrict__ ray_o, const float* __restrict__ ray_d, int n,
                           const float* __restrict__ bounds, uint8_t* __restrict__ mask,
                           float* __restrict__ near_, float* __restrict__ far_) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double b[2][3];
  for (int c = 0; c < 3; ++c) {
    b[0][c] = (double)bounds[c] + (-0.01);
    b[1][c] = (double)bounds[3 + c] + 0.01;
  }
  const double o[3] = {(double)ray_o[3 * i], (double)ray_o[3 * i + 1], (double)ray_o[3 * i + 2]};
  const double d[3] = {(double)ray_d[3 * i], (double)ray_d[3 * i + 1], (double)ray_d[3 * i + 2]};
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
  const bool hit = hits == 2;
  mask[i] = hit ? 1 : 0;
  // np.linalg.norm(axis=1): sqrt((x0*x0 + x1*x1) + x2*x2); ray_d is float32 in the test split,
  // so |d| is evaluated in float32 and promoted at the division (if_nerf_data_utils.py:189-191)
  const float df[3] = {ray_d[3 * i], ray_d[3 * i + 1], ray_d[3 * i + 2]};
  const double nd = (double)sqrtf((df[0] * df[0] + df[1] * df[1]) + df[2] * df[2]);
  double dd[2];
  for (int h = 0; h < 2; ++h) {
    const double e0 = pin[h][0] - o[0], e1 = pin[h][1] - o[1], e2 = pin[h][2] - o[2];
    dd[h] = sqrt((e0 * e0 + e1 * e1) + e2 * e2) / nd;
  }
  near_[i] = (float)fmin(dd[0], dd[1]);
  far_[i] = (float)fmax(dd[0], dd[1]);
}

// ------------------------------------------------------------------------------------------
// A4-A6 front-end: one wave per ray, lane = sample.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_frontend(FrontArgs a) {
  const int lane = threadIdx.x & 63;
  const int ray = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= a.n_rays) return;
  float z, dist, pts[3], pose[3];
  sample_point(a.ray_o, a.ray_d, a.near_, a.far_, a.t_rand, ray, lane, 64, z, dist, pts);
  world_to_pose(pts, a.R, a.Th, pose);
  float lo[3], hi[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) { lo[c] = a.pbounds[c]; hi[c] = a.pbounds[3 + c]; }
  TriCell cell;
  tri_cell(pose, lo, hi, a.X, a.Y, a.Z, cell);
  const float pn = tri_channel(a.pbw, 25, 24, cell);
  const bool keep = pn < a.norm_th;
  const uint64_t m = __ballot(keep);
  if (lane == 0) a.mask[ray] = m;
  if (a.raw != nullptr && !keep) a.raw[(size_t)ray * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  // per-chunk argmin of pnorm (first index on ties): key = bits(pn) << 32 | index-in-chunk
  const int rc = ray % a.chunk;
  uint64_t key = ((uint64_t)__float_as_uint(pn) << 32) | (uint32_t)(rc * 64 + lane);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(key, off);
    key = o < key ? o : key;
  }
  if (lane == 0) atomicMin((unsigned long long*)&a.chunk_min[ray / a.chunk], (unsigned long long)key);
}

// ------------------------------------------------------------------------------------------
// ordered compaction of kept samples: count (+ forced argmin bit), scan, write
// ------------------------------------------------------------------------------------------
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

__global__ __launch_bounds__(256) void k_count(CompactArgs a) {
  __shared__ int sh[4];
  const int ray = blockIdx.x * 256 + threadIdx.x;
  int cnt = 0;
  if (ray < a.n_rays) {
    uint64_t m = a.mask[ray];
    const int c = ray / a.chunk;
    const uint64_t key = a.chunk_min[c];
    const uint32_t idx = (uint32_t)(key & 0xffffffffu);
    if ((int)(idx >> 6) == ray % a.chunk) m |= 1ull << (idx & 63);
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
    const uint64_t key = ((uint64_t)ordered_bits(a.sigma[i]) << 32) | (uint32_t)(~(uint32_t)(i - s0));
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
  const int s0 = a.ray_off[r0], s1 = a.ray_off[min(a.n_rays, r0 + a.chunk)];
  if (s1 <= s0) return;
  const int i = s0 + (int)(~(uint32_t)(key & 0xffffffffu));
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
