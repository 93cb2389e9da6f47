// anr_train.hip — per-sample kernels of the training executor (A16/A17, configs 3/4).
//
// Forward: the exact front-end of the render path selects and compacts the kept samples
// (tpose_nerf_network.py:143-157); then, per compact sample, point prep -> BW MLP (GEMMs) ->
// softmax + LBS -> BW MLP on the T-pose -> NeRF MLP (GEMMs) -> raw; every activation is kept in
// HBM for the backward (training batches are 1,024 rays: ~24k kept samples, ~28 KB each).
// Backward: compositing (wave per ray, suffix scan), raw activations, heads and MLP layers
// (GEMMs, anr_gemm.hip), gamma and grid_sample input gradients, LBS (3x3 inverse) and softmax,
// latent-row gradients from column sums; Adam (torch.optim.Adam semantics) + clip_grad_value_.
#include "anr_common.h"
#include "anr_train.h"

#pragma clang fp contract(off)

namespace anr {

// fp32 -> bf16, round to nearest even (the rounding every bf16 consumer applies)
__device__ __forceinline__ unsigned short f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

// ------------------------------------------------------------------------------------------
// forward point kernels
// ------------------------------------------------------------------------------------------
// one wave per kept sample: lane f -> gamma(pose)_f, init_pbw_f (f<24), gamma(dir)_f (f<27)
__device__ __forceinline__ void point_prep_one(const TrainBufs& b, int i, int lane) {
  const int pid = b.list[i];
  float dist, pose[3], dir[3];
  if (b.dists) {  // free samples (Network.forward)
    world_to_pose_pt(b.wpts, pid, b.n_pts, (int)b.n_pts, b.R, b.Th, pose);
    dist = b.dists[pid];
    for (int c = 0; c < 3; ++c) dir[c] = b.vdir[3 * (long)pid + c];
  } else {
    const int ray = pid >> 6, s = pid & 63;
    float z, pts[3];
    sample_point(b.ray_o, b.ray_d, b.near_, b.far_, b.t_rand, ray, s, 64, z, dist, pts);
    world_to_pose(pts, b.R, b.Th, pose);
    for (int c = 0; c < 3; ++c) dir[c] = b.ray_d[3 * ray + c];
  }
  const float gp = lane < 63 ? embed_feature(pose, lane, 10) : 0.f;
  if (b.hbp) ((unsigned short*)b.Gp)[(long)i * 64 + lane] = f2bf(gp);
  else b.Gp[(long)i * 64 + lane] = gp;
  if (lane < 32) {
    float lo[3], hi[3];
    for (int c = 0; c < 3; ++c) { lo[c] = b.pbounds[c]; hi[c] = b.pbounds[3 + c]; }
    TriCell cell;
    tri_cell(pose, lo, hi, b.pX, b.pY, b.pZ, cell);
    b.Ip[(long)i * 32 + lane] = lane < 24 ? tri_channel(b.pbw, 25, lane, cell) : 0.f;
    const float gv = lane < 27 ? embed_feature(dir, lane, 4) : 0.f;
    if (b.hb) ((unsigned short*)b.Gv)[(long)i * 64 + lane] = f2bf(gv);  // rows of 64 (the row GEMM's K chunk)
    else b.Gv[(long)i * 32 + lane] = gv;
  }
  if (lane == 0) {
    float* p = b.pt + (long)i * 8;
    p[0] = pose[0]; p[1] = pose[1]; p[2] = pose[2]; p[3] = dist;
  }
}

// one wave per sample over a capacity-sized grid (a grid-stride loop over a capped grid ran 38 instead
// of ~29 us: the per-sample work is latency-bound and wants every wave in flight at once)
__global__ __launch_bounds__(256) void k_tr_point_prep(TrainBufs b) {
  if (blockIdx.x == 0 && b.zero4) {
    if (threadIdx.x < 4) b.zero4[threadIdx.x] = 0.f;
    for (int k = threadIdx.x; k < 2048; k += 256) b.zero2048[k] = 0.f;
  }
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i < *b.n_kept) point_prep_one(b, i, lane);
}

__device__ __forceinline__ void softmax24(const float* __restrict__ logits, const float* __restrict__ init, float* out) {
#pragma clang fp contract(fast)
  float l[24];
  float m = -INFINITY;
  for (int j = 0; j < 24; ++j) {
    l[j] = logf(init[j] + 1e-9f) + logits[j];
    m = fmaxf(m, l[j]);
  }
  float s = 0.f;
  for (int j = 0; j < 24; ++j) {
    l[j] = expf(l[j] - m);
    s += l[j];
  }
  for (int j = 0; j < 24; ++j) out[j] = l[j] / s;
}

// sums / max over the 64 lanes of a wave, or over the 32 lanes of a half-wave (every lane gets it)
__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float half_sum(float v) {
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// one wave per sample: pbw softmax (lane = joint), LBS to the T-pose, gamma(x_T) (lane = feature),
// init_tbw (lane = channel); every row written by consecutive lanes
__device__ __forceinline__ void softmax_lbs_one(const TrainBufs& b, int i, int lane) {
#pragma clang fp contract(fast)
  // softmax(log(init + 1e-9) + logits) over the 24 joints
  const float l = lane < 24 ? logf(b.Ip[(long)i * 32 + lane] + 1e-9f) + b.Lp[(long)i * 32 + lane] : -INFINITY;
  const float m = wave_max(l);
  const float ex = lane < 24 ? expf(l - m) : 0.f;
  const float bw = ex / wave_sum(ex);
  if (lane < 24) b.Bp[(long)i * 24 + lane] = bw;
  // blended transform sum_j bw_j A_j: lane q < 16 accumulates entry q
  float ab = 0.f;
  for (int j = 0; j < 24; ++j) ab += __shfl(bw, j) * b.A[j * 16 + (lane & 15)];
  float Ab[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) Ab[q] = __shfl(ab, q);
  const float a = Ab[0], bb = Ab[1], c = Ab[2], d = Ab[4], e = Ab[5], f = Ab[6], g = Ab[8], h = Ab[9], k = Ab[10];
  const float c00 = e * k - f * h, c01 = c * h - bb * k, c02 = bb * f - c * e;
  const float c10 = f * g - d * k, c11 = a * k - c * g, c12 = c * d - a * f;
  const float c20 = d * h - e * g, c21 = bb * g - a * h, c22 = a * e - bb * d;
  const float rd = 1.0f / (a * c00 + bb * c10 + c * c20);
  const float Ri[9] = {c00 * rd, c01 * rd, c02 * rd, c10 * rd, c11 * rd, c12 * rd, c20 * rd, c21 * rd, c22 * rd};
  float* pt = b.pt + (long)i * 8;
  const float y[3] = {pt[0] - Ab[3], pt[1] - Ab[7], pt[2] - Ab[11]};
  float tp[3];
  for (int r = 0; r < 3; ++r) tp[r] = Ri[3 * r] * y[0] + Ri[3 * r + 1] * y[1] + Ri[3 * r + 2] * y[2];
  if (lane == 0) {
    float* L = b.lbs + (long)i * 16;
    for (int q = 0; q < 9; ++q) L[q] = Ri[q];
    L[9] = y[0]; L[10] = y[1]; L[11] = y[2];
    bool inside = true;
    for (int r = 0; r < 3; ++r) inside = inside && tp[r] > b.tbounds[r] && tp[r] < b.tbounds[3 + r];
    pt[4] = tp[0]; pt[5] = tp[1]; pt[6] = tp[2]; pt[7] = inside ? 1.f : 0.f;
  }
  const float gt = lane < 63 ? embed_feature(tp, lane, 10) : 0.f;
  if (b.hb) ((unsigned short*)b.Gt)[(long)i * 64 + lane] = f2bf(gt);
  else b.Gt[(long)i * 64 + lane] = gt;
  if (lane < 32) {
    float lo[3], hi[3];
    for (int r = 0; r < 3; ++r) { lo[r] = b.tbounds[r]; hi[r] = b.tbounds[3 + r]; }
    TriCell cell;
    tri_cell(tp, lo, hi, b.tX, b.tY, b.tZ, cell);
    b.It[(long)i * 32 + lane] = lane < 24 ? tri_channel(b.tbw, 25, lane, cell) : 0.f;
  }
}

__global__ __launch_bounds__(256) void k_tr_softmax_lbs(TrainBufs b) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i < *b.n_kept) softmax_lbs_one(b, i, lane);
}

// free points (Network.calculate_neural_blend_weights / TPoseHuman.calculate_alpha): one wave per
// point, lane f -> gamma(x)_f (embedder.py:5-54), init row f < 24 from the reference's (24, n) layout
__global__ __launch_bounds__(256) void k_pt_prep(const float* __restrict__ pts, const float* __restrict__ smpl_bw, int n,
                                                 float* G, float* I) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const float x[3] = {pts[3 * (long)i], pts[3 * (long)i + 1], pts[3 * (long)i + 2]};
  G[(long)i * 64 + lane] = lane < 63 ? embed_feature(x, lane, 10) : 0.f;
  if (I && lane < 32) I[(long)i * 32 + lane] = lane < 24 ? smpl_bw[(long)lane * n + i] : 0.f;
}

__global__ __launch_bounds__(256) void k_pt_softmax_out(const float* __restrict__ logits, const float* __restrict__ I,
                                                        int n, float* bw_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float bw[24];
  softmax24(logits + (long)i * 32, I + (long)i * 32, bw);
  for (int j = 0; j < 24; ++j) bw_out[(long)j * n + i] = bw[j];
}

// the latent columns of layers 0 (191 inputs) and 5 (447) times table[row (+ add)], plus the bias:
// the per-call constant part of get_bw_feature's [gamma(x), latent] input (tpose_nerf_network.py:40-53)
__global__ __launch_bounds__(256) void k_fold_latent(FoldArgs a) {
  const int row = (int)a.row[0] + a.add;
  const float* lat = a.table + (size_t)row * 128;
  for (int k = threadIdx.x; k < 512; k += blockDim.x) {
    const int which = k >> 8, nn = k & 255;
    const float* W = which ? a.w5 : a.w0;
    const int ld = which ? 447 : 191;
    float acc = (which ? a.b5 : a.b0)[nn];
    for (int q = 0; q < 128; ++q) acc = fmaf(W[(size_t)nn * ld + 63 + q], lat[q], acc);
    a.fold[k] = acc;
  }
}

__global__ __launch_bounds__(256) void k_tr_softmax_t(TrainBufs b) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *b.n_kept;
  if (i >= n) return;
  float bw[24];
  softmax24(b.Lt + (long)i * 32, b.It + (long)i * 32, bw);
  for (int j = 0; j < 24; ++j) b.Bt[(long)i * 24 + j] = bw[j];
}

// sigma' (T-pose bbox mask), raw = (sigmoid(rgb), 1 - exp(-relu(sigma') dist)) at the sample id
__global__ __launch_bounds__(256) void k_tr_raw(TrainBufs b) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *b.n_kept;
  if (i >= n) return;
  const float* pt = b.pt + (long)i * 8;
  const float sig = pt[7] > 0.f ? b.Alpha[i] : 0.f;
  const float* l = b.Rgbl + (long)i * 4;
  float4 r;
  r.x = 1.0f / (1.0f + expf(-l[0]));
  r.y = 1.0f / (1.0f + expf(-l[1]));
  r.z = 1.0f / (1.0f + expf(-l[2]));
  r.w = 1.0f - expf(-fmaxf(sig, 0.f) * pt[3]);
  b.raw[b.list[i]] = r;
  b.sigma[i] = sig;
}

// ------------------------------------------------------------------------------------------
// losses (tpose_trainer.py:50-63): img MSE over mask_at_box rays, smooth-L1(pbw rows, tbw rows)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tr_loss(TrainBufs b, const float* rgb_gt, const uint8_t* mask, float* acc3) {
  __shared__ float sh[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float v0 = 0.f, v1 = 0.f;
  if (blockIdx.y == 0) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r < b.n_rays && (mask == nullptr || mask[r])) {
      for (int c = 0; c < 3; ++c) {
        const float d = b.rgb_map[3 * r + c] - rgb_gt[3 * r + c];
        v0 += d * d;
      }
      v1 = 1.f;
    }
  } else {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < *b.n_kept && b.out_row[i] >= 0)
      for (int c = 0; c < 24; ++c) {
        const float x = b.Bp[(long)i * 24 + c] - b.Bt[(long)i * 24 + c];
        const float ax = fabsf(x);
        v0 += ax < 1.f ? 0.5f * x * x : ax - 0.5f;
      }
  }
  for (int off = 32; off > 0; off >>= 1) {
    v0 += __shfl_xor(v0, off);
    v1 += __shfl_xor(v1, off);
  }
  if (lane == 0) { sh[0][w] = v0; sh[1][w] = v1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float s0 = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
    const float s1 = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
    if (blockIdx.y == 0) {
      atomicAdd(acc3 + 0, s0);
      atomicAdd(acc3 + 1, s1);
    } else {
      atomicAdd(acc3 + 2, s0);
      if (blockIdx.x == 0) acc3[3] = (float)*b.m_rows;  // the rows count beside the sums (a ray split sums all four)
    }
  }
}

// acc3 = {sum sq. error, mask rays, sum smooth-L1, alpha_ind rows} (summed over the ranks of a ray split)
__device__ __forceinline__ void loss_final(const float* acc3, float* loss3) {
  const float img = acc3[0] / (3.0f * acc3[1]);
  const float bw = acc3[2] / (24.0f * acc3[3]);
  loss3[0] = bw + img;
  loss3[1] = img;
  loss3[2] = bw;
}
__global__ void k_tr_loss_final(const float* acc3, const int* m_rows, float* loss3) {
  (void)m_rows;
  loss_final(acc3, loss3);
}

// upstream gradients of the fused loss: d rgb_map (R,3), d pbw / d tbw rows (m,24)
__global__ __launch_bounds__(256) void k_tr_loss_grads(TrainBufs b, const float* rgb_gt, const uint8_t* mask,
                                                       const float* acc3, float* d_rgb, float* d_pbw, float* d_tbw) {
  if (b.loss3_out && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) loss_final(acc3, b.loss3_out);
  if (blockIdx.y == 0) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= b.n_rays) return;
    const bool on = mask == nullptr || mask[r];
    const float sc = 2.0f / (3.0f * acc3[1]);
    for (int c = 0; c < 3; ++c) d_rgb[3 * r + c] = on ? sc * (b.rgb_map[3 * r + c] - rgb_gt[3 * r + c]) : 0.f;
  } else {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= *b.n_kept) return;
    const int row = b.out_row[i];
    if (row < 0) return;
    const float sc = 1.0f / (24.0f * acc3[3]);
    for (int c = 0; c < 24; ++c) {
      const float x = b.Bp[(long)i * 24 + c] - b.Bt[(long)i * 24 + c];
      const float d = (fabsf(x) < 1.f ? x : (x > 0.f ? 1.f : -1.f)) * sc;
      d_pbw[(long)row * 24 + c] = d;
      d_tbw[(long)row * 24 + c] = -d;
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward point kernels
// ------------------------------------------------------------------------------------------
// raw2outputs backward (nerf_net_utils.py:22-26), wave per ray: w = a T, T_s = prod_{j<s}(1-a_j+1e-10)
//   dc_s = w_s g;  da_s = T_s (g.c_s) - (sum_{k>s} (g.c_k) w_k) / (1 - a_s + 1e-10)
__global__ __launch_bounds__(256) void k_tr_composite_bwd(TrainBufs b) {
#pragma clang fp contract(fast)
  const int lane = threadIdx.x & 63;
  const int ray = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= b.n_rays) return;
  const float4 r = b.raw[(long)ray * 64 + lane];
  const float p = (1.0f - r.w) + 1e-10f;
  float incl = p;
  for (int off = 1; off < 64; off <<= 1) {
    const float y = __shfl_up(incl, off);
    if (lane >= off) incl *= y;
  }
  float T = __shfl_up(incl, 1);
  if (lane == 0) T = 1.0f;
  const float w = r.w * T;
  float g0 = 0.f, g1 = 0.f, g2 = 0.f;
  if (b.d_rgb_map) {
    g0 = b.d_rgb_map[3 * ray];
    g1 = b.d_rgb_map[3 * ray + 1];
    g2 = b.d_rgb_map[3 * ray + 2];
  }
  const float e = g0 * r.x + g1 * r.y + g2 * r.z;
  float suf = e * w;  // inclusive suffix sum
  for (int off = 1; off < 64; off <<= 1) {
    const float y = __shfl_down(suf, off);
    if (lane + off < 64) suf += y;
  }
  const float S = suf - e * w;
  float4 d;
  d.x = w * g0;
  d.y = w * g1;
  d.z = w * g2;
  d.w = T * e - S / p;
  b.draw[(long)ray * 64 + lane] = d;
}

// sigmoid / alpha backward per kept sample -> d rgb logits, d sigma (alpha_fc output)
__global__ __launch_bounds__(256) void k_tr_raw_bwd(TrainBufs b) {
#pragma clang fp contract(fast)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *b.n_kept;
  if (i >= n) return;
  const float4 d = b.draw[b.list[i]];
  const float* l = b.Rgbl + (long)i * 4;
  float* o = b.dRgb + (long)i * 4;
  const float dc[3] = {d.x, d.y, d.z};
  for (int c = 0; c < 3; ++c) {
    const float s = 1.0f / (1.0f + expf(-l[c]));
    o[c] = dc[c] * s * (1.0f - s);
  }
  o[3] = 0.f;
  const float* pt = b.pt + (long)i * 8;
  const float sig = b.sigma[i], dist = pt[3];
  const float ds = sig > 0.f ? d.w * expf(-sig * dist) * dist : 0.f;
  b.dAlpha[i] = pt[7] > 0.f ? ds : 0.f;
  if (b.hb) b.dAlpha16[(long)i * 64] = f2bf(pt[7] > 0.f ? ds : 0.f);
}

// upstream pbw / tbw row gradients scattered to the compact samples (alpha_ind rows); half a wave per
// sample, lane = joint
__global__ __launch_bounds__(256) void k_tr_rows_bwd(TrainBufs b) {
  const int hl = threadIdx.x & 31;
  const int i = blockIdx.x * 8 + (threadIdx.x >> 5);
  const int n = *b.n_kept;
  if (i >= n || hl >= 24) return;
  const int row = b.out_row[i];
  b.dBp[(long)i * 24 + hl] = (row >= 0 && b.d_pbw) ? b.d_pbw[(long)row * 24 + hl] : 0.f;
  b.dBt[(long)i * 24 + hl] = (row >= 0 && b.d_tbw) ? b.d_tbw[(long)row * 24 + hl] : 0.f;
}

// softmax(log(init + 1e-9) + logits) backward (T-pose pass): d logits and d init_tbw; half a wave per
// sample, lane = joint
__global__ __launch_bounds__(256) void k_tr_softmax_bwd_t(TrainBufs b) {
#pragma clang fp contract(fast)
  const int hl = threadIdx.x & 31;
  const int i = blockIdx.x * 8 + (threadIdx.x >> 5);
  const int n = *b.n_kept;
  if (i >= n) return;
  const float B = hl < 24 ? b.Bt[(long)i * 24 + hl] : 0.f;
  const float dB = hl < 24 ? b.dBt[(long)i * 24 + hl] : 0.f;
  const float dot = half_sum(dB * B);
  const float dl = hl < 24 ? B * (dB - dot) : 0.f;
  b.dLt[(long)i * (b.ldl ? b.ldl : 32) + hl] = dl;
  b.dIt[(long)i * 32 + hl] = hl < 24 ? dl / (b.It[(long)i * 32 + hl] + 1e-9f) : 0.f;
}

__global__ __launch_bounds__(256) void k_tr_softmax_bwd_p(TrainBufs b) {
#pragma clang fp contract(fast)
  const int hl = threadIdx.x & 31;
  const int i = blockIdx.x * 8 + (threadIdx.x >> 5);
  const int n = *b.n_kept;
  if (i >= n) return;
  const float B = hl < 24 ? b.Bp[(long)i * 24 + hl] : 0.f;
  const float dB = hl < 24 ? b.dBp[(long)i * 24 + hl] : 0.f;
  const float dot = half_sum(dB * B);
  b.dLp[(long)i * (b.ldl ? b.ldl : 32) + hl] = hl < 24 ? B * (dB - dot) : 0.f;
}

// d x_T from gamma(x_T) and from the init_tbw lookup (grid_sampler_3d backward w.r.t. the grid),
// then LBS backward into d pbw (accumulated onto the row gradients already in dBp). One wave per
// sample: lane = gamma feature; lane = (corner, channel group) for the lookup; lane = joint for d pbw.
__global__ __launch_bounds__(256) void k_tr_tpose_bwd(TrainBufs b) {
#pragma clang fp contract(fast)
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = *b.n_kept;
  if (i >= n) return;
  const float* pt = b.pt + (long)i * 8;
  const float tp[3] = {pt[4], pt[5], pt[6]};
  float gc[3] = {0.f, 0.f, 0.f};
  if (lane < 63) {
    const float d = b.dGt[(long)i * 64 + lane] + (b.dGt2 ? b.dGt2[(long)i * 64 + lane] : 0.f);
    if (lane < 3) {
      gc[lane] = d;
    } else {
      const int q = lane - 3, k = q / 6, w = q - 6 * (q / 6), comp = w >= 3 ? w - 3 : w;
      const float sc = (float)(1 << k);
      const float v = tp[comp] * sc;
      gc[comp] = w < 3 ? d * sc * cosf(v) : -d * sc * sinf(v);
    }
  }
  float g[3] = {wave_sum(gc[0]), wave_sum(gc[1]), wave_sum(gc[2])};
  // grid_sample backward (align_corners, border): ATen grid_sampler_3d_backward
  {
    float lo[3], hi[3], gg[3];
    for (int c = 0; c < 3; ++c) {
      lo[c] = b.tbounds[c];
      hi[c] = b.tbounds[3 + c];
      gg[c] = ((tp[c] - lo[c]) / (hi[c] - lo[c])) * 2.0f - 1.0f;
    }
    const int sizes[3] = {b.tZ, b.tY, b.tX};  // ix <- x_T[2], iy <- x_T[1], iz <- x_T[0]
    float src[3], mult[3];
    for (int a = 0; a < 3; ++a) {
      const float raw = ((gg[2 - a] + 1.0f) / 2.0f) * (float)(sizes[a] - 1);
      const float mx = (float)(sizes[a] - 1);
      mult[a] = (raw <= 0.f || raw >= mx) ? 0.f : (float)(sizes[a] - 1) / 2.0f;
      src[a] = fminf(mx, fmaxf(raw, 0.f));
    }
    const float ix = src[0], iy = src[1], iz = src[2];
    const int x0 = (int)floorf(ix), y0 = (int)floorf(iy), z0 = (int)floorf(iz);
    const float wx[2] = {(float)(x0 + 1) - ix, ix - (float)x0};
    const float wy[2] = {(float)(y0 + 1) - iy, iy - (float)y0};
    const float wz[2] = {(float)(z0 + 1) - iz, iz - (float)z0};
    const float* dI = b.dIt + (long)i * 32;
    // lane = corner k (lane >> 3) x channel group cg (lane & 7): channels cg, cg + 8, cg + 16
    const int k = lane >> 3, cg = lane & 7;
    const int ax = k & 1, ay = (k >> 1) & 1, az = k >> 2;
    const int cx = x0 + ax, cy = y0 + ay, cz = z0 + az;
    float sv = 0.f;
    if (!(cx < 0 || cx >= b.tZ || cy < 0 || cy >= b.tY || cz < 0 || cz >= b.tX)) {
      const float* v = b.tbw + (long)((cz * b.tY + cy) * b.tZ + cx) * 25;
      sv = v[cg] * dI[cg] + v[cg + 8] * dI[cg + 8] + v[cg + 16] * dI[cg + 16];
    }
    sv += __shfl_xor(sv, 1);
    sv += __shfl_xor(sv, 2);
    sv += __shfl_xor(sv, 4);
    const float sx = ax ? 1.f : -1.f, sy = ay ? 1.f : -1.f, sz = az ? 1.f : -1.f;
    const bool own = cg == 0;
    const float gix = wave_sum(own ? sx * wy[ay] * wz[az] * sv : 0.f);
    const float giy = wave_sum(own ? wx[ax] * sy * wz[az] * sv : 0.f);
    const float giz = wave_sum(own ? wx[ax] * wy[ay] * sz * sv : 0.f);
    g[2] += gix * mult[0] * 2.0f / (hi[2] - lo[2]);
    g[1] += giy * mult[1] * 2.0f / (hi[1] - lo[1]);
    g[0] += giz * mult[2] * 2.0f / (hi[0] - lo[0]);
  }
  // LBS backward (blend_utils.py:41-59): x_T = Rinv y, y = x - t, [R|t] = sum_j bw_j A_j
  if (lane >= 24) return;
  const float* L = b.lbs + (long)i * 16;
  float dy[3];
  for (int c = 0; c < 3; ++c) dy[c] = L[0 * 3 + c] * g[0] + L[1 * 3 + c] * g[1] + L[2 * 3 + c] * g[2];
  float dAb[12];  // rows 0..2 of the 4x4 blend: dR[a][c] = -dy[a] x_T[c]; dt[a] = -dy[a]
  for (int a = 0; a < 3; ++a) {
    for (int c = 0; c < 3; ++c) dAb[4 * a + c] = -dy[a] * tp[c];
    dAb[4 * a + 3] = -dy[a];
  }
  float sum = 0.f;
  for (int q = 0; q < 12; ++q) sum += dAb[q] * b.A[lane * 16 + q];
  b.dBp[(long)i * 24 + lane] += sum;
}

// latent columns folded into the bias (row = li[0] + add when li, else add):
//   d table[row][k] += sum_n dysum[n] W[n][col0+k];  d W[n][col0+k] += dysum[n] table[row][k]
// (dysum = column sum over samples of the layer's d pre-activation)
// grid = nout + 128 blocks of 128 threads: blocks < nout update one dW row, block nout + k reduces
// the 128-wide table column k over the nout outputs
__global__ __launch_bounds__(128) void k_tr_latent_grad(const float* dysum, const float* W, int in_ch, int col0,
                                                        int nout, const float* table, const int64_t* li, int add,
                                                        float* dW, float* dtable) {
  const long row = (li ? li[0] : 0) + add;
  if ((int)blockIdx.x < nout) {
    const int k = threadIdx.x;
    const int nn = blockIdx.x;
    dW[(long)nn * in_ch + col0 + k] += dysum[nn] * table[row * 128 + k];
    return;
  }
  __shared__ float sh[2];
  const int k = blockIdx.x - nout;
  float acc = 0.f;
  for (int nn = threadIdx.x; nn < nout; nn += 128) acc += dysum[nn] * W[(long)nn * in_ch + col0 + k];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) dtable[row * 128 + k] += sh[0] + sh[1];
}

// the latent-row updates queued with one weight-gradient flush, one launch: grid (256 + 128, n), post
// blockIdx.y as k_tr_latent_grad. Posts of one launch can share outputs (the blend-weight MLP's pose and
// T-pose passes update the same dW latent columns, layers 0 and 5 the same table row), so every update
// is an atomic add (sequential launches ordered them; here they run concurrently)
__global__ __launch_bounds__(128) void k_tr_latent_grads(LatentPosts P) {
  const int q = blockIdx.y;
  const long row = (P.li[q] ? P.li[q][0] : 0) + P.add[q];
  const int nout = P.nout[q], in_ch = P.in_ch[q], col0 = P.col0[q];
  if ((int)blockIdx.x < nout) {
    const int k = threadIdx.x;
    const int nn = blockIdx.x;
    atomicAdd(P.dW[q] + (long)nn * in_ch + col0 + k, P.dysum[q][nn] * P.table[q][row * 128 + k]);
    return;
  }
  __shared__ float sh[2];
  const int k = blockIdx.x - nout;
  if (k >= 128) return;
  float acc = 0.f;
  for (int nn = threadIdx.x; nn < nout; nn += 128) acc += P.dysum[q][nn] * P.W[q][(long)nn * in_ch + col0 + k];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(P.dtable[q] + row * 128 + k, sh[0] + sh[1]);
}

// clip_grad_value_(clip) + torch.optim.Adam step (decoupled bias corrections as in torch)
__global__ __launch_bounds__(256) void k_adam(float* p, float* g, float* m, float* v, long n, float lr, float b1, float b2,
                                              float eps, float wd, float bc1, float bc2_sqrt, float clip) {
#pragma clang fp contract(fast)
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // clip_grad_value_ is torch.clamp: a NaN gradient stays NaN (fminf/fmaxf would turn it into
  // -clip and hide a diverged loss behind a full-size Adam step)
  const float g0 = g[i];
  float gi = g0 != g0 ? g0 : fminf(fmaxf(g0, -clip), clip);
  g[i] = gi;
  if (wd != 0.f) gi += wd * p[i];
  const float mi = m[i] + (1.0f - b1) * (gi - m[i]);
  const float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] -= (lr / bc1) * mi / denom;
}

// ------------------------------------------------------------------------------------------
// (f) animation stage (lib/train/trainers/aninerf_animation_trainer.py:33-140): free points, no
// compaction (every point of a path is processed; n = b.n_kept[0]), frozen network except
// novel_pose_bw. Buffers are the training executor's (TrainBufs), reused by the two paths.
// ------------------------------------------------------------------------------------------
// path 1 (observation space): world -> pose ((x - Th) R, :132-139), gamma(pose), init_pbw and pnorm
// (pt[3]); wave per point, lane = feature
__global__ __launch_bounds__(256) void k_an_prep_obs(TrainBufs b, const float* __restrict__ wpts) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = *b.n_kept;
  if (i >= n) return;
  float pose[3];
  world_to_pose_pt(wpts, i, n, n, b.R, b.Th, pose);
  const float gp = lane < 63 ? embed_feature(pose, lane, 10) : 0.f;
  if (b.hbp) ((unsigned short*)b.Gp)[(long)i * 64 + lane] = f2bf(gp);
  else b.Gp[(long)i * 64 + lane] = gp;
  if (lane < 32) {
    float lo[3], hi[3];
    for (int c = 0; c < 3; ++c) { lo[c] = b.pbounds[c]; hi[c] = b.pbounds[3 + c]; }
    TriCell cell;
    tri_cell(pose, lo, hi, b.pX, b.pY, b.pZ, cell);
    const float v = lane < 25 ? tri_channel(b.pbw, 25, lane, cell) : 0.f;
    b.Ip[(long)i * 32 + lane] = lane < 24 ? v : 0.f;
    if (lane == 24) b.pt[(long)i * 8 + 3] = v;  // pnorm
  }
  if (lane == 0) {
    float* p = b.pt + (long)i * 8;
    p[0] = pose[0]; p[1] = pose[1]; p[2] = pose[2];
  }
}

// path 2 (canonical space): x_T given; gamma(x_T), init_tbw (:82-88)
__global__ __launch_bounds__(256) void k_an_prep_can(TrainBufs b, const float* __restrict__ tpts) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = *b.n_kept;
  if (i >= n) return;
  const float tp[3] = {tpts[3 * (long)i], tpts[3 * (long)i + 1], tpts[3 * (long)i + 2]};
  b.Gt[(long)i * 64 + lane] = lane < 63 ? embed_feature(tp, lane, 10) : 0.f;
  if (lane < 32) {
    float lo[3], hi[3];
    for (int c = 0; c < 3; ++c) { lo[c] = b.tbounds[c]; hi[c] = b.tbounds[3 + c]; }
    TriCell cell;
    tri_cell(tp, lo, hi, b.tX, b.tY, b.tZ, cell);
    b.It[(long)i * 32 + lane] = lane < 24 ? tri_channel(b.tbw, 25, lane, cell) : 0.f;
  }
  if (lane == 0) {
    float* p = b.pt + (long)i * 8;
    p[4] = tp[0]; p[5] = tp[1]; p[6] = tp[2];
  }
}

// path 2: tpose_points_to_pose_points (blend_utils.py:77-90) with the frozen tbw, then gamma(pose)
// and init_pbw of the posed point
__global__ __launch_bounds__(256) void k_an_lbs_fwd(TrainBufs b) {
#pragma clang fp contract(fast)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *b.n_kept;
  if (i >= n) return;
  float Ab[16];
  for (int m = 0; m < 16; ++m) Ab[m] = 0.f;
  for (int j = 0; j < 24; ++j) {
    const float w = b.Bt[(long)i * 24 + j];
    for (int m = 0; m < 16; ++m) Ab[m] += w * b.A[j * 16 + m];
  }
  const float* pt = b.pt + (long)i * 8;
  const float tp[3] = {pt[4], pt[5], pt[6]};
  float pose[3];
  for (int r = 0; r < 3; ++r) pose[r] = (Ab[4 * r] * tp[0] + Ab[4 * r + 1] * tp[1] + Ab[4 * r + 2] * tp[2]) + Ab[4 * r + 3];
  for (int q = 0; q < 64; ++q) b.Gp[(long)i * 64 + q] = q < 63 ? embed_feature(pose, q, 10) : 0.f;
  float lo[3], hi[3];
  for (int r = 0; r < 3; ++r) { lo[r] = b.pbounds[r]; hi[r] = b.pbounds[3 + r]; }
  TriCell cell;
  tri_cell(pose, lo, hi, b.pX, b.pY, b.pZ, cell);
  for (int j = 0; j < 32; ++j) b.Ip[(long)i * 32 + j] = j < 24 ? tri_channel(b.pbw, 25, j, cell) : 0.f;
}

__global__ __launch_bounds__(256) void k_an_softmax_p(TrainBufs b) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *b.n_kept;
  if (i >= n) return;
  float bw[24];
  softmax24(b.Lp + (long)i * 32, b.Ip + (long)i * 32, bw);
  for (int j = 0; j < 24; ++j) b.Bp[(long)i * 24 + j] = bw[j];
}

// float -> order-preserving uint32
__device__ __forceinline__ uint32_t ord_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// alpha (path 1: zeroed outside the T-pose bbox or where pnorm >= norm_th, :117-124; path 2: as
// is), then the argmax key (first index on ties, torch.argmax)
__global__ __launch_bounds__(256) void k_an_select(TrainBufs b, int masked, float norm_th, unsigned long long* amax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *b.n_kept;
  unsigned long long key = 0ull;
  if (i < n) {
    float a = b.Alpha[i];
    if (masked) {
      const float* pt = b.pt + (long)i * 8;
      bool inside = true;
      for (int r = 0; r < 3; ++r) inside = inside && pt[4 + r] > b.tbounds[r] && pt[4 + r] < b.tbounds[3 + r];
      inside = inside && pt[3] < norm_th;
      a = inside ? a : 0.f;
      b.Alpha[i] = a;
    }
    key = ((unsigned long long)ord_bits(a) << 32) | (0xffffffffu - (uint32_t)i);
  }
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(key, off);
    key = o > key ? o : key;
  }
  if ((threadIdx.x & 63) == 0 && key) atomicMax(amax, key);
}

// alpha_ind = alpha > train_th plus the argmax (:126-130); smooth-L1 sum and row count (m) into acc
__global__ __launch_bounds__(256) void k_an_loss(TrainBufs b, float train_th, const unsigned long long* amax,
                                                 float* acc, int* rows) {
  __shared__ float sh[4];
  __shared__ int shc[4];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *b.n_kept;
  const int forced = (int)(0xffffffffu - (uint32_t)(*amax & 0xffffffffull));
  float v = 0.f;
  int c = 0;
  if (i < n) {
    const bool sel = b.Alpha[i] > train_th || i == forced;
    b.sigma[i] = sel ? 1.f : 0.f;
    if (sel) {
      c = 1;
      for (int j = 0; j < 24; ++j) {
        const float x = b.Bp[(long)i * 24 + j] - b.Bt[(long)i * 24 + j];
        const float ax = fabsf(x);
        v += ax < 1.f ? 0.5f * x * x : ax - 0.5f;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    v += __shfl_xor(v, off);
    c += __shfl_xor(c, off);
  }
  if ((threadIdx.x & 63) == 0) { sh[threadIdx.x >> 6] = v; shc[threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(acc, sh[0] + sh[1] + sh[2] + sh[3]);
    atomicAdd(rows, shc[0] + shc[1] + shc[2] + shc[3]);
  }
}

// d loss / d pbw rows and d tbw rows (smooth_l1_loss mean over m x 24) scattered per point
__global__ __launch_bounds__(256) void k_an_loss_grads(TrainBufs b, const int* rows, int need_dt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *b.n_kept;
  if (i >= n) return;
  const bool sel = b.sigma[i] > 0.f;
  const float sc = 1.0f / (24.0f * (float)(*rows));
  for (int j = 0; j < 24; ++j) {
    const float x = b.Bp[(long)i * 24 + j] - b.Bt[(long)i * 24 + j];
    const float d = sel ? (fabsf(x) < 1.f ? x : (x > 0.f ? 1.f : -1.f)) * sc : 0.f;
    b.dBp[(long)i * 24 + j] = d;
    if (need_dt) b.dBt[(long)i * 24 + j] = -d;
  }
}

__global__ void k_an_set(int* c, int n) { c[0] = n; }

__global__ void k_an_loss_final(const float* acc, const int* rows, float* loss3) {
  const float l0 = acc[0] / (24.0f * (float)rows[0]);
  const float l1 = acc[1] / (24.0f * (float)rows[1]);
  loss3[0] = l0 + l1;
  loss3[1] = l0;
  loss3[2] = l1;
}

}  // namespace anr
