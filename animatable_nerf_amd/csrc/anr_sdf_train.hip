// anr_sdf_train.hip — one training step of the sdf_pdf variant (config 5, SURVEY.md §8(e) "Training
// (3/4/5)"): tpose_trainer.NetworkWrapper.forward + loss.backward() over anisdf_pdf_network.Network
// (lib/train/trainers/tpose_trainer.py:21-73, crit.py:5-19, anisdf_pdf_network.py:49-224).
//
// The loss reaches the parameters through second-order paths: the eikonal loss and the colour net
// read gradients = d sdf / d x (create_graph, :306-321), and the observed-gradient loss reads
// d sdf(x + resd(x)) / d x (:140-154). Each such term is differentiated forward-over-reverse: with
// the upstream adjoint dg of g = grad_x s(x), dg . g = J_s(x) dg is the directional derivative of s
// along dg, so one forward tangent pass (tangent input dg) and one reverse pass over the stacked
// [primal; tangent] activations give every parameter's gradient. Per softplus layer
// (h = sp(z), hdot = sp'(z) zdot): zdot_bar = sp'(z) hdot_bar, z_bar = sp'(z) h_bar + sp''(z) zdot
// hdot_bar, and sp''(z) zdot = 100 (1 - sp'(z)) hdot, so only the stored factor d = exp(100 z) and
// the tangent activation hdot are needed. ReLU layers have no second-order term; tanh has one.
//
// Layer-wise: every activation stays in HBM (a 1,024-ray batch keeps ~46k samples), exact fp32
// MFMA GEMMs (anr_gemm.hip k_gemm_t: weights and activations shared by the primal and tangent
// rows, which are stacked into one 2n-row operand wherever the epilogue allows); per-sample work in
// the kernels below. Two host reads of counts (kept samples, observed-gradient rows).
#include <cstdio>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/aninerf.h"
#include "anr_common.h"
#include "anr_kernels.h"
#include "anr_sdf.h"
#include "anr_train.h"
#include "anr_ws.h"

#pragma clang fp contract(off)

using namespace anr;

namespace anr {

// ------------------------------------------------------------------------------------------
// per-sample kernels
// ------------------------------------------------------------------------------------------
// inv[list[i]] = i: a sample id -> its compact row (the msk_sdf argmin scatter)
__global__ void k_st_inv(const int* __restrict__ list, const int* __restrict__ n_dev, int* inv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < *n_dev) inv[list[i]] = i;
}

// gamma_F feature f of x and its first and second derivatives along x[comp(f)] (embedder.py:5-54)
__device__ __forceinline__ void embed_d(const float x[3], int f, int& comp, float& v, float& d1, float& d2) {
  if (f < 3) {
    comp = f; v = x[f]; d1 = 1.f; d2 = 0.f;
    return;
  }
  const int g = f - 3, fr = g / 6, w = g - fr * 6;
  comp = w >= 3 ? w - 3 : w;
  const float om = (float)(1 << fr);
  const float a = x[comp] * om;
  const float sa = sinf(a), ca = cosf(a);
  if (w < 3) { v = sa; d1 = om * ca; d2 = -om * om * sa; }
  else { v = ca; d1 = -om * sa; d2 = -om * om * ca; }
}

// tangent of gamma_F: out[i][col0 + f] = scale * J_gamma(x_i) xd_i  (f < 3 + 6 F)
__global__ void k_st_embed_tan(const float* __restrict__ x, long ldx, const float* __restrict__ xd, long ldxd, int nf,
                               int n, float* out, long ldo, int col0, float scale) {
  const int F = 3 + 6 * nf;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * F) return;
  const int i = (int)(e / F), f = (int)(e - (long)i * F);
  const float p[3] = {x[i * ldx], x[i * ldx + 1], x[i * ldx + 2]};
  int c;
  float v, d1, d2;
  embed_d(p, f, c, v, d1, d2);
  out[(long)i * ldo + col0 + f] = scale * (d1 * xd[i * ldxd + c]);
}

// reverse of [gamma_6(t); J_gamma_6(t) tdot] (the SDF input, primal rows 0..n-1, tangent rows n..2n-1
// of the adjoints): the gamma adjoint is lin0's input adjoint (A0, ld 40) plus lin4's gamma columns
// (A4 cols 217.., ld 256, times 1/sqrt2). tbar += J^T abar + (d/dt J tdot)^T atbar; ttbar = J^T atbar.
__global__ void k_st_embed_rev6(const float* __restrict__ t, long ldt, const float* __restrict__ td, long ldtd,
                                const float* __restrict__ A0, const float* __restrict__ A4, int n, float* tbar,
                                float* ttbar) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float p[3] = {t[i * ldt], t[i * ldt + 1], t[i * ldt + 2]};
  const float pd[3] = {td[i * ldtd], td[i * ldtd + 1], td[i * ldtd + 2]};
  const float rs2 = 0.70710678118654752f;
  float tb[3] = {0.f, 0.f, 0.f}, ttb[3] = {0.f, 0.f, 0.f};
  for (int f = 0; f < 39; ++f) {
    const float ab = A0[(long)i * 40 + f] + A4[(long)i * 256 + 217 + f] * rs2;
    const float atb = A0[(long)(n + i) * 40 + f] + A4[(long)(n + i) * 256 + 217 + f] * rs2;
    int c;
    float v, d1, d2;
    embed_d(p, f, c, v, d1, d2);
    tb[c] += d1 * ab + d2 * pd[c] * atb;
    ttb[c] += d1 * atb;
  }
  for (int c = 0; c < 3; ++c) {
    tbar[i * 4 + c] += tb[c];
    if (ttbar) ttbar[i * 4 + c] = ttb[c];
  }
}

// first-order reverse of gamma_10 (the residual net's input): xbar = J^T (G0 + G5) over 63 columns
__global__ void k_st_embed_bwd10(const float* __restrict__ x, long ldx, const float* __restrict__ G, long ldg, int n,
                                 float* xbar, long ldxb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float p[3] = {x[i * ldx], x[i * ldx + 1], x[i * ldx + 2]};
  float xb[3] = {0.f, 0.f, 0.f};
  for (int f = 0; f < 63; ++f) {
    int c;
    float v, d1, d2;
    embed_d(p, f, c, v, d1, d2);
    xb[c] += d1 * G[(long)i * ldg + f];
  }
  for (int c = 0; c < 3; ++c) xbar[i * ldxb + c] = xb[c];
}

// softplus reverse of one layer over the stacked adjoints: rows 0..n-1 primal (A), n..2n-1 tangent
// (At, row stride ldat: 0 broadcasts one row, NULL = 0). Z = [z_bar; zdot_bar] (ld 256).
//   zdot_bar = sp' at;  z_bar = sp' a + 100 / (d + 1) hdot at  (d = exp(100 z) >= 0; above torch's
//   threshold d = -1: sp' = 1, sp'' = 0). hdot = the tangent activation (Hd, times hscale).
__global__ void k_st_sp_rev(const float* __restrict__ A, long lda, const float* __restrict__ At, long ldat, float ascale,
                            const float* __restrict__ D, const float* __restrict__ Hd, long ldh, float hscale, int n,
                            int width, float* Z) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * width) return;
  const int i = (int)(e / width), c = (int)(e - (long)i * width);
  const float a = A ? A[(long)i * lda + c] * ascale : 0.f;
  const float at = At ? At[(long)i * ldat + c] * ascale : 0.f;
  const float d = D[(long)i * 256 + c];
  float zb, ztb;
  if (d < 0.f) {
    zb = a;
    ztb = at;
  } else {
    const float r = 1.f / (d + 1.f);
    const float sp1 = d * r;
    const float hd = Hd[(long)i * ldh + c] * hscale;
    ztb = sp1 * at;
    zb = sp1 * a + 100.f * r * hd * at;
  }
  Z[(long)i * 256 + c] = zb;
  Z[(long)(n + i) * 256 + c] = ztb;
}

// dW[o][col0 + q] += bsum[o] * v[q] (the folded constant columns: poses of the residual net)
__global__ void k_st_outer_add(const float* __restrict__ bsum, const float* __restrict__ v, int nq, int nout, float* dW,
                               int in_ch, int col0) {
  const int o = blockIdx.x, q = threadIdx.x;
  if (o < nout && q < nq) dW[(long)o * in_ch + col0 + q] += bsum[o] * v[q];
}

// dst[c] += sum over n rows of H[r][c] (c < 256): the tangent output adjoint e0 of lin8 (row 0 of dW8)
__global__ void k_st_colsum(const float* __restrict__ H, long ldh, int n, float* dst) {
  const int c = threadIdx.x;
  float acc = 0.f;
  for (int r = blockIdx.x; r < n; r += gridDim.x) acc += H[(long)r * ldh + c];
  atomicAdd(dst + c, acc);
}

// weight norm backward (torch._weight_norm, dim 0): W = g v / |v|_row; from dW (effective):
//   dg = (dW . v) / |v|;  dv = (g / |v|) (dW - (dW . v) v / |v|^2)
__global__ __launch_bounds__(256) void k_st_wn_grad(const float* __restrict__ v, const float* __restrict__ gw,
                                                    const float* __restrict__ dW, int in_ch, float* dg, float* dv) {
  __shared__ float sh[2][4];
  const int row = blockIdx.x;
  const float* vr = v + (long)row * in_ch;
  const float* dr = dW + (long)row * in_ch;
  float s = 0.f, q = 0.f;
  for (int k = threadIdx.x; k < in_ch; k += 256) {
    s += dr[k] * vr[k];
    q += vr[k] * vr[k];
  }
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    q += __shfl_xor(q, off);
  }
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = s;
    sh[1][threadIdx.x >> 6] = q;
  }
  __syncthreads();
  s = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
  q = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
  const float nrm = sqrtf(q);
  const float g = gw[row];
  if (threadIdx.x == 0) dg[row] += s / nrm;
  const float a = g / nrm, b = s / q;
  for (int k = threadIdx.x; k < in_ch; k += 256) dv[(long)row * in_ch + k] += a * (dr[k] - b * vr[k]);
}

struct StRaw {
  const int* list;
  const int* n_kept;
  int chunk;
  const float4* draw;   // (R*64) d raw from the compositing backward
  const float* C0;      // [n][40] tpose
  const float* tbtab;
  const float* Y8;      // [n][264] sdf = col 0
  const float* Yc;      // [n][4] colour logits
  const float* beta;    // device scalar
  float* dYc;           // [n][4]
  float* ds;            // [n]
  float* dbeta;         // device scalar (atomic)
};

// raw = (sigmoid(yc), 1 - exp(-relu(sigma(s, beta)) 0.005)), zero outside the widened tbounds
// (anisdf_pdf_network.py:204-210, :271-331): d logits, d sdf, d beta per kept sample
__global__ __launch_bounds__(256) void k_st_raw_bwd(StRaw a) {
  __shared__ float sb[4];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float db = 0.f;
  if (i < *a.n_kept) {
    const int pid = a.list[i];
    const float4 d = a.draw[pid];
    const float* tb = a.tbtab + (size_t)((pid >> 6) / a.chunk) * 6;
    const float* c = a.C0 + (size_t)i * 40;
    bool inside = true;
    for (int r = 0; r < 3; ++r) inside = inside && c[r] > tb[r] && c[r] < tb[3 + r];
    float* dy = a.dYc + (size_t)i * 4;
    if (!inside) {
      dy[0] = dy[1] = dy[2] = dy[3] = 0.f;
      a.ds[i] = 0.f;
    } else {
      const float dc[3] = {d.x, d.y, d.z};
      for (int r = 0; r < 3; ++r) {
        const float sg = 1.0f / (1.0f + expf(-a.Yc[(size_t)i * 4 + r]));
        dy[r] = dc[r] * (sg * (1.f - sg));
      }
      dy[3] = 0.f;
      const float braw = *a.beta;
      const float beta = fminf(fmaxf(braw, 1e-9f), 1e6f);
      const float x = -a.Y8[(size_t)i * 264];
      float sig, dsig_dx, dsig_db;
      if (x <= 0.f) {
        const float e = expf(x / beta);
        sig = 1.0f / beta * (0.5f * e);
        dsig_dx = sig / beta;
        dsig_db = -sig / beta - sig * x / (beta * beta);
      } else {
        const float e = expf(-x / beta);
        sig = 1.0f / beta * (1.0f - 0.5f * e);
        dsig_dx = 0.5f * e / (beta * beta);
        dsig_db = -sig / beta - 0.5f * e * x / (beta * beta * beta);
      }
      const float dsig = sig > 0.f ? d.w * expf(-sig * 0.005f) * 0.005f : 0.f;
      a.ds[i] = -dsig * dsig_dx;
      if (braw >= 1e-9f && braw <= 1e6f) db = dsig * dsig_db;
    }
  }
  for (int off = 32; off > 0; off >>= 1) db += __shfl_xor(db, off);
  if ((threadIdx.x & 63) == 0) sb[threadIdx.x >> 6] = db;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(a.dbeta, sb[0] + sb[1] + sb[2] + sb[3]);
}

// loss accumulators (acc): 0 offset |r| sum, 1 eikonal sum, 2 observed-eikonal sum, 3 BCE sum,
// 4 img sq-err sum, 5 img rays, 6 msk entries (count)
struct StLoss {
  const int* n_kept;
  const float* resd;   // [n][3]
  const float* C0;     // [n][40] gradients at 30..32
  const float* dC0;    // [n][40] colour input adjoint (normal at 30..32)
  const float* ds;     // [n]
  float* rbar;         // [n][4] out: offset-loss adjoint of resd
  float* dG;           // [n][4] out: normal adjoint (colour + eikonal)
  float* dZ8;          // [n][264] col 0 out: sdf adjoint
  float* acc;
};

__device__ __forceinline__ void block_add(float v, float* dst) {
  __shared__ float sb[4];
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sb[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(dst, sb[0] + sb[1] + sb[2] + sb[3]);
}

// offset_loss = mean |resd|, grad_loss = mean (|g| - 1)^2 (tpose_trainer.py:26-36) and their adjoints
__global__ __launch_bounds__(256) void k_st_sample_loss(StLoss a) {
  const int n = *a.n_kept;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float lo = 0.f, lg = 0.f;
  if (i < n) {
    const float* r = a.resd + (size_t)i * 3;
    const float rn = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    lo = rn;
    const float so = rn > 0.f ? 0.01f / ((float)n * rn) : 0.f;
    const float* g = a.C0 + (size_t)i * 40 + 30;
    const float gn = sqrtf(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]);
    lg = (gn - 1.f) * (gn - 1.f);
    const float sg = gn > 0.f ? 0.01f * 2.f * (gn - 1.f) / ((float)n * gn) : 0.f;
    for (int c = 0; c < 3; ++c) {
      a.rbar[(size_t)i * 4 + c] = r[c] * so;
      a.dG[(size_t)i * 4 + c] = a.dC0[(size_t)i * 40 + 30 + c] + g[c] * sg;
    }
    a.rbar[(size_t)i * 4 + 3] = 0.f;
    a.dG[(size_t)i * 4 + 3] = 0.f;
    a.dZ8[(size_t)i * 264] = a.ds[i];
  }
  block_add(lo, a.acc + 0);
  block_add(lg, a.acc + 1);
}

// observed gradients: ograd_loss = mean (|og| - 1)^2 and its adjoint dog (tpose_trainer.py:38-43)
__global__ __launch_bounds__(256) void k_st_obs_loss(const float* __restrict__ og, int n_o, float* dog, float* acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float l = 0.f;
  if (i < n_o) {
    const float* g = og + (size_t)i * 4;
    const float gn = sqrtf(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]);
    l = (gn - 1.f) * (gn - 1.f);
    const float sg = gn > 0.f ? 0.01f * 2.f * (gn - 1.f) / ((float)n_o * gn) : 0.f;
    for (int c = 0; c < 3; ++c) dog[(size_t)i * 4 + c] = g[c] * sg;
    dog[(size_t)i * 4 + 3] = 0.f;
  }
  block_add(l, acc + 2);
}

// msk_sdf (tpose_renderer.py:134-152): per ray the min sdf over its 64 samples and the first sample
// holding it (torch.min's index), the intersection test, the list an entry goes to; count entries
__global__ __launch_bounds__(256) void k_st_msk_rays(const float* __restrict__ sdf, const uint8_t* __restrict__ occ,
                                                     int R, float* mn_out, int* am_out, uint8_t* flags, float* acc) {
  const int lane = threadIdx.x & 63;
  const int ray = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= R) return;
  const float s = sdf[(size_t)ray * 64 + lane];
  const float nx = __shfl_down(s, 1);
  float mn = s;
  for (int off = 32; off > 0; off >>= 1) mn = fminf(mn, __shfl_xor(mn, off));
  const uint64_t at = __ballot(s == mn);
  const bool neg = lane < 63 && s * nx < 0.f;
  const bool inter = __ballot(neg) != 0ull;
  if (lane == 0) {
    const uint8_t o = occ[ray];
    const uint8_t f = (uint8_t)(((!inter && o == 1) ? 1 : 0) | (o == 0 ? 2 : 0));
    mn_out[ray] = mn;
    am_out[ray] = ray * 64 + (at ? __builtin_ctzll(at) : 0);
    flags[ray] = f;
    if (f) atomicAdd(acc + 6, 1.f);
  }
}

// mask_loss = BCE_with_logits(-alpha msk_sdf, label).mean() / alpha (crit.py:5-19); its adjoint goes
// to the argmin sample's sdf when that sample was kept (dropped samples hold the constant 10)
__global__ __launch_bounds__(256) void k_st_msk_loss(const float* __restrict__ mn, const int* __restrict__ am,
                                                     const uint8_t* __restrict__ flags, const int* __restrict__ inv,
                                                     int R, float alpha, float* ds, float* acc) {
  const int ray = blockIdx.x * blockDim.x + threadIdx.x;
  float l = 0.f;
  if (ray < R && flags[ray]) {
    const float y = (flags[ray] & 1) ? 1.f : 0.f;
    const float z = -alpha * mn[ray];
    l = fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z)));
    const float L = acc[6];
    const float sg = 1.f / (1.f + expf(-z));
    const int i = inv[am[ray]];
    if (i >= 0) ds[i] += -(sg - y) / L;
  }
  block_add(l, acc + 3);
}

// loss vector (include/aninerf.h anr_sdf_train_step)
__global__ void k_st_loss_final(const float* acc, const float* acc3, const int* n_kept, int n_o, float alpha, float* loss) {
  const float n = (float)*n_kept;
  const float off = acc[0] / n, gl = acc[1] / n, og = n_o > 0 ? acc[2] / (float)n_o : 0.f;
  const float ml = acc[3] / acc[6] / alpha;
  const float img = acc3[0] / (3.0f * acc3[1]);
  float tot = 0.f;
  tot += 0.01f * off;
  tot += 0.01f * gl;
  if (n_o > 0) tot += 0.01f * og;
  tot += ml;
  tot += img;
  loss[0] = tot; loss[1] = off; loss[2] = gl; loss[3] = og; loss[4] = ml; loss[5] = img;
  loss[6] = (float)n_o; loss[7] = acc[6]; loss[8] = n; loss[9] = 0.f;
}

// tanh head of the residual net, r = 0.05 tanh(y): tangent rdot = 0.05 (1 - tau^2) ydot, t = x + r
__global__ void k_st_resd_tan(const float* __restrict__ Y, const float* __restrict__ Yd, const float* __restrict__ xd,
                              int n, float* td) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int c = 0; c < 3; ++c) {
    const float t = tanhf(Y[(size_t)i * 4 + c]);
    td[(size_t)i * 4 + c] = xd[(size_t)i * 4 + c] + 0.05f * (1.f - t * t) * Yd[(size_t)i * 4 + c];
  }
  td[(size_t)i * 4 + 3] = 0.f;
}

// reverse of r = 0.05 tanh(y) (and of its tangent when Yd != NULL): rows 0..n-1 y_bar, n..2n-1 ydot_bar
//   ydot_bar = 0.05 (1 - tau^2) rdot_bar;  y_bar = 0.05 (1 - tau^2) r_bar - 0.1 tau (1 - tau^2) ydot rdot_bar
__global__ void k_st_tanh_rev(const float* __restrict__ Y, const float* __restrict__ Yd, const float* __restrict__ rb,
                              const float* __restrict__ rb2, const float* __restrict__ rdb, int n, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int c = 0; c < 3; ++c) {
    const float t = tanhf(Y[(size_t)i * 4 + c]);
    const float s = 1.f - t * t;
    float r = rb[(size_t)i * 4 + c];
    if (rb2) r += rb2[(size_t)i * 4 + c];
    float yb = 0.05f * s * r;
    if (Yd) {
      const float rd = rdb[(size_t)i * 4 + c];
      yb += -0.1f * t * s * Yd[(size_t)i * 4 + c] * rd;
      out[(size_t)(n + i) * 4 + c] = 0.05f * s * rd;
    }
    out[(size_t)i * 4 + c] = yb;
  }
  out[(size_t)i * 4 + 3] = 0.f;
  if (Yd) out[(size_t)(n + i) * 4 + 3] = 0.f;
}

// observed-gradient rows: kept samples with |sdf| < 0.02 (anisdf_pdf_network.py:194), compact order
__global__ __launch_bounds__(256) void k_st_obs_count(const float* __restrict__ Y8, const int* __restrict__ n_dev,
                                                      int* block_sum) {
  __shared__ int sh[4];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int v = (i < *n_dev && fabsf(Y8[(size_t)i * 264]) < 0.02f) ? 1 : 0;
  int tot;
  block_excl_scan_256(v, sh, tot);
  if (threadIdx.x == 0) block_sum[blockIdx.x] = tot;
}

// gather: ptb_o / Gro rows of the observed samples (init_bigpose, its gamma_10 -- the same values the
// reference recomputes from the detached copy)
__global__ __launch_bounds__(256) void k_st_obs_gather(const float* __restrict__ Y8, const int* __restrict__ n_dev,
                                                       const int* __restrict__ block_off, const float* __restrict__ ptb,
                                                       const float* __restrict__ Gr, float* ptb_o, float* Gro) {
  __shared__ int sh[4];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int v = (i < *n_dev && fabsf(Y8[(size_t)i * 264]) < 0.02f) ? 1 : 0;
  int tot;
  const int ex = block_excl_scan_256(v, sh, tot);
  if (!v) return;
  const int o = block_off[blockIdx.x] + ex;
  for (int k = 0; k < 8; ++k) ptb_o[(size_t)o * 8 + k] = ptb[(size_t)i * 8 + k];
  for (int k = 0; k < 64; ++k) Gro[(size_t)o * 64 + k] = Gr[(size_t)i * 64 + k];
}

// anr_sdf_points rows: big-pose point x in columns 0..2 of ptb (stride 8, directions 0), gamma_10(x) (stride 64)
__global__ void k_st_pts_rows(const float* __restrict__ x, int n, float* ptb, float* Gr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float p[3] = {x[3 * i], x[3 * i + 1], x[3 * i + 2]};
  for (int c = 0; c < 8; ++c) ptb[(size_t)i * 8 + c] = c < 3 ? p[c] : 0.f;
  for (int c = 0; c < 64; ++c) Gr[(size_t)i * 64 + c] = c < 63 ? embed_feature(p, c, 10) : 0.f;
}

__global__ void k_st_add_bias(const float* __restrict__ src, int n, float* dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] += src[i];
}

__global__ void k_st_add3(const float* __restrict__ a, long lda, const float* __restrict__ b, long ldb, int n, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int c = 0; c < 3; ++c) out[(size_t)i * 4 + c] = a[i * lda + c] + b[i * ldb + c];
  out[(size_t)i * 4 + 3] = 0.f;
}

// ---- Network.forward under autograd (anr_sdf_network_train_bwd): the upstream adjoints of the
// call's outputs take the place of the loss adjoints
// d sdf of a kept sample (sdf[pind] = ret['sdf'], :219): ds[i] += d_sdf[list[i]]
__global__ void k_st_cotan_sdf(const int* __restrict__ list, const int* __restrict__ n_dev, const float* __restrict__ d_sdf,
                               float* ds) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < *n_dev) ds[i] += d_sdf[list[i]];
}

// rbar = d resd, dG = colour-normal adjoint + d gradients, lin8's sdf column adjoint = ds
__global__ void k_st_cotan_rows(const int* __restrict__ n_dev, const float* __restrict__ d_resd,
                                const float* __restrict__ d_grad, const float* __restrict__ dC0, const float* __restrict__ ds,
                                float* rbar, float* dG, float* dZ8) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *n_dev) return;
  for (int c = 0; c < 3; ++c) {
    rbar[(size_t)i * 4 + c] = d_resd ? d_resd[(size_t)i * 3 + c] : 0.f;
    dG[(size_t)i * 4 + c] = dC0[(size_t)i * 40 + 30 + c] + (d_grad ? d_grad[(size_t)i * 3 + c] : 0.f);
  }
  rbar[(size_t)i * 4 + 3] = 0.f;
  dG[(size_t)i * 4 + 3] = 0.f;
  dZ8[(size_t)i * 264] = ds[i];
}

// (n,3) -> (n,4) rows (zero 4th column; src NULL: zeros)
__global__ void k_st_rows3to4(const float* __restrict__ src, int n, float* dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int c = 0; c < 3; ++c) dst[(size_t)i * 4 + c] = src ? src[(size_t)i * 3 + c] : 0.f;
  dst[(size_t)i * 4 + 3] = 0.f;
}

}  // namespace anr

namespace {

// exact fp32 layer GEMMs (anr_gemm.hip)
struct Epi {
  int relu = 0;
  float* deriv = nullptr;   // softplus(beta=100) epilogue writing its factor exp(100 z) (-1 above the threshold)
  bool softplus = false;
  const float* spd = nullptr;  // v *= sp'(z) from the stored factor (n < spd_n)
  int spd_n = 0;
  const float* mask = nullptr;  // v = 0 where mask <= 0 (a ReLU layer's output)
  long ldm = 0;
  float div_post = 0.f;
};

// x3 (o->precision ANR_BF16X3): the forward / input-gradient products as split-bf16 tiles (k_gemm_b
// X3: lo*bh + hi*bl + hi*bh, fp32 accumulation, the same epilogues) and the weight gradients on the
// split-bf16 slab kernel (anr_tgemm.hip k_wgrad X3) where its operand shapes fit; otherwise exact fp32
// x3 products whose operands fit anr_lgemm.hip (no accumulate / mask, 16-B addressable rows) run on
// k_lgemm, the weights' hi/lo fragment image resident in LDS: each distinct weight view (operand
// pointers, strides, depths, N, bias) is packed into the arena once per call and reused by every
// later product on it (the weights do not change inside one step).
struct LgImage {
  const float *B0, *B1, *bias;
  long r0, c0, r1, c1;
  int K0, K1, N;
  void* img;
  int f32;                          // fp32 image (F32 kernels) or hi / lo bf16
  long blocks;                      // its pack launch's blocks
  alignas(8) unsigned char desc[192];  // its pack descriptor (lgemm_pack_describe)
};

// Per-call pack plans: a call packs each distinct weight view once, ~60 k_limg_pack launches per sdf_pdf
// training step. The views a call packs depend only on the parameter pointers, the workspace and the
// precision switches, so the list is recorded at the end of a call under that key (descriptors and block
// starts copied to device memory once) and the next call with the same key packs all of them in ONE
// k_limg_pack_multi launch right after the per-call weights (weight norm, folds) are formed, before its
// first product. A product the plan does not hold is still packed on first use (and re-records the plan).
struct LgPlan {
  std::string key;
  void* dev = nullptr;  // descriptors, then n + 1 block starts (long)
  int n = 0;
  long blocks = 0;
  size_t used = 0;
  std::vector<LgImage> entries;
};
std::mutex lg_plan_mu;
std::vector<LgPlan> lg_plans;  // least recently recorded first, at most 8

struct TG {
  hipStream_t s;
  int x3 = 0;
  int wg_x3 = 0;          // the weight gradients split-bf16 (set per part)
  float* slab = nullptr;  // k_wgrad partial slabs (x3)
  char* lg_arena = nullptr;  // k_lgemm weight images (x3)
  size_t lg_cap = 0, lg_used = 0;
  int cus = 256;
  LgImage lg[64];
  int nlg = 0;
  void* lg_image(const GemmArgs& g) {
    const GemmSeg& a = g.seg[0];
    const GemmSeg& b = g.seg[1];
    const bool two = g.nseg > 1;
    const int f32 = !g.x3 && !g.bf16;
    for (int i = 0; i < nlg; ++i) {
      const LgImage& q = lg[i];
      if (q.B0 == a.B && q.r0 == a.b_rs && q.c0 == a.b_cs && q.K0 == a.K && q.N == g.N && q.bias == g.bias &&
          q.f32 == f32 && q.B1 == (two ? b.B : nullptr) && (!two || (q.r1 == b.b_rs && q.c1 == b.b_cs && q.K1 == b.K)))
        return q.img;
    }
    const size_t bytes = (lgemm_image_bytes(g) + 255) / 256 * 256;
    if (nlg >= 64 || lg_used + bytes > lg_cap) return nullptr;
    void* img = lg_arena + lg_used;
    if (lgemm_pack(g, img, s) != 0) return nullptr;
    lg_used += bytes;
    LgImage& q = lg[nlg++];
    q = LgImage{a.B, two ? b.B : nullptr, g.bias, a.b_rs, a.b_cs, two ? b.b_rs : 0, two ? b.b_cs : 0,
                a.K, two ? b.K : 0, g.N, img, f32, 0, {}};
    if (lgemm_pack_desc_bytes() <= sizeof(q.desc)) q.blocks = lgemm_pack_describe(g, img, q.desc);
    plan_dirty = true;
    return img;
  }
  // the pack plan of this call's key (LgPlan): every recorded image packed in one launch
  std::string plan_key;
  bool plan_dirty = false;
  int plan_begin(const std::string& key) {
    plan_key = key;
    std::lock_guard<std::mutex> lk(lg_plan_mu);
    for (const LgPlan& P : lg_plans) {
      if (P.key != key) continue;
      const size_t D = lgemm_pack_desc_bytes();
      const long* starts = (const long*)((const char*)P.dev + (P.n * D + 7) / 8 * 8);
      if (lgemm_pack_batch(P.dev, starts, P.n, P.blocks, s) != 0) return -1;
      nlg = (int)P.entries.size();
      for (int i = 0; i < nlg; ++i) lg[i] = P.entries[i];
      lg_used = P.used;
      return 0;
    }
    return 0;
  }
  // record (or re-record) the plan once the call has issued every product
  void plan_end() {
    if (plan_key.empty() || !plan_dirty || nlg == 0) return;
    const size_t D = lgemm_pack_desc_bytes();
    for (int i = 0; i < nlg; ++i)
      if (D > sizeof(lg[i].desc) || lg[i].blocks <= 0) return;
    const size_t off = (nlg * D + 7) / 8 * 8;
    std::vector<unsigned char> host(off + (nlg + 1) * sizeof(long));
    long* starts = (long*)(host.data() + off);
    long b = 0;
    for (int i = 0; i < nlg; ++i) {
      std::memcpy(host.data() + i * D, lg[i].desc, D);
      starts[i] = b;
      b += lg[i].blocks;
    }
    starts[nlg] = b;
    void* dev = nullptr;
    if (hipMalloc(&dev, host.size()) != hipSuccess) return;
    if (hipMemcpy(dev, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(dev);
      return;
    }
    LgPlan P;
    P.key = plan_key; P.dev = dev; P.n = nlg; P.blocks = b; P.used = lg_used;
    P.entries.assign(lg, lg + nlg);
    std::lock_guard<std::mutex> lk(lg_plan_mu);
    for (size_t i = 0; i < lg_plans.size(); ++i)
      if (lg_plans[i].key == plan_key) {  // hipFree waits for the device: a batch still reading it finishes first
        (void)hipFree(lg_plans[i].dev);
        lg_plans.erase(lg_plans.begin() + i);
        break;
      }
    if (lg_plans.size() >= 8) {
      (void)hipFree(lg_plans.front().dev);
      lg_plans.erase(lg_plans.begin());
    }
    lg_plans.push_back(std::move(P));
  }
  ~TG() { plan_end(); }
  int lg32 = 0;  // exact fp32 products on k_lgemm's F32 kernels (resident fp32 weight image) where they fit
  int wg32 = 0;  // exact fp32 weight gradients on k_wgrad_f32 (slab + reduce) where they fit
  int run(GemmArgs g, int M) {
    if (M <= 0 || g.N <= 0) return ANR_OK;
    g.M = M;
    if (g.ksplit < 1) g.ksplit = 1;
    if (x3 && !g.atomic) g.x3 = 1;
    if ((g.x3 || lg32) && lg_arena && lgemm_supported(g)) {
      g.prof = 1;  // the step's clock (anr_profile_read_clock) from these launches' stamps
      if (void* img = lg_image(g)) {
        if (lgemm_run(g, img, cus, s) != 0) return check_launch("k_lgemm (sdf train)");
        return ANR_OK;
      }
    }
    static const bool log_fb = getenv("ANR_SDF_LOG_FALLBACK") != nullptr;  // which products k_lgemm does not take
    if (log_fb)
      fprintf(stderr, "sdf train k_gemm: M %d N %d nseg %d K0 %d a_rs0 %ld K1 %d atomic %d softplus %d spd %d mask %d ldc %ld "
              "acc %d div_post %g x3 %d\n", M, g.N, g.nseg, g.seg[0].K, (long)g.seg[0].a_rs, g.nseg > 1 ? g.seg[1].K : 0,
              g.atomic, g.softplus, g.spd ? 1 : 0, g.mask ? 1 : 0, (long)g.ldc, g.accumulate, (double)g.div_post, g.x3);
    launch_gemm(g, dim3((g.N + 63) / 64, (M + 63) / 64, g.ksplit), s);
    return check_launch("k_gemm (sdf train)");
  }
  // Y[M][N] = epi(X0[:, :K0] W[:, c0:c0+K0]^T (+ X1[:, :K1] W[:, c1:c1+K1]^T) + bias)
  int fwd(int M, float* Y, long ldY, int N, const float* W, int in_ch, const float* bias, const float* X0, long ld0,
          int K0, int c0, const Epi& e = Epi(), const float* X1 = nullptr, long ld1 = 0, int K1 = 0, int c1 = 0) {
    GemmArgs g{};
    g.N = N;
    g.nseg = X1 ? 2 : 1;
    g.seg[0] = GemmSeg{X0, ld0, 1, W + c0, 1, in_ch, K0};
    if (X1) g.seg[1] = GemmSeg{X1, ld1, 1, W + c1, 1, in_ch, K1};
    g.C = Y; g.ldc = ldY; g.bias = bias; g.relu = e.relu;
    if (e.softplus) { g.softplus = 1; g.deriv = e.deriv; g.ldd = 256; }
    g.spd = e.spd; g.ldsd = 256; g.spd_n = e.spd_n;
    g.mask = e.mask; g.ldm = e.ldm;
    g.div_post = e.div_post;
    return run(g, M);
  }
  // dW[:, c0:c0+K] (row stride in_ch) += dY^T X over M samples; bsum (+)= column sums of dY
  int wgrad(int M, float* dW, int in_ch, int c0, int Nout, const float* dY, long ldY, const float* X, long ldX, int K,
            float* bsum = nullptr) {
    if (M <= 0) return ANR_OK;
    if (wg_x3 && slab && Nout <= 256 && K <= 256 && ldY % 4 == 0 && ldX % 4 == 0 && ((uintptr_t)dY & 15) == 0 &&
        ((uintptr_t)X & 15) == 0) {
      WGrad w{};
      w.x3 = 1;
      w.dY = dY; w.ldY = ldY; w.nout = Nout; w.X = X; w.ldX = ldX; w.K = K;
      w.dW = dW + c0; w.ldw = in_ch; w.bsum = bsum; w.slab = slab;
      if (launch_wgrad(w, M, s) != 0) return check_launch("k_wgrad (sdf train)");
      return ANR_OK;
    }
    if (!wg_x3 && wg32 && slab) {
      // exact fp32: k_wgrad_f32 over blocks of <= 256 outputs x <= 256 inputs (lin8's 257 outputs, the
      // colour net's 289 inputs), each block's column sums once (its first input block); the blocks run
      // one after another on s, reusing the slab region in stream order
      // X off a 16-B boundary (the colour net's feature, Y8 + 1): the product starts `off` columns early at
      // the boundary and the reduction skips those columns (WGrad::j0)
      const int off = (int)(((uintptr_t)X & 15) / 4);
      const bool shift = ((uintptr_t)X & 3) == 0 && off > 0 && c0 >= off;
      const float* Xs = shift ? X - off : X;
      const int Ks = shift ? K + off : K;
      const int cs = shift ? c0 - off : c0;
      WGrad w{};
      w.ldY = ldY; w.ldX = ldX; w.ldw = in_ch; w.slab = slab;
      bool fits = true;
      for (int pass = 0; pass < 2 && fits; ++pass)
        for (int r0 = 0; r0 < Nout && fits; r0 += 256)
          for (int k0 = 0; k0 < Ks && fits; k0 += 256) {
            w.dY = dY + r0; w.nout = std::min(256, Nout - r0);
            w.X = Xs + k0; w.K = std::min(256, Ks - k0);
            w.j0 = k0 == 0 && shift ? off : 0;
            w.dW = dW + cs + (long)r0 * in_ch + k0;
            w.bsum = bsum && k0 == 0 ? bsum + r0 : nullptr;
            if (pass == 0) fits = wgrad_f32_fits(w);
            else if (launch_wgrad_f32(w, M, s) != 0) return check_launch("k_wgrad_f32 (sdf train)");
          }
      if (fits) return ANR_OK;
    }
    GemmArgs g{};
    g.rowsum = bsum;
    g.N = K;
    g.nseg = 1;
    g.seg[0] = GemmSeg{dY, 1, ldY, X, ldX, 1, M};
    g.C = dW + c0; g.ldc = in_ch; g.atomic = 1;
    g.ksplit = (M + 511) / 512;
    return run(g, Nout);
  }
  // dX[M][K] (+)= dY W[:, c0:c0+K] (masked by mask > 0), / div_post
  int xgrad(int M, float* dX, long ldX, int K, const float* dY, long ldY, int Nout, const float* W, int in_ch, int c0,
            const float* mask = nullptr, long ldm = 0, bool acc = false) {
    GemmArgs g{};
    g.N = K;
    g.nseg = 1;
    g.seg[0] = GemmSeg{dY, ldY, 1, W + c0, in_ch, 1, Nout};
    g.C = dX; g.ldc = ldX; g.mask = mask; g.ldm = ldm; g.accumulate = acc ? 1 : 0;
    return run(g, M);
  }
};

constexpr float SQRT2 = 1.41421356237309515f;
constexpr size_t kLgArena = (size_t)32 << 20;  // k_lgemm weight images of one call (x3)

struct STLayout {
  size_t counts, mask, chunk_min, ray_off, block_sum, list, knn, tbtab, wimg, fold, inv;
  size_t ptb, Gr, Hr, Yr, resd, C0, Xs0, Hs, D, Y8, Ga, Gb, Gc, gB, grow, Hc, Yc;
  size_t raw, sdf, draw, drgb, rmin, ramin, rflag;
  size_t dYc, dHa, dHb, dC0, dZ8, ds, dG, rbar, tbar, ttbar, Ab, Zb, AX4, Ain, dWe, bsum, acc, acc3, dbeta, zero;
  size_t oblock, ptbo, Gro, Grt, ro, og, dog, tdot, Gbar, Yd, gro, wslab, lgimg;
  long N;
  size_t total;
};

STLayout stlayout(int R, int chunk) {
  STLayout L{};
  const size_t N = (size_t)R * 64;
  L.N = (long)N;
  const size_t nch = (R + chunk - 1) / (size_t)std::max(chunk, 1);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align256(o + bytes);
    return at;
  };
  auto f = [&](size_t floats) { return take(floats * 4); };
  L.counts = take(16); L.mask = take(R * 8); L.chunk_min = take(nch * 8); L.ray_off = take((R + 1) * 4);
  L.block_sum = take(((N + 255) / 256 + 1) * 4); L.list = take(N * 4); L.knn = take(N * 32); L.tbtab = f(nch * 6);
  L.wimg = f(SDF_WN_FLOATS); L.fold = f(768); L.inv = take(N * 4);
  L.ptb = f(N * 8); L.Gr = f(N * 64); L.Hr = f(8 * 2 * N * 256); L.Yr = f(2 * N * 4); L.resd = f(N * 3);
  L.C0 = f(N * 40); L.Xs0 = f(2 * N * 40); L.Hs = f(8 * 2 * N * 256); L.D = f(8 * N * 256); L.Y8 = f(N * 264);
  L.Ga = f(N * 256); L.Gb = f(N * 256); L.Gc = f(N * 256); L.gB = f(N * 40); L.grow = f(N * 3);
  L.Hc = f(4 * N * 256); L.Yc = f(N * 4);
  L.raw = f(N * 4); L.sdf = f(N); L.draw = f(N * 4); L.drgb = f(R * 3); L.rmin = f(R); L.ramin = take(R * 4);
  L.rflag = take(R);
  L.dYc = f(N * 4); L.dHa = f(N * 256); L.dHb = f(N * 256); L.dC0 = f(N * 40); L.dZ8 = f(N * 264); L.ds = f(N);
  L.dG = f(N * 4); L.rbar = f(N * 4); L.tbar = f(N * 4); L.ttbar = f(N * 4); L.Ab = f(2 * N * 256);
  L.Zb = f(2 * N * 256); L.AX4 = f(2 * N * 256); L.Ain = f(2 * N * 40); L.dWe = f(SDF_WN_FLOATS); L.bsum = f(4 * 256);
  L.acc = f(16); L.acc3 = f(4); L.dbeta = f(4); L.zero = take(64);
  L.oblock = take(((N + 255) / 256 + 1) * 4); L.ptbo = f(N * 8); L.Gro = f(N * 64); L.Grt = f(N * 64);
  L.ro = f(N * 3); L.og = f(N * 4); L.dog = f(N * 4); L.tdot = f(N * 4); L.Gbar = f(N * 64); L.Yd = f(N * 4);
  L.gro = f(N * 3);
  L.wslab = f(wgrad_slab_floats());
  L.lgimg = take(kLgArena);
  L.total = o;
  return L;
}

int check_train(const anr_sdf_params* p, float* const* grads, const anr_sdf_frame* f, const float* ray_o,
                const float* ray_d, const float* near_, const float* far_, int R, const anr_render_opts* o,
                const float* rgb_gt, const anr_sdf_render_out* out, const float* loss, void* ws) {
  if (!p || !grads || !f || !o || !out || !ws || !ray_o || !ray_d || !near_ || !far_ || !rgb_gt || !loss)
    return fail(ANR_E_ARG, "sdf train: NULL argument");
  if (o->n_samples != 64) return fail(ANR_E_ARG, "sdf train: only N_samples == 64 is supported");
  if (o->chunk <= 0 || R <= 0 || (long)R * 64 > (1L << 24)) return fail(ANR_E_ARG, "sdf train: bad chunk / n_rays");
  if (o->novel_pose) return fail(ANR_E_ARG, "sdf train: novel_pose is an aninerf option");
  for (int i = 0; i < ANR_SDF_NUM_TENSORS; ++i) {
    if (!p->t[i] && i != SDF_RESD_LAT) return fail(ANR_E_ARG, "sdf train: NULL parameter tensor");
    if (!grads[i] && i != SDF_RESD_LAT) return fail(ANR_E_ARG, "sdf train: NULL gradient tensor");
  }
  if (!f->A || !f->big_A || !f->R || !f->Th || !f->poses || !f->pvertices || !f->weights || !f->tbounds ||
      !f->latent_index || !f->occupancy)
    return fail(ANR_E_ARG, "sdf train: NULL frame tensor");
  if (f->n_verts <= 0 || f->n_verts > 6912) return fail(ANR_E_ARG, "sdf train: n_verts must be in [1, 6912]");
  if (!out->rgb_map || !out->acc_map || !out->depth_map) return fail(ANR_E_ARG, "sdf train: NULL output");
  return ANR_OK;
}

int read_int(const void* dev, int* host, hipStream_t s) {
  if (hipMemcpyAsync(host, dev, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return fail(ANR_E_HIP, "sdf train: count readback failed");
  return ANR_OK;
}


// one pass of the layer-wise sdf_pdf executor. STEP: the training step over rays (losses computed
// here, their adjoints drive the backward). Free samples of one Network.forward call (wpts != NULL,
// n_pts points in R = ceil(n_pts / 64) groups = one chunk, no compositing / msk_sdf): NET_FWD runs
// the forward (with the observed gradients) into the caller's raw / sdf and the workspace rows;
// NET_BWD re-runs that forward (deterministic: same counts, same rows) and the backward from the
// caller's upstream adjoints.
// PTS: the network's point helpers on n free points x (anr_sdf_points; pts_mode ANR_SDFP_*): no
// front-end / compaction (every point is a row), the SDF (and residual) layers of this executor.
enum CoreMode { STEP = 0, NET_FWD = 1, NET_BWD = 2, PTS = 3 };

struct TrainCore {
  int mode;
  const anr_sdf_params* p;
  float* const* grads;
  const anr_sdf_frame* f;
  const float *ray_o, *ray_d, *near_, *far_;
  const float *wpts, *vdir;
  int n_pts;
  int R, chunk;
  const anr_render_opts* o;
  const float* rgb_gt;
  const uint8_t* mask_at_box;
  int iter_step;
  const anr_sdf_render_out* out;  // STEP
  float* loss;                    // STEP
  float *raw_out, *sdf_out, *tb_out;  // NET_FWD
  const float *d_raw, *d_sdf, *d_resd, *d_grad, *d_og;  // NET_BWD (any NULL = 0)
  int pts_mode;                      // PTS: ANR_SDFP_NETWORK / _GRADIENT / _DEFORMED_GRADIENT
  float *pts_out, *pts_out2;         // PTS outputs
  const anr_sdf_train_hooks* hooks;  // STEP: the colour net's gradients final (anr_sdf_train_step_hooked), or NULL
  void* ws;
  size_t ws_bytes;
  hipStream_t s;
};

int sdf_train_core(const TrainCore& C) {
  const anr_sdf_params* p = C.p;
  float* const* grads = C.grads;
  const anr_sdf_frame* f = C.f;
  const float *ray_o = C.ray_o, *ray_d = C.ray_d, *near_ = C.near_, *far_ = C.far_;
  const int R = C.R;
  const anr_render_opts* o = C.o;
  const bool step = C.mode == STEP, net_fwd = C.mode == NET_FWD;
  const STLayout L = stlayout(R, C.chunk);
  if (C.ws_bytes < L.total) return fail(ANR_E_WORKSPACE, "sdf train: workspace too small");
  hipStream_t s = C.s;
  char* ws = (char*)C.ws;
  auto F = [&](size_t off) { return (float*)(ws + off); };
  const long N = L.N;
  const int nch = (R + C.chunk - 1) / C.chunk;
  int* counts = (int*)(ws + L.counts);
  const float* const* tp = p->t;
  float* wimg = F(L.wimg);
  float* fold = F(L.fold);
  float* tbtab = F(L.tbtab);
  float4* raw = net_fwd ? (float4*)C.raw_out : (float4*)F(L.raw);
  float* sdf = net_fwd ? C.sdf_out : F(L.sdf);
  float* acc = F(L.acc);
  float* acc3 = F(L.acc3);
  if (hipMemsetAsync(ws + L.counts, 0, 16, s) != hipSuccess ||
      hipMemsetAsync(ws + L.chunk_min, 0xff, (size_t)nch * 8, s) != hipSuccess ||
      hipMemsetAsync(ws + L.inv, 0xff, (size_t)N * 4, s) != hipSuccess || hipMemsetAsync(acc, 0, 64, s) != hipSuccess ||
      hipMemsetAsync(acc3, 0, 16, s) != hipSuccess || hipMemsetAsync(F(L.dbeta), 0, 16, s) != hipSuccess ||
      hipMemsetAsync(ws + L.zero, 0, 64, s) != hipSuccess ||
      hipMemsetAsync(F(L.dWe), 0, SDF_WN_FLOATS * 4, s) != hipSuccess)
    return fail(ANR_E_HIP, "sdf train: memset");

  // ---- per-call weights: weight norm, folds, per-chunk tbounds (anr_sdf_capi.hip)
  SdfTensors T{};
  for (int i = 0; i < ANR_SDF_NUM_TENSORS; ++i) T.t[i] = tp[i];
  hipLaunchKernelGGL(k_sdf_wnorm, dim3(sdf_wn_rows()), dim3(256), 0, s, T, wimg);
  hipLaunchKernelGGL(k_sdf_fold, dim3(3), dim3(256), 0, s, T, (const float*)wimg, f->poses, f->latent_index, fold);
  const bool pts = C.mode == PTS;
  if (!pts)
    hipLaunchKernelGGL(k_sdf_tbtab, dim3(1), dim3(64), 0, s, f->tbounds, nch, tbtab,
                       step ? C.out->tbounds_out : (net_fwd ? C.tb_out : nullptr));
  ANR_TRY(check_launch("sdf train prep"));

  // ---- B1 front-end (KNN keep mask) + ordered compaction; one host read of n'
  SdfFrontArgs fa{};
  fa.ray_o = ray_o; fa.ray_d = ray_d; fa.near_ = near_; fa.far_ = far_; fa.t_rand = o->t_rand;
  fa.wpts = C.wpts; fa.n_pts = C.n_pts;
  fa.n_rays = R; fa.chunk = C.chunk; fa.R = f->R; fa.Th = f->Th; fa.verts = f->pvertices; fa.nv = f->n_verts;
  fa.norm_th = o->norm_th; fa.mask = (uint64_t*)(ws + L.mask); fa.chunk_min = (uint64_t*)(ws + L.chunk_min);
  fa.knn = (uint32_t*)(ws + L.knn); fa.raw = raw; fa.sdf = sdf;
  int cus = 256;
  {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      cus = v;
  }
  CompactArgs ca{};
  int n = 0;
  int* inv = (int*)(ws + L.inv);
  if (pts) {
    n = C.n_pts;
  } else {
    hipLaunchKernelGGL(k_sdf_front, dim3(std::min(cus, (R + 15) / 16)), dim3(1024), 0, s, fa);
    ANR_TRY(check_launch("k_sdf_front (train)"));
    ca.n_rays = R; ca.chunk = C.chunk; ca.mask = fa.mask; ca.chunk_min = fa.chunk_min;
    ca.ray_off = (int*)(ws + L.ray_off); ca.block_sum = (int*)(ws + L.block_sum); ca.list = (int*)(ws + L.list);
    const int nb = (R + 255) / 256;
    hipLaunchKernelGGL(k_count, dim3(nb), dim3(256), 0, s, ca);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, ca.block_sum, nb, counts);
    hipLaunchKernelGGL(k_compact, dim3((R + 3) / 4), dim3(256), 0, s, ca);
    ANR_TRY(check_launch("k_compact (sdf train)"));
    ANR_TRY(read_int(counts, &n, s));
    hipLaunchKernelGGL(k_st_inv, dim3((n + 255) / 256 + 1), dim3(256), 0, s, (const int*)ca.list, (const int*)counts, inv);
  }

  TG g{s};
  // which products run split-bf16 (bits, ANR_SDF_X3_PARTS): 1 residual MLP, 2 SDF forward, 4 SDF input
  // gradient, 8 colour net, 16 SDF tangent pass, 32 stacked SDF reverse, 64 the weight gradients of the
  // split parts. Default 252: all but the residual MLP's and the SDF forward's products (exact fp32). The residual MLP's parameter
  // gradients are ~1e-5 in magnitude and lose tests/test_gpu_sdf_train.py's 5e-3-of-max bar to split
  // products in any of those two (the softplus(beta=100) factors of the SDF forward feed every
  // second-order term); each other part split alone, and all of them together, keep it (profiles/r4e,
  // r4g, r4h bisection). Bit 128 (default on): the weight gradients split-bf16 in every part, the
  // fp32-level ones included (test green at the same tolerances, 11.1 -> 10.9 ms, profiles/r4y)
  static const int x3_parts = [] {
    const char* v = getenv("ANR_SDF_X3_PARTS");
    return v ? atoi(v) : 252;
  }();
  const bool x3_on = o->precision == ANR_BF16X3;
  auto part = [&](int bit) {
    g.x3 = x3_on && (x3_parts & bit) ? 1 : 0;
    g.wg_x3 = x3_on && ((g.x3 && (x3_parts & 64)) || (x3_parts & 128)) ? 1 : 0;
  };
  // ANR_SDF_LG32 (read per call, default 1): the exact-fp32 forward / input-gradient products that fit
  // k_lgemm (no accumulate / atomics, 16-B addressable rows) run on its F32 kernels — the layer's fp32
  // weight image resident in LDS, activations streamed to registers, v_mfma_f32_16x16x4_f32 — instead of
  // k_gemm_t's register-staged 64 x 64 tiles (8.0 VALU instructions per MFMA, profiles/r4q_sq_k_gemm_t)
  const char* lg32_env = getenv("ANR_SDF_LG32");
  g.lg32 = !(lg32_env && lg32_env[0] == '0');
  if (x3_on || g.lg32) {
    g.lg_arena = ws + L.lgimg;
    g.lg_cap = kLgArena;
    g.cus = cus;
    // the pack plan key: parameter pointers, workspace arena, precision switches (ANR_SDF_PACK_PLAN=0: off)
    static const bool plan_on = [] {
      const char* v = getenv("ANR_SDF_PACK_PLAN");
      return !(v && v[0] == '0');
    }();
    if (plan_on) {
      std::string key;
      key.append((const char*)tp, sizeof(const float*) * ANR_SDF_NUM_TENSORS);
      const void* arena = g.lg_arena;
      const int sw[4] = {x3_on ? 1 : 0, g.lg32, x3_parts, (int)C.mode};
      key.append((const char*)&arena, sizeof(arena));
      key.append((const char*)sw, sizeof(sw));
      if (g.plan_begin(key) != 0) return fail(ANR_E_HIP, "sdf train: batched weight-image pack failed");
    }
  }
  // ANR_SDF_WG32 (read per call, default 1): the exact weight gradients on k_wgrad_f32 instead of k_gemm_t's
  // atomic split-K (~4.7 M fp32 atomics per 36k-row 256 x 256 product)
  const char* wg32_env = getenv("ANR_SDF_WG32");
  g.wg32 = !(wg32_env && wg32_env[0] == '0');
  g.slab = F(L.wslab);
  const dim3 pb(256), pg((n + 255) / 256 + 1);
  auto WN = [&](int l) { return (const float*)wimg + wn_layer(l).off; };
  float* dWe = F(L.dWe);
  auto dWN = [&](int l) { return dWe + wn_layer(l).off; };
  const size_t S2 = (size_t)2 * N * 256;  // one stacked [2N][256] activation
  auto Hr = [&](int l) { return F(L.Hr) + (size_t)l * S2; };
  auto Hs = [&](int l) { return F(L.Hs) + (size_t)l * S2; };  // l = 3: X4 = [h3, gamma_6] / sqrt2
  auto Dl = [&](int l) { return F(L.D) + (size_t)l * N * 256; };
  auto Hc = [&](int l) { return F(L.Hc) + (size_t)l * N * 256; };
  const float* Wr[8];
  for (int l = 0; l < 8; ++l) Wr[l] = tp[SDF_RLIN0 + 2 * l];
  const int rin[8] = {135, 256, 256, 256, 256, 391, 256, 256};

  SdfPointArgs a{};
  a.list = ca.list; a.b0 = 0; a.cnt = n;
  a.ray_o = ray_o; a.ray_d = ray_d; a.near_ = near_; a.far_ = far_; a.t_rand = o->t_rand; a.chunk = C.chunk;
  a.wpts = C.wpts; a.vdir = C.vdir; a.n_pts = C.n_pts;
  a.R = f->R; a.Th = f->Th; a.A = f->A; a.bigA = f->big_A; a.weights = f->weights; a.knn = fa.knn;
  a.wimg = wimg; a.tbtab = tbtab;
  a.ptb = F(L.ptb); a.Gr = F(L.Gr); a.Yr = F(L.Yr); a.Xs0 = F(L.Xs0); a.X4 = Hs(3); a.C0 = F(L.C0);
  a.D7 = Dl(7); a.G7 = F(L.Ga); a.Gc = F(L.Gc); a.gB = F(L.gB); a.Y8 = F(L.Y8); a.Yc = F(L.Yc); a.beta = 0.f;
  a.resd_rows = F(L.resd); a.grad_rows = F(L.grow); a.raw = raw; a.sdf = sdf;

  // residual MLP forward on n rows (primal half of Hr); poses folded into the biases of layers 0, 5
  auto resd_forward = [&](int m, const float* G, float* Y) -> int {
    part(1);
    Epi r;
    r.relu = 1;
    ANR_TRY(g.fwd(m, Hr(0), 256, 256, Wr[0], 135, fold, G, 64, 63, 0, r));
    for (int l = 1; l < 8; ++l) {
      if (l == 5) ANR_TRY(g.fwd(m, Hr(5), 256, 256, Wr[5], 391, fold + 256, G, 64, 63, 0, r, Hr(4), 256, 256, 135));
      else ANR_TRY(g.fwd(m, Hr(l), 256, 256, Wr[l], 256, tp[SDF_RLIN0 + 2 * l + 1], Hr(l - 1), 256, 256, 0, r));
    }
    return g.fwd(m, Y, 4, 3, tp[SDF_RFC_W], 256, tp[SDF_RFC_B], Hr(7), 256, 256, 0);
  };
  // SDF forward on m rows with the stored softplus factors (lin8 into Y8 when given)
  auto sdf_forward = [&](int m, float* Y8) -> int {
    part(2);
    Epi e;
    e.softplus = true;
    const float* hin = F(L.Xs0);
    long ldin = 40;
    for (int l = 0; l < 8; ++l) {
      e.deriv = Dl(l);
      if (l == 3) {
        Epi e3 = e;
        e3.div_post = SQRT2;
        ANR_TRY(g.fwd(m, Hs(3), 256, 217, WN(3), 256, tp[9], hin, 256, 256, 0, e3));
      } else {
        ANR_TRY(g.fwd(m, Hs(l), 256, 256, WN(l), l == 0 ? 39 : 256, tp[3 * l], hin, ldin, l == 0 ? 39 : 256, 0, e));
      }
      hin = Hs(l);
      ldin = 256;
    }
    if (Y8) ANR_TRY(g.fwd(m, Y8, 264, 257, WN(8), 256, tp[24], Hs(7), 256, 256, 0));
    return ANR_OK;
  };
  // first-order input gradient of the SDF (the eval path's reverse chain): gradients -> C0[:, 30:33]
  auto sdf_input_grad = [&](SdfPointArgs& pa, int m) -> int {
    if (m <= 0) return ANR_OK;
    part(4);
    pa.cnt = m;
    pa.d7_h = 0;
    hipLaunchKernelGGL(k_sdf_gtop, dim3((unsigned)(((long)m * 256 + 255) / 256)), pb, 0, s, pa);
    ANR_TRY(check_launch("k_sdf_gtop (train)"));
    auto bwd = [&](float* dX, int K, const float* dY, int Nout, const float* W, int in_ch, const float* spd, int spd_n,
                   float div_pre) {
      GemmArgs q{};
      q.N = K; q.nseg = 1; q.seg[0] = GemmSeg{dY, 256, 1, W, in_ch, 1, Nout};
      q.C = dX; q.ldc = K == 39 ? 40 : 256; q.spd = spd; q.ldsd = 256; q.spd_n = spd_n; q.div_pre = div_pre;
      return g.run(q, m);
    };
    float *Ga = F(L.Ga), *Gb = F(L.Gb), *Gc = F(L.Gc);
    ANR_TRY(bwd(Gb, 256, Ga, 256, WN(7), 256, Dl(6), 256, 0.f));
    ANR_TRY(bwd(Ga, 256, Gb, 256, WN(6), 256, Dl(5), 256, 0.f));
    ANR_TRY(bwd(Gb, 256, Ga, 256, WN(5), 256, Dl(4), 256, 0.f));
    ANR_TRY(bwd(Gc, 256, Gb, 256, WN(4), 256, Dl(3), 217, SQRT2));
    ANR_TRY(bwd(Ga, 256, Gc, 217, WN(3), 256, Dl(2), 256, 0.f));
    ANR_TRY(bwd(Gb, 256, Ga, 256, WN(2), 256, Dl(1), 256, 0.f));
    ANR_TRY(bwd(Ga, 256, Gb, 256, WN(1), 256, Dl(0), 256, 0.f));
    ANR_TRY(bwd(F(L.gB), 39, Ga, 256, WN(0), 39, nullptr, 0, 0.f));
    hipLaunchKernelGGL(k_sdf_gamma_bwd, dim3((m + 255) / 256), pb, 0, s, pa);
    return check_launch("k_sdf_gamma_bwd (train)");
  };
  // tangent forward of the SDF from the input tangent tdot (n,4): tangent rows of Xs0 / Hs
  auto sdf_tangent = [&](int m, const float* t, long ldt, const float* td) -> int {
    part(16);
    float* Xt = F(L.Xs0) + (size_t)m * 40;
    hipLaunchKernelGGL(k_st_embed_tan, dim3((unsigned)(((long)m * 39 + 255) / 256)), pb, 0, s, t, ldt, td, 4L, 6, m, Xt,
                       40L, 0, 1.f);
    hipLaunchKernelGGL(k_st_embed_tan, dim3((unsigned)(((long)m * 39 + 255) / 256)), pb, 0, s, t, ldt, td, 4L, 6, m,
                       Hs(3) + (size_t)m * 256, 256L, 217, 1.f / SQRT2);
    ANR_TRY(check_launch("k_st_embed_tan"));
    const float* hin = Xt;
    long ldin = 40;
    for (int l = 0; l < 8; ++l) {
      Epi e;
      e.spd = Dl(l);
      e.spd_n = l == 3 ? 217 : 256;
      if (l == 3) e.div_post = SQRT2;
      ANR_TRY(g.fwd(m, Hs(l) + (size_t)m * 256, 256, l == 3 ? 217 : 256, WN(l), l == 0 ? 39 : 256, nullptr, hin, ldin,
                    l == 0 ? 39 : 256, 0, e));
      hin = Hs(l) + (size_t)m * 256;
      ldin = 256;
    }
    return ANR_OK;
  };
  // reverse of the SDF over the stacked [primal; tangent] rows. Z8 (m x 257, ld 264) = lin8's output
  // adjoint (NULL = 0); the tangent output adjoint is e0 (the directional derivative of sdf).
  // -> dW (effective) / bias grads, tbar (+=, (m,4)), ttbar ((m,4), or NULL)
  auto sdf_reverse = [&](int m, const float* Z8, const float* t, long ldt, const float* td, float* tbar,
                         float* ttbar) -> int {
    part(32);
    float* Ab = F(L.Ab);
    float* Zb = F(L.Zb);
    float* AX4 = F(L.AX4);
    float* Ain = F(L.Ain);
    // lin8: primal dW / bias from Z8, tangent row 0 from the column sums of hdot7; A7 = Z8 W8
    if (Z8) {
      ANR_TRY(g.wgrad(m, dWN(8), 256, 0, 257, Z8, 264, Hs(7), 256, 256, grads[24]));
      ANR_TRY(g.xgrad(m, Ab, 256, 256, Z8, 264, 257, WN(8), 256, 0));
    }
    hipLaunchKernelGGL(k_st_colsum, dim3(std::min(1024, m)), dim3(256), 0, s, (const float*)(Hs(7) + (size_t)m * 256),
                       256L, m, dWN(8));
    ANR_TRY(check_launch("k_st_colsum"));
    const float* Aprim = Z8 ? Ab : nullptr;
    const float* Atan = WN(8);  // row 0 of W8, broadcast
    long ldat = 0;
    for (int l = 7; l >= 0; --l) {
      const int width = l == 3 ? 217 : 256;
      const float sc = l == 3 ? 1.f / SQRT2 : 1.f;
      const float* Hd = Hs(l) + (size_t)m * 256;
      hipLaunchKernelGGL(k_st_sp_rev, dim3((unsigned)(((long)m * width + 255) / 256)), pb, 0, s, Aprim, 256L, Atan, ldat,
                         sc, (const float*)Dl(l), Hd, 256L, l == 3 ? SQRT2 : 1.f, m, width, Zb);
      ANR_TRY(check_launch("k_st_sp_rev"));
      const int in_ch = l == 0 ? 39 : 256;
      const float* Xp = l == 0 ? F(L.Xs0) : Hs(l - 1);
      const long ldx = l == 0 ? 40 : 256;
      ANR_TRY(g.wgrad(m, dWN(l), in_ch, 0, width, Zb, 256, Xp, ldx, in_ch, grads[3 * l]));
      ANR_TRY(g.wgrad(m, dWN(l), in_ch, 0, width, Zb + (size_t)m * 256, 256, Xp + (size_t)m * ldx, ldx, in_ch));
      float* Aout = l == 0 ? Ain : (l == 4 ? AX4 : Ab);
      ANR_TRY(g.xgrad(2 * m, Aout, l == 0 ? 40 : 256, in_ch, Zb, 256, width, WN(l), in_ch, 0));
      Aprim = l == 4 ? AX4 : Ab;
      Atan = Aprim + (size_t)m * 256;
      ldat = 256;
    }
    hipLaunchKernelGGL(k_st_embed_rev6, dim3((m + 255) / 256), pb, 0, s, t, ldt, td, 4L, (const float*)Ain,
                       (const float*)AX4, m, tbar, ttbar);
    return check_launch("k_st_embed_rev6");
  };

  if (pts) {
    // ---- the network's point helpers (anr_sdf_points): every point is a row, x in big-pose space
    const dim3 og_((n + 255) / 256);
    SdfPointArgs ao = a;
    ao.list = nullptr; ao.cnt = n; ao.ptb = F(L.ptbo); ao.Gr = F(L.Gro); ao.Yr = F(L.Yr); ao.resd_rows = F(L.ro);
    ao.grad_rows = F(L.gro);
    hipLaunchKernelGGL(k_st_pts_rows, og_, pb, 0, s, C.wpts, n, F(L.ptbo), F(L.Gro));
    ANR_TRY(check_launch("k_st_pts_rows"));
    const bool deformed = C.pts_mode == ANR_SDFP_DEFORMED_GRADIENT;
    if (deformed) {
      ANR_TRY(resd_forward(n, F(L.Gro), F(L.Yr)));  // tpose = x + 0.05 tanh(resd_fc) (k_sdf_mid)
    } else if (hipMemsetAsync(F(L.Yr), 0, (size_t)n * 16, s) != hipSuccess) {  // tanh(0) = 0: tpose = x exactly
      return fail(ANR_E_HIP, "memset");
    }
    hipLaunchKernelGGL(k_sdf_mid, og_, pb, 0, s, ao);
    ANR_TRY(check_launch("k_sdf_mid (points)"));
    ANR_TRY(sdf_forward(n, F(L.Y8)));
    if (C.pts_mode == ANR_SDFP_NETWORK) {  // [sdf / scale (scale 1) || feature]
      if (hipMemcpy2DAsync(C.pts_out, 257 * 4, F(L.Y8), 264 * 4, 257 * 4, (size_t)n, hipMemcpyDeviceToDevice, s) !=
          hipSuccess)
        return fail(ANR_E_HIP, "anr_sdf_points: copy");
      return ANR_OK;
    }
    ANR_TRY(sdf_input_grad(ao, n));  // d sdf / d tpose -> C0[:, 30:33]
    const float* gout = F(L.C0) + 30;
    long ldg = 40;
    if (deformed) {  // og = g_t + J_resd^T g_t, as the observed-gradient pass below
      part(1);
      float *dHa = F(L.dHa), *dHb = F(L.dHb), *Gbar = F(L.Gbar);
      float* yb = F(L.Yd);
      hipLaunchKernelGGL(k_st_add3, og_, pb, 0, s, (const float*)(F(L.C0) + 30), 40L, (const float*)(ws + L.zero), 0L, n,
                         F(L.tdot));
      hipLaunchKernelGGL(k_st_tanh_rev, og_, pb, 0, s, (const float*)F(L.Yr), (const float*)nullptr,
                         (const float*)F(L.tdot), (const float*)nullptr, (const float*)nullptr, n, yb);
      ANR_TRY(g.xgrad(n, dHa, 256, 256, yb, 4, 3, tp[SDF_RFC_W], 256, 0, Hr(7), 256));
      float* cur = dHa;
      float* nxt = dHb;
      for (int l = 7; l >= 1; --l) {
        if (l == 5) {
          ANR_TRY(g.xgrad(n, Gbar, 64, 63, cur, 256, 256, Wr[5], 391, 0));
          ANR_TRY(g.xgrad(n, nxt, 256, 256, cur, 256, 256, Wr[5], 391, 135, Hr(4), 256));
        } else {
          ANR_TRY(g.xgrad(n, nxt, 256, 256, cur, 256, 256, Wr[l], 256, 0, Hr(l - 1), 256));
        }
        std::swap(cur, nxt);
      }
      ANR_TRY(g.xgrad(n, Gbar, 64, 63, cur, 256, 256, Wr[0], 135, 0, nullptr, 0, true));
      float* og = F(L.og);
      hipLaunchKernelGGL(k_st_embed_bwd10, og_, pb, 0, s, (const float*)F(L.ptbo), 8L, (const float*)Gbar, 64L, n, og, 4L);
      hipLaunchKernelGGL(k_st_add3, og_, pb, 0, s, (const float*)F(L.tdot), 4L, (const float*)og, 4L, n, og);
      ANR_TRY(check_launch("anr_sdf_points: deformed gradient"));
      gout = og;
      ldg = 4;
    }
    if (hipMemcpy2DAsync(C.pts_out, 12, gout, ldg * 4, 12, (size_t)n, hipMemcpyDeviceToDevice, s) != hipSuccess ||
        (C.pts_out2 && hipMemcpy2DAsync(C.pts_out2, 4, F(L.Y8), 264 * 4, 4, (size_t)n, hipMemcpyDeviceToDevice, s) != hipSuccess))
      return fail(ANR_E_HIP, "anr_sdf_points: copy");
    return ANR_OK;
  }

  if (n > 0) {
    // ---- forward: B2/B3 residual deformation, B4 SDF + its input gradient, B6 colour, B5 raw
    hipLaunchKernelGGL(k_sdf_prep, pg, pb, 0, s, a);
    ANR_TRY(check_launch("k_sdf_prep (train)"));
    ANR_TRY(resd_forward(n, F(L.Gr), F(L.Yr)));
    hipLaunchKernelGGL(k_sdf_mid, pg, pb, 0, s, a);
    ANR_TRY(check_launch("k_sdf_mid (train)"));
    ANR_TRY(sdf_forward(n, F(L.Y8)));
    ANR_TRY(sdf_input_grad(a, n));
    {
      part(8);
      Epi r;
      r.relu = 1;
      ANR_TRY(g.fwd(n, Hc(0), 256, 256, WN(9), 289, tp[29], F(L.C0), 40, 33, 0, r, F(L.Y8) + 1, 264, 256, 33));
      ANR_TRY(g.fwd(n, Hc(1), 256, 256, WN(10), 256, tp[32], Hc(0), 256, 256, 0, r));
      ANR_TRY(g.fwd(n, Hc(2), 256, 256, WN(11), 256, tp[35], Hc(1), 256, 256, 0, r));
      ANR_TRY(g.fwd(n, Hc(3), 256, 256, WN(12), 384, fold + 512, Hc(2), 256, 256, 0, r));
      ANR_TRY(g.fwd(n, F(L.Yc), 4, 3, WN(13), 256, tp[41], Hc(3), 256, 256, 0));
    }
    // k_sdf_raw reads beta from the host struct: pass it through the device scalar instead
    float beta_h = 0.f;
    if (hipMemcpyAsync(&beta_h, tp[SDF_BETA], 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return fail(ANR_E_HIP, "sdf train: beta readback");
    a.beta = beta_h;
    hipLaunchKernelGGL(k_sdf_raw, pg, pb, 0, s, a);
    ANR_TRY(check_launch("k_sdf_raw (train)"));
  }
  float alpha = 50.f;
  const float4* draw = (const float4*)F(L.draw);
  if (step) {
    // compositing, image loss and d rgb_map
    const anr_sdf_render_out* out = C.out;
    const anr_render_out ro{out->rgb_map, out->acc_map, out->depth_map, nullptr};
    ANR_TRY(stage_composite(near_, far_, R, o, raw, &ro, nullptr, s));
    TrainBufs tb{};
    tb.raw = raw; tb.draw = (float4*)F(L.draw); tb.n_rays = R; tb.rgb_map = out->rgb_map; tb.d_rgb_map = F(L.drgb);
    tb.n_kept = counts;
    const int gx = (R + 255) / 256;
    hipLaunchKernelGGL(k_tr_loss, dim3(gx, 1), dim3(256), 0, s, tb, C.rgb_gt, C.mask_at_box, acc3);
    hipLaunchKernelGGL(k_tr_loss_grads, dim3(gx, 1), dim3(256), 0, s, tb, C.rgb_gt, C.mask_at_box, (const float*)acc3,
                       F(L.drgb), nullptr, nullptr);
    hipLaunchKernelGGL(k_tr_composite_bwd, dim3((R + 3) / 4), dim3(256), 0, s, tb);
    ANR_TRY(check_launch("sdf train: image loss / compositing backward"));
    // msk_sdf lists: per-ray min / argmin / flags, entry count
    hipLaunchKernelGGL(k_st_msk_rays, dim3((R + 3) / 4), dim3(256), 0, s, (const float*)sdf, f->occupancy, R, F(L.rmin),
                       (int*)(ws + L.ramin), (uint8_t*)(ws + L.rflag), acc);
    ANR_TRY(check_launch("k_st_msk_rays"));
    for (int m : {10000, 20000, 30000, 40000, 50000})
      if (C.iter_step > m) alpha *= 2.f;
  } else if (!net_fwd) {
    if (C.d_raw) {
      draw = (const float4*)C.d_raw;
    } else if (hipMemsetAsync(F(L.draw), 0, (size_t)N * 16, s) != hipSuccess) {
      return fail(ANR_E_HIP, "memset");
    }
  }

  bool colour_wn = false;  // the colour net's weight-norm gradients converted (after its backward)
  if (n > 0 && !net_fwd) {
    // ---- backward: raw -> colour logits, sdf, beta; msk_sdf -> sdf
    StRaw sr{};
    sr.list = ca.list; sr.n_kept = counts; sr.chunk = C.chunk; sr.draw = draw;
    sr.C0 = F(L.C0); sr.tbtab = tbtab; sr.Y8 = F(L.Y8); sr.Yc = F(L.Yc); sr.beta = tp[SDF_BETA];
    sr.dYc = F(L.dYc); sr.ds = F(L.ds); sr.dbeta = F(L.dbeta);
    hipLaunchKernelGGL(k_st_raw_bwd, pg, pb, 0, s, sr);
    if (step)
      hipLaunchKernelGGL(k_st_msk_loss, dim3((R + 255) / 256), pb, 0, s, (const float*)F(L.rmin),
                         (const int*)(ws + L.ramin), (const uint8_t*)(ws + L.rflag), (const int*)inv, R, alpha, F(L.ds),
                         acc);
    else if (C.d_sdf)
      hipLaunchKernelGGL(k_st_cotan_sdf, pg, pb, 0, s, (const int*)ca.list, (const int*)counts, C.d_sdf, F(L.ds));
    ANR_TRY(check_launch("sdf train: raw / msk backward"));
    // ---- colour net backward (weight-normed lin4..lin0; color_latent folded into lin3)
    part(8);
    float *dHa = F(L.dHa), *dHb = F(L.dHb), *bsum = F(L.bsum);
    ANR_TRY(g.wgrad(n, dWN(13), 256, 0, 3, F(L.dYc), 4, Hc(3), 256, 256, grads[41]));
    ANR_TRY(g.xgrad(n, dHa, 256, 256, F(L.dYc), 4, 3, WN(13), 256, 0, Hc(3), 256));
    if (hipMemsetAsync(bsum, 0, 256 * 4, s) != hipSuccess) return fail(ANR_E_HIP, "memset");
    ANR_TRY(g.wgrad(n, dWN(12), 384, 0, 256, dHa, 256, Hc(2), 256, 256, bsum));
    hipLaunchKernelGGL(k_tr_latent_grad, dim3(256 + 128), dim3(128), 0, s, (const float*)bsum, WN(12), 384, 256, 256,
                       tp[SDF_COLOR_LAT], f->latent_index, 0, dWN(12), grads[SDF_COLOR_LAT]);
    ANR_TRY(check_launch("k_tr_latent_grad (colour)"));
    hipLaunchKernelGGL(k_st_add_bias, dim3(1), dim3(256), 0, s, (const float*)bsum, 256, grads[38]);
    ANR_TRY(g.xgrad(n, dHb, 256, 256, dHa, 256, 256, WN(12), 384, 0, Hc(2), 256));
    ANR_TRY(g.wgrad(n, dWN(11), 256, 0, 256, dHb, 256, Hc(1), 256, 256, grads[35]));
    ANR_TRY(g.xgrad(n, dHa, 256, 256, dHb, 256, 256, WN(11), 256, 0, Hc(1), 256));
    ANR_TRY(g.wgrad(n, dWN(10), 256, 0, 256, dHa, 256, Hc(0), 256, 256, grads[32]));
    ANR_TRY(g.xgrad(n, dHb, 256, 256, dHa, 256, 256, WN(10), 256, 0, Hc(0), 256));
    ANR_TRY(g.wgrad(n, dWN(9), 289, 0, 256, dHb, 256, F(L.C0), 40, 33, grads[29]));
    ANR_TRY(g.wgrad(n, dWN(9), 289, 33, 256, dHb, 256, F(L.Y8) + 1, 264, 256));
    ANR_TRY(g.xgrad(n, F(L.dC0), 40, 33, dHb, 256, 256, WN(9), 289, 0));
    ANR_TRY(g.xgrad(n, F(L.dZ8) + 1, 264, 256, dHb, 256, 256, WN(9), 289, 33));
    // the colour net's weight-norm gradients now (nothing after this point reaches tensors 28..43: the
    // SDF, residual and observed passes below touch the SDF and residual weights only), so the caller can
    // all-reduce them while the rest of the backward runs (anr_sdf_train_step_hooked)
    for (int l = 9; l < SDF_NUM_WN; ++l) {
      const WnLayer d = wn_layer(l);
      hipLaunchKernelGGL(k_st_wn_grad, dim3(d.out), dim3(256), 0, s, tp[d.v], tp[d.g], (const float*)dWN(l), d.in,
                         grads[d.g], grads[d.v]);
    }
    ANR_TRY(check_launch("k_st_wn_grad (colour)"));
    colour_wn = true;
    if (C.hooks) {
      hipEvent_t ev = (hipEvent_t)C.hooks->colour_grads_ready;
      if (ev && hipEventRecord(ev, s) != hipSuccess) return fail(ANR_E_HIP, "colour event record");
      if (C.hooks->colour_ready && C.hooks->colour_ready(C.hooks->user, (void*)ev, (void*)s) != 0)
        return fail(ANR_E_ARG, "anr_sdf_train_hooks.colour_ready failed");
    }
    // ---- loss adjoints of resd (offset) and gradients (eikonal + colour normals); d sdf into Z8 col 0
    if (step) {
      StLoss sl{};
      sl.n_kept = counts; sl.resd = F(L.resd); sl.C0 = F(L.C0); sl.dC0 = F(L.dC0); sl.ds = F(L.ds);
      sl.rbar = F(L.rbar); sl.dG = F(L.dG); sl.dZ8 = F(L.dZ8); sl.acc = acc;
      hipLaunchKernelGGL(k_st_sample_loss, pg, pb, 0, s, sl);
    } else {
      hipLaunchKernelGGL(k_st_cotan_rows, pg, pb, 0, s, (const int*)counts, C.d_resd, C.d_grad, (const float*)F(L.dC0),
                         (const float*)F(L.ds), F(L.rbar), F(L.dG), F(L.dZ8));
    }
    ANR_TRY(check_launch("k_st_sample_loss"));
    // ---- SDF: tangent pass along dG, stacked reverse -> SDF weights, d tpose
    if (hipMemsetAsync(F(L.tbar), 0, (size_t)n * 16, s) != hipSuccess) return fail(ANR_E_HIP, "memset");
    ANR_TRY(sdf_tangent(n, F(L.C0), 40, F(L.dG)));
    ANR_TRY(sdf_reverse(n, F(L.dZ8), F(L.C0), 40, F(L.dG), F(L.tbar), nullptr));
    // ---- residual net: r_bar = t_bar + offset adjoint -> tanh -> ReLU layers (first order)
    part(1);
    float* yb = F(L.Yd);
    hipLaunchKernelGGL(k_st_tanh_rev, pg, pb, 0, s, (const float*)F(L.Yr), (const float*)nullptr,
                       (const float*)F(L.tbar), (const float*)F(L.rbar), (const float*)nullptr, n, yb);
    ANR_TRY(check_launch("k_st_tanh_rev"));
    ANR_TRY(g.wgrad(n, grads[SDF_RFC_W], 256, 0, 3, yb, 4, Hr(7), 256, 256, grads[SDF_RFC_B]));
    ANR_TRY(g.xgrad(n, dHa, 256, 256, yb, 4, 3, tp[SDF_RFC_W], 256, 0, Hr(7), 256));
    float* cur = dHa;
    float* nxt = dHb;
    for (int l = 7; l >= 0; --l) {
      float* dW = grads[SDF_RLIN0 + 2 * l];
      float* db = grads[SDF_RLIN0 + 2 * l + 1];
      if (l == 0 || l == 5) {
        if (hipMemsetAsync(bsum, 0, 256 * 4, s) != hipSuccess) return fail(ANR_E_HIP, "memset");
        ANR_TRY(g.wgrad(n, dW, rin[l], 0, 256, cur, 256, F(L.Gr), 64, 63, bsum));
        hipLaunchKernelGGL(k_st_outer_add, dim3(256), dim3(128), 0, s, (const float*)bsum, f->poses, 72, 256, dW, rin[l], 63);
        hipLaunchKernelGGL(k_st_add_bias, dim3(1), dim3(256), 0, s, (const float*)bsum, 256, db);
        ANR_TRY(check_launch("sdf train: residual folded columns"));
        if (l == 5) {
          ANR_TRY(g.wgrad(n, dW, 391, 135, 256, cur, 256, Hr(4), 256, 256));
          ANR_TRY(g.xgrad(n, nxt, 256, 256, cur, 256, 256, Wr[5], 391, 135, Hr(4), 256));
        }
      } else {
        ANR_TRY(g.wgrad(n, dW, 256, 0, 256, cur, 256, Hr(l - 1), 256, 256, db));
        ANR_TRY(g.xgrad(n, nxt, 256, 256, cur, 256, 256, Wr[l], 256, 0, Hr(l - 1), 256));
      }
      std::swap(cur, nxt);
    }
  }

  // ---- observed gradients (anisdf_pdf_network.py:194-199, 140-154): samples with |sdf| < 0.02
  int n_o = 0;
  if (n > 0) {
    const int nbo = (n + 255) / 256;
    int* oblock = (int*)(ws + L.oblock);
    hipLaunchKernelGGL(k_st_obs_count, dim3(nbo), pb, 0, s, (const float*)F(L.Y8), (const int*)counts, oblock);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, oblock, nbo, counts + 2);
    hipLaunchKernelGGL(k_st_obs_gather, dim3(nbo), pb, 0, s, (const float*)F(L.Y8), (const int*)counts,
                       (const int*)oblock, (const float*)F(L.ptb), (const float*)F(L.Gr), F(L.ptbo), F(L.Gro));
    ANR_TRY(check_launch("sdf train: observed rows"));
    ANR_TRY(read_int(counts + 2, &n_o, s));
  }
  if (n_o > 0) {
    const dim3 og_((n_o + 255) / 256);
    // forward: x_o -> resd -> t_o -> SDF (factors) -> g_t = grad_t sdf; og = g_t + J_resd^T g_t
    SdfPointArgs ao = a;
    ao.cnt = n_o; ao.ptb = F(L.ptbo); ao.Gr = F(L.Gro); ao.Yr = F(L.Yr); ao.resd_rows = F(L.ro);
    ao.grad_rows = F(L.gro);  // (not read: the main pass's gradient rows stay the call's output)
    ANR_TRY(resd_forward(n_o, F(L.Gro), F(L.Yr)));
    hipLaunchKernelGGL(k_sdf_mid, og_, pb, 0, s, ao);
    ANR_TRY(check_launch("k_sdf_mid (observed)"));
    ANR_TRY(sdf_forward(n_o, nullptr));
    ANR_TRY(sdf_input_grad(ao, n_o));
    part(1);
    float *dHa = F(L.dHa), *dHb = F(L.dHb), *Gbar = F(L.Gbar);
    float* yb = F(L.Yd);
    // y_bar = 0.05 (1 - tau^2) g_t; reverse of the ReLU net to its gamma_10 input (input gradient only)
    hipLaunchKernelGGL(k_st_add3, og_, pb, 0, s, (const float*)(F(L.C0) + 30), 40L, (const float*)(ws + L.zero), 0L, n_o,
                       F(L.tdot));
    hipLaunchKernelGGL(k_st_tanh_rev, og_, pb, 0, s, (const float*)F(L.Yr), (const float*)nullptr,
                       (const float*)F(L.tdot), (const float*)nullptr, (const float*)nullptr, n_o, yb);
    ANR_TRY(g.xgrad(n_o, dHa, 256, 256, yb, 4, 3, tp[SDF_RFC_W], 256, 0, Hr(7), 256));
    float* cur = dHa;
    float* nxt = dHb;
    for (int l = 7; l >= 1; --l) {
      if (l == 5) {
        ANR_TRY(g.xgrad(n_o, Gbar, 64, 63, cur, 256, 256, Wr[5], 391, 0));
        ANR_TRY(g.xgrad(n_o, nxt, 256, 256, cur, 256, 256, Wr[5], 391, 135, Hr(4), 256));
      } else {
        ANR_TRY(g.xgrad(n_o, nxt, 256, 256, cur, 256, 256, Wr[l], 256, 0, Hr(l - 1), 256));
      }
      std::swap(cur, nxt);
    }
    ANR_TRY(g.xgrad(n_o, Gbar, 64, 63, cur, 256, 256, Wr[0], 135, 0, nullptr, 0, true));
    float* og = F(L.og);
    hipLaunchKernelGGL(k_st_embed_bwd10, og_, pb, 0, s, (const float*)F(L.ptbo), 8L, (const float*)Gbar, 64L, n_o, og, 4L);
    hipLaunchKernelGGL(k_st_add3, og_, pb, 0, s, (const float*)F(L.tdot), 4L, (const float*)og, 4L, n_o, og);
    if (net_fwd) return ANR_OK;  // og (n_o, 4) is an output of the call; the backward re-runs this
    if (step)
      hipLaunchKernelGGL(k_st_obs_loss, og_, pb, 0, s, (const float*)og, n_o, F(L.dog), acc);
    else
      hipLaunchKernelGGL(k_st_rows3to4, og_, pb, 0, s, C.d_og, n_o, F(L.dog));
    ANR_TRY(check_launch("sdf train: observed-gradient loss"));
    // tangent forward along dog: gamma_10 -> ReLU net (masks of the primal) -> tanh -> tdot -> SDF
    float* Grt = F(L.Grt);
    if (hipMemsetAsync(Grt, 0, (size_t)n_o * 64 * 4, s) != hipSuccess) return fail(ANR_E_HIP, "memset");
    hipLaunchKernelGGL(k_st_embed_tan, dim3((unsigned)(((long)n_o * 63 + 255) / 256)), pb, 0, s, (const float*)F(L.ptbo),
                       8L, (const float*)F(L.dog), 4L, 10, n_o, Grt, 64L, 0, 1.f);
    ANR_TRY(check_launch("k_st_embed_tan (gamma_10)"));
    auto HrT = [&](int l) { return Hr(l) + (size_t)n_o * 256; };
    {
      Epi e;
      e.mask = Hr(0); e.ldm = 256;
      ANR_TRY(g.fwd(n_o, HrT(0), 256, 256, Wr[0], 135, nullptr, Grt, 64, 63, 0, e));
      for (int l = 1; l < 8; ++l) {
        e.mask = Hr(l);
        if (l == 5) ANR_TRY(g.fwd(n_o, HrT(5), 256, 256, Wr[5], 391, nullptr, Grt, 64, 63, 0, e, HrT(4), 256, 256, 135));
        else ANR_TRY(g.fwd(n_o, HrT(l), 256, 256, Wr[l], 256, nullptr, HrT(l - 1), 256, 256, 0, e));
      }
    }
    float* Yd = F(L.Yr) + (size_t)n_o * 4;  // ydot in the stacked Yr rows
    ANR_TRY(g.fwd(n_o, Yd, 4, 3, tp[SDF_RFC_W], 256, nullptr, HrT(7), 256, 256, 0));
    hipLaunchKernelGGL(k_st_resd_tan, og_, pb, 0, s, (const float*)F(L.Yr), (const float*)Yd, (const float*)F(L.dog), n_o,
                       F(L.tdot));
    ANR_TRY(check_launch("k_st_resd_tan"));
    ANR_TRY(sdf_tangent(n_o, F(L.C0), 40, F(L.tdot)));
    // stacked reverse: SDF (output adjoint: tangent e0 only) -> t_bar, tdot_bar -> tanh -> ReLU net
    float* tbar = F(L.tbar);
    float* ttbar = F(L.ttbar);
    if (hipMemsetAsync(tbar, 0, (size_t)n_o * 16, s) != hipSuccess) return fail(ANR_E_HIP, "memset");
    ANR_TRY(sdf_reverse(n_o, nullptr, F(L.C0), 40, F(L.tdot), tbar, ttbar));
    part(1);
    float* ybs = F(L.Ab);  // [2 n_o][4]: y_bar, ydot_bar (the SDF adjoint buffer is free again)
    hipLaunchKernelGGL(k_st_tanh_rev, og_, pb, 0, s, (const float*)F(L.Yr), (const float*)Yd, (const float*)tbar,
                       (const float*)nullptr, (const float*)ttbar, n_o, ybs);
    ANR_TRY(check_launch("k_st_tanh_rev (observed)"));
    const float* ybt = ybs + (size_t)n_o * 4;
    float* bsum = F(L.bsum);
    ANR_TRY(g.wgrad(n_o, grads[SDF_RFC_W], 256, 0, 3, ybs, 4, Hr(7), 256, 256, grads[SDF_RFC_B]));
    ANR_TRY(g.wgrad(n_o, grads[SDF_RFC_W], 256, 0, 3, ybt, 4, HrT(7), 256, 256));
    float* Zr = F(L.Zb);  // stacked [2 n_o][256] ReLU-layer adjoints: z_bar rows then zdot_bar rows
    float* Zr2 = F(L.AX4);
    ANR_TRY(g.xgrad(n_o, Zr, 256, 256, ybs, 4, 3, tp[SDF_RFC_W], 256, 0, Hr(7), 256));
    ANR_TRY(g.xgrad(n_o, Zr + (size_t)n_o * 256, 256, 256, ybt, 4, 3, tp[SDF_RFC_W], 256, 0, Hr(7), 256));
    for (int l = 7; l >= 0; --l) {
      float* dW = grads[SDF_RLIN0 + 2 * l];
      float* db = grads[SDF_RLIN0 + 2 * l + 1];
      const float* Zt = Zr + (size_t)n_o * 256;
      if (l == 0 || l == 5) {
        if (hipMemsetAsync(bsum, 0, 256 * 4, s) != hipSuccess) return fail(ANR_E_HIP, "memset");
        ANR_TRY(g.wgrad(n_o, dW, rin[l], 0, 256, Zr, 256, F(L.Gro), 64, 63, bsum));
        ANR_TRY(g.wgrad(n_o, dW, rin[l], 0, 256, Zt, 256, Grt, 64, 63));
        hipLaunchKernelGGL(k_st_outer_add, dim3(256), dim3(128), 0, s, (const float*)bsum, f->poses, 72, 256, dW, rin[l],
                           63);
        hipLaunchKernelGGL(k_st_add_bias, dim3(1), dim3(256), 0, s, (const float*)bsum, 256, db);
        ANR_TRY(check_launch("sdf train: residual folded columns (observed)"));
        if (l == 5) {
          ANR_TRY(g.wgrad(n_o, dW, 391, 135, 256, Zr, 256, Hr(4), 256, 256));
          ANR_TRY(g.wgrad(n_o, dW, 391, 135, 256, Zt, 256, HrT(4), 256, 256));
          ANR_TRY(g.xgrad(n_o, Zr2, 256, 256, Zr, 256, 256, Wr[5], 391, 135, Hr(4), 256));
          ANR_TRY(g.xgrad(n_o, Zr2 + (size_t)n_o * 256, 256, 256, Zt, 256, 256, Wr[5], 391, 135, Hr(4), 256));
        }
      } else {
        ANR_TRY(g.wgrad(n_o, dW, 256, 0, 256, Zr, 256, Hr(l - 1), 256, 256, db));
        ANR_TRY(g.wgrad(n_o, dW, 256, 0, 256, Zt, 256, HrT(l - 1), 256, 256));
        ANR_TRY(g.xgrad(n_o, Zr2, 256, 256, Zr, 256, 256, Wr[l], 256, 0, Hr(l - 1), 256));
        ANR_TRY(g.xgrad(n_o, Zr2 + (size_t)n_o * 256, 256, 256, Zt, 256, 256, Wr[l], 256, 0, Hr(l - 1), 256));
      }
      std::swap(Zr, Zr2);
    }
  }

  if (net_fwd) return ANR_OK;
  // ---- weight norm: effective-weight gradients -> weight_g / weight_v; beta; loss vector
  if (n > 0) {
    for (int l = 0; l < (colour_wn ? 9 : SDF_NUM_WN); ++l) {
      const WnLayer d = wn_layer(l);
      hipLaunchKernelGGL(k_st_wn_grad, dim3(d.out), dim3(256), 0, s, tp[d.v], tp[d.g], (const float*)dWN(l), d.in,
                         grads[d.g], grads[d.v]);
    }
    hipLaunchKernelGGL(k_st_add_bias, dim3(1), dim3(256), 0, s, (const float*)F(L.dbeta), 1, grads[SDF_BETA]);
    ANR_TRY(check_launch("k_st_wn_grad"));
  }
  if (!step) return check_launch("k_st_wn_grad");
  hipLaunchKernelGGL(k_st_loss_final, dim3(1), dim3(1), 0, s, (const float*)acc, (const float*)acc3, (const int*)counts,
                     n_o, alpha, C.loss);
  return check_launch("k_st_loss_final");
}

int check_net(const anr_sdf_params* p, const anr_sdf_frame* f, const anr_samples* x, const anr_render_opts* o, void* ws) {
  if (!p || !f || !x || !o || !ws || !x->wpts || !x->viewdir) return fail(ANR_E_ARG, "sdf network train: NULL argument");
  if (x->n_pts <= 0 || x->n_pts > (1 << 24)) return fail(ANR_E_ARG, "sdf network train: n must be in [1, 2^24]");
  for (int i = 0; i < ANR_SDF_NUM_TENSORS; ++i)
    if (!p->t[i] && i != SDF_RESD_LAT) return fail(ANR_E_ARG, "sdf network train: NULL parameter tensor");
  if (!f->A || !f->big_A || !f->R || !f->Th || !f->poses || !f->pvertices || !f->weights || !f->tbounds ||
      !f->latent_index)
    return fail(ANR_E_ARG, "sdf network train: NULL frame tensor");
  if (f->n_verts <= 0 || f->n_verts > 6912) return fail(ANR_E_ARG, "sdf network train: n_verts must be in [1, 6912]");
  return ANR_OK;
}

TrainCore net_core(int mode, const anr_sdf_params* p, const anr_sdf_frame* f, const anr_samples* x,
                   const anr_render_opts* o, void* ws, size_t ws_bytes, void* stream) {
  TrainCore c{};
  c.mode = mode; c.p = p; c.f = f; c.o = o;
  c.wpts = x->wpts; c.vdir = x->viewdir; c.n_pts = x->n_pts;
  c.R = (x->n_pts + 63) / 64; c.chunk = c.R;
  c.ws = ws; c.ws_bytes = ws_bytes; c.s = (hipStream_t)stream;
  return c;
}

}  // namespace

extern "C" {

size_t anr_sdf_train_workspace_bytes(int n_rays, const anr_render_opts* o) {
  if (n_rays <= 0 || !o || o->chunk <= 0) return 0;
  return stlayout(n_rays, o->chunk).total;
}

int anr_sdf_train_step(const anr_sdf_params* p, float* const* grads, const anr_sdf_frame* f, const float* ray_o,
                       const float* ray_d, const float* near_, const float* far_, int R, const anr_render_opts* o,
                       const float* rgb_gt, const uint8_t* mask_at_box, int iter_step, const anr_sdf_render_out* out,
                       float* loss, void* workspace, size_t ws_bytes, void* stream) {
  ANR_TRY(check_train(p, grads, f, ray_o, ray_d, near_, far_, R, o, rgb_gt, out, loss, workspace));
  TrainCore c{};
  c.mode = STEP; c.p = p; c.grads = grads; c.f = f;
  c.ray_o = ray_o; c.ray_d = ray_d; c.near_ = near_; c.far_ = far_; c.R = R; c.chunk = o->chunk; c.o = o;
  c.rgb_gt = rgb_gt; c.mask_at_box = mask_at_box; c.iter_step = iter_step; c.out = out; c.loss = loss;
  c.ws = workspace; c.ws_bytes = ws_bytes; c.s = (hipStream_t)stream;
  return sdf_train_core(c);
}

int anr_sdf_train_step_hooked(const anr_sdf_params* p, float* const* grads, const anr_sdf_frame* f, const float* ray_o,
                              const float* ray_d, const float* near_, const float* far_, int R, const anr_render_opts* o,
                              const float* rgb_gt, const uint8_t* mask_at_box, int iter_step,
                              const anr_sdf_render_out* out, float* loss, const anr_sdf_train_hooks* hooks,
                              void* workspace, size_t ws_bytes, void* stream) {
  ANR_TRY(check_train(p, grads, f, ray_o, ray_d, near_, far_, R, o, rgb_gt, out, loss, workspace));
  if (hooks && hooks->struct_size != sizeof(anr_sdf_train_hooks))
    return fail(ANR_E_ARG, "anr_sdf_train_step_hooked: hooks->struct_size != sizeof(anr_sdf_train_hooks)");
  TrainCore c{};
  c.mode = STEP; c.p = p; c.grads = grads; c.f = f;
  c.ray_o = ray_o; c.ray_d = ray_d; c.near_ = near_; c.far_ = far_; c.R = R; c.chunk = o->chunk; c.o = o;
  c.rgb_gt = rgb_gt; c.mask_at_box = mask_at_box; c.iter_step = iter_step; c.out = out; c.loss = loss;
  c.hooks = hooks;
  c.ws = workspace; c.ws_bytes = ws_bytes; c.s = (hipStream_t)stream;
  return sdf_train_core(c);
}

size_t anr_sdf_network_train_workspace_bytes(int n_pts) {
  if (n_pts <= 0) return 0;
  const int G = (n_pts + 63) / 64;
  return stlayout(G, G).total;
}

int anr_sdf_network_train_fwd(const anr_sdf_params* p, const anr_sdf_frame* f, const anr_samples* x,
                              const anr_render_opts* o, float* raw, float* sdf, float* tbounds_out, void* workspace,
                              size_t ws_bytes, void* stream) {
  ANR_TRY(check_net(p, f, x, o, workspace));
  if (!raw || !sdf) return fail(ANR_E_ARG, "sdf network train: NULL output");
  TrainCore c = net_core(NET_FWD, p, f, x, o, workspace, ws_bytes, stream);
  c.raw_out = raw; c.sdf_out = sdf; c.tb_out = tbounds_out;
  return sdf_train_core(c);
}

const int32_t* anr_sdf_network_train_counts(const void* workspace, int n_pts) {
  if (!workspace || n_pts <= 0) return nullptr;
  const int G = (n_pts + 63) / 64;
  return (const int32_t*)((const char*)workspace + stlayout(G, G).counts);
}

int anr_sdf_network_train_rows(const void* workspace, int n_pts, float* resd, float* gradients,
                               float* observed_gradients, void* stream) {
  if (!workspace || n_pts <= 0) return fail(ANR_E_ARG, "anr_sdf_network_train_rows: bad arguments");
  const int G = (n_pts + 63) / 64;
  const STLayout L = stlayout(G, G);
  const char* ws = (const char*)workspace;
  hipStream_t s = (hipStream_t)stream;
  int cnt[4];
  if (hipMemcpyAsync(cnt, ws + L.counts, 16, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return fail(ANR_E_HIP, "anr_sdf_network_train_rows: count readback");
  const int n = cnt[0], n_o = cnt[2];
  if (resd && n > 0 && hipMemcpyAsync(resd, ws + L.resd, (size_t)n * 12, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return fail(ANR_E_HIP, "anr_sdf_network_train_rows: copy");
  if (gradients && n > 0 && hipMemcpyAsync(gradients, ws + L.grow, (size_t)n * 12, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return fail(ANR_E_HIP, "anr_sdf_network_train_rows: copy");
  if (observed_gradients && n_o > 0 &&
      hipMemcpy2DAsync(observed_gradients, 12, ws + L.og, 16, 12, (size_t)n_o, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return fail(ANR_E_HIP, "anr_sdf_network_train_rows: copy");
  return ANR_OK;
}

size_t anr_sdf_points_workspace_bytes(int n) {
  if (n <= 0) return 0;
  const int G = (n + 63) / 64;
  return stlayout(G, G).total;
}

int anr_sdf_points(const anr_sdf_params* p, const anr_sdf_frame* f, const float* x, int n, int mode, float* out,
                   float* out2, void* workspace, size_t ws_bytes, void* stream) {
  if (!p || !f || !x || !out || !workspace) return fail(ANR_E_ARG, "anr_sdf_points: NULL argument");
  if (n <= 0 || n > (1 << 24)) return fail(ANR_E_ARG, "anr_sdf_points: n must be in [1, 2^24]");
  if (mode != ANR_SDFP_NETWORK && mode != ANR_SDFP_GRADIENT && mode != ANR_SDFP_DEFORMED_GRADIENT)
    return fail(ANR_E_ARG, "anr_sdf_points: unknown mode");
  for (int i = 0; i < ANR_SDF_NUM_TENSORS; ++i)
    if (!p->t[i] && i != SDF_RESD_LAT) return fail(ANR_E_ARG, "anr_sdf_points: NULL parameter tensor");
  if (!f->poses || !f->latent_index) return fail(ANR_E_ARG, "anr_sdf_points: needs poses and latent_index");
  static const anr_render_opts o0{};  // exact fp32 products
  TrainCore c{};
  c.mode = PTS; c.p = p; c.f = f; c.o = &o0;
  c.wpts = x; c.n_pts = n;
  c.R = (n + 63) / 64; c.chunk = c.R;
  c.pts_mode = mode; c.pts_out = out; c.pts_out2 = out2;
  c.ws = workspace; c.ws_bytes = ws_bytes; c.s = (hipStream_t)stream;
  return sdf_train_core(c);
}

int anr_sdf_network_train_bwd(const anr_sdf_params* p, float* const* grads, const anr_sdf_frame* f, const anr_samples* x,
                              const anr_render_opts* o, const float* d_raw, const float* d_sdf, const float* d_resd,
                              const float* d_gradients, const float* d_observed_gradients, void* workspace,
                              size_t ws_bytes, void* stream) {
  ANR_TRY(check_net(p, f, x, o, workspace));
  if (!grads) return fail(ANR_E_ARG, "sdf network train: NULL gradients");
  for (int i = 0; i < ANR_SDF_NUM_TENSORS; ++i)
    if (!grads[i] && i != SDF_RESD_LAT) return fail(ANR_E_ARG, "sdf network train: NULL gradient tensor");
  TrainCore c = net_core(NET_BWD, p, f, x, o, workspace, ws_bytes, stream);
  c.grads = grads;
  c.d_raw = d_raw; c.d_sdf = d_sdf; c.d_resd = d_resd; c.d_grad = d_gradients; c.d_og = d_observed_gradients;
  return sdf_train_core(c);
}

}  // extern "C"
