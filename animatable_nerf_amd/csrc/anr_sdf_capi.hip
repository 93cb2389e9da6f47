// anr_sdf_capi.hip — C-ABI of the sdf_pdf render path (include/aninerf.h, "sdf_pdf variant").
//
// Sequence per render call (anisdf_pdf_network.py:156-223 under tpose_renderer.py:159-186):
//   k_sdf_front (KNN keep mask, all samples) -> ordered compaction -> one host read of n'
//   -> per batch of <= SDF_BATCH kept samples: prep, the residual MLP (split-bf16: one fused
//      k_resd_b16 launch; exact fp32: 9 layer GEMMs), mid, the SDF network forward (split-bf16: one
//      fused k_sdfnet_b16 launch writing the softplus outputs, and its input gradient as one fused
//      k_sdfgrad_b16 launch, the colour net as one fused k_color_b16 launch; exact fp32: 9 SDF GEMMs
//      (softplus + its backward factor in the epilogue), 8 input-gradient GEMMs (reverse mode
//      through the stored factors), gamma backward, 5 colour GEMMs, raw
//   -> compositing (k_composite) -> msk_sdf lists.
// Layer-wise GEMMs (anr_gemm.hip exact fp32 MFMA, or anr_lgemm.hip split-bf16) keep each activation in HBM: the input gradient
// needs every softplus factor of the forward, which does not fit a fused register pipeline.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "../../include/aninerf.h"
#include "anr_common.h"
#include "anr_kernels.h"
#include "anr_sdf.h"
#include "anr_train.h"
#include "anr_ws.h"

using namespace anr;

namespace {

#ifndef ANR_SDF_BATCH_LOG2
#define ANR_SDF_BATCH_LOG2 19
#endif
constexpr long SDF_BATCH = 1L << ANR_SDF_BATCH_LOG2;  // kept samples per layer-GEMM batch
constexpr size_t SDF_LIMG_BYTES = 16u << 20;  // split-bf16 layer-GEMM weight images (31 GEMMs, <= 384 KiB each)

struct SLayout {
  size_t counts, mask, chunk_min, ray_off, block_sum, list, knn, tbtab, wimg, fold, limg, rimg, simg, gimg, cimg, resd_rows, grad_rows;
  size_t min_sdf, flags, chunk_cnt, msk_sdf, msk_label;
  size_t ptb, Gr, Ha, Hb, Yr, Xs0, X4, D, Y8, Ga, Gb, Gc, gB, C0, Yc;
  long P;
  size_t total;
};

SLayout slayout(int n_rays, int chunk) {
  SLayout L{};
  const size_t R = (size_t)n_rays, N = R * 64;
  const size_t nch = (R + chunk - 1) / (size_t)std::max(chunk, 1);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align256(o + bytes);
    return at;
  };
  L.counts = take(16);
  L.mask = take(R * 8);
  L.chunk_min = take(nch * 8);
  L.ray_off = take((R + 1) * 4);
  L.block_sum = take(((R + 255) / 256) * 4);
  L.list = take(N * 4);
  L.knn = take(N * 32);
  L.tbtab = take(nch * 6 * 4);
  L.wimg = take(SDF_WN_FLOATS * 4);
  L.fold = take(768 * 4);
  L.limg = take(SDF_LIMG_BYTES);
  // the fused programs' images: bf16x3 (k_pack_seq) or bf16x6 (k_pack_seq_x6), sized for the larger
  auto img = [&](int L0, int nl) { return take((size_t)std::max(seq_image_bytes(L0, nl), x6seq_image_bytes(L0, nl))); };
  L.rimg = img(ANR_L_RESD0, ANR_RESD_LAYERS);
  L.simg = img(ANR_L_SDF0, ANR_SDF_LAYERS);
  L.gimg = img(ANR_L_SREV0, ANR_SREV_LAYERS);
  L.cimg = img(ANR_L_COL0, ANR_COL_LAYERS);
  L.resd_rows = take(N * 3 * 4);
  L.grad_rows = take(N * 3 * 4);
  L.min_sdf = take(R * 4);
  L.flags = take(R);
  L.chunk_cnt = take(nch * 4);
  L.msk_sdf = take(R * 4);
  L.msk_label = take(R * 4);
  const long P = (long)std::min<size_t>(N, SDF_BATCH);
  L.P = P;
  auto f = [&](long w) { return take((size_t)P * w * 4); };
  L.ptb = f(8); L.Gr = f(64); L.Ha = f(256); L.Hb = f(256); L.Yr = f(4); L.Xs0 = f(40); L.X4 = f(256);
  L.D = f(8 * 256); L.Y8 = f(264); L.Ga = f(256); L.Gb = f(256); L.Gc = f(256); L.gB = f(40); L.C0 = f(40);
  L.Yc = f(4);
  L.total = o;
  return L;
}

int sdf_cus() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) return 256;
  return v;
}

// weight (and bias) images of the split-bf16 layer GEMM (anr_lgemm.hip), packed on first use in a render call
// (the weights are fixed for its batches) and reused by every later batch
struct LImgCache {
  char* base = nullptr;
  size_t cap = 0, used = 0;
  struct E {
    const float* B[2];
    const float* bias;
    long rs[2], cs[2];
    int K[2], N;
    size_t off;
  } e[48];
  int n = 0;
  const void* get(const GemmArgs& g, hipStream_t s) {
    E k{};
    for (int i = 0; i < g.nseg; ++i) {
      k.B[i] = g.seg[i].B; k.rs[i] = g.seg[i].b_rs; k.cs[i] = g.seg[i].b_cs; k.K[i] = g.seg[i].K;
    }
    k.N = g.N;
    k.bias = g.bias;
    for (int i = 0; i < n; ++i) {
      const E& c = e[i];
      bool same = c.N == k.N && c.bias == k.bias;
      for (int j = 0; j < 2; ++j) same = same && c.B[j] == k.B[j] && c.rs[j] == k.rs[j] && c.cs[j] == k.cs[j] && c.K[j] == k.K[j];
      if (same) return base + c.off;
    }
    const size_t bytes = lgemm_image_bytes(g);
    if (n == 48 || used + bytes > cap) return nullptr;
    k.off = used;
    if (lgemm_pack(g, base + used, s) != 0) return nullptr;
    used = align256(used + bytes);
    e[n++] = k;
    return base + k.off;
  }
};

struct G {
  hipStream_t s;
  int M;
  int x3;  // render precision ANR_BF16X3: split-bf16 MFMA GEMMs (k_lgemm; k_gemm_b<.., .., true> otherwise)
  LImgCache* limg;
  int cus;
  int spd_h = 0;  // the spd operands of bwd / bwd_top hold softplus outputs h (GemmArgs::spd_h)
  float spd_scale = 0.f;  // ... stored as h / spd_scale (GemmArgs::spd_scale)
  // exact fp32 precision: the layer GEMMs that fit k_lgemm run on its F32 kernels (exact fp32 MFMA,
  // fp32 weight image resident in LDS) instead of k_gemm_t (ANR_SDF_LG32=0: k_gemm_t throughout)
  bool lg() const {
    if (x3) return true;
    const char* v = getenv("ANR_SDF_LG32");
    return !(v && v[0] == '0');
  }
  int run(GemmArgs g) {
    if (M <= 0 || g.N <= 0) return ANR_OK;
    g.M = M;
    g.x3 = x3;
    g.ksplit = 1;
    if (lg() && limg && lgemm_supported(g)) {
      g.prof = !x3;  // the exact render's clock (anr_profile_read_clock) from these launches' stamps
      if (const void* img = limg->get(g, s)) {
        (void)lgemm_run(g, img, cus, s);
        return check_launch("k_lgemm (sdf)");
      }
    }
    launch_gemm(g, dim3((g.N + 63) / 64, (M + 63) / 64, 1), s);
    return check_launch("k_gemm (sdf)");
  }
  // the first reverse GEMM with d sdf / d z7 = softplus_backward(W8[0], z7) applied to the stored
  // lin7 factors D7 as they are loaded (k_lgemm ATR); false (nothing launched) where k_lgemm does not
  // run, and the caller materialises G7 with k_sdf_gtop instead
  bool bwd_top(float* dX, long ldX, int K, const float* D7, const float* w8, int Nout, const float* W, int in_ch,
               const float* spd, int spd_n) {
    if (!lg() || !limg || M <= 0) return false;
    GemmArgs g{};
    g.M = M; g.N = K; g.nseg = 1; g.x3 = x3; g.ksplit = 1; g.prof = !x3;
    g.seg[0] = GemmSeg{D7, 256, 1, W, in_ch, 1, Nout};
    g.C = dX; g.ldc = ldX;
    g.spd = spd; g.ldsd = 256; g.spd_n = spd_n; g.spd_h = spd_h;
    g.a_softplus_w = w8;
    if (!lgemm_supported(g)) return false;
    const void* img = limg->get(g, s);
    if (!img) return false;
    (void)lgemm_run(g, img, cus, s);
    return true;
  }
  // Y = epi([X0 | X1] [W[:, c0:c0+K0] | W[:, c1:c1+K1]]^T + bias)
  // (sp_out_only: softplus with no factor written — deriv only selects the softplus epilogue)
  int fwd(float* Y, long ldY, int N, const float* W, int in_ch, const float* bias, const float* X0, long ld0, int K0,
          int c0, bool relu, float* deriv = nullptr, float div_post = 0.f, bool sp_out_only = false,
          const float* X1 = nullptr, long ld1 = 0, int K1 = 0, int c1 = 0) {
    GemmArgs g{};
    g.N = N;
    g.nseg = X1 ? 2 : 1;
    g.seg[0] = GemmSeg{X0, ld0, 1, W + c0, 1, in_ch, K0};
    if (X1) g.seg[1] = GemmSeg{X1, ld1, 1, W + c1, 1, in_ch, K1};
    g.C = Y; g.ldc = ldY; g.bias = bias; g.relu = relu ? 1 : 0;
    if (deriv) { g.softplus = 1; g.deriv = sp_out_only ? nullptr : deriv; g.ldd = 256; }
    g.div_post = div_post;
    return run(g);
  }
  // split-bf16 only: Yh = Wh relu(X W^T + bias) + bh with the 256-wide hidden activation never stored
  // (k_lgemm HEAD epilogue, two column groups adding into a zeroed Yh); false: nothing launched, the
  // caller runs the two GEMMs
  bool fwd_head(float* Yh, long ldh, int nh, const float* Wh, const float* bh, const float* W, int in_ch,
                const float* bias, const float* X, long ldX, int K) {
    if (!lg() || !limg || M <= 0) return false;
    GemmArgs g{};
    g.M = M; g.N = 256; g.nseg = 1; g.x3 = x3; g.ksplit = 1; g.prof = !x3;
    g.seg[0] = GemmSeg{X, ldX, 1, W, 1, in_ch, K};
    g.C = Yh; g.ldc = 4;  // not written (HEAD); kept valid for the support checks
    g.bias = bias; g.relu = 1;
    g.head_w = Wh; g.head_b = bh; g.head_out = Yh; g.ldh = ldh; g.head_n = nh;
    if (!lgemm_supported(g)) return false;
    const void* img = limg->get(g, s);
    if (!img) return false;
    if (hipMemsetAsync(Yh, 0, (size_t)M * ldh * sizeof(float), s) != hipSuccess) return false;
    (void)lgemm_run(g, img, cus, s);
    return true;
  }
  // Y[:, :256] = softplus(X W^T + bias), with its backward factors in deriv (or none: deriv NULL)
  int fwd_sp(float* Y, const float* W, int in_ch, const float* bias, const float* X, long ldX, float* deriv) {
    GemmArgs g{};
    g.N = 256;
    g.nseg = 1;
    g.seg[0] = GemmSeg{X, ldX, 1, W, 1, in_ch, in_ch};
    g.C = Y; g.ldc = 256; g.bias = bias;
    g.softplus = 1; g.deriv = deriv; g.ldd = 256;
    return run(g);
  }
  // dX[:, :K] = softplus_bwd((dY W[:, :K]) / div_pre, spd) (pass-through at n >= spd_n)
  int bwd(float* dX, long ldX, int K, const float* dY, long ldY, int Nout, const float* W, int in_ch, const float* spd,
          int spd_n, float div_pre = 0.f) {
    GemmArgs g{};
    g.N = K;
    g.nseg = 1;
    g.seg[0] = GemmSeg{dY, ldY, 1, W, in_ch, 1, Nout};
    g.C = dX; g.ldc = ldX;
    g.spd = spd; g.ldsd = 256; g.spd_n = spd_n; g.spd_h = spd ? spd_h : 0; g.spd_scale = spd_scale;
    g.div_pre = div_pre;
    return run(g);
  }
};

int check(const anr_sdf_params* p, const anr_sdf_frame* f, const float* ray_o, const float* ray_d, const float* near_,
          const float* far_, int R, const anr_render_opts* o, const anr_sdf_render_out* out, void* ws) {
  if (!p || !f || !o || !out || !ws || !ray_o || !ray_d || !near_ || !far_)
    return fail(ANR_E_ARG, "sdf render: NULL argument");
  if (o->n_samples != 64) return fail(ANR_E_ARG, "sdf render: only N_samples == 64 is supported");
  if (o->chunk <= 0 || R <= 0) return fail(ANR_E_ARG, "sdf render: bad chunk / n_rays");
  if (o->novel_pose) return fail(ANR_E_ARG, "sdf render: novel_pose is an aninerf option");
  for (int i = 0; i < ANR_SDF_NUM_TENSORS; ++i)
    if (!p->t[i] && i != SDF_RESD_LAT) return fail(ANR_E_ARG, "sdf render: NULL parameter tensor");
  if (!f->A || !f->big_A || !f->R || !f->Th || !f->poses || !f->pvertices || !f->weights || !f->tbounds ||
      !f->latent_index || !f->occupancy)
    return fail(ANR_E_ARG, "sdf render: NULL frame tensor");
  if (f->n_verts <= 0 || f->n_verts > 6912) return fail(ANR_E_ARG, "sdf render: n_verts must be in [1, 6912]");
  if (!out->rgb_map || !out->acc_map || !out->depth_map || !out->raw || !out->sdf)
    return fail(ANR_E_ARG, "sdf render: NULL output");
  if (f->n_views < 0 || (f->n_views > 0 && (!f->Ks || !f->RT || !f->msks || f->img_h <= 0 || f->img_w <= 0)))
    return fail(ANR_E_ARG, "sdf render: bad visibility-filter views");
  return ANR_OK;
}

}  // namespace

extern "C" {

size_t anr_sdf_render_workspace_bytes(int n_rays, const anr_render_opts* o) {
  if (n_rays <= 0 || !o || o->chunk <= 0) return 0;
  return slayout(n_rays, o->chunk).total;
}

const int32_t* anr_sdf_render_counts(const void* workspace, int n_rays, const anr_render_opts* o) {
  if (!workspace || !o || o->chunk <= 0) return nullptr;
  return (const int32_t*)((const char*)workspace + slayout(n_rays, o->chunk).counts);
}

const uint32_t* anr_sdf_render_knn(const void* workspace, int n_rays, const anr_render_opts* o) {
  if (!workspace || !o || o->chunk <= 0 || n_rays <= 0) return nullptr;
  return (const uint32_t*)((const char*)workspace + slayout(n_rays, o->chunk).knn);
}

int anr_sdf_render_rows(const void* workspace, int n_rays, const anr_render_opts* o, float* resd, float* gradients,
                        float* msk_sdf, float* msk_label, void* stream) {
  if (!workspace || !o || o->chunk <= 0) return fail(ANR_E_ARG, "anr_sdf_render_rows: bad arguments");
  const SLayout L = slayout(n_rays, o->chunk);
  const char* ws = (const char*)workspace;
  int cnt[2];
  hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyAsync(cnt, ws + L.counts, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return fail(ANR_E_HIP, "anr_sdf_render_rows: count readback");
  auto cp = [&](void* dst, size_t off, size_t bytes) {
    if (!dst || bytes == 0) return hipSuccess;
    return hipMemcpyAsync(dst, ws + off, bytes, hipMemcpyDeviceToDevice, s);
  };
  if (cp(resd, L.resd_rows, (size_t)cnt[0] * 12) != hipSuccess || cp(gradients, L.grad_rows, (size_t)cnt[0] * 12) != hipSuccess ||
      cp(msk_sdf, L.msk_sdf, (size_t)cnt[1] * 4) != hipSuccess || cp(msk_label, L.msk_label, (size_t)cnt[1] * 4) != hipSuccess)
    return fail(ANR_E_HIP, "anr_sdf_render_rows: copy");
  return ANR_OK;
}

}  // extern "C"

namespace {

// the render sequence over rays (wpts NULL) or over the free samples of one Network.forward call
// (wpts / vdir, n_pts points in R = ceil(n_pts / 64) groups that form one chunk: no compositing, no
// msk_sdf lists; raw / sdf are the caller's (n_pts) outputs)
int sdf_render_core(const anr_sdf_params* p, const anr_sdf_frame* f, const float* ray_o, const float* ray_d,
                    const float* near_, const float* far_, int R, int chunk, const anr_render_opts* o,
                    const anr_sdf_render_out* out, void* workspace, size_t ws_bytes, hipStream_t s,
                    const float* wpts, const float* vdir, int n_pts) {
  const SLayout L = slayout(R, chunk);
  if (ws_bytes < L.total) return fail(ANR_E_WORKSPACE, "sdf render: workspace too small");
  char* ws = (char*)workspace;
  const int nch = (R + chunk - 1) / chunk;
  int* counts = (int*)(ws + L.counts);
  float4* raw = (float4*)out->raw;

  if (hipMemsetAsync(ws + L.counts, 0, 16, s) != hipSuccess ||
      hipMemsetAsync(ws + L.chunk_min, 0xff, (size_t)nch * 8, s) != hipSuccess)
    return fail(ANR_E_HIP, "sdf render: memset");

  // per-call weight preparation (weight norm, folds, per-chunk tbounds)
  const float* const* tp = p->t;
  float* wimg = (float*)(ws + L.wimg);
  float* fold = (float*)(ws + L.fold);
  float* tbtab = (float*)(ws + L.tbtab);
  SdfTensors T{};
  for (int i = 0; i < ANR_SDF_NUM_TENSORS; ++i) T.t[i] = tp[i];
  hipLaunchKernelGGL(k_sdf_wnorm, dim3(sdf_wn_rows()), dim3(256), 0, s, T, wimg);
  ANR_TRY(check_launch("k_sdf_wnorm"));
  hipLaunchKernelGGL(k_sdf_fold, dim3(3), dim3(256), 0, s, T, (const float*)wimg, f->poses, f->latent_index, fold);
  ANR_TRY(check_launch("k_sdf_fold"));
  const bool filt = !wpts && f->n_views > 0;  // visibility filter: widening depends on the front-end
  if (!filt) {
    hipLaunchKernelGGL(k_sdf_tbtab, dim3(1), dim3(64), 0, s, f->tbounds, nch, tbtab, out->tbounds_out, nullptr);
    ANR_TRY(check_launch("k_sdf_tbtab"));
  }

  // B1 front-end + ordered compaction
  SdfFrontArgs fa{};
  fa.ray_o = ray_o; fa.ray_d = ray_d; fa.near_ = near_; fa.far_ = far_; fa.t_rand = o->t_rand;
  fa.wpts = wpts; fa.n_pts = n_pts;
  fa.n_rays = R; fa.chunk = chunk; fa.R = f->R; fa.Th = f->Th; fa.verts = f->pvertices; fa.nv = f->n_verts;
  fa.norm_th = o->norm_th; fa.mask = (uint64_t*)(ws + L.mask); fa.chunk_min = (uint64_t*)(ws + L.chunk_min);
  fa.knn = (uint32_t*)(ws + L.knn); fa.raw = raw; fa.sdf = out->sdf;
  const int grid_front = std::min(sdf_cus(), (R + 15) / 16);
  if (filt) {
    fa.n_views = f->n_views; fa.Ks = f->Ks; fa.RT = f->RT; fa.msks = f->msks; fa.img_h = f->img_h; fa.img_w = f->img_w;
  }
  hipLaunchKernelGGL(k_sdf_front, dim3(grid_front), dim3(1024), 0, s, fa);
  ANR_TRY(check_launch("k_sdf_front"));
  if (filt) {
    hipLaunchKernelGGL(k_sdf_tbtab, dim3(1), dim3(64), 0, s, f->tbounds, nch, tbtab, out->tbounds_out,
                       (const uint64_t*)fa.chunk_min);
    ANR_TRY(check_launch("k_sdf_tbtab (visible chunks)"));
  }
  CompactArgs ca{};
  ca.n_rays = R; ca.chunk = chunk; ca.mask = fa.mask; ca.chunk_min = fa.chunk_min;
  ca.ray_off = (int*)(ws + L.ray_off); ca.block_sum = (int*)(ws + L.block_sum); ca.list = (int*)(ws + L.list);
  const int nb = (R + 255) / 256;
  hipLaunchKernelGGL(k_count, dim3(nb), dim3(256), 0, s, ca);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, ca.block_sum, nb, counts);
  hipLaunchKernelGGL(k_compact, dim3((R + 3) / 4), dim3(256), 0, s, ca);
  ANR_TRY(check_launch("k_compact (sdf)"));
  int n = 0;
  if (hipMemcpyAsync(&n, counts, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return fail(ANR_E_HIP, "sdf render: kept-count readback");

  // per batch of kept samples
  float beta = 0.f;
  if (hipMemcpyAsync(&beta, tp[SDF_BETA], 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return fail(ANR_E_HIP, "sdf render: beta readback");
  auto F = [&](size_t off) { return (float*)(ws + off); };
  float *Ha = F(L.Ha), *Hb = F(L.Hb), *Ga = F(L.Ga), *Gb = F(L.Gb), *Gc = F(L.Gc), *D = F(L.D);
  const long P = L.P;
  auto Dl = [&](int l) { return D + (size_t)l * P * 256; };
  auto WN = [&](int l) { return (const float*)wimg + wn_layer(l).off; };
  const float sqrt2 = 1.41421356237309515f;
  LImgCache limg;
  limg.base = ws + L.limg;
  limg.cap = SDF_LIMG_BYTES;
  const int cus = sdf_cus();
  // split-bf16: the residual MLP, the SDF network forward, its input gradient and the colour net as
  // one fused launch per batch each (anr_resd_b16.hip), their weight images packed once per call;
  // ANR_BF16X6: the same four fused launches as fp32-level bf16x6 programs (anr_resd_x6.hip)
  const bool x6 = o->precision == ANR_BF16X6;
  const bool fused = x6 || o->precision == ANR_BF16X3;
  // the bf16x6 images' weight bytes (the bias section follows them)
  auto wbytes = [&](int L0, int nl) { return x6 ? x6seq_wbytes(L0, nl) : seq_wbytes(L0, nl); };
  auto pack = [&](const PackArgs& pa, int L0, int nl, int sl, float sc) {
    const int nt = x6 ? seq_x6_pack_threads(L0, nl) : seq_pack_threads(L0, nl);
    if (x6) hipLaunchKernelGGL(k_pack_seq_x6, dim3((nt + 255) / 256), dim3(256), 0, s, pa, L0, nl, sl, sc);
    else hipLaunchKernelGGL(k_pack_seq, dim3((nt + 255) / 256), dim3(256), 0, s, pa, L0, nl, sl, sc);
    return check_launch(x6 ? "k_pack_seq_x6" : "k_pack_seq");
  };
  unsigned char* rimg = (unsigned char*)(ws + L.rimg);
  unsigned char* simg = (unsigned char*)(ws + L.simg);
  unsigned char* gimg = (unsigned char*)(ws + L.gimg);
  unsigned char* cimg = (unsigned char*)(ws + L.cimg);
  if (fused) {
    PackArgs pa{};
    for (int l = 0; l < 8; ++l) {
      pa.t[l] = tp[SDF_RLIN0 + 2 * l];
      pa.t[9 + l] = l == 0 || l == 5 ? nullptr : tp[SDF_RLIN0 + 2 * l + 1];  // folded with the poses
    }
    pa.t[8] = tp[SDF_RFC_W];
    pa.t[17] = tp[SDF_RFC_B];
    pa.out = rimg;
    ANR_TRY(pack(pa, ANR_L_RESD0, ANR_RESD_LAYERS, -1, 1.0f));
    PackArgs ps{};
    for (int l = 0; l < 9; ++l) {
      ps.t[l] = WN(l);
      ps.t[9 + l] = tp[3 * l];
    }
    ps.out = simg;
    ANR_TRY(pack(ps, ANR_L_SDF0, ANR_SDF_LAYERS, 4, 1.0f / sqrt2));
    for (int l = 9; l < 18; ++l) ps.t[l] = nullptr;  // no biases in the gradient pass
    ps.out = gimg;  // lin7 .. lin0 transposed, lin4's with the skip's 1/sqrt2 (entry 3)
    ANR_TRY(pack(ps, ANR_L_SREV0, ANR_SREV_LAYERS, 3, 1.0f / sqrt2));
    PackArgs pc{};
    for (int l = 0; l < 5; ++l) {
      pc.t[l] = WN(9 + l);
      pc.t[9 + l] = l == 3 ? nullptr : tp[SDF_CLIN0 + 3 * l];  // lin3's bias: the latent fold
    }
    pc.out = cimg;
    ANR_TRY(pack(pc, ANR_L_COL0, ANR_COL_LAYERS, -1, 1.0f));
  }
  for (long b0 = 0; b0 < n; b0 += P) {
    const int cnt = (int)std::min<long>(P, n - b0);
    SdfPointArgs a{};
    a.list = ca.list; a.b0 = (int)b0; a.cnt = cnt;
    a.ray_o = ray_o; a.ray_d = ray_d; a.near_ = near_; a.far_ = far_; a.t_rand = o->t_rand; a.chunk = chunk;
    a.wpts = wpts; a.vdir = vdir; a.n_pts = n_pts;
    a.R = f->R; a.Th = f->Th; a.A = f->A; a.bigA = f->big_A; a.weights = f->weights; a.knn = fa.knn;
    a.wimg = wimg; a.tbtab = tbtab;
    a.ptb = F(L.ptb); a.Gr = fused ? nullptr : F(L.Gr); a.Yr = F(L.Yr); a.skip_sdf_in = fused ? 1 : 0; a.Xs0 = F(L.Xs0); a.X4 = F(L.X4); a.C0 = F(L.C0);
    a.D7 = Dl(7); a.G7 = Ga; a.Gc = Gc; a.gB = F(L.gB); a.Y8 = F(L.Y8); a.Yc = F(L.Yc); a.beta = beta;
    a.resd_rows = F(L.resd_rows); a.grad_rows = F(L.grad_rows); a.raw = raw; a.sdf = out->sdf;
    const dim3 pg((cnt + 255) / 256), pb(256);
    G g{s, cnt, o->precision == ANR_BF16X3 ? 1 : 0, &limg, cus};

    // B2 + B3: LBS to the big pose, residual deformation MLP (poses folded into layers 0 / 5)
    hipLaunchKernelGGL(k_sdf_prep, pg, pb, 0, s, a);
    ANR_TRY(check_launch("k_sdf_prep"));
    if (fused) {
      MlpArgs ra{};
      ra.wimg = rimg;
      ra.bias = (const float*)(rimg + wbytes(ANR_L_RESD0, ANR_RESD_LAYERS));
      ra.fold = fold;
      ra.ptb = a.ptb;
      ra.ptb_ld = 8;
      ra.yr = F(L.Yr);
      ra.n_rows = cnt;
      if (launch_resd(ra, cus, s, x6) != 0) return fail(ANR_E_HIP, "k_resd launch failed");
    } else {
    const float* Wr[8];
    for (int l = 0; l < 8; ++l) Wr[l] = tp[SDF_RLIN0 + 2 * l];
    ANR_TRY(g.fwd(Ha, 256, 256, Wr[0], 135, fold, a.Gr, 64, 63, 0, true));
    ANR_TRY(g.fwd(Hb, 256, 256, Wr[1], 256, tp[SDF_RLIN0 + 3], Ha, 256, 256, 0, true));
    ANR_TRY(g.fwd(Ha, 256, 256, Wr[2], 256, tp[SDF_RLIN0 + 5], Hb, 256, 256, 0, true));
    ANR_TRY(g.fwd(Hb, 256, 256, Wr[3], 256, tp[SDF_RLIN0 + 7], Ha, 256, 256, 0, true));
    ANR_TRY(g.fwd(Ha, 256, 256, Wr[4], 256, tp[SDF_RLIN0 + 9], Hb, 256, 256, 0, true));
    ANR_TRY(g.fwd(Hb, 256, 256, Wr[5], 391, fold + 256, a.Gr, 64, 63, 0, true, nullptr, 0.f, false, Ha, 256, 256, 135));
    ANR_TRY(g.fwd(Ha, 256, 256, Wr[6], 256, tp[SDF_RLIN0 + 13], Hb, 256, 256, 0, true));
    if (g.fwd_head(F(L.Yr), 4, 3, tp[SDF_RFC_W], tp[SDF_RFC_B], Wr[7], 256, tp[SDF_RLIN0 + 15], Ha, 256, 256)) {
      ANR_TRY(check_launch("k_lgemm (sdf, resd_linears.7 + resd_fc)"));
    } else {
      ANR_TRY(g.fwd(Hb, 256, 256, Wr[7], 256, tp[SDF_RLIN0 + 15], Ha, 256, 256, 0, true));
      ANR_TRY(g.fwd(F(L.Yr), 4, 3, tp[SDF_RFC_W], 256, tp[SDF_RFC_B], Hb, 256, 256, 0, false));
    }
    }
    hipLaunchKernelGGL(k_sdf_mid, pg, pb, 0, s, a);
    ANR_TRY(check_launch("k_sdf_mid"));

    // B4 SDF network forward. Split-bf16 precision: every softplus layer but lin3 writes its output h
    // to its own D slot and nothing else; the next layer reads it there and the reverse pass recomputes
    // the backward factor from it (softplus_factor_h) — one 0.54 GB write per layer fewer than storing
    // exp(100 z) beside a ping-pong activation. lin3 (217 outputs, /sqrt2 and the gamma columns in X4)
    // and the exact-fp32 precision keep the stored factors.
    const bool sph = g.x3 != 0;
    const float* hin = nullptr;
    if (fused) {
      MlpArgs sa{};
      sa.wimg = simg;
      sa.bias = (const float*)(simg + wbytes(ANR_L_SDF0, ANR_SDF_LAYERS));
      sa.ptb = a.C0;
      sa.ptb_ld = 40;
      for (int l = 0; l < 8; ++l) sa.sdf_h[l] = Dl(l);
      sa.x4 = a.X4;
      sa.y8 = F(L.Y8);
      sa.n_rows = cnt;
      if (launch_sdfnet(sa, cus, s, x6) != 0) return fail(ANR_E_HIP, "k_sdfnet launch failed");
    } else {
    auto sp_fwd = [&](int l, int K, float* pingpong) -> int {
      float* out = sph ? Dl(l) : pingpong;
      const int r = g.fwd_sp(out, WN(l), K, tp[3 * l], l == 0 ? a.Xs0 : hin, l == 0 ? 40 : 256, sph ? nullptr : Dl(l));
      hin = out;
      return r;
    };
    ANR_TRY(sp_fwd(0, 39, Ha));
    ANR_TRY(sp_fwd(1, 256, Hb));
    ANR_TRY(sp_fwd(2, 256, Ha));
    ANR_TRY(g.fwd(a.X4, 256, 217, WN(3), 256, tp[9], hin, 256, 256, 0, false, Dl(3), sqrt2, sph));
    hin = a.X4;
    ANR_TRY(sp_fwd(4, 256, Ha));
    ANR_TRY(sp_fwd(5, 256, Hb));
    ANR_TRY(sp_fwd(6, 256, Ha));
    ANR_TRY(sp_fwd(7, 256, Hb));
    ANR_TRY(g.fwd(F(L.Y8), 264, 257, WN(8), 256, tp[24], hin, 256, 256, 0, false));
    }

    // B4 gradient of sdf w.r.t. the canonical point (reverse mode through the stored factors / outputs)
    if (fused) {
      MlpArgs ga{};
      ga.wimg = gimg;
      ga.bias = (const float*)(gimg + wbytes(ANR_L_SREV0, ANR_SREV_LAYERS));
      for (int l = 0; l < 8; ++l) ga.sdf_h[l] = Dl(l);
      ga.x4 = a.X4;
      ga.w8row = WN(8);
      ga.gb = F(L.gB);
      ga.gc = Gc;
      ga.n_rows = cnt;
      if (launch_sdfgrad(ga, cus, s, x6) != 0) return fail(ANR_E_HIP, "k_sdfgrad launch failed");
    } else {
    g.spd_h = sph ? 1 : 0;
    a.d7_h = sph ? 1 : 0;
    if (g.bwd_top(Gb, 256, 256, Dl(7), WN(8), 256, WN(7), 256, Dl(6), 256)) {
      ANR_TRY(check_launch("k_lgemm (sdf, fused top)"));
    } else {
      hipLaunchKernelGGL(k_sdf_gtop, dim3((unsigned)(((long)cnt * 256 + 255) / 256)), pb, 0, s, a);
      ANR_TRY(check_launch("k_sdf_gtop"));
      ANR_TRY(g.bwd(Gb, 256, 256, Ga, 256, 256, WN(7), 256, Dl(6), 256));
    }
    ANR_TRY(g.bwd(Ga, 256, 256, Gb, 256, 256, WN(6), 256, Dl(5), 256));
    ANR_TRY(g.bwd(Gb, 256, 256, Ga, 256, 256, WN(5), 256, Dl(4), 256));
    if (sph) {  // lin3's outputs h3 / sqrt2 in X4
      g.spd_scale = sqrt2;
      ANR_TRY(g.bwd(Gc, 256, 256, Gb, 256, 256, WN(4), 256, a.X4, 217, sqrt2));
      g.spd_scale = 0.f;
    } else {
      ANR_TRY(g.bwd(Gc, 256, 256, Gb, 256, 256, WN(4), 256, Dl(3), 217, sqrt2));
    }
    ANR_TRY(g.bwd(Ga, 256, 256, Gc, 256, 217, WN(3), 256, Dl(2), 256));
    ANR_TRY(g.bwd(Gb, 256, 256, Ga, 256, 256, WN(2), 256, Dl(1), 256));
    ANR_TRY(g.bwd(Ga, 256, 256, Gb, 256, 256, WN(1), 256, Dl(0), 256));
    g.spd_h = 0;
    ANR_TRY(g.bwd(F(L.gB), 40, 39, Ga, 256, 256, WN(0), 39, nullptr, 0));
    }
    hipLaunchKernelGGL(k_sdf_gamma_bwd, pg, pb, 0, s, a);
    ANR_TRY(check_launch("k_sdf_gamma_bwd"));

    // B6 colour network (color_latent folded into lin3)
    if (fused) {
      MlpArgs ca{};
      ca.wimg = cimg;
      ca.bias = (const float*)(cimg + wbytes(ANR_L_COL0, ANR_COL_LAYERS));
      ca.fold = fold;
      ca.ptb = a.C0;
      ca.ptb_ld = 40;
      ca.y8 = F(L.Y8);
      ca.yr = F(L.Yc);
      ca.n_rows = cnt;
      if (launch_color(ca, cus, s, x6) != 0) return fail(ANR_E_HIP, "k_color launch failed");
    } else {
    ANR_TRY(g.fwd(Ha, 256, 256, WN(9), 289, tp[29], a.C0, 40, 33, 0, true, nullptr, 0.f, false, F(L.Y8) + 1, 264, 256, 33));
    ANR_TRY(g.fwd(Hb, 256, 256, WN(10), 256, tp[32], Ha, 256, 256, 0, true));
    ANR_TRY(g.fwd(Ha, 256, 256, WN(11), 256, tp[35], Hb, 256, 256, 0, true));
    if (g.fwd_head(F(L.Yc), 4, 3, WN(13), tp[41], WN(12), 384, fold + 512, Ha, 256, 256)) {
      ANR_TRY(check_launch("k_lgemm (sdf, colour lin3 + lin4)"));
    } else {
      ANR_TRY(g.fwd(Hb, 256, 256, WN(12), 384, fold + 512, Ha, 256, 256, 0, true));
      ANR_TRY(g.fwd(F(L.Yc), 4, 3, WN(13), 256, tp[41], Hb, 256, 256, 0, false));
    }
    }

    // B5 density, raw assembly with the (widened) tbounds mask
    hipLaunchKernelGGL(k_sdf_raw, pg, pb, 0, s, a);
    ANR_TRY(check_launch("k_sdf_raw"));
  }

  if (wpts) return ANR_OK;  // a Network.forward call: no compositing, no msk_sdf lists
  // A12 compositing over the full raw, then B7 msk_sdf / msk_label
  const anr_render_out ro{out->rgb_map, out->acc_map, out->depth_map, out->raw};
  ANR_TRY(stage_composite(near_, far_, R, o, raw, &ro, nullptr, s));
  SdfMskArgs ma{};
  ma.sdf = out->sdf; ma.occ = f->occupancy; ma.n_rays = R; ma.chunk = chunk;
  ma.min_sdf = F(L.min_sdf); ma.flags = (uint8_t*)(ws + L.flags); ma.chunk_cnt = (int*)(ws + L.chunk_cnt);
  ma.total = counts + 1; ma.msk_sdf = F(L.msk_sdf); ma.msk_label = F(L.msk_label);
  hipLaunchKernelGGL(k_sdf_msk_rays, dim3((R + 3) / 4), dim3(256), 0, s, ma);
  hipLaunchKernelGGL(k_sdf_msk_count, dim3(nch), dim3(1024), 0, s, ma);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, ma.chunk_cnt, nch, ma.total);
  hipLaunchKernelGGL(k_sdf_msk_write, dim3(nch), dim3(1024), 0, s, ma);
  return check_launch("k_sdf_msk_write");
}

int check_points(const anr_sdf_params* p, const anr_sdf_frame* f, const anr_samples* x, const anr_render_opts* o,
                 void* ws) {
  if (!p || !f || !x || !o || !ws || !x->wpts || !x->viewdir) return fail(ANR_E_ARG, "sdf network: NULL argument");
  if (x->n_pts <= 0 || x->n_pts > (1 << 24)) return fail(ANR_E_ARG, "sdf network: n must be in [1, 2^24]");
  for (int i = 0; i < ANR_SDF_NUM_TENSORS; ++i)
    if (!p->t[i] && i != SDF_RESD_LAT) return fail(ANR_E_ARG, "sdf network: NULL parameter tensor");
  if (!f->A || !f->big_A || !f->R || !f->Th || !f->poses || !f->pvertices || !f->weights || !f->tbounds ||
      !f->latent_index)
    return fail(ANR_E_ARG, "sdf network: NULL frame tensor");
  if (f->n_verts <= 0 || f->n_verts > 6912) return fail(ANR_E_ARG, "sdf network: n_verts must be in [1, 6912]");
  if (f->n_views) return fail(ANR_E_ARG, "sdf network: the visibility filter is a renderer option (n_views must be 0)");
  return ANR_OK;
}

int groups_of(int n) { return (n + 63) / 64; }

}  // namespace

extern "C" {

int anr_sdf_render_fwd(const anr_sdf_params* p, const anr_sdf_frame* f, const float* ray_o, const float* ray_d,
                       const float* near_, const float* far_, int R, const anr_render_opts* o,
                       const anr_sdf_render_out* out, void* workspace, size_t ws_bytes, void* stream) {
  ANR_TRY(check(p, f, ray_o, ray_d, near_, far_, R, o, out, workspace));
  return sdf_render_core(p, f, ray_o, ray_d, near_, far_, R, o->chunk, o, out, workspace, ws_bytes,
                         (hipStream_t)stream, nullptr, nullptr, 0);
}

size_t anr_sdf_network_workspace_bytes(int n, const anr_render_opts* o) {
  if (n <= 0 || !o) return 0;
  const int G = groups_of(n);
  return slayout(G, G).total;
}

int anr_sdf_network_fwd(const anr_sdf_params* p, const anr_sdf_frame* f, const anr_samples* x, const anr_render_opts* o,
                        float* raw, float* sdf, float* tbounds_out, void* workspace, size_t ws_bytes, void* stream) {
  ANR_TRY(check_points(p, f, x, o, workspace));
  if (!raw || !sdf) return fail(ANR_E_ARG, "sdf network: NULL output");
  const int G = groups_of(x->n_pts);
  const anr_sdf_render_out out{nullptr, nullptr, nullptr, raw, sdf, tbounds_out};
  return sdf_render_core(p, f, nullptr, nullptr, nullptr, nullptr, G, G, o, &out, workspace, ws_bytes,
                         (hipStream_t)stream, x->wpts, x->viewdir, x->n_pts);
}

const int32_t* anr_sdf_network_counts(const void* workspace, int n) {
  if (!workspace || n <= 0) return nullptr;
  const int G = groups_of(n);
  return (const int32_t*)((const char*)workspace + slayout(G, G).counts);
}

// KNN blend of free points: [R | Th identity (12 floats)] [mask (G x 8)] [chunk_min 8] [knn (64 G x 32)]
//   [raw (64 G x 16)] [sdf (64 G x 4)]
size_t anr_knn_blend_workspace_bytes(int n) {
  if (n <= 0) return 0;
  const size_t G = (size_t)groups_of(n);
  return align256(64) + align256(G * 8) + align256(8) + align256(64 * G * 32) + align256(64 * G * 16) + align256(64 * G * 4);
}

int anr_knn_blend(const float* verts, const float* weights, int nv, const float* pts, int n, float norm_th, float* bw,
                  uint8_t* inside, void* workspace, size_t ws_bytes, void* stream) {
  if (!verts || !weights || !pts || !workspace || n <= 0 || (!bw && !inside))
    return fail(ANR_E_ARG, "anr_knn_blend: bad arguments");
  if (nv <= 0 || nv > 6912) return fail(ANR_E_ARG, "anr_knn_blend: nv must be in [1, 6912]");
  if (ws_bytes < anr_knn_blend_workspace_bytes(n)) return fail(ANR_E_WORKSPACE, "anr_knn_blend: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int G = groups_of(n);
  char* w = (char*)workspace;
  float* rt = (float*)w;
  w += align256(64);
  uint64_t* mask = (uint64_t*)w;
  w += align256((size_t)G * 8);
  uint64_t* cmin = (uint64_t*)w;
  w += align256(8);
  uint32_t* knn = (uint32_t*)w;
  w += align256((size_t)64 * G * 32);
  float4* raw = (float4*)w;
  w += align256((size_t)64 * G * 16);
  float* sdf = (float*)w;
  static const float ident[12] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f};
  if (hipMemcpyAsync(rt, ident, sizeof(ident), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemsetAsync(cmin, 0xff, 8, s) != hipSuccess)
    return fail(ANR_E_HIP, "anr_knn_blend: setup");
  SdfFrontArgs fa{};
  fa.wpts = pts; fa.n_pts = n; fa.n_rays = G; fa.chunk = G;
  fa.R = rt; fa.Th = rt + 9;  // world -> pose with R = I, Th = 0 is the identity in fp32 (x * 1 + y * 0 + z * 0)
  fa.verts = verts; fa.nv = nv; fa.norm_th = norm_th;
  fa.mask = mask; fa.chunk_min = cmin; fa.knn = knn; fa.raw = raw; fa.sdf = sdf;
  hipLaunchKernelGGL(k_sdf_front, dim3(std::min(sdf_cus(), (G + 15) / 16)), dim3(1024), 0, s, fa);
  ANR_TRY(check_launch("k_sdf_front (knn blend)"));
  hipLaunchKernelGGL(k_knn_blend_out, dim3((n + 255) / 256), dim3(256), 0, s, (const uint32_t*)knn, (const uint64_t*)mask,
                     weights, n, bw, inside);
  return check_launch("k_knn_blend_out");
}

int anr_sdf_mesh_pose(const float* pts, const float* bw, int n, const float* big_A, const float* A, const float* R,
                      const float* Th, float* out, void* stream) {
  if (!pts || !bw || !big_A || !A || !R || !Th || !out || n < 0) return fail(ANR_E_ARG, "anr_sdf_mesh_pose: bad arguments");
  if (n == 0) return ANR_OK;
  hipLaunchKernelGGL(k_mesh_pose, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, pts, bw, n, big_A, A, R, Th, out);
  return check_launch("k_mesh_pose");
}

int anr_sdf_network_rows(const void* workspace, int n, float* resd, float* gradients, void* stream) {
  if (!workspace || n <= 0) return fail(ANR_E_ARG, "anr_sdf_network_rows: bad arguments");
  const int G = groups_of(n);
  anr_render_opts o{};
  o.chunk = G;
  return anr_sdf_render_rows(workspace, G, &o, resd, gradients, nullptr, nullptr, stream);
}

}  // extern "C"
