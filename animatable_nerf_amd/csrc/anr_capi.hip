// anr_capi.hip — the C-ABI (include/aninerf.h): argument checks, workspace layout, launch order.
// All launches are asynchronous on the caller's stream; no allocation, no synchronisation, so a
// caller may capture a whole render into a hipGraph.
#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "../../include/aninerf.h"
#include "anr_common.h"
#include "anr_kernels.h"
#include "anr_layers.h"
#include "anr_ws.h"

using namespace anr;

namespace anr {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(ANR_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return ANR_OK;
}

}  // namespace anr

namespace {


int num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cached[dev] = v;
  }
  return cached[dev];
}

bool mlp_attr_set = false;

// measurement: event pairs around the fused network launches (anr_profile_enable / anr_profile_read),
// and each launch's per-workgroup clock stamps (MlpArgs::clk) in a device arena of kProfSlots slots
constexpr int kProfSlots = 512, kProfGroups = 1024;
struct Prof {
  bool on = false;
  std::vector<anr::ProfSlot> slot;
  std::vector<int> groups;  // workgroups stamped per used slot
  size_t used = 0;
  unsigned long long* arena = nullptr;
} g_prof;

}  // namespace

namespace anr {

ProfSlot* prof_begin(hipStream_t s, int grid) {
  if (!g_prof.on) return nullptr;
  if (!g_prof.arena &&
      hipMalloc((void**)&g_prof.arena, (size_t)kProfSlots * kProfGroups * 4 * sizeof(unsigned long long)) != hipSuccess) {
    g_prof.arena = nullptr;
    (void)hipGetLastError();
  }
  if (g_prof.used == g_prof.slot.size()) {
    ProfSlot q{};
    if (hipEventCreate(&q.b) != hipSuccess || hipEventCreate(&q.e) != hipSuccess) return nullptr;
    g_prof.slot.push_back(q);
    g_prof.groups.push_back(0);
  }
  const size_t i = g_prof.used++;
  ProfSlot* q = &g_prof.slot[i];
  q->clk = g_prof.arena && i < (size_t)kProfSlots && grid <= kProfGroups
               ? g_prof.arena + i * (size_t)kProfGroups * 4 : nullptr;
  g_prof.groups[i] = q->clk ? grid : 0;
  if (q->clk && hipMemsetAsync(q->clk, 0, (size_t)grid * 4 * sizeof(unsigned long long), s) != hipSuccess) return nullptr;
  if (hipEventRecord(q->b, s) != hipSuccess) return nullptr;
  return q;
}

int prof_end(ProfSlot* q, hipStream_t s) {
  if (q && hipEventRecord(q->e, s) != hipSuccess) return fail(ANR_E_HIP, "hipEventRecord failed");
  return ANR_OK;
}

// A2-A6 + per-frame prep: memsets, volumes/folds, front-end, ordered compaction (counts[0] = n')
int RaySplit::run(void* buf, int count, int op, hipStream_t s) const {
  if (!reduce) return ANR_OK;
  if (check_launch("before the ray-split reduction") != ANR_OK) return ANR_E_HIP;
  if (reduce(user, buf, count, op, (void*)s) != 0) return fail(ANR_E_ARG, "ray split: the reduce hook failed");
  return ANR_OK;
}

int stage_frontend(const anr_params* p, const anr_frame* f, const float* ray_o, const float* ray_d, const float* near_,
                   const float* far_, int R, const anr_render_opts* o, char* ws, const Layout& L, float4* raw,
                   hipStream_t s, const anr_samples* x, const RaySplit* split) {
  const long np = (long)f->pbw_dims[0] * f->pbw_dims[1] * f->pbw_dims[2];
  const long nt = (long)f->tbw_dims[0] * f->tbw_dims[1] * f->tbw_dims[2];
  const int nch = (R + o->chunk - 1) / o->chunk;
  int* counts = (int*)(ws + L.counts);

  PrepArgs pa{};
  pa.counts = counts;  // counts, chunk_min and chunk_max reset by k_prep's block 0
  pa.chunk_min = (uint64_t*)(ws + L.chunk_min);
  pa.chunk_max = (uint64_t*)(ws + L.chunk_max);
  pa.nch = nch;
  pa.pbw = f->pbw; pa.tbw = f->tbw;
  pa.pbw32 = (float*)(ws + L.pbw32); pa.tbw32 = (float*)(ws + L.tbw32);
  pa.np = (int)np; pa.nt = (int)nt;
  pa.w_bw0 = p->t[28]; pa.b_bw0 = p->t[29]; pa.w_bw5 = p->t[38]; pa.b_bw5 = p->t[39];
  pa.bw_latent = p->t[27]; pa.w_lat = p->t[21]; pa.b_lat = p->t[22]; pa.nf_latent = p->t[0];
  pa.latent_index = f->latent_index;
  pa.fold = (float*)(ws + L.fold);
  pa.pn24 = (float*)(ws + L.pn24);
  if (p->packed) {  // the bf16x3 program's folded head (anr_layers.h ANR_L_HEAD)
    const float* head = (const float*)((const unsigned char*)p->packed + head_base());
    pa.head_P = head + ANR_HEAD_P_OFF;
    pa.head_q = head + ANR_HEAD_Q_OFF;
    pa.b_alpha = p->t[18];
  }
  if (o->novel_pose) {
    pa.novel = 1;
    pa.n_latent = p->novel[0];
    pa.nw_bw0 = p->novel[1]; pa.nb_bw0 = p->novel[2];
    pa.nw_bw5 = p->novel[11]; pa.nb_bw5 = p->novel[12];
    pa.bw_latent_index = f->bw_latent_index;
  }
  hipLaunchKernelGGL(k_prep, dim3(prep_blocks(np, nt)), dim3(256), 0, s, pa);
  ANR_TRY(check_launch("k_prep"));

  FrontArgs fa{};
  fa.ray_o = ray_o; fa.ray_d = ray_d; fa.near_ = near_; fa.far_ = far_; fa.t_rand = o->t_rand;
  fa.n_rays = R; fa.chunk = o->chunk;
  fa.ray_offset = split ? split->ray_offset : 0;
  fa.R = f->R; fa.Th = f->Th; fa.pbw = f->pbw; fa.pbounds = f->pbounds;
  fa.pn24 = pa.pn24;
  fa.X = f->pbw_dims[0]; fa.Y = f->pbw_dims[1]; fa.Z = f->pbw_dims[2];
  fa.norm_th = o->norm_th;
  fa.mask = (uint64_t*)(ws + L.mask);
  fa.chunk_min = (uint64_t*)(ws + L.chunk_min);
  fa.raw = raw;
  fa.n_views = f->n_views;
  fa.Ks = f->Ks; fa.RT = f->RT; fa.msks = f->msks;
  fa.img_h = f->img_h; fa.img_w = f->img_w;
  if (f->n_views < 0 || (f->n_views > 0 && (!f->Ks || !f->RT || !f->msks || f->img_h <= 0 || f->img_w <= 0)))
    return fail(ANR_E_ARG, "render: bad visibility-filter views");
  if (x) {  // free samples: world->pose with the matmul path of an n_pts-point call, argmin over the call
    if (f->n_views) return fail(ANR_E_ARG, "network forward: the visibility filter is a renderer option");
    fa.wpts = x->wpts;
    fa.n_pts = x->n_pts;
    fa.chunk_pts = x->n_pts;
    hipLaunchKernelGGL(k_frontend_pts, dim3((R + 3) / 4), dim3(256), 0, s, fa);
    ANR_TRY(check_launch("k_frontend_pts"));
  } else {
    hipLaunchKernelGGL(k_frontend, dim3((R + 15) / 16), dim3(1024), 0, s, fa);
    ANR_TRY(check_launch("k_frontend"));
  }

  // ray split: the chunk's argmin over every rank's samples
  if (split) ANR_TRY(split->run(fa.chunk_min, (R + o->chunk - 1) / o->chunk, ANR_REDUCE_MIN_U64, s));
  CompactArgs ca{};
  ca.n_rays = R; ca.chunk = o->chunk;
  ca.ray_offset = fa.ray_offset;
  ca.mask = fa.mask; ca.chunk_min = fa.chunk_min;
  ca.ray_off = (int*)(ws + L.ray_off);
  ca.block_sum = (int*)(ws + L.block_sum);
  ca.list = (int*)(ws + L.list);
  if (R <= 1024) {  // a training batch: one launch
    hipLaunchKernelGGL(k_compact1, dim3(1), dim3(1024), 0, s, ca, counts);
    return check_launch("k_compact1");
  }
  const int nb = (R + 255) / 256;
  hipLaunchKernelGGL(k_count, dim3(nb), dim3(256), 0, s, ca);
  ANR_TRY(check_launch("k_count"));
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, ca.block_sum, nb, counts);
  ANR_TRY(check_launch("k_scan_blocks"));
  hipLaunchKernelGGL(k_compact, dim3((R + 3) / 4), dim3(256), 0, s, ca);
  return check_launch("k_compact");
}

// the fused network kernel (render path)
int stage_mlp(const anr_params* p, const anr_frame* f, const float* ray_o, const float* ray_d, const float* near_,
              const float* far_, int R, const anr_render_opts* o, char* ws, const Layout& L, float4* raw,
              hipStream_t s, const anr_samples* x) {
  const long N = (long)R * 64;
  MlpArgs ma{};
  if (x) {
    ma.wpts = x->wpts; ma.vdir = x->viewdir; ma.dists = x->dists;
    ma.n_pts = x->n_pts; ma.chunk_pts = x->n_pts;
  }
  ma.wimg = (const unsigned char*)p->packed;
  ma.bias = (const float*)((const unsigned char*)p->packed + weights_bytes());
  ma.fold = (const float*)(ws + L.fold);
  ma.A = f->A; ma.R = f->R; ma.Th = f->Th;
  ma.pbw32 = (const float*)(ws + L.pbw32); ma.pbounds = f->pbounds;
  ma.tbw32 = (const float*)(ws + L.tbw32); ma.tbounds = f->tbounds;
  ma.pX = f->pbw_dims[0]; ma.pY = f->pbw_dims[1]; ma.pZ = f->pbw_dims[2];
  ma.tX = f->tbw_dims[0]; ma.tY = f->tbw_dims[1]; ma.tZ = f->tbw_dims[2];
  ma.ray_o = ray_o; ma.ray_d = ray_d; ma.near_ = near_; ma.far_ = far_; ma.t_rand = o->t_rand;
  ma.list = (const int*)(ws + L.list); ma.n_kept = (const int*)(ws + L.counts);
  ma.raw = raw;
  ma.sigma = (float*)(ws + L.sigma);
  ma.pbw_rows = (float*)(ws + L.pbw_rows);
  ma.tbw_rows = (float*)(ws + L.tbw_rows);
  const bool x6 = o->precision == ANR_BF16X6;
  const bool b16 = o->precision == ANR_BF16X3 || x6;
  ma.pose_woff = o->novel_pose ? (x6 || (b16 && ANR_POSE_MODE == 2) ? ANR_X6_NOVEL_WOFF : b16 ? ANR_B16_NOVEL_WOFF : ANR_NOVEL_WOFF) : 0;
  ma.pose_boff = o->novel_pose ? ANR_NOVEL_BOFF : 0;
  const int lds = b16 ? mlp_lds_bytes<true>() : mlp_lds_bytes<false>();
  if (!mlp_attr_set) {
    if (hipFuncSetAttribute((const void*)k_mlp, hipFuncAttributeMaxDynamicSharedMemorySize, mlp_lds_bytes<false>()) !=
            hipSuccess ||
        hipFuncSetAttribute((const void*)k_mlp_b16, hipFuncAttributeMaxDynamicSharedMemorySize, mlp_lds_bytes<true>()) !=
            hipSuccess ||
        hipFuncSetAttribute((const void*)k_mlp_x6, hipFuncAttributeMaxDynamicSharedMemorySize, mlp_lds_bytes<true>()) !=
            hipSuccess)
      return fail(ANR_E_HIP, "hipFuncSetAttribute(k_mlp) failed");
    mlp_attr_set = true;
  }
  const long max_tiles = (N + 127) / 128;
  const int grid = (int)(max_tiles < num_cus() ? max_tiles : num_cus());
  ProfSlot* ps = prof_begin(s, grid);
  ma.clk = ps ? ps->clk : nullptr;
  if (x6) hipLaunchKernelGGL(k_mlp_x6, dim3(grid), dim3(512), lds, s, ma);
  else if (b16) hipLaunchKernelGGL(k_mlp_b16, dim3(grid), dim3(512), lds, s, ma);
  else hipLaunchKernelGGL(k_mlp, dim3(grid), dim3(512), lds, s, ma);
  ANR_TRY(check_launch("k_mlp"));
  return prof_end(ps, s);
}

// A11 alpha_ind rows: sigma' > train_th plus per-chunk argmax (counts[1] = m)
int stage_alpha_ind(int R, const anr_render_opts* o, char* ws, const Layout& L, hipStream_t s, const RaySplit* split) {
  const long N = (long)R * 64;
  const int nch = (R + o->chunk - 1) / o->chunk;
  int* counts = (int*)(ws + L.counts);
  AlphaArgs aa{};
  aa.n_rays = R; aa.chunk = o->chunk;
  aa.ray_off = (const int*)(ws + L.ray_off); aa.n_kept = counts;
  aa.sigma = (const float*)(ws + L.sigma);
  aa.chunk_max = (uint64_t*)(ws + L.chunk_max);
  aa.train_th = o->train_th;
  aa.flags = (uint8_t*)(ws + L.flags);
  aa.block_sum = (int*)(ws + L.block_sum2);
  aa.out_row = (int*)(ws + L.out_row);
  aa.list = (const int*)(ws + L.list);
  aa.mask = (const uint64_t*)(ws + L.mask);
  aa.ray_offset = split ? split->ray_offset : 0;
  const int nb2 = (int)((N + 1023) / 1024);
  if (nch == 1 && nb2 <= 64 && !split) {  // a training batch: two launches (chunk_max[0] is 0 from k_prep)
    hipLaunchKernelGGL(k_alpha_count1, dim3(nb2), dim3(256), 0, s, aa);
    ANR_TRY(check_launch("k_alpha_count1"));
    hipLaunchKernelGGL(k_alpha_scatter1, dim3(nb2), dim3(256), 0, s, aa, counts + 1);
    return check_launch("k_alpha_scatter1");
  }
  hipLaunchKernelGGL(k_chunk_argmax, dim3(nch, 16), dim3(256), 0, s, aa);
  ANR_TRY(check_launch("k_chunk_argmax"));
  if (split) ANR_TRY(split->run(aa.chunk_max, nch, ANR_REDUCE_MAX_U64, s));  // the chunk's argmax over every rank
  hipLaunchKernelGGL(k_flag_count, dim3(nb2), dim3(256), 0, s, aa);
  ANR_TRY(check_launch("k_flag_count"));
  hipLaunchKernelGGL(k_flag_force, dim3((nch + 255) / 256), dim3(256), 0, s, aa, nch);
  ANR_TRY(check_launch("k_flag_force"));
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, aa.block_sum, nb2, counts + 1);
  ANR_TRY(check_launch("k_scan_blocks(alpha)"));
  hipLaunchKernelGGL(k_flag_scatter, dim3(nb2), dim3(256), 0, s, aa);
  return check_launch("k_flag_scatter");
}

// A12 compositing
int stage_composite(const float* near_, const float* far_, int R, const anr_render_opts* o, const float4* raw,
                    const anr_render_out* out, float* weights, hipStream_t s) {
  CompositeArgs co{};
  co.raw = raw; co.near_ = near_; co.far_ = far_; co.t_rand = o->t_rand; co.n_rays = R;
  co.rgb = out->rgb_map; co.acc = out->acc_map; co.depth = out->depth_map; co.weights = weights;
  hipLaunchKernelGGL(k_composite, dim3((R + 3) / 4), dim3(256), 0, s, co);
  return check_launch("k_composite");
}

}  // namespace anr

extern "C" {

int anr_version(void) { return 2; }  // 2: anr_train_hooks.struct_size

const char* anr_last_error(void) { return g_err.c_str(); }

int anr_near_far(const float* ray_o, const float* ray_d, int n, const float* bounds, uint8_t* mask, float* near_,
                 float* far_, void* stream) {
  if (n < 0 || (n > 0 && (!ray_o || !ray_d || !bounds || !mask || !near_ || !far_)))
    return fail(ANR_E_ARG, "anr_near_far: bad arguments");
  if (n == 0) return ANR_OK;
  hipLaunchKernelGGL(k_near_far, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, ray_o, ray_d, n, bounds, mask,
                     near_, far_);
  return check_launch("k_near_far");
}

size_t anr_camera_rays_workspace_bytes(int H, int W) {
  if (H <= 0 || W <= 0) return 0;
  const size_t P = (size_t)H * W;
  return align256(P * 12) * 2 + align256(P * 4) * 2 + align256(((P + 255) / 256) * 4);
}

int anr_camera_rays(int H, int W, const double* Kinv, const double* R, const double* T, const double* origin, int fp64,
                    const float* bounds, float* ray_o, float* ray_d, float* near_, float* far_, int32_t* coord,
                    uint8_t* mask, int32_t* count, void* workspace, size_t ws_bytes, void* stream) {
  if (H <= 0 || W <= 0 || !Kinv || !R || !T || !origin || !bounds || !ray_o || !ray_d || !near_ || !far_ || !coord ||
      !mask || !count || !workspace)
    return fail(ANR_E_ARG, "anr_camera_rays: bad arguments");
  if ((long)H * W > (1L << 30)) return fail(ANR_E_ARG, "anr_camera_rays: image too large");
  if (ws_bytes < anr_camera_rays_workspace_bytes(H, W)) return fail(ANR_E_WORKSPACE, "anr_camera_rays: workspace");
  const size_t P = (size_t)H * W;
  char* ws = (char*)workspace;
  CamArgs a{};
  a.H = H; a.W = W; a.fp64 = fp64 ? 1 : 0;
  for (int k = 0; k < 9; ++k) { a.Kinv[k] = Kinv[k]; a.R[k] = R[k]; }
  for (int k = 0; k < 3; ++k) { a.T[k] = T[k]; a.o[k] = origin[k]; }
  a.bounds = bounds;
  a.all_o = (float*)ws;
  a.all_d = (float*)(ws + align256(P * 12));
  a.all_near = (float*)(ws + 2 * align256(P * 12));
  a.all_far = (float*)(ws + 2 * align256(P * 12) + align256(P * 4));
  a.block_sum = (int*)(ws + 2 * align256(P * 12) + 2 * align256(P * 4));
  a.mask = mask;
  a.ray_o = ray_o; a.ray_d = ray_d; a.near_ = near_; a.far_ = far_; a.coord = coord;
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)((P + 255) / 256);
  hipLaunchKernelGGL(k_cam_rays, dim3(nb), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_cam_count, dim3(nb), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, a.block_sum, nb, count);
  hipLaunchKernelGGL(k_cam_scatter, dim3(nb), dim3(256), 0, s, a);
  return check_launch("anr_camera_rays");
}

size_t anr_train_ray_workspace_bytes(int H, int W) {
  if (H <= 0 || W <= 0) return 0;
  return align256((((size_t)H * W + 255) / 256) * 4 * 3);
}

int anr_train_ray_lists(int H, int W, const uint8_t* msk, const uint8_t* bound_mask, int32_t* lists, int32_t* counts,
                        void* workspace, size_t ws_bytes, void* stream) {
  if (H <= 0 || W <= 0 || !msk || !bound_mask || !lists || !counts || !workspace)
    return fail(ANR_E_ARG, "anr_train_ray_lists: bad arguments");
  if ((long)H * W > (1L << 29)) return fail(ANR_E_ARG, "anr_train_ray_lists: image too large");
  if (ws_bytes < anr_train_ray_workspace_bytes(H, W)) return fail(ANR_E_WORKSPACE, "anr_train_ray_lists: workspace");
  TrainRayArgs a{};
  a.cam.H = H; a.cam.W = W;
  a.msk = msk; a.bound_mask = bound_mask;
  a.block_sum = (int*)workspace;
  a.lists = lists;
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)(((size_t)H * W + 255) / 256);
  hipLaunchKernelGGL(k_trl_count, dim3(nb), dim3(256), 0, s, a);
  for (int k = 0; k < 3; ++k)
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, a.block_sum + k * nb, nb, counts + k);
  hipLaunchKernelGGL(k_trl_scatter, dim3(nb), dim3(256), 0, s, a);
  return check_launch("anr_train_ray_lists");
}

int anr_train_ray_gather(int H, int W, const double* Kinv, const double* R, const double* T, const double* origin,
                         int fp64, const float* bounds, const float* img, const uint8_t* bound_mask, int mask_bkgd,
                         const int32_t* lists, const int32_t* draws, int n_body, int n_face, int n_rand, int cap,
                         float* ray_o, float* ray_d, float* rgb, float* near_, float* far_, int32_t* coord,
                         int32_t* n_out, void* stream) {
  if (H <= 0 || W <= 0 || !Kinv || !R || !T || !origin || !bounds || !img || !bound_mask || !lists || !ray_o ||
      !ray_d || !rgb || !near_ || !far_ || !coord || !n_out || n_body < 0 || n_face < 0 || n_rand < 0 || cap < 0)
    return fail(ANR_E_ARG, "anr_train_ray_gather: bad arguments");
  const long n = (long)n_body + n_face + n_rand;
  if (n > 0 && !draws) return fail(ANR_E_ARG, "anr_train_ray_gather: draws is NULL");
  if (n > (1L << 24)) return fail(ANR_E_ARG, "anr_train_ray_gather: too many draws");
  if (n == 0) return ANR_OK;
  TrainRayArgs a{};
  a.cam.H = H; a.cam.W = W; a.cam.fp64 = fp64 ? 1 : 0;
  for (int k = 0; k < 9; ++k) { a.cam.Kinv[k] = Kinv[k]; a.cam.R[k] = R[k]; }
  for (int k = 0; k < 3; ++k) { a.cam.T[k] = T[k]; a.cam.o[k] = origin[k]; }
  a.cam.bounds = bounds;
  a.img = img; a.bound_mask = bound_mask; a.mask_bkgd = mask_bkgd ? 1 : 0;
  a.lists = const_cast<int*>(lists); a.draws = draws;
  a.n_seg[0] = n_body; a.n_seg[1] = n_face; a.n_seg[2] = n_rand;
  a.cap = cap; a.n_out = n_out;
  a.ray_o = ray_o; a.ray_d = ray_d; a.rgb = rgb; a.near_ = near_; a.far_ = far_; a.coord = coord;
  hipLaunchKernelGGL(k_trl_gather, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
  return check_launch("anr_train_ray_gather");
}

size_t anr_params_packed_bytes(void) { return (size_t)packed_bytes_all(); }

int anr_params_pack(const anr_params* p, void* packed, void* stream) {
  if (!p || !packed) return fail(ANR_E_ARG, "anr_params_pack: NULL");
  PackArgs a{};
  for (int i = 0; i < ANR_NUM_TENSORS; ++i) {
    if (!p->t[i]) return fail(ANR_E_ARG, "anr_params_pack: tensor " + std::to_string(i) + " is NULL");
    a.t[i] = p->t[i];
  }
  for (int i = 0; i < ANR_NUM_NOVEL_TENSORS; ++i) a.t[ANR_NOVEL_T0 + i] = p->novel[i];  // may be NULL
  a.out = (unsigned char*)packed;
  a.t[ANR_HEAD_T] = (const float*)((unsigned char*)packed + head_base());
  hipLaunchKernelGGL(k_pack_head_a, dim3((128 * 256 + 256 + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  ANR_TRY(check_launch("k_pack_head_a"));
  hipLaunchKernelGGL(k_pack_head_b, dim3((ANR_HEAD_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  ANR_TRY(check_launch("k_pack_head_b"));
  const int nw = weights_bytes() / 4;
  hipLaunchKernelGGL(k_pack_weights, dim3((nw + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  ANR_TRY(check_launch("k_pack_weights"));
  hipLaunchKernelGGL(k_pack_bias, dim3((bias_floats() + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  ANR_TRY(check_launch("k_pack_bias"));
  hipLaunchKernelGGL(k_pack_b16, dim3((b16_bytes() / 32 + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  ANR_TRY(check_launch("k_pack_b16"));
  hipLaunchKernelGGL(k_pack_x6, dim3((x6_bytes() / 48 + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("k_pack_x6");
}

size_t anr_render_workspace_bytes(int n_rays, const anr_render_opts* o, const anr_frame* f) {
  if (!o || !f || n_rays < 0) return 0;
  const long np = (long)f->pbw_dims[0] * f->pbw_dims[1] * f->pbw_dims[2];
  const long nt = (long)f->tbw_dims[0] * f->tbw_dims[1] * f->tbw_dims[2];
  return layout(n_rays, o->chunk, np, nt, true).total;
}

const int32_t* anr_render_counts(const void* workspace, int n_rays) {
  return (const int32_t*)((const char*)workspace + layout(n_rays, 1, 0, 0, false).counts);
}

int anr_render_fwd(const anr_params* p, const anr_frame* f, const float* ray_o, const float* ray_d, const float* near_,
                   const float* far_, int n_rays, const anr_render_opts* o, const anr_render_out* out, void* workspace,
                   size_t ws_bytes, void* stream) {
  if (!p || !f || !o || !out || !workspace) return fail(ANR_E_ARG, "anr_render_fwd: NULL argument");
  if (o->n_samples != 64) return fail(ANR_E_ARG, "anr_render_fwd: only N_samples == 64 is supported");
  if (o->chunk <= 0) return fail(ANR_E_ARG, "anr_render_fwd: chunk must be > 0");
  if (n_rays <= 0) return fail(ANR_E_ARG, "anr_render_fwd: n_rays must be > 0");
  if ((long)n_rays * 64 > 0x7fffffffL / 24) return fail(ANR_E_ARG, "anr_render_fwd: too many rays for one call");
  if (!ray_o || !ray_d || !near_ || !far_ || !out->rgb_map || !out->acc_map || !out->depth_map || !p->packed)
    return fail(ANR_E_ARG, "anr_render_fwd: NULL tensor");
  for (int i = 0; i < 3; ++i)
    if (f->pbw_dims[i] <= 0 || f->tbw_dims[i] <= 0) return fail(ANR_E_ARG, "anr_render_fwd: bad volume dims");
  if (!f->A || !f->R || !f->Th || !f->pbw || !f->tbw || !f->pbounds || !f->tbounds || !f->latent_index)
    return fail(ANR_E_ARG, "anr_render_fwd: NULL frame tensor");
  if (o->novel_pose) {
    for (int i = 0; i < ANR_NUM_NOVEL_TENSORS; ++i)
      if (!p->novel[i]) return fail(ANR_E_ARG, "anr_render_fwd: novel_pose needs the novel_pose_bw tensors");
    if (!f->bw_latent_index) return fail(ANR_E_ARG, "anr_render_fwd: novel_pose needs bw_latent_index");
  }
  const long np = (long)f->pbw_dims[0] * f->pbw_dims[1] * f->pbw_dims[2];
  const long nt = (long)f->tbw_dims[0] * f->tbw_dims[1] * f->tbw_dims[2];
  const Layout L = layout(n_rays, o->chunk, np, nt, out->raw == nullptr);
  if (ws_bytes < L.total) return fail(ANR_E_WORKSPACE, "anr_render_fwd: workspace too small");

  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float4* raw = out->raw ? (float4*)out->raw : (float4*)(ws + L.raw);
  ANR_TRY(stage_frontend(p, f, ray_o, ray_d, near_, far_, n_rays, o, ws, L, raw, s));
  ANR_TRY(stage_mlp(p, f, ray_o, ray_d, near_, far_, n_rays, o, ws, L, raw, s));
  ANR_TRY(stage_alpha_ind(n_rays, o, ws, L, s));
  return stage_composite(near_, far_, n_rays, o, raw, out, nullptr, s);
}

// ---- Network.forward over free samples (include/aninerf.h) --------------------------------
static int check_network_args(const anr_params* p, const anr_frame* f, const anr_samples* x, const anr_render_opts* o,
                              const void* ws, const char* who) {
  const std::string w(who);
  if (!p || !f || !x || !o || !ws) return fail(ANR_E_ARG, w + ": NULL argument");
  if (!x->wpts || !x->viewdir || !x->dists) return fail(ANR_E_ARG, w + ": NULL sample tensor");
  if (x->n_pts <= 0 || (long)x->n_pts > 0x7fffffffL / 24 - 64) return fail(ANR_E_ARG, w + ": bad n_pts");
  for (int i = 0; i < 3; ++i)
    if (f->pbw_dims[i] <= 0 || f->tbw_dims[i] <= 0) return fail(ANR_E_ARG, w + ": bad volume dims");
  if (!f->A || !f->R || !f->Th || !f->pbw || !f->tbw || !f->pbounds || !f->tbounds || !f->latent_index)
    return fail(ANR_E_ARG, w + ": NULL frame tensor");
  if (f->n_views) return fail(ANR_E_ARG, w + ": the visibility filter is a renderer option (n_views must be 0)");
  for (int i = 0; i < ANR_NUM_TENSORS; ++i)
    if (!p->t[i]) return fail(ANR_E_ARG, w + ": NULL parameter tensor");
  return ANR_OK;
}

size_t anr_network_workspace_bytes(int n_pts, const anr_render_opts* o, const anr_frame* f) {
  if (!o || !f || n_pts <= 0) return 0;
  const int G = (n_pts + 63) / 64;
  const long np = (long)f->pbw_dims[0] * f->pbw_dims[1] * f->pbw_dims[2];
  const long nt = (long)f->tbw_dims[0] * f->tbw_dims[1] * f->tbw_dims[2];
  return layout(G, G, np, nt, true).total;
}

const int32_t* anr_network_counts(const void* workspace, int n_pts) {
  return anr_render_counts(workspace, (n_pts + 63) / 64);
}

int anr_network_bw_rows(const void* workspace, int n_pts, float* pbw, float* tbw, void* stream) {
  return anr_render_bw_rows(workspace, (n_pts + 63) / 64, pbw, tbw, stream);
}

int anr_network_fwd(const anr_params* p, const anr_frame* f, const anr_samples* x, const anr_render_opts* o, float* raw,
                    void* workspace, size_t ws_bytes, void* stream) {
  ANR_TRY(check_network_args(p, f, x, o, workspace, "anr_network_fwd"));
  if (!raw || !p->packed) return fail(ANR_E_ARG, "anr_network_fwd: NULL raw / weights not packed");
  if (o->novel_pose) {
    for (int i = 0; i < ANR_NUM_NOVEL_TENSORS; ++i)
      if (!p->novel[i]) return fail(ANR_E_ARG, "anr_network_fwd: novel_pose needs the novel_pose_bw tensors");
    if (!f->bw_latent_index) return fail(ANR_E_ARG, "anr_network_fwd: novel_pose needs bw_latent_index");
  }
  const int G = (x->n_pts + 63) / 64;
  anr_render_opts oo = *o;
  oo.chunk = G;  // one call = one reference chunk
  oo.t_rand = nullptr;
  const long np = (long)f->pbw_dims[0] * f->pbw_dims[1] * f->pbw_dims[2];
  const long nt = (long)f->tbw_dims[0] * f->tbw_dims[1] * f->tbw_dims[2];
  const Layout L = layout(G, G, np, nt, true);
  if (ws_bytes < L.total) return fail(ANR_E_WORKSPACE, "anr_network_fwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float4* wraw = (float4*)(ws + L.raw);
  ANR_TRY(stage_frontend(p, f, nullptr, nullptr, nullptr, nullptr, G, &oo, ws, L, wraw, s, x));
  ANR_TRY(stage_mlp(p, f, nullptr, nullptr, nullptr, nullptr, G, &oo, ws, L, wraw, s, x));
  ANR_TRY(stage_alpha_ind(G, &oo, ws, L, s));
  if (hipMemcpyAsync(raw, wraw, (size_t)x->n_pts * 16, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return fail(ANR_E_HIP, "anr_network_fwd: raw copy failed");
  return ANR_OK;
}

int anr_profile_enable(int on) {
  g_prof.on = on != 0;
  return ANR_OK;
}

int anr_profile_read_clock(double* mlp_ms, int* launches, double* clk_mhz) {
  double tot = 0.0;
  std::vector<double> mhz;
  std::vector<unsigned long long> h;
  for (size_t i = 0; i < g_prof.used; ++i) {
    const ProfSlot& q = g_prof.slot[i];
    if (hipEventSynchronize(q.e) != hipSuccess) return fail(ANR_E_HIP, "hipEventSynchronize failed");
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, q.b, q.e) != hipSuccess) return fail(ANR_E_HIP, "hipEventElapsedTime failed");
    tot += ms;
    const int ng = g_prof.groups[i];
    if (clk_mhz && q.clk && ng > 0) {
      h.resize((size_t)ng * 4);
      if (hipMemcpy(h.data(), q.clk, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(ANR_E_HIP, "hipMemcpy (clock stamps) failed");
      for (int g = 0; g < ng; ++g) {
        const unsigned long long* c = &h[(size_t)g * 4];
        // a workgroup that ran at least 20 us (2,000 realtime ticks: the ratio to 0.05 %) of its own — the
        // training chains and layer GEMMs run 30-80 us, the render kernel's workgroups ~140 ms
        if (c[2] > c[0] && c[3] > c[1] + 2000) mhz.push_back((double)(c[2] - c[0]) / (double)(c[3] - c[1]) * 100.0);
      }
    }
  }
  if (mlp_ms) *mlp_ms = tot;
  if (launches) *launches = (int)g_prof.used;
  if (clk_mhz) {
    *clk_mhz = 0.0;
    if (!mhz.empty()) {
      std::nth_element(mhz.begin(), mhz.begin() + mhz.size() / 2, mhz.end());
      *clk_mhz = mhz[mhz.size() / 2];
    }
  }
  g_prof.used = 0;
  return ANR_OK;
}

int anr_profile_read(double* mlp_ms, int* launches) { return anr_profile_read_clock(mlp_ms, launches, nullptr); }

int anr_render_bw_rows(const void* workspace, int n_rays, float* pbw, float* tbw, void* stream) {
  if (!workspace || n_rays <= 0 || !pbw || !tbw) return fail(ANR_E_ARG, "anr_render_bw_rows: bad arguments");
  const Layout L = layout(n_rays, 1, 0, 0, false);
  const char* ws = (const char*)workspace;
  const long N = (long)n_rays * 64;
  const int grid = (int)((N * 6 + 255) / 256);
  hipLaunchKernelGGL(k_gather_rows, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const int*)(ws + L.out_row),
                     (const int*)(ws + L.counts), (const float4*)(ws + L.pbw_rows), (const float4*)(ws + L.tbw_rows),
                     (float4*)pbw, (float4*)tbw);
  return check_launch("k_gather_rows");
}

int anr_sample_volume(const float* vol, int X, int Y, int Z, int C, const float* bounds, const float* pts, int n,
                      float* out, void* stream) {
  if (!vol || !bounds || !pts || !out || X <= 0 || Y <= 0 || Z <= 0 || C <= 0 || n < 0)
    return fail(ANR_E_ARG, "anr_sample_volume: bad arguments");
  if (n == 0) return ANR_OK;
  hipLaunchKernelGGL(k_sample_volume, dim3((unsigned)(((long)n * C + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     vol, X, Y, Z, C, bounds, pts, n, out);
  return check_launch("k_sample_volume");
}

int anr_render_row_ids(const void* workspace, int n_rays, int32_t* ids, void* stream) {
  if (!workspace || n_rays <= 0 || !ids) return fail(ANR_E_ARG, "anr_render_row_ids: bad arguments");
  const Layout L = layout(n_rays, 1, 0, 0, false);
  const char* ws = (const char*)workspace;
  const long N = (long)n_rays * 64;
  hipLaunchKernelGGL(k_row_ids, dim3((int)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const int*)(ws + L.out_row), (const int*)(ws + L.counts), (const int*)(ws + L.list), (int*)ids);
  return check_launch("k_row_ids");
}

}  // extern "C"
