// anr_mesh.hip — (f) mesh path: the density of free points and the
// marching-cubes extraction of lib/networks/renderer/aninerf_mesh_renderer.py:26-63.
//
//   anr_alpha_points   Network.get_alpha (tpose_nerf_network.py:105-137) over batchify chunks of
//                      free points: world->pose, pbw prefilter (pnorm < 0.1 plus the per-chunk
//                      argmin, k_frontend_pts), ordered compaction, then the density program of the
//                      fused network kernel (k_alpha / k_alpha_b16) scattering raw alpha by point id.
//                      No host synchronisation (graph-capturable), like anr_render_fwd.
//   anr_mc_count/emit  mcubes.marching_cubes(np.pad(cube, pad), iso) (aninerf_mesh_renderer.py:43-45)
//                      in two launches each: per grid point its crossing edges (one vertex each,
//                      owned by the edge's lower end) and per cube its case (anr_mc_table.h), block
//                      scans of both counts, then vertices and triangles written in grid order.
//                      The padding is virtual (values outside the cube read as 0).
#include <string>

#include "../../include/aninerf.h"
#include "anr_common.h"
#include "anr_kernels.h"
#include "anr_layers.h"
#include "anr_mc_table.h"
#include "anr_ws.h"

#pragma clang fp contract(off)

namespace anr {

struct McArgs {
  const float* vol;
  int X, Y, Z, pad;
  int Xp, Yp, Zp;
  double iso;
  uint8_t* flags;   // (P) bit a: the edge from this point along axis a crosses the iso level
  uint8_t* cases;   // (P) case index of the cube whose lower corner is this point (0 if none)
  int* voff;        // (P) block-local vertex offsets
  int* toff;        // (P) block-local triangle offsets
  int* vblock;      // (nb) vertex block sums -> exclusive offsets
  int* tblock;      // (nb) triangle block sums -> exclusive offsets
  int* counts;      // [V, T]
  double* verts;    // (V, 3)
  int64_t* tris;    // (T, 3)
};

__device__ __forceinline__ double mc_val(const McArgs& a, int i, int j, int k) {
  i -= a.pad;
  j -= a.pad;
  k -= a.pad;
  if (i < 0 || j < 0 || k < 0 || i >= a.X || j >= a.Y || k >= a.Z) return 0.0;
  return (double)a.vol[((size_t)i * a.Y + j) * a.Z + k];
}

__global__ __launch_bounds__(256) void k_mc_count(McArgs a) {
  __shared__ int sh[4];
  const long P = (long)a.Xp * a.Yp * a.Zp;
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  int nv = 0, nt = 0;
  if (q < P) {
    const int k = (int)(q % a.Zp);
    const int j = (int)((q / a.Zp) % a.Yp);
    const int i = (int)(q / ((long)a.Zp * a.Yp));
    const bool o0 = mc_val(a, i, j, k) <= a.iso;
    int f = 0;
    if (i + 1 < a.Xp && (mc_val(a, i + 1, j, k) <= a.iso) != o0) f |= 1;
    if (j + 1 < a.Yp && (mc_val(a, i, j + 1, k) <= a.iso) != o0) f |= 2;
    if (k + 1 < a.Zp && (mc_val(a, i, j, k + 1) <= a.iso) != o0) f |= 4;
    int c = 0;
    if (i + 1 < a.Xp && j + 1 < a.Yp && k + 1 < a.Zp) {
      // corners c0..c7 = (0,0,0) (1,0,0) (1,1,0) (0,1,0) (0,0,1) (1,0,1) (1,1,1) (0,1,1)
      const int dx[8] = {0, 1, 1, 0, 0, 1, 1, 0}, dy[8] = {0, 0, 1, 1, 0, 0, 1, 1}, dz[8] = {0, 0, 0, 0, 1, 1, 1, 1};
#pragma unroll
      for (int m = 0; m < 8; ++m)
        if (mc_val(a, i + dx[m], j + dy[m], k + dz[m]) <= a.iso) c |= 1 << m;
    }
    a.flags[q] = (uint8_t)f;
    a.cases[q] = (uint8_t)c;
    nv = __popc(f);
    nt = kMcCount[c];
  }
  int tv, tt;
  const int ev = block_excl_scan_256(nv, sh, tv);
  const int et = block_excl_scan_256(nt, sh, tt);
  if (q < P) {
    a.voff[q] = ev;
    a.toff[q] = et;
  }
  if (threadIdx.x == 0) {
    a.vblock[blockIdx.x] = tv;
    a.tblock[blockIdx.x] = tt;
  }
}

__global__ __launch_bounds__(256) void k_mc_emit(McArgs a) {
  const long P = (long)a.Xp * a.Yp * a.Zp;
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= P) return;
  const int k = (int)(q % a.Zp);
  const int j = (int)((q / a.Zp) % a.Yp);
  const int i = (int)(q / ((long)a.Zp * a.Yp));
  const int f = a.flags[q];
  if (f) {
    long v = (long)a.vblock[blockIdx.x] + a.voff[q];
    const double f0 = mc_val(a, i, j, k);
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      if (!(f >> ax & 1)) continue;
      const double f1 = mc_val(a, i + (ax == 0), j + (ax == 1), k + (ax == 2));
      const double t = (a.iso - f0) / (f1 - f0);
      a.verts[3 * v + 0] = (double)i + (ax == 0 ? t : 0.0);
      a.verts[3 * v + 1] = (double)j + (ax == 1 ? t : 0.0);
      a.verts[3 * v + 2] = (double)k + (ax == 2 ? t : 0.0);
      ++v;
    }
  }
  const int c = a.cases[q];
  const int nt = kMcCount[c];
  if (nt) {
    long t = (long)a.tblock[blockIdx.x] + a.toff[q];
    for (int m = 0; m < nt; ++m, ++t) {
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const int edge = kMcTris[c][3 * m + e];
        const long o = (((long)(i + kMcEdgeOwner[edge][0]) * a.Yp) + (j + kMcEdgeOwner[edge][1])) * a.Zp +
                       (k + kMcEdgeOwner[edge][2]);
        const int ax = kMcEdgeOwner[edge][3];
        const int below = __popc(a.flags[o] & ((1 << ax) - 1));
        a.tris[3 * t + e] = (int64_t)a.vblock[o / 256] + a.voff[o] + below;
      }
    }
  }
}

}  // namespace anr

using namespace anr;

namespace {

struct AlphaLayout {
  Layout L;  // the render layout's fields the free-point pipeline uses (groups of 64 points)
};

AlphaLayout alpha_layout(long n_pts, int chunk_pts, long np) {
  const size_t G = (size_t)((n_pts + 63) / 64), N = G * 64;
  const size_t nch = (G + chunk_pts / 64 - 1) / (chunk_pts / 64);
  AlphaLayout A{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align256(o + bytes);
    return at;
  };
  A.L.counts = take(16);
  A.L.mask = take(G * 8);
  A.L.ray_off = take((G + 1) * 4);
  A.L.block_sum = take(((G + 255) / 256) * 4);
  A.L.list = take(N * 4);
  A.L.chunk_min = take(nch * 8);
  A.L.pbw32 = take((size_t)np * 32 * 4);
  A.L.fold = take(1280 * 4);
  A.L.total = o;
  return A;
}

bool alpha_attr_set = false;

int num_cus_here() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
    return 256;
  return v;
}

struct McLayout {
  size_t flags, cases, voff, toff, vblock, tblock, counts, total;
};

McLayout mc_layout(int X, int Y, int Z, int pad) {
  const size_t P = (size_t)(X + 2 * pad) * (Y + 2 * pad) * (Z + 2 * pad);
  const size_t nb = (P + 255) / 256;
  McLayout M{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align256(o + bytes);
    return at;
  };
  M.counts = take(16);
  M.flags = take(P);
  M.cases = take(P);
  M.voff = take(P * 4);
  M.toff = take(P * 4);
  M.vblock = take(nb * 4);
  M.tblock = take(nb * 4);
  M.total = o;
  return M;
}

McArgs mc_args(const float* vol, int X, int Y, int Z, int pad, double iso, char* ws) {
  const McLayout M = mc_layout(X, Y, Z, pad);
  McArgs a{};
  a.vol = vol; a.X = X; a.Y = Y; a.Z = Z; a.pad = pad;
  a.Xp = X + 2 * pad; a.Yp = Y + 2 * pad; a.Zp = Z + 2 * pad;
  a.iso = iso;
  a.flags = (uint8_t*)(ws + M.flags); a.cases = (uint8_t*)(ws + M.cases);
  a.voff = (int*)(ws + M.voff); a.toff = (int*)(ws + M.toff);
  a.vblock = (int*)(ws + M.vblock); a.tblock = (int*)(ws + M.tblock);
  a.counts = (int*)(ws + M.counts);
  return a;
}

int mc_check(const float* vol, int X, int Y, int Z, int pad, void* ws, size_t ws_bytes) {
  if (!vol || !ws || X <= 0 || Y <= 0 || Z <= 0 || pad < 0) return fail(ANR_E_ARG, "anr_mc: bad arguments");
  if ((double)(X + 2 * pad) * (Y + 2 * pad) * (Z + 2 * pad) > 2.0e9) return fail(ANR_E_ARG, "anr_mc: grid too large");
  if (ws_bytes < mc_layout(X, Y, Z, pad).total) return fail(ANR_E_WORKSPACE, "anr_mc: workspace too small");
  return ANR_OK;
}

}  // namespace

extern "C" {

size_t anr_alpha_workspace_bytes(long n_pts, const anr_alpha_opts* o, const anr_frame* f) {
  if (!o || !f || n_pts <= 0 || o->chunk_pts <= 0 || o->chunk_pts % 64) return 0;
  const long np = (long)f->pbw_dims[0] * f->pbw_dims[1] * f->pbw_dims[2];
  return alpha_layout(n_pts, o->chunk_pts, np).L.total;
}

int anr_alpha_points(const anr_params* p, const anr_frame* f, const float* wpts, long n_pts, const anr_alpha_opts* o,
                     float* alpha, void* workspace, size_t ws_bytes, void* stream) {
  if (!p || !f || !o || !wpts || !alpha || !workspace) return fail(ANR_E_ARG, "anr_alpha_points: NULL argument");
  if (n_pts <= 0 || n_pts > (1L << 31) - 64) return fail(ANR_E_ARG, "anr_alpha_points: bad point count");
  if (o->chunk_pts <= 0 || o->chunk_pts % 64) return fail(ANR_E_ARG, "anr_alpha_points: chunk_pts must be a positive multiple of 64");
  if (!p->packed) return fail(ANR_E_ARG, "anr_alpha_points: weights not packed");
  for (int i = 0; i < 3; ++i)
    if (f->pbw_dims[i] <= 0) return fail(ANR_E_ARG, "anr_alpha_points: bad pbw dims");
  if (!f->A || !f->R || !f->Th || !f->pbw || !f->pbounds || !f->latent_index)
    return fail(ANR_E_ARG, "anr_alpha_points: NULL frame tensor");
  if (o->novel_pose) {
    for (int i = 0; i < ANR_NUM_NOVEL_TENSORS; ++i)
      if (!p->novel[i]) return fail(ANR_E_ARG, "anr_alpha_points: novel_pose needs the novel_pose_bw tensors");
    if (!f->bw_latent_index) return fail(ANR_E_ARG, "anr_alpha_points: novel_pose needs bw_latent_index");
  }
  const long np = (long)f->pbw_dims[0] * f->pbw_dims[1] * f->pbw_dims[2];
  const Layout L = alpha_layout(n_pts, o->chunk_pts, np).L;
  if (ws_bytes < L.total) return fail(ANR_E_WORKSPACE, "anr_alpha_points: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const int G = (int)((n_pts + 63) / 64);  // groups of 64 points
  const int chunk = o->chunk_pts / 64;
  const int nch = (G + chunk - 1) / chunk;
  if (hipMemsetAsync(ws + L.counts, 0, 16, s) != hipSuccess ||
      hipMemsetAsync(ws + L.chunk_min, 0xff, (size_t)nch * 8, s) != hipSuccess ||
      hipMemsetAsync(alpha, 0, (size_t)n_pts * 4, s) != hipSuccess)
    return fail(ANR_E_HIP, "hipMemsetAsync failed");

  // pbw volume repack + the pose-pass folded biases (k_prep with no T-pose volume)
  PrepArgs pa{};
  pa.pbw = f->pbw; pa.pbw32 = (float*)(ws + L.pbw32); pa.np = (int)np; pa.nt = 0;
  pa.w_bw0 = p->t[28]; pa.b_bw0 = p->t[29]; pa.w_bw5 = p->t[38]; pa.b_bw5 = p->t[39];
  pa.bw_latent = p->t[27]; pa.w_lat = p->t[21]; pa.b_lat = p->t[22]; pa.nf_latent = p->t[0];
  pa.latent_index = f->latent_index;
  pa.fold = (float*)(ws + L.fold);
  if (o->novel_pose) {
    pa.novel = 1;
    pa.n_latent = p->novel[0];
    pa.nw_bw0 = p->novel[1]; pa.nb_bw0 = p->novel[2];
    pa.nw_bw5 = p->novel[11]; pa.nb_bw5 = p->novel[12];
    pa.bw_latent_index = f->bw_latent_index;
  }
  hipLaunchKernelGGL(k_prep, dim3(prep_blocks(np, 0)), dim3(256), 0, s, pa);
  ANR_TRY(check_launch("k_prep"));

  FrontArgs fa{};
  fa.n_rays = G; fa.chunk = chunk;
  fa.R = f->R; fa.Th = f->Th; fa.pbw = f->pbw; fa.pbounds = f->pbounds;
  fa.X = f->pbw_dims[0]; fa.Y = f->pbw_dims[1]; fa.Z = f->pbw_dims[2];
  fa.norm_th = o->norm_th;
  fa.mask = (uint64_t*)(ws + L.mask);
  fa.chunk_min = (uint64_t*)(ws + L.chunk_min);
  fa.wpts = wpts; fa.n_pts = n_pts; fa.chunk_pts = o->chunk_pts;
  hipLaunchKernelGGL(k_frontend_pts, dim3((G + 3) / 4), dim3(256), 0, s, fa);
  ANR_TRY(check_launch("k_frontend_pts"));

  CompactArgs ca{};
  ca.n_rays = G; ca.chunk = chunk;
  ca.mask = fa.mask; ca.chunk_min = fa.chunk_min;
  ca.ray_off = (int*)(ws + L.ray_off);
  ca.block_sum = (int*)(ws + L.block_sum);
  ca.list = (int*)(ws + L.list);
  const int nb = (G + 255) / 256;
  hipLaunchKernelGGL(k_count, dim3(nb), dim3(256), 0, s, ca);
  ANR_TRY(check_launch("k_count"));
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, ca.block_sum, nb, (int*)(ws + L.counts));
  ANR_TRY(check_launch("k_scan_blocks"));
  hipLaunchKernelGGL(k_compact, dim3((G + 3) / 4), dim3(256), 0, s, ca);
  ANR_TRY(check_launch("k_compact"));

  MlpArgs ma{};
  ma.wimg = (const unsigned char*)p->packed;
  ma.bias = (const float*)((const unsigned char*)p->packed + weights_bytes());
  ma.fold = (const float*)(ws + L.fold);
  ma.A = f->A; ma.R = f->R; ma.Th = f->Th;
  ma.pbw32 = (const float*)(ws + L.pbw32); ma.pbounds = f->pbounds;
  ma.pX = f->pbw_dims[0]; ma.pY = f->pbw_dims[1]; ma.pZ = f->pbw_dims[2];
  ma.list = (const int*)(ws + L.list); ma.n_kept = (const int*)(ws + L.counts);
  ma.wpts = wpts; ma.n_pts = n_pts; ma.chunk_pts = o->chunk_pts; ma.alpha_out = alpha;
  const bool x6 = o->precision == ANR_BF16X6;
  const bool b16 = o->precision == ANR_BF16X3 || x6;
  ma.pose_woff = o->novel_pose ? (x6 || (b16 && ANR_POSE_MODE == 2) ? ANR_X6_NOVEL_WOFF : b16 ? ANR_B16_NOVEL_WOFF : ANR_NOVEL_WOFF) : 0;
  ma.pose_boff = o->novel_pose ? ANR_NOVEL_BOFF : 0;
  if (!alpha_attr_set) {
    if (hipFuncSetAttribute((const void*)k_alpha, hipFuncAttributeMaxDynamicSharedMemorySize, mlp_lds_bytes<false>()) !=
            hipSuccess ||
        hipFuncSetAttribute((const void*)k_alpha_b16, hipFuncAttributeMaxDynamicSharedMemorySize,
                            mlp_lds_bytes<true>()) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_alpha_x6, hipFuncAttributeMaxDynamicSharedMemorySize,
                            mlp_lds_bytes<true>()) != hipSuccess)
      return fail(ANR_E_HIP, "hipFuncSetAttribute(k_alpha) failed");
    alpha_attr_set = true;
  }
  const long max_tiles = ((long)G * 64 + 127) / 128;
  const int cus = num_cus_here();
  const int grid = (int)(max_tiles < cus ? max_tiles : cus);
  if (x6) hipLaunchKernelGGL(k_alpha_x6, dim3(grid), dim3(512), mlp_lds_bytes<true>(), s, ma);
  else if (b16) hipLaunchKernelGGL(k_alpha_b16, dim3(grid), dim3(512), mlp_lds_bytes<true>(), s, ma);
  else hipLaunchKernelGGL(k_alpha, dim3(grid), dim3(512), mlp_lds_bytes<false>(), s, ma);
  return check_launch("k_alpha");
}

const int32_t* anr_alpha_counts(const void* workspace) { return (const int32_t*)workspace; }

size_t anr_mc_workspace_bytes(int X, int Y, int Z, int pad) {
  if (X <= 0 || Y <= 0 || Z <= 0 || pad < 0) return 0;
  return mc_layout(X, Y, Z, pad).total;
}

int anr_mc_count(const float* vol, int X, int Y, int Z, int pad, double iso, int32_t* counts, void* workspace,
                 size_t ws_bytes, void* stream) {
  ANR_TRY(mc_check(vol, X, Y, Z, pad, workspace, ws_bytes));
  if (!counts) return fail(ANR_E_ARG, "anr_mc_count: NULL counts");
  McArgs a = mc_args(vol, X, Y, Z, pad, iso, (char*)workspace);
  hipStream_t s = (hipStream_t)stream;
  const long P = (long)a.Xp * a.Yp * a.Zp;
  const int nb = (int)((P + 255) / 256);
  hipLaunchKernelGGL(k_mc_count, dim3(nb), dim3(256), 0, s, a);
  ANR_TRY(check_launch("k_mc_count"));
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, a.vblock, nb, a.counts);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, a.tblock, nb, a.counts + 1);
  ANR_TRY(check_launch("k_scan_blocks(mc)"));
  if (hipMemcpyAsync(counts, a.counts, 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return fail(ANR_E_HIP, "anr_mc_count: copy failed");
  return ANR_OK;
}

int anr_mc_emit(const float* vol, int X, int Y, int Z, int pad, double iso, double* vertices, int64_t* triangles,
                void* workspace, size_t ws_bytes, void* stream) {
  ANR_TRY(mc_check(vol, X, Y, Z, pad, workspace, ws_bytes));
  if (!vertices || !triangles) return fail(ANR_E_ARG, "anr_mc_emit: NULL output");
  McArgs a = mc_args(vol, X, Y, Z, pad, iso, (char*)workspace);
  a.verts = vertices;
  a.tris = triangles;
  const long P = (long)a.Xp * a.Yp * a.Zp;
  hipLaunchKernelGGL(k_mc_emit, dim3((int)((P + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("k_mc_emit");
}

}  // extern "C"
