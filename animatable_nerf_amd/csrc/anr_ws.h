// anr_ws.h — render workspace layout (shared by the render and training entry points).
#pragma once
#include <stddef.h>
#include <string>

#include <hip/hip_runtime.h>

#include "../../include/aninerf.h"
#include "anr_layers.h"

namespace anr {

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Workspace layout. Fields up to `tbw_rows` depend only on n_rays (anr_render_counts/bw_rows).
struct Layout {
  size_t counts, mask, ray_off, block_sum, list, sigma, flags, block_sum2, out_row, pbw_rows, tbw_rows;
  size_t chunk_min, chunk_max, raw, pbw32, tbw32, pn24, fold, total;
};

inline Layout layout(int n_rays, int chunk, long np, long nt, bool need_raw) {
  Layout L{};
  const size_t R = (size_t)n_rays, N = R * 64;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align256(o + bytes);
    return at;
  };
  L.counts = take(16);
  L.mask = take(R * 8);
  L.ray_off = take((R + 1) * 4);
  L.block_sum = take(((R + 255) / 256) * 4);
  L.list = take(N * 4);
  L.sigma = take(N * 4);
  L.flags = take(N);
  L.block_sum2 = take(((N + 1023) / 1024) * 4);
  L.out_row = take(N * 4);
  L.pbw_rows = take(N * 24 * 4);
  L.tbw_rows = take(N * 24 * 4);
  const size_t nch = (R + chunk - 1) / (chunk > 0 ? chunk : 1);
  L.chunk_min = take(nch * 8);
  L.chunk_max = take(nch * 8);
  L.raw = need_raw ? take(N * 16) : 0;
  L.pbw32 = take((size_t)np * 32 * 4);
  L.tbw32 = take((size_t)nt * 32 * 4);
  L.pn24 = take((size_t)np * 4);
  L.fold = take(ANR_FOLD_FLOATS * 4);
  L.total = o;
  return L;
}


int fail(int code, const std::string& msg);
int check_launch(const char* what);
#define ANR_TRY(x)                  \
  do {                              \
    const int _rc = (x);            \
    if (_rc != ANR_OK) return _rc;  \
  } while (0)

// ray split of one reference chunk over ranks (anr_train_hooks): ray offset + the host reduction hook
struct RaySplit {
  int ray_offset;
  anr_reduce_fn reduce;
  void* user;
  int run(void* buf, int count, int op, hipStream_t s) const;
};

// x != NULL: free samples (Network.forward): R = ceil(n_pts / 64) groups of 64 samples, the caller's
// opts with chunk = R (the whole call is one reference chunk) and no t_rand; ray pointers unused
int stage_frontend(const anr_params* p, const anr_frame* f, const float* ray_o, const float* ray_d, const float* near_,
                   const float* far_, int R, const anr_render_opts* o, char* ws, const Layout& L, float4* raw,
                   hipStream_t s, const anr_samples* x = nullptr, const RaySplit* split = nullptr);
int stage_mlp(const anr_params* p, const anr_frame* f, const float* ray_o, const float* ray_d, const float* near_,
              const float* far_, int R, const anr_render_opts* o, char* ws, const Layout& L, float4* raw,
              hipStream_t s, const anr_samples* x = nullptr);
int stage_alpha_ind(int R, const anr_render_opts* o, char* ws, const Layout& L, hipStream_t s,
                    const RaySplit* split = nullptr);
int stage_composite(const float* near_, const float* far_, int R, const anr_render_opts* o, const float4* raw,
                    const anr_render_out* out, float* weights, hipStream_t s);

}  // namespace anr
