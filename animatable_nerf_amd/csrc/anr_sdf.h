// anr_sdf.h — internal structures of the sdf_pdf render path (config 5).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace anr {

// state_dict order of anisdf_pdf_network.Network (include/aninerf.h, anr_sdf_params)
enum : int {
  SDF_LIN0 = 0,        // sdf_network.lin{l}: bias 3l, weight_g 3l+1, weight_v 3l+2 (l = 0..8)
  SDF_BETA = 27,       // tpose_human.beta_network.beta
  SDF_COLOR_LAT = 28,  // color_network.color_latent.weight (num_latent_code, 128)
  SDF_CLIN0 = 29,      // color_network.lin{l}: bias 29+3l, weight_g 30+3l, weight_v 31+3l (l = 0..4)
  SDF_RESD_LAT = 44,   // resd_latent.weight (unused by the render)
  SDF_RLIN0 = 45,      // resd_linears.{l}: weight 45+2l, bias 46+2l (l = 0..7)
  SDF_RFC_W = 61,
  SDF_RFC_B = 62,
  SDF_NUM_TENSORS = 63,
};

// weight-normed layers: 9 SDF + 5 colour, effective weights v * (g / |v|_row) packed back to back
struct WnLayer {
  int v, g, in, out;
  long off;  // float offset in the effective-weight image
};
constexpr int SDF_NUM_WN = 14;
__host__ __device__ constexpr WnLayer wn_layer(int i) {
  constexpr int ins[14] = {39, 256, 256, 256, 256, 256, 256, 256, 256, 289, 256, 256, 384, 256};
  constexpr int outs[14] = {256, 256, 256, 217, 256, 256, 256, 256, 257, 256, 256, 256, 256, 3};
  long off = 0;
  for (int k = 0; k < i; ++k) off += (long)ins[k] * outs[k];
  const int base = i < 9 ? 3 * i : SDF_CLIN0 + 3 * (i - 9);
  return WnLayer{base + 2, base + 1, ins[i], outs[i], off};
}
constexpr long SDF_WN_FLOATS = wn_layer(13).off + 256L * 3;
__host__ __device__ constexpr int sdf_wn_rows() {
  int r = 0;
  for (int i = 0; i < SDF_NUM_WN; ++i) r += wn_layer(i).out;
  return r;
}

// Free-sample mode (Network.forward(wpts, viewdir, dists, batch), anisdf_pdf_network.py:156-224):
// wpts != NULL replaces the rays: "ray" g is the group of points [64 g, 64 g + 64) of the call (n_pts
// points, the last group partial), chunk = the number of groups (the call is one reference chunk:
// its forced argmin spans every point), world -> pose by torch's matmul rule for an (n_pts, 3) product.
struct SdfFrontArgs {
  const float *ray_o, *ray_d, *near_, *far_, *t_rand;
  const float* wpts;    // (n_pts, 3) free samples or NULL
  int n_pts;
  int n_rays, chunk;
  const float *R, *Th;
  const float* verts;  // pvertices (nv, 3)
  int nv;
  float norm_th;
  uint64_t* mask;       // (R) keep ballots
  uint64_t* chunk_min;  // (nchunks) argmin keys, preset to ~0
  uint32_t* knn;        // (R*64, 8): w[5] (float bits), idx (3 x u32, u16 pairs)
  float4* raw;          // (R*64) zero at non-kept samples
  float* sdf;           // (R*64) 10 at non-kept samples
  int n_views;          // novel-view visibility filter (anr_sdf_frame), 0 = off
  const float *Ks, *RT;
  const uint8_t* msks;
  int img_h, img_w;
};

// per-point kernels over one batch [b0, b0 + cnt) of the compact kept-sample list
struct SdfPointArgs {
  const int* list;
  int b0, cnt;
  const float *ray_o, *ray_d, *near_, *far_, *t_rand;
  const float *wpts, *vdir;  // free-sample mode (SdfFrontArgs): points and world view directions, or NULL
  int n_pts;
  int chunk;
  const float *R, *Th, *A, *bigA;
  const float* weights;  // (nv, 24)
  const uint32_t* knn;
  const float* wimg;     // effective weight-normed weights
  const float* tbtab;    // (nchunks, 6) tbounds after this chunk's widening
  float* ptb;            // [P][8]: bigpose xyz, bigdir xyz
  float* Gr;             // [P][64] gamma_10(bigpose)
  const float* Yr;       // [P][4] resd_fc output
  float* Xs0;            // [P][40] gamma_6(tpose)
  float* X4;             // [P][256] lin4 input: cols 217..255 = gamma_6 / sqrt(2)
  int skip_sdf_in;       // the fused SDF forward forms gamma_6 itself: k_sdf_mid writes no Xs0 / X4 columns
  float* C0;             // [P][40] colour input: tpose, gamma_4(bigdir), gradient
  const float* D7;       // [P][256] softplus factor of lin7 (d7_h: lin7's softplus output h)
  int d7_h;
  float* G7;             // [P][256]
  const float* Gc;       // [P][256] lin4 input gradient (cols 217..255: gamma part)
  const float* gB;       // [P][40] lin0 input gradient
  const float* Y8;       // [P][264] lin8 output: sdf, feature
  const float* Yc;       // [P][4] colour logits
  float beta;
  float* resd_rows;      // (n', 3) compact output
  float* grad_rows;      // (n', 3)
  float4* raw;           // (R*64)
  float* sdf;            // (R*64)
};

struct SdfTensors {
  const float* t[SDF_NUM_TENSORS];  // kernel argument by value (504 B)
};

__global__ void k_sdf_front(SdfFrontArgs a);
__global__ void k_sdf_wnorm(SdfTensors T, float* wimg);
__global__ void k_sdf_fold(SdfTensors T, const float* wimg, const float* poses, const int64_t* li, float* fold);
__global__ void k_sdf_tbtab(const float* tbounds, int nchunks, float* tbtab, float* tb_out, const uint64_t* chunk_min = nullptr);
__global__ void k_sdf_prep(SdfPointArgs a);
__global__ void k_knn_blend_out(const uint32_t* knn, const uint64_t* mask, const float* weights, int n, float* bw,
                                uint8_t* inside);
__global__ void k_mesh_pose(const float* pts, const float* bw, int n, const float* bigA, const float* A, const float* R,
                            const float* Th, float* out);
__global__ void k_sdf_mid(SdfPointArgs a);
__global__ void k_sdf_gtop(SdfPointArgs a);
__global__ void k_sdf_gamma_bwd(SdfPointArgs a);
__global__ void k_sdf_raw(SdfPointArgs a);

struct SdfMskArgs {
  const float* sdf;        // (R*64)
  const uint8_t* occ;      // (R)
  int n_rays, chunk;
  float* min_sdf;          // (R)
  uint8_t* flags;          // (R): bit0 = no intersection & occ == 1, bit1 = occ == 0
  int* chunk_cnt;          // (nchunks) -> exclusive offsets after k_scan_blocks
  int* total;
  float* msk_sdf;          // (R) compact
  float* msk_label;
};
__global__ void k_sdf_msk_rays(SdfMskArgs a);
__global__ void k_sdf_msk_count(SdfMskArgs a);
__global__ void k_sdf_msk_write(SdfMskArgs a);

}  // namespace anr
