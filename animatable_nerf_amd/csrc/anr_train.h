// anr_train.h — internal structures of the layer-wise training executor (anr_train.hip, anr_gemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace anr {

struct GemmSeg {
  const float* A;
  long a_rs, a_cs;
  const float* B;
  long b_rs, b_cs;
  int K;
};

struct GemmArgs {
  int M;
  const int* M_dev;  // if set, M is read from device memory
  const int* K_dev;  // if set, segment 0's K is read from device memory (sample-reduction GEMMs)
  int N;
  int nseg;
  GemmSeg seg[2];
  float* C;
  long ldc;
  const float* bias;   // (N) or NULL
  int relu;            // apply ReLU
  const float* mask;   // multiply by (mask > 0) (ReLU derivative), or NULL
  long ldm;
  int accumulate;      // C += result (non-atomic)
  int atomic;          // atomicAdd into C (split-K)
  int ksplit;          // number of K splits (grid.z)
  int kper;            // > 0: each split covers kper of K (splits past K exit); 0: K / ksplit rounded up
  // sdf_pdf epilogues (anr_sdf*.hip); all off when zero / NULL
  float div_pre;       // v = v / div_pre before the activation (backward of cat(...)/sqrt(2))
  int softplus;        // v = Softplus(beta=100)(v); deriv[m][n] = exp(100 v) or -1 above the threshold (deriv may be NULL)
  float* deriv;
  long ldd;
  const float* spd;    // softplus backward: v = d < 0 ? v : v * d / (d + 1), d = spd[m][n], n < spd_n
  long ldsd;
  int spd_n;
  int spd_h;           // spd (and the ATR activations) hold softplus OUTPUTS h instead: factor = softplus_factor_h(h)
  float spd_scale;     // spd_h: the stored values are h / spd_scale (0: 1), e.g. lin3's cat(...)/sqrt(2) output
  float div_post;      // v = v / div_post after the activation (cat(...)/sqrt(2) forward)
  // activations are softplus factors d: A(m, k) = d >= 0 ? w[k] d / (d + 1) : w[k] (k_lgemm only)
  const float* a_softplus_w;
  // k_lgemm only: a following small layer (head_n <= 4 outputs of head_w (head_n, N) + head_b) fused into
  // the epilogue; C is then not written and head_out (ld ldh, zeroed by the caller) receives the result
  const float* head_w;
  const float* head_b;
  float* head_out;
  long ldh;
  int head_n;
  int bf16;            // operands rounded to bf16, bf16 MFMA, fp32 accumulate (training precision)
  int x3;              // operands split hi + lo (bf16 each), three bf16 MFMAs per product (fp32-level)
  int prof;            // k_lgemm: a profiling slot (anr_profile_*: events + per-workgroup clock stamps)
  // weight-gradient GEMMs (A(m,k) = dY[k][m]): the fp32 row sums of A over this launch's k range
  // (= the bias gradient, the column sums of dY) are atomically added into rowsum[m] (and rowsum2[m])
  // by the workgroups of the first N tile; NULL: off
  float* rowsum;
  float* rowsum2;
  // per segment: the operand tiles may be read with 16-B loads (aligned base, stride a multiple of 4)
  int a_vec[2], b_vec[2];
  int vec_out;  // set by launch_gemm: non-atomic epilogue with 16-B accesses
};

void launch_gemm(GemmArgs g, dim3 grid, hipStream_t s);

// bf16 row GEMM with a weight-image B operand (anr_tgemm.hip): C[M][N] = epi(sum_s A_s[M][K_s] B_s^T),
// A_s fp32 (or, abf, bf16) rows (stride lda elements, 16-B aligned, lda >= K_s rounded up to 64), B_s bf16 image rows
// (k-contiguous, stride ldb, chunk-aligned column offset bcol, `rows` valid rows), N <= 256
struct RGemmSeg {
  const float* A;
  long lda;
  int K;
  const unsigned short* B;
  long ldb;
  int bcol;
  int rows;
  long lo_off;  // elements from B to the same rows of the lo image (x3)
};
struct RGemm {
  int M;
  const int* M_dev;
  int N;
  int nseg;
  RGemmSeg seg[2];
  float* C;
  long ldc;
  const float* bias;
  int relu;
  const float* mask;
  long ldm;
  int accumulate;
  int vec_out;  // set by launch_rgemm: C (and mask) rows 16-B addressable, N % 4 == 0
  int vec16;    // set by launch_rgemm: bf16 C rows take 16-B stores (ldc % 8 == 0, C 16-B aligned)
  int x3;       // split-bf16 products (fp32-level): activations hi/lo, weights hi/lo images
  // bf16 storage (training precision 'bf16': every consumer rounds these to bf16 anyway): A rows,
  // C rows (RNE from the fp32 result) and the mask rows hold bf16 (C / mask reinterpreted as
  // unsigned short*). Not with x3; C bf16 excludes accumulate.
  int abf, cbf, mbf;
};
void launch_rgemm(const RGemm& g, int M_host, hipStream_t s);
// bf16 weight images of the training GEMM weights: forward (rows = outputs, k = used input columns,
// segments padded to 64) and backward (rows = input columns, k = outputs padded to 64). t: the
// ANR_NUM_TENSORS network tensors followed by the ANR_NUM_NOVEL_TENSORS novel_pose_bw tensors
// (NULL when absent: their images are then neither packed nor viewable)
size_t wimg_bytes();
int wimg_pack(const float* const* t, void* dst, hipStream_t s);
struct WView {
  const unsigned short* B;
  long ldb;
  int bcol;
  int rows;
  long lo_off;
};
bool wimg_view(const void* base, const float* const* t, const float* W, int c0, int K, bool bwd, WView* v);

// bf16 weight gradient with per-sample-range partial slabs (anr_tgemm.hip): dW[i][j] (ldw) +=
// sum_s dY[s][i] X[s][j], i < nout <= 256, j < K <= 256; column sums of dY into bsum / bsum2.
// dY, X: fp32 rows, 16-B aligned, ld % 4 == 0. slab: wgrad_slab_floats() of workspace.
#define WG_MAX_Z 64
struct WGrad {
  const float* dY;
  long ldY;
  int nout;
  const float* X;
  long ldX;
  int K;
  float* dW;
  long ldw;
  float* bsum;
  float* bsum2;
  int n;
  const int* M_dev;
  float* slab;
  float* rs_slab;
  int spb, nz, tiles, tj;
  int x3;  // split-bf16 products (fp32-level)
  int ybf, xbf;  // dY / X rows hold bf16 (reinterpreted as unsigned short*), not with x3
  int j0;        // k_wgrad_f32: columns j < j0 are not written (X starts j0 columns early, at a 16-B boundary)
};
size_t wgrad_slab_floats();
int launch_wgrad(WGrad g, int n_host, hipStream_t s);
// exact-fp32 weight gradient (k_wgrad_f32 + k_wgrad_reduce; fp32 rows, nout / K <= 256, 16-B addressable
// rows): the exact executors' dW += dY^T X (+ bsum / bsum2 column sums), ACCUMULATED like the atomic
// split-K GEMM it replaces; -1 (nothing launched) for a product it does not take
bool wgrad_f32_fits(const WGrad& g);
int launch_wgrad_f32(WGrad g, int n_host, hipStream_t s);
// several weight gradients in two launches (k_wgrad_group + k_wgrad_reduce_group): d[0..nd) as for
// launch_wgrad (dY, X, dW, bsum, M_dev, formats; slab fields ignored) with nz sample ranges each, their
// partial slabs packed into slab[0, slab_floats); more descriptors than fit one launch (WG_GROUP_MAX, or
// the slab region) are issued as consecutive groups on s, reusing the region in stream order
#define WG_GROUP_MAX 16
struct WGradGroup {
  WGrad d[WG_GROUP_MAX];
  int n;
  int start[WG_GROUP_MAX + 1];   // first workgroup of descriptor k (k_wgrad_group)
  int rstart[WG_GROUP_MAX + 1];  // first reduce block of descriptor k (k_wgrad_reduce_group)
};
int launch_wgrad_group(const WGrad* d, int nd, int n_host, int nz, float* slab, size_t slab_floats, hipStream_t s);

// fused chains of the bf16 training executor (anr_tchain.hip): program 0 = the blend-weight MLP forward
// (9 layers), 1 = the canonical NeRF forward (8 layers + feature||alpha, latent, view, rgb), 2 / 3 their
// input-gradient chains (transposed weights, ReLU masks from the stored activations). Weight image per
// program (tchain_image_bytes), packed from the layers' fp32 weights every call (tchain_pack).
struct TcPackLayer {
  // forward layers: output rows 0 .. n1-1 of W, n1 .. n1+n2-1 of W2 (feature_fc || alpha_fc); inputs at
  // columns cmem (memory operand, kmem_cols wide) and cprev (previous layer, kprev_cols wide).
  // transposed layers (input gradients): the k side is W's output rows (previous-layer k-steps,
  // kprev_cols) or W2's (memory k-steps, kmem_cols); output neuron m < oa is input column oc0 + m,
  // m in [ob_b0, ob_b0 + nb) is column oc1 + m - ob_b0
  const float* W;
  int in_ch, n1;
  const float* W2;
  int in_ch2, n2;
  int cmem, kmem_cols;
  int cprev, kprev_cols;
  int oc0, oa, oc1, nb, ob_b0;
  long start;             // filled by tchain_pack
  int ob, kmem, kprev, mem_first, trans;
};
struct TcPackArgs {
  TcPackLayer L[12];
  int nl;
  long total;
  unsigned short* out;
};
struct TcArgs {
  const unsigned char* img;
  const float* bias[12];  // per layer (nout[l] floats)
  const float* bias2;     // program 1: alpha_fc's bias (row 256 of feature || alpha)
  int nout[12];
  void* out[12];          // per layer: bf16 rows (hidden, feature, latent) or fp32 rows (heads)
  int ldo[12];
  float* out2;            // program 1: alpha (fp32, one per sample)
  const unsigned short* mem;   // gamma rows (bf16)
  int ld_mem, kmem_cols;
  const unsigned short* mem2;  // program 1: gamma(dir) rows (bf16)
  int ld_mem2, kmem2_cols;
  int mem_f32, mem2_f32;  // the memory operands are fp32 rows (else bf16)
  // ReLU mask bits per layer, rows of 32 B (lane h of a sample: 8 B; packed word i = 4 s + j of the epilogue
  // (neurons 32 s + 8 h + 2 j + {0, 1}) at bits (i & 15) and 16 + (i & 15) of dword i >> 4),
  // at least ceil(rows / 128) x 128 rows: forward programs write them for their ReLU layers (when set),
  // backward programs read the mask of each masked layer's outputs
  void* bits[12];
  float* aux;             // backward: the gamma gradient rows (fp32): layer 5 stores (adds when aux_acc), layer 0 adds
  int ld_aux, aux_cols, aux_acc;
  const int* M_dev;       // kept-sample count (device)
  unsigned long long* clk;  // anr_profile_*: per-workgroup clock stamps (set by tchain_run when profiling)
};
size_t tchain_image_bytes(int prog);
int tchain_pack(int prog, TcPackArgs a, void* dst, hipStream_t s);
int tchain_run(int prog, const TcArgs& a, int cap, int cus, hipStream_t s);

// split-bf16 layer GEMM with LDS-resident weight images for large M (anr_lgemm.hip; the sdf_pdf
// batches): lgemm_supported(g) (g.x3, no accumulate / mask / atomics, 16-B addressable operands),
// the weight image (lgemm_image_bytes, packed once per weight set by lgemm_pack), then lgemm_run.
bool lgemm_supported(const GemmArgs& g);
size_t lgemm_image_bytes(const GemmArgs& g);
int lgemm_pack(const GemmArgs& g, void* img, hipStream_t s);
// batched packing (anr_sdf_train.hip's per-call plan): lgemm_pack_describe writes g's pack descriptor
// (lgemm_pack_desc_bytes bytes) for image img and returns its block count; lgemm_pack_batch packs n
// described images (descriptors and block starts in device memory, starts[n] = blocks) in one launch
size_t lgemm_pack_desc_bytes();
long lgemm_pack_describe(const GemmArgs& g, void* img, void* desc);
int lgemm_pack_batch(const void* descs, const long* starts, int n, long blocks, hipStream_t s);
int lgemm_run(const GemmArgs& g, const void* img, int cus, hipStream_t s);

// per-point training buffers (row-major, compact kept-sample order)
struct TrainBufs {
  const int* list;
  const int* n_kept;
  const float *ray_o, *ray_d, *near_, *far_, *t_rand;
  const float *R, *Th, *A;
  const float *pbw, *pbounds, *tbw, *tbounds;  // original (X,Y,Z,25) volumes
  int pX, pY, pZ, tX, tY, tZ;
  float* pt;     // [N][8]: pose xyz, dist, tpose xyz, inside
  float* Gp;     // [N][64] gamma(pose)
  float* Ip;     // [N][32] init_pbw
  float* Gv;     // [N][32] gamma(dir)
  float* Lp;     // [N][32] pose logits
  float* Bp;     // [N][24] pbw (softmax)
  float* lbs;    // [N][16] Rinv (9), y (3)
  float* Gt;     // [N][64] gamma(tpose)
  float* It;     // [N][32] init_tbw
  float* Lt;     // [N][32]
  float* Bt;     // [N][24]
  float* Rgbl;   // [N][4] rgb logits
  float* Alpha;  // [N] sigma (raw, before the bbox mask)
  float* sigma;  // [N] sigma'
  float4* raw;   // [R*64]
  // backward
  float4* draw;  // [R*64] (dc, dalpha)
  float* dRgb;   // [N][4]
  float* dAlpha; // [N]
  float* dBp;    // [N][24]
  float* dBt;    // [N][24]
  float* dLp;    // [N][32]
  float* dLt;    // [N][32]
  float* dIt;    // [N][32]
  float* dGt;    // [N][64]
  float* dGt2;   // [N][64] second contribution (T-pose BW chain), summed by k_tr_tpose_bwd; NULL: none
  unsigned short* dAlpha16;  // [N][64] bf16 d alpha in column 0 (written when hb)
  int hb;        // bf16 storage (training precision bf16): Gt, Gv and d alpha (dAlpha16) are written as bf16
  int hbp;       // bf16 storage of the pose space too (precision bf16_all): Gp written as bf16
  int ldl;       // row stride of dLp / dLt (0: 32); the training executor uses 64, the row GEMM's K chunk
  const int* out_row;
  const int* m_rows;
  const float* d_rgb_map;  // (R,3) upstream or NULL
  const float* d_pbw;      // (m,24) upstream or NULL
  const float* d_tbw;
  const float *rgb_map, *acc_map;
  int n_rays;
  // free samples (anr_network_train_fwd, Network.forward under autograd): sample id -> wpts[id],
  // vdir[id], dists[id] (n_pts of them, one reference call) instead of a ray sample; NULL: rays
  const float *wpts, *vdir, *dists;
  long n_pts;
  // fused step only (NULL elsewhere): k_tr_point_prep's block 0 zeroes zero4[0..4) (the loss sums) and
  // zero2048[0..2048) (the latent column-sum scratch) instead of two memset launches; k_tr_loss_grads'
  // first thread writes loss3_out (was k_tr_loss_final)
  float* zero4;
  float* zero2048;
  float* loss3_out;
};

__global__ void k_tr_point_prep(TrainBufs b);
// free-point helpers (anr_blend_weights / anr_canonical_alpha): gamma(x) rows [n][64] and the initial
// blend weights (24,n) -> rows [n][32]; softmax(log(init + 1e-9) + logits) -> (24,n); the latent row
// of one blend-weight field folded into the biases of its layers 0 and 5
__global__ void k_pt_prep(const float* pts, const float* smpl_bw, int n, float* G, float* I);
__global__ void k_pt_softmax_out(const float* logits, const float* I, int n, float* bw_out);
struct FoldArgs {
  const float *w0, *b0, *w5, *b5, *table;
  const int64_t* row;
  int add;
  float* fold;  // [2][256]
};
__global__ void k_fold_latent(FoldArgs a);
__global__ void k_tr_softmax_lbs(TrainBufs b);
__global__ void k_tr_softmax_t(TrainBufs b);
__global__ void k_tr_raw(TrainBufs b);
__global__ void k_tr_composite_bwd(TrainBufs b);
__global__ void k_tr_raw_bwd(TrainBufs b);
__global__ void k_tr_rows_bwd(TrainBufs b);
__global__ void k_tr_softmax_bwd_t(TrainBufs b);
__global__ void k_tr_tpose_bwd(TrainBufs b);
__global__ void k_tr_softmax_bwd_p(TrainBufs b);
struct LatentPosts {
  const float* dysum[8];
  const float* W[8];
  int in_ch[8], col0[8], nout[8];
  const float* table[8];
  const int64_t* li[8];
  int add[8];
  float* dW[8];
  float* dtable[8];
};
__global__ void k_tr_latent_grads(LatentPosts P);
__global__ void k_tr_latent_grad(const float* dysum, const float* W, int in_ch, int col0, int nout, const float* table,
                                 const int64_t* li, int add, float* dW, float* dtable);
__global__ void k_an_prep_obs(TrainBufs b, const float* wpts);
__global__ void k_an_prep_can(TrainBufs b, const float* tpts);
__global__ void k_an_lbs_fwd(TrainBufs b);
__global__ void k_an_softmax_p(TrainBufs b);
__global__ void k_an_select(TrainBufs b, int masked, float norm_th, unsigned long long* amax);
__global__ void k_an_loss(TrainBufs b, float train_th, const unsigned long long* amax, float* acc, int* rows);
__global__ void k_an_loss_grads(TrainBufs b, const int* rows, int need_dt);
__global__ void k_an_set(int* c, int n);
__global__ void k_an_loss_final(const float* acc, const int* rows, float* loss3);
__global__ void k_adam(float* p, float* g, float* m, float* v, long n, float lr, float b1, float b2, float eps, float wd,
                       float bc1, float bc2_sqrt, float clip);
__global__ void k_tr_loss(TrainBufs b, const float* rgb_gt, const uint8_t* mask, float* acc3);
__global__ void k_tr_loss_final(const float* acc3, const int* m_rows, float* loss3);
__global__ void k_tr_loss_grads(TrainBufs b, const float* rgb_gt, const uint8_t* mask, const float* acc3, float* d_rgb,
                                float* d_pbw_rows, float* d_tbw_rows);

}  // namespace anr
