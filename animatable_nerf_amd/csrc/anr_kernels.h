// anr_kernels.h — kernel argument blocks and launch declarations (internal to libaninerf_hip.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace anr {

struct FrontArgs {
  const float *ray_o, *ray_d, *near_, *far_, *t_rand;
  int n_rays, chunk;
  const float *R, *Th, *pbw, *pbounds;
  int X, Y, Z;
  float norm_th;
  uint64_t* mask;        // (R) keep ballots
  uint64_t* chunk_min;   // (nchunks) argmin keys, preset to ~0
  float4* raw;           // (R*64) zeroed at non-kept samples (may be NULL)
  int n_views;           // visibility filter (anr_frame), 0 = off
  const float *Ks, *RT;
  const uint8_t* msks;
  int img_h, img_w;
  // free-point mode (k_frontend_pts, the mesh path's get_alpha): n_rays = ceil(n_pts / 64) groups
  // of 64 points, chunk = chunk_pts / 64 groups
  const float* wpts;     // (n_pts, 3) world points
  long n_pts;
  int chunk_pts;
  const float* pn24;     // channel 24 of pbw as a compact (X,Y,Z) array (k_prep), or NULL: read pbw
  // (k_frontend_pts also zeroes raw at the dropped points when raw != NULL: Network.forward's raw_full)
  int ray_offset;        // ray split (anr_train_hooks): index of ray 0 within its reference chunk
};

struct CompactArgs {
  int n_rays, chunk;
  uint64_t* mask;
  const uint64_t* chunk_min;
  int* ray_off;    // (R+1) exclusive offsets (global after k_compact)
  int* block_sum;  // (ceil(R/256))
  int* list;       // (R*64) kept point ids (ray*64+sample)
  int ray_offset;  // as FrontArgs::ray_offset
};

struct AlphaArgs {
  int n_rays, chunk;
  const int* ray_off;
  const int* n_kept;
  const float* sigma;    // (n') sigma' in compact order
  uint64_t* chunk_max;   // (nchunks) preset to 0
  float train_th;
  uint8_t* flags;        // (n')
  int* block_sum;        // (ceil(n'/1024))
  int* out_row;          // (n') output row or -1
  // the argmax key's tie-break index is the sample's index within its reference chunk, (ray +
  // ray_offset) % chunk * 64 + lane (compaction keeps sample order, so within one call it orders
  // like the compact index; across the ranks of a ray split it is the global one)
  const int* list;
  const uint64_t* mask;  // keep ballots after k_count (forced argmin bit included)
  int ray_offset;
};

// (f) eval-split camera rays (get_rays_within_bounds)
struct CamArgs {
  int H, W, fp64;
  double Kinv[9], R[9], T[3], o[3];
  const float* bounds;            // (2,3) or NULL (rays only)
  float *all_o, *all_d;           // (H*W, 3)
  uint8_t* mask;                  // (H*W)
  float *all_near, *all_far;      // (H*W)
  int* block_sum;                 // (ceil(H*W/256))
  float *ray_o, *ray_d, *near_, *far_;  // compacted hits
  int* coord;                     // (n, 2) (row, col)
};

// (f) train-split ray sampler (anr_rays.hip, k_trl_*)
struct TrainRayArgs {
  CamArgs cam;                    // H, W, fp64, Kinv, R, T, o, bounds
  const uint8_t *msk, *bound_mask;  // (H*W) u8
  const float* img;               // (H*W, 3)
  int mask_bkgd;
  int* block_sum;                 // 3 x ceil(H*W/256)
  int* lists;                     // 3 x H*W pixel ids: body, face, bound
  const int* draws;               // one round of list-relative draws
  int n_seg[3];
  int cap;                        // output capacity (nrays)
  int* n_out;                     // device: rays so far (in/out)
  float *ray_o, *ray_d, *rgb, *near_, *far_;
  int* coord;
};

struct CompositeArgs {
  const float4* raw;
  const float *near_, *far_, *t_rand;
  int n_rays;
  float *rgb, *acc, *depth, *weights;
};

// the fused deform + NeRF MLP kernel (anr_mlp.hip)
struct MlpArgs {
  const unsigned char* wimg;  // packed weight image (anr_layers.h)
  const float* bias;          // packed bias section
  const float* fold;          // per-frame folded biases: bw0[2][256], bw5[2][256], nlat[256]
  const float *A, *R, *Th;
  const float *pbw32, *pbounds, *tbw32, *tbounds;
  int pX, pY, pZ, tX, tY, tZ;
  const float *ray_o, *ray_d, *near_, *far_, *t_rand;
  const int* list;
  const int* n_kept;
  float4* raw;
  float* sigma;      // (n') sigma' (after the T-pose bbox mask)
  float* pbw_rows;   // (n', 24)
  float* tbw_rows;   // (n', 24)
  int pose_woff;     // byte offset of the pose-pass BW weight slices (novel_pose_bw copy or 0)
  int pose_boff;     // float offset of the pose-pass BW biases
  // density program (k_alpha*, get_alpha): kept point ids index wpts; alpha_out[id] = raw sigma
  const float* wpts;
  long n_pts;
  int chunk_pts;
  float* alpha_out;
  // free samples (anr_network_fwd, Network.forward): when dists != NULL the render program reads
  // sample id's world point wpts[id], view direction vdir[id] and dists[id] instead of a ray sample
  const float* vdir;
  const float* dists;
  // sdf residual program (k_resd_b16): rows [0, n_rows) of ptb ([n][8], big-pose xyz in 0..2) in,
  // the resd_fc outputs (before 0.05 tanh) to yr ([n][4], columns 0..2)
  const float* ptb;
  float* yr;
  int n_rows;
  // sdf network program (k_sdfnet_b16): point xyz in columns 0..2 of ptb rows of stride ptb_ld (C0);
  // softplus outputs h of lin l to sdf_h[l] ([n][256], l != 3), lin3's h / sqrt2 to x4[:, :217],
  // lin8's [sdf || feature] to y8 ([n][264])
  int ptb_ld;
  float* sdf_h[8];
  float* x4;
  float* y8;
  // sdf input-gradient program (k_sdfgrad_b16): reads sdf_h / x4 of the forward and lin8's row 0
  // (w8row); writes the gamma_6 gradients of lin0 to gb ([n][40]) and of lin4's skip to gc[:, 217:256]
  const float* w8row;
  float* gb;
  float* gc;
  // measurement (anr_profile_*): when set, thread 0 of every workgroup stamps (s_memtime, s_memrealtime)
  // at kernel entry and exit into clk[blockIdx.x * 4 + {0, 1, 2, 3}]: the in-kernel shader clock is
  // d memtime / d realtime x 100 MHz (MI355X_MICROARCH.md, DVFS item 6)
  unsigned long long* clk;
};

__device__ __forceinline__ void clk_stamp(unsigned long long* clk, int k) {
  if (clk && threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    clk[(size_t)blockIdx.x * 4 + 2 * k] = t;
    clk[(size_t)blockIdx.x * 4 + 2 * k + 1] = r;
  }
}
#ifdef ANR_NO_CLK_STAMP  // A/B builds: the kernels without the stamp code
#define ANR_STAMPED(...) __VA_ARGS__
#else
#define ANR_STAMPED(...) \
  clk_stamp(a.clk, 0);   \
  __VA_ARGS__;           \
  clk_stamp(a.clk, 1)
#endif

// profiling slot of one fused launch (anr_capi.hip; NULL from prof_begin when profiling is off): events
// around the launch and the clock-stamp area handed to the kernel as MlpArgs::clk (NULL past the arena)
struct ProfSlot {
  hipEvent_t b, e;
  unsigned long long* clk;
};
ProfSlot* prof_begin(hipStream_t s, int grid);
int prof_end(ProfSlot* q, hipStream_t s);

struct PrepArgs {
  const float *pbw, *tbw;  // (X,Y,Z,25)
  float *pbw32, *tbw32;    // (X,Y,Z,32)
  int np, nt;              // voxel counts
  const float *w_bw0, *b_bw0, *w_bw5, *b_bw5, *bw_latent;
  const float *w_lat, *b_lat, *nf_latent;
  const int64_t* latent_index;
  float* fold;
  // novel pose: pose-pass folds from novel_pose_bw with bw_latent_index (no +1)
  int novel;
  const float *nw_bw0, *nb_bw0, *nw_bw5, *nb_bw5, *n_latent;
  const int64_t* bw_latent_index;
  // folded colour head (anr_layers.h ANR_L_HEAD): fold[ANR_FOLD_HEAD + i] = P nf_latent[li] + q, row 128
  // = alpha_fc's bias; skipped when head_P is NULL (callers without the bf16x3 render program)
  const float *head_P, *head_q, *b_alpha;
  float* pn24;  // (np) channel 24 of pbw, compact, for the front-end's prefilter lookups (or NULL)
  // the render front-end's per-call state, reset here instead of by three memset launches ahead of this
  // one (block 0; NULL: nothing): counts[0..3] = 0, chunk_min[0..nch) = ~0, chunk_max[0..nch) = 0
  int* counts;
  uint64_t *chunk_min, *chunk_max;
  int nch;
};
// k_prep launch size for np + nt voxels (the folded biases and head included)
int prep_blocks(long np, long nt);


__global__ void k_near_far(const float*, const float*, int, const float*, uint8_t*, float*, float*);
__global__ void k_cam_rays(CamArgs a);
__global__ void k_cam_count(CamArgs a);
__global__ void k_cam_scatter(CamArgs a);
__global__ void k_trl_count(TrainRayArgs a);
__global__ void k_trl_scatter(TrainRayArgs a);
__global__ void k_trl_gather(TrainRayArgs a);
__global__ void k_frontend(FrontArgs a);
__global__ void k_frontend_pts(FrontArgs a);
__global__ void k_count(CompactArgs a);
__global__ void k_scan_blocks(int* sums, int nb, int* total_out);
__global__ void k_compact(CompactArgs a);
// R <= 1024 rays (a training batch): k_count + k_scan_blocks + k_compact as one 1024-thread workgroup
__global__ void k_compact1(CompactArgs a, int* total_out);
// one chunk of <= 65,536 compact samples: the alpha_ind stage's five launches as two (anr_rays.hip)
__global__ void k_alpha_count1(AlphaArgs a);
__global__ void k_alpha_scatter1(AlphaArgs a, int* total_out);
__global__ void k_chunk_argmax(AlphaArgs a);
__global__ void k_flag_count(AlphaArgs a);
__global__ void k_flag_force(AlphaArgs a, int nchunks);
__global__ void k_flag_scatter(AlphaArgs a);
__global__ void k_gather_rows(const int*, const int*, const float4*, const float4*, float4*, float4*);
__global__ void k_row_ids(const int*, const int*, const int*, int*);
__global__ void k_sample_volume(const float*, int, int, int, int, const float*, const float*, int, float*);
__global__ void k_composite(CompositeArgs a);
__global__ void k_prep(PrepArgs a);
__global__ void k_mlp(MlpArgs a);
__global__ void k_mlp_b16(MlpArgs a);  // T-pose BW + NeRF in bf16x3 (render precision ANR_BF16X3)
__global__ void k_mlp_x6(MlpArgs a);   // every layer in bf16x6, fp32-level (render precision ANR_BF16X6)
__global__ void k_alpha(MlpArgs a);      // density program (get_alpha), exact fp32 MFMA
__global__ void k_alpha_b16(MlpArgs a);  // density program, NeRF trunk in bf16x3
__global__ void k_alpha_x6(MlpArgs a);   // density program, every layer in bf16x6

struct PackArgs {
  const float* t[66];  // 46 core tensors + 19 novel_pose_bw tensors (NULL when absent) + the head H
  unsigned char* out;
};
__global__ void k_pack_head_a(PackArgs a);
__global__ void k_pack_head_b(PackArgs a);
__global__ void k_pack_weights(PackArgs a);
__global__ void k_pack_bias(PackArgs a);
__global__ void k_pack_b16(PackArgs a);
// layer sequences of the sdf render (anr_layers.h resd_desc / sdfnet_desc): bf16x3 image + biases of
// seq_image_bytes(L0, nl) at a.out (t[l] = weight of layer L0 + l, t[9 + l] its bias; layer L0 + sl
// scaled by sc), and the fused programs over one batch (residual MLP; SDF network forward)
__global__ void k_pack_seq(PackArgs a, int L0, int nl, int sl, float sc);
int seq_pack_threads(int L0, int nl);
// the same sequence as a bf16x6 image (anr_layers.h x6seq_*) for the fp32-level programs
__global__ void k_pack_seq_x6(PackArgs a, int L0, int nl, int sl, float sc);
int seq_x6_pack_threads(int L0, int nl);
__global__ void k_resd_x6(MlpArgs a);
__global__ void k_sdfnet_x6(MlpArgs a);
__global__ void k_sdfgrad_x6(MlpArgs a);
__global__ void k_color_x6(MlpArgs a);
// x6: the bf16x6 programs (image from k_pack_seq_x6), else bf16x3 (k_pack_seq)
int launch_resd(const MlpArgs& a, int grid, hipStream_t s, bool x6 = false);
int launch_sdfnet(const MlpArgs& a, int grid, hipStream_t s, bool x6 = false);
int launch_sdfgrad(const MlpArgs& a, int grid, hipStream_t s, bool x6 = false);
int launch_color(const MlpArgs& a, int grid, hipStream_t s, bool x6 = false);
__global__ void k_pack_x6(PackArgs a);

}  // namespace anr
