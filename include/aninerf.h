/*
 * aninerf.h — C-ABI of the MI355X-native Animatable-NeRF volume-rendering hot path.
 *
 * Plain C: device pointers + sizes + a hipStream_t passed as void*; no torch types. Every entry
 * point is asynchronous on the given stream and returns 0 or an ANR_E* code (a hipError_t is
 * returned as ANR_E_HIP, its text via anr_last_error()).
 *
 * Reference interfaces each entry point replaces (paths relative to the reference tree):
 *   anr_near_far            lib/utils/if_nerf/if_nerf_data_utils.py:156-196   get_near_far (A14)
 *   anr_camera_rays         if_nerf_data_utils.py:64-89, 310-339  get_rays + get_rays_within_bounds
 *   anr_params_pack         lib/networks/bw_deform/tpose_nerf_network.py:11-38, 218-239
 *                           (state_dict -> the kernel's weight image; called when weights change)
 *   anr_render_fwd          lib/networks/renderer/tpose_renderer.py:159-186   Renderer.render (A1)
 *                             -> get_wsampling_points :14-39, get_density_color :41-69,
 *                                Network.forward tpose_nerf_network.py:139-215,
 *                                raw2outputs nerf_net_utils.py:6-36
 *   anr_render_counts       the host syncs the reference makes at pind/alpha_ind (:153-157, :192-196)
 *   anr_render_bw_rows      tpose_nerf_network.py:195-196 (pbw/tbw rows selected by alpha_ind)
 *   anr_sdf_render_fwd      the same Renderer.render over the sdf_pdf network (config 5):
 *                             lib/networks/bw_deform/anisdf_pdf_network.py:156-223 Network.forward,
 *                             sample_utils.py:309-348 (KNN blend), TPoseHuman :288-338,
 *                             tpose_renderer.py:134-152 (msk_sdf / msk_label)
 *   anr_sdf_train_step      lib/train/trainers/tpose_trainer.py:21-73 over the sdf_pdf network
 *                             (configs/sdf_pdf/anisdf_pdf_s9p.yaml:13-14), forward + loss.backward()
 *   anr_sdf_render_counts / anr_sdf_render_rows   the compact outputs 'resd', 'gradients',
 *                             'msk_sdf', 'msk_label' (sizes known only after the keep mask)
 *   anr_network_fwd         lib/networks/bw_deform/tpose_nerf_network.py:139-215 Network.forward
 *                             (wpts, viewdir, dists, batch), the per-chunk call of tpose_renderer.py:95
 *   anr_network_train_fwd/bwd  the same call under autograd (forward + loss.backward() through it)
 *   anr_blend_weights       tpose_nerf_network.py:55-77 calculate_neural_blend_weights and
 *                             :304-315 BackwardBlendWeight.forward (novel_pose_bw)
 *   anr_canonical_alpha     tpose_nerf_network.py:241-250 TPoseHuman.calculate_alpha
 *   anr_alpha_points        lib/networks/bw_deform/tpose_nerf_network.py:105-137 Network.get_alpha
 *                             over the batchify chunks of aninerf_mesh_renderer.py:14-23, 34-36
 *   anr_anim_step           lib/train/trainers/aninerf_animation_trainer.py:33-140 (forward + backward)
 *   anr_mc_count/anr_mc_emit  mcubes.marching_cubes(np.pad(cube, 10), cfg.mesh_th)
 *                             (aninerf_mesh_renderer.py:38-45; PyMCubes, third-party, not installed)
 *
 * All float tensors are fp32, contiguous, row-major, with the reference's shapes (batch dim 1).
 */
#ifndef ANINERF_H
#define ANINERF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ANR_OK = 0,
  ANR_E_HIP = 1,        /* a HIP runtime call failed; see anr_last_error() */
  ANR_E_ARG = 2,        /* bad shape / NULL pointer / unsupported option */
  ANR_E_WORKSPACE = 3   /* workspace too small */
};

/* Number of tensors of the aninerf Network state_dict (tpose_nerf_network.py:11-38, 218-239),
 * in this order (weights are Conv1d (out, in, 1), embeddings (rows, 128)):
 *   0 tpose_human.nf_latent.weight (F,128)
 *   1..16  tpose_human.pts_linears.{0..7}.{weight,bias}   in: 63,256,256,256,256,319,256,256
 *   17,18 tpose_human.alpha_fc.{weight,bias} (1,256,1)
 *   19,20 tpose_human.feature_fc.{weight,bias} (256,256,1)
 *   21,22 tpose_human.latent_fc.{weight,bias} (256,384,1)
 *   23,24 tpose_human.view_fc.{weight,bias} (128,283,1)
 *   25,26 tpose_human.rgb_fc.{weight,bias} (3,128,1)
 *   27 bw_latent.weight (F+1,128)
 *   28..43 bw_linears.{0..7}.{weight,bias}   in: 191,256,256,256,256,447,256,256
 *   44,45 bw_fc.{weight,bias} (24,256,1)                                                     */
#define ANR_NUM_TENSORS 46
/* novel_pose_bw (BackwardBlendWeight, tpose_nerf_network.py:278-315; present when
 * cfg.aninerf_animation): bw_latent.weight (E,128), bw_linears.{0..7}.{weight,bias},
 * bw_fc.{weight,bias} — 19 tensors, state_dict order. */
#define ANR_NUM_NOVEL_TENSORS 19

typedef struct anr_params {
  const float* t[ANR_NUM_TENSORS];  /* device pointers, state_dict order above */
  int num_train_frame;              /* F: rows of nf_latent (bw_latent has F+1) */
  const void* packed;               /* device weight image written by anr_params_pack */
  const float* novel[ANR_NUM_NOVEL_TENSORS];  /* novel_pose_bw tensors or all NULL */
} anr_params;

typedef struct anr_frame {
  const float* A;          /* (24,4,4) device */
  const float* R;          /* (3,3) device (smpl->world rotation, Rodrigues(Rh)) */
  const float* Th;         /* (3) device */
  const float* pbw;        /* (X,Y,Z,25) device: posed blend-weight volume, ch 24 = distance */
  int pbw_dims[3];
  const float* pbounds;    /* (2,3) device */
  const float* tbw;        /* (X',Y',Z',25) device: T-pose blend-weight volume */
  int tbw_dims[3];
  const float* tbounds;    /* (2,3) device */
  const int64_t* latent_index;  /* (1) device: batch['latent_index'] */
  const int64_t* bw_latent_index;  /* (1) device: batch['bw_latent_index'] (novel pose only) */
  /* novel-view visibility filter (tpose_renderer_mmsk.py:14-57); n_views = 0 disables it:
   * a sample is kept only if it projects inside every training view's mask. */
  int n_views;
  const float* Ks;         /* (V,3,3) device */
  const float* RT;         /* (V,3,4) device, world -> camera */
  const uint8_t* msks;     /* (V,img_h,img_w) device */
  int img_h, img_w;
} anr_frame;

typedef struct anr_render_opts {
  int n_samples;     /* cfg.N_samples; only 64 is supported */
  int chunk;         /* rays per reference chunk (2048, tpose_renderer.py:170); semantics depend on it */
  float norm_th;     /* cfg.norm_th (0.05) */
  float train_th;    /* cfg.train_th (0) */
  const float* t_rand;  /* (R, n_samples) device stratification draws, or NULL (eval / perturb 0) */
  int novel_pose;    /* cfg.test_novel_pose: pose-space blend weights from novel_pose_bw
                        with bw_latent_index (tpose_nerf_network.py:93-94); render only */
  int precision;     /* training GEMM operands: ANR_FP32 (exact fp32 MFMA); ANR_BF16 (config 3:
                        operands rounded to bf16, fp32 accumulation, fp32 master weights and Adam,
                        the pose-space blend-weight MLP kept fp32); ANR_BF16_ALL (every GEMM bf16).
                        anr_render_fwd / anr_alpha_points: ANR_FP32 (exact fp32 MFMA everywhere) or
                        ANR_BF16X3 (every MLP layer as hi/lo-split bf16 MFMA, lo*bh + hi*bl + hi*bh
                        with fp32 accumulation: ~2^-16 relative per product, outputs within the
                        1e-4 fp32 tolerance); anr_render_fwd / anr_network_fwd / anr_alpha_points
                        also ANR_BF16X6
                        (hi/mid/lo-split bf16, six products per multiply-add, fp32 accumulation:
                        fp32-level products, <= ~2^-23 relative, on the bf16 MFMA pipe).
                        anr_sdf_render_fwd: ANR_BF16X3 splits its layer GEMMs the same way (the
                        residual MLP as one fused launch). Other entry points treat ANR_BF16X3 /
                        ANR_BF16X6 as ANR_FP32. */
} anr_render_opts;

enum { ANR_FP32 = 0, ANR_BF16 = 1, ANR_BF16_ALL = 2, ANR_BF16X3 = 3, ANR_BF16X6 = 4 };

/* Outputs (device). raw may be NULL (then kept in the workspace). */
typedef struct anr_render_out {
  float* rgb_map;    /* (R,3) */
  float* acc_map;    /* (R)   */
  float* depth_map;  /* (R)   */
  float* raw;        /* (R*n_samples, 4) or NULL */
} anr_render_out;

/* ---- A14: ray / box intersection in float64 (bit-exact with numpy) ---------------------
 * rays (n,3) f32, bounds (2,3) f32 -> mask (n) u8, near/far (n) f32 at EVERY ray
 * (garbage where mask==0). */
int anr_near_far(const float* ray_o, const float* ray_d, int n, const float* bounds,
                 uint8_t* mask, float* near_, float* far_, void* stream);

/* ---- (f) eval-split ray pipeline: get_rays_within_bounds (if_nerf_data_utils.py:310-339) ------
 * get_rays (:64-89) for every pixel of an H x W camera, the A14 box test, and the ordered list of
 * the hit pixels (row-major, like np.argwhere). Kinv = np.linalg.inv(K) and origin = -R^T T are
 * passed in as the reference computes them on the host (LAPACK / BLAS results); fp64 selects the
 * float64 arithmetic of float64 camera annotations, else float32 (float32 cameras). Outputs
 * (device, capacity H*W): ray_o/ray_d (n,3), near/far (n), coord (n,2) (row, col), mask (H*W);
 * count (device int32) = n. */
size_t anr_camera_rays_workspace_bytes(int H, int W);
int anr_camera_rays(int H, int W, const double* Kinv, const double* R, const double* T, const double* origin, int fp64,
                    const float* bounds, float* ray_o, float* ray_d, float* near_, float* far_, int32_t* coord,
                    uint8_t* mask, int32_t* count, void* workspace, size_t ws_bytes, void* stream);

/* ---- (f) train-split ray sampler: sample_ray_h36m(split='train') (if_nerf_data_utils.py:198-283) ----
 * Replaces the float64 numpy sampler the reference runs in its DataLoader workers
 * (tpose_dataset.py:228). Two calls, both asynchronous on `stream`:
 *  anr_train_ray_lists: the pixel lists np.argwhere(msk == 1), (msk == 13), (bound_mask == 1) of
 *    :238-249 (row-major), after msk = msk * bound_mask and bound_mask[msk == 100] = 0 (:230-231).
 *    msk / bound_mask (H*W) u8 device; lists (3 * H*W) int32 device; counts (3) int32 device.
 *  anr_train_ray_gather: one round of the sampling loop (:236-271). draws (n_body + n_face + n_rand)
 *    int32 device = the np.random.randint draws into lists 0, 1, 2 in that order (the caller makes
 *    them with numpy, so the random stream is the reference's); per draw get_rays (:64-89) at the
 *    pixel, get_near_far (:156-196) on get_rays' arrays (float64 for a float64 camera), rgb = img
 *    (H*W,3) f32, zero outside bound_mask when mask_bkgd (:228). Hits are appended in draw order
 *    at index *n_out (device int32, updated), at most cap; outputs ray_o/ray_d/rgb (cap,3),
 *    near/far (cap), coord (cap,2) (row, col). Camera arguments as anr_camera_rays. */
size_t anr_train_ray_workspace_bytes(int H, int W);
int anr_train_ray_lists(int H, int W, const uint8_t* msk, const uint8_t* bound_mask, int32_t* lists, int32_t* counts,
                        void* workspace, size_t ws_bytes, void* stream);
int anr_train_ray_gather(int H, int W, const double* Kinv, const double* R, const double* T, const double* origin,
                         int fp64, const float* bounds, const float* img, const uint8_t* bound_mask, int mask_bkgd,
                         const int32_t* lists, const int32_t* draws, int n_body, int n_face, int n_rand, int cap,
                         float* ray_o, float* ray_d, float* rgb, float* near_, float* far_, int32_t* coord,
                         int32_t* n_out, void* stream);

/* ---- weights --------------------------------------------------------------------------- */
size_t anr_params_packed_bytes(void);
int anr_params_pack(const anr_params* p, void* packed, void* stream);

/* ---- render ---------------------------------------------------------------------------- */
size_t anr_render_workspace_bytes(int n_rays, const anr_render_opts* o, const anr_frame* f);
int anr_render_fwd(const anr_params* p, const anr_frame* f, const float* ray_o, const float* ray_d,
                   const float* near_, const float* far_, int n_rays, const anr_render_opts* o,
                   const anr_render_out* out, void* workspace, size_t ws_bytes, void* stream);
/* device int32[2] inside the workspace: {kept points n', alpha_ind rows m}. */
const int32_t* anr_render_counts(const void* workspace, int n_rays);
/* Gather the m alpha_ind rows of pbw / tbw (each (m,24)) after the counts were read. */
int anr_render_bw_rows(const void* workspace, int n_rays, float* pbw, float* tbw, void* stream);
/* The sample id (ray * N_samples + sample, frame order) of each of the m alpha_ind rows, ids (m) int32:
 * which samples tpose_nerf_network.py:192-196 selected (rows compared by sample in tests). */
int anr_render_row_ids(const void* workspace, int n_rays, int32_t* ids, void* stream);

/* ---- Network.forward over free samples (tpose_nerf_network.py:139-215) ----------------------
 * The call a reference renderer makes per chunk, self.net(wpts, viewdir, dists, batch)
 * (tpose_renderer.py:95): n_pts samples given by world points wpts (n,3), view directions viewdir
 * (n,3) and interval lengths dists (n). The prefilter's forced argmin and the alpha_ind argmax run
 * over the whole call, as the reference's pnorm.argmin(dim=1) / argmax(alpha, dim=1) do (one call =
 * one reference chunk); o->chunk and o->t_rand are ignored. raw (n,4) is zero at dropped samples
 * (raw_full). anr_network_counts: device int32 {kept n', alpha_ind rows m} in the workspace;
 * anr_network_bw_rows: the m rows of pbw / tbw (each (m,24)) after the counts were read; both work on
 * either workspace below.
 *  anr_network_fwd: the fused network kernel (o->precision ANR_FP32 or ANR_BF16X3), no host sync.
 *  anr_network_train_fwd / _bwd: the layer-wise training executor (o->precision as for training),
 *    activations kept in the workspace until the backward; n' stays on the device (no host sync). _bwd
 *    ACCUMULATES the parameter gradients (anr_params order) from the upstream d raw (n,4) and d pbw /
 *    d tbw rows (m,24); any of the three may be NULL (zero). */
typedef struct anr_samples {
  const float* wpts;     /* (n,3) device, world frame */
  const float* viewdir;  /* (n,3) device */
  const float* dists;    /* (n) device */
  int n_pts;
} anr_samples;
size_t anr_network_workspace_bytes(int n_pts, const anr_render_opts* o, const anr_frame* f);
int anr_network_fwd(const anr_params* p, const anr_frame* f, const anr_samples* x, const anr_render_opts* o, float* raw,
                    void* workspace, size_t ws_bytes, void* stream);
const int32_t* anr_network_counts(const void* workspace, int n_pts);
int anr_network_bw_rows(const void* workspace, int n_pts, float* pbw, float* tbw, void* stream);
size_t anr_network_train_workspace_bytes(int n_pts, const anr_render_opts* o, const anr_frame* f);
int anr_network_train_fwd(const anr_params* p, const anr_frame* f, const anr_samples* x, const anr_render_opts* o,
                          float* raw, void* workspace, size_t ws_bytes, void* stream);
int anr_network_train_bwd(const anr_params* p, float* const* grads, const anr_frame* f, const anr_samples* x,
                          const anr_render_opts* o, const float* d_raw, const float* d_pbw, const float* d_tbw,
                          void* workspace, size_t ws_bytes, void* stream);

/* ---- network helpers the reference's other trainers / renderers call --------------------------
 * anr_blend_weights: field 0 = calculate_neural_blend_weights(pts, smpl_bw, latent_index)
 *   (tpose_nerf_network.py:55-77; bw_latent, bw_linears, bw_fc), field 1 = novel_pose_bw(pts, smpl_bw,
 *   latent_index) (BackwardBlendWeight.forward :304-315): pts (n,3), smpl_bw (24,n) (the reference's
 *   (1,24,n)) -> bw (24,n) = softmax(log(smpl_bw + 1e-9) + MLP([gamma(pts), latent row])), latent row =
 *   latent_row[0] + row_add (latent_row: device int64, the caller's index tensor).
 * anr_canonical_alpha: TPoseHuman.calculate_alpha(nf_pts) (:241-250): raw alpha (n) of canonical points.
 * Forward only, exact fp32 MFMA layer GEMMs, no host sync. */
size_t anr_points_workspace_bytes(int n);
int anr_blend_weights(const anr_params* p, int field, const float* pts, const float* smpl_bw, int n,
                      const int64_t* latent_row, int row_add, float* bw, void* workspace, size_t ws_bytes, void* stream);
int anr_canonical_alpha(const anr_params* p, const float* pts, int n, float* alpha, void* workspace, size_t ws_bytes,
                        void* stream);

/* ---- training (A16/A17; lib/train/trainers/tpose_trainer.py:21-73, trainer.py:50-68) ------
 * anr_train_fwd: the render forward of the training step (perturb via o->t_rand), keeping every
 *   activation in the workspace; same outputs as anr_render_fwd (+ anr_render_counts /
 *   anr_render_bw_rows on this workspace). Reads the kept-sample count once (host sync).
 * anr_train_bwd: given upstream gradients d rgb_map (R,3) and d pbw / d tbw rows (m,24) (any may
 *   be NULL = zero), ACCUMULATES parameter gradients into grads[ANR_NUM_TENSORS] (state_dict
 *   order, same shapes as anr_params.t) — what loss.backward() does in the reference.
 * anr_train_step: forward + the reference losses (img MSE over mask_at_box rays + smooth-L1 of
 *   the pbw/tbw rows; loss3 = {loss, img_loss, bw_loss} on device) + backward, one call.
 * anr_adam: clip_grad_value_(clip) then torch.optim.Adam on a flat parameter blob (trainer.py:64-68). */
size_t anr_train_workspace_bytes(int n_rays, const anr_render_opts* o, const anr_frame* f);
int anr_train_fwd(const anr_params* p, const anr_frame* f, const float* ray_o, const float* ray_d,
                  const float* near_, const float* far_, int n_rays, const anr_render_opts* o,
                  const anr_render_out* out, void* workspace, size_t ws_bytes, void* stream);
int anr_train_bwd(const anr_params* p, float* const* grads, const anr_frame* f, const float* ray_o,
                  const float* ray_d, const float* near_, const float* far_, int n_rays,
                  const anr_render_opts* o, const float* d_rgb_map, const float* d_pbw, const float* d_tbw,
                  void* workspace, size_t ws_bytes, void* stream);
int anr_train_step(const anr_params* p, float* const* grads, const anr_frame* f, const float* ray_o,
                   const float* ray_d, const float* near_, const float* far_, int n_rays,
                   const anr_render_opts* o, const float* rgb_gt, const uint8_t* mask_at_box,
                   const anr_render_out* out, float* loss3, void* workspace, size_t ws_bytes, void* stream);
/* anr_train_step_hooked: anr_train_step plus events for overlapping the gradient all-reduce with
 * the backward (DDP's reverse-order buckets): nerf_grads_ready (a hipEvent_t or
 * NULL) is recorded on the stream once the gradients of tensors 0..26 (tpose_human.*, the canonical
 * NeRF) are final; the blend-weight backward (tensors 27..45) follows on the stream. */
typedef int (*anr_reduce_fn)(void* user, void* device_buf, int count, int op, void* stream);
#define ANR_REDUCE_MIN_U64 0 /* unsigned 64-bit keys, min over ranks (all-ones = empty) */
#define ANR_REDUCE_MAX_U64 1 /* unsigned 64-bit keys, max over ranks */
#define ANR_REDUCE_SUM_F32 2 /* float sums over ranks */
/* struct_size must be sizeof(anr_train_hooks) (ANR_TRAIN_HOOKS_VERSION 2, anr_version() >= 2): the struct
 * grew from version 1's single nerf_grads_ready field, and a caller built against another layout is
 * rejected with ANR_E_ARG instead of having its memory read as the newer fields. */
#define ANR_TRAIN_HOOKS_VERSION 2
typedef struct anr_train_hooks {
  size_t struct_size;
  void* nerf_grads_ready;
  /* Ray split of ONE reference chunk over ranks (north_star "rays-per-iteration shard"; strong scaling of
   * a 1,024-ray step): this call's rays are rays [ray_offset, ray_offset + n_rays) of a
   * batch that is a single reference chunk (ray_offset + n_rays <= o->chunk). The chunk-wide decisions are
   * exchanged through reduce (NULL: no split), which the library calls on the host, in issue order, with
   * a device buffer of the workspace; it must make `stream` wait for the reduction over all ranks (e.g. an
   * RCCL all-reduce on that stream): the per-chunk argmin key of the prefilter (tpose_nerf_network.py:154,
   * MIN_U64) before compaction, the per-chunk argmax key of sigma' (:193-194, MAX_U64) before the
   * alpha_ind rows are flagged, and the loss sums {squared error, mask rays, smooth-L1 sum, alpha_ind
   * rows} (SUM_F32) before the loss and its gradients. Losses are then the batch's on every rank and
   * the gradients are this rank's share of the batch gradient (sum them over ranks). */
  int ray_offset;
  anr_reduce_fn reduce;
  void* reduce_user;
} anr_train_hooks;
int anr_train_step_hooked(const anr_params* p, float* const* grads, const anr_frame* f, const float* ray_o,
                          const float* ray_d, const float* near_, const float* far_, int n_rays,
                          const anr_render_opts* o, const float* rgb_gt, const uint8_t* mask_at_box,
                          const anr_render_out* out, float* loss3, const anr_train_hooks* hooks, void* workspace,
                          size_t ws_bytes, void* stream);
int anr_adam(float* param, float* grad, float* exp_avg, float* exp_avg_sq, long n, float lr, float beta1,
             float beta2, float eps, float weight_decay, int step, float clip_value, void* stream);

/* ---- (f) animation stage (lib/train/trainers/aninerf_animation_trainer.py:33-140) -------------
 * anr_anim_step: NetworkWrapper.forward + loss.backward of the second training stage, which fits
 *   novel_pose_bw with every other parameter frozen. wpts (n_obs,3): points drawn in wbounds
 *   (observation space, world frame; get_sampling_points :143-160); tpts (n_can,3): points drawn in
 *   tbounds (canonical). Path 1 (ppts_to_tpose :63-99): pbw0 = novel_pose_bw at the posed point,
 *   tbw0 = the frozen blend-weight MLP at its LBS-inverse T-pose point (differentiable through x_T),
 *   rows where alpha (zeroed outside tbounds or pnorm >= o->norm_th) > o->train_th plus the argmax.
 *   Path 2 (tpose_to_ppts :102-131): tbw1 frozen at the canonical point, pbw1 = novel_pose_bw at its
 *   forward-LBS posed point, rows alpha > train_th plus the argmax. loss3 = {bw_loss0 + bw_loss1,
 *   bw_loss0, bw_loss1} (smooth_l1 means, device). ACCUMULATES the gradients of the 19
 *   novel_pose_bw tensors into grads (anr_params.novel order). Reads frame A, R, Th, pbw, pbounds,
 *   tbw, tbounds, bw_latent_index; o->precision as for training (ANR_BF16 keeps the pose-space
 *   novel_pose_bw MLP fp32). No host sync. */
size_t anr_anim_workspace_bytes(int n_points);
int anr_anim_step(const anr_params* p, float* const* grads, const anr_frame* f, const float* wpts, int n_obs,
                  const float* tpts, int n_can, const anr_render_opts* o, float* loss3, void* workspace,
                  size_t ws_bytes, void* stream);

/* ---- sdf_pdf variant (config 5, anisdf_pdf_network.py) ------------------------------------
 * Parameters: the 63 tensors of anisdf_pdf_network.Network's state_dict, in order:
 *   0..26  tpose_human.sdf_network.lin{0..8}.{bias, weight_g (o,1), weight_v (o,i)}
 *          i/o: 39/256, 256/256, 256/256, 256/217, 256/256 x4, 256/257
 *   27     tpose_human.beta_network.beta ()
 *   28     tpose_human.color_network.color_latent.weight (L,128)
 *   29..43 tpose_human.color_network.lin{0..4}.{bias, weight_g, weight_v}  i: 289,256,256,384,256
 *   44     resd_latent.weight (L,128)            (not read by the render)
 *   45..60 resd_linears.{0..7}.{weight,bias}     Conv1d, in: 135,256,256,256,256,391,256,256
 *   61,62  resd_fc.{weight,bias} (3,256,1)                                                   */
#define ANR_SDF_NUM_TENSORS 63

typedef struct anr_sdf_params {
  const float* t[ANR_SDF_NUM_TENSORS];  /* device pointers, state_dict order above */
} anr_sdf_params;

typedef struct anr_sdf_frame {
  const float* A;          /* (24,4,4) device */
  const float* big_A;      /* (24,4,4) device: big pose (tpose_pdf_dataset.py:91-100) */
  const float* R;          /* (3,3) */
  const float* Th;         /* (3) */
  const float* poses;      /* (72) batch['poses'] */
  const float* pvertices;  /* (V,3) posed SMPL vertices in the pose frame, V <= 6912 */
  const float* weights;    /* (V,24) skin weights */
  int n_verts;
  const float* tbounds;    /* (2,3) batch['tbounds'] as passed in */
  const int64_t* latent_index;  /* (1) colour latent row */
  const uint8_t* occupancy;     /* (R) batch['occupancy'] */
  /* novel-view visibility filter of tpose_renderer_mmsk (:14-57, the config-5 novel_view_cfg /
   * pose_sequence_cfg renderer over this network), anr_sdf_render_fwd only; n_views = 0 disables it. A
   * sample reaches the network only if it projects inside every training view's mask: the KNN keep and
   * the per-chunk forced argmin range over the visible samples (one Network.forward call per chunk on
   * them), and tbounds widens only at chunks with a visible sample (a chunk without one makes no call). */
  int n_views;
  const float* Ks;         /* (V,3,3) device */
  const float* RT;         /* (V,3,4) device, world -> camera */
  const uint8_t* msks;     /* (V,img_h,img_w) device */
  int img_h, img_w;
} anr_sdf_frame;

typedef struct anr_sdf_render_out {
  float* rgb_map;      /* (R,3) */
  float* acc_map;      /* (R) */
  float* depth_map;    /* (R) */
  float* raw;          /* (R*64,4) */
  float* sdf;          /* (R*64) (10 at samples the KNN filter drops) */
  float* tbounds_out;  /* (2,3) or NULL: batch['tbounds'] after the reference's in-place widening
                          by 0.05 per chunk (anisdf_pdf_network.py:203-205) */
} anr_sdf_render_out;

/* o->norm_th is the KNN distance threshold (0.1 in the reference, :172). Reads the kept-sample
 * count once (host sync) to size the layer GEMMs. Eval path: the training-only
 * 'observed_gradients' (:187-193) are not produced. */
size_t anr_sdf_render_workspace_bytes(int n_rays, const anr_render_opts* o);
int anr_sdf_render_fwd(const anr_sdf_params* p, const anr_sdf_frame* f, const float* ray_o, const float* ray_d,
                       const float* near_, const float* far_, int n_rays, const anr_render_opts* o,
                       const anr_sdf_render_out* out, void* workspace, size_t ws_bytes, void* stream);
/* device int32[2] inside the workspace: {kept samples n', msk_sdf length}. */
const int32_t* anr_sdf_render_counts(const void* workspace, int n_rays, const anr_render_opts* o);
/* device uint32 (R*64, 8) inside the workspace: the front-end's per-sample KNN records (w0..w4 float
 * bits, i0 | i1 << 16, i2 | i3 << 16, i4) of the last anr_sdf_render_fwd -- a debugging / test view of
 * the pytorch3d knn_points boundary (sample_utils.py:309-348). */
const uint32_t* anr_sdf_render_knn(const void* workspace, int n_rays, const anr_render_opts* o);
/* copy resd (n',3), gradients (n',3), msk_sdf / msk_label (len) out of the workspace */
int anr_sdf_render_rows(const void* workspace, int n_rays, const anr_render_opts* o, float* resd, float* gradients,
                        float* msk_sdf, float* msk_label, void* stream);

/* ---- sdf_pdf Network.forward over free samples (anisdf_pdf_network.py:156-224) -----------------
 * The call tpose_renderer makes per chunk over the sdf_pdf network, self.net(wpts, viewdir, dists,
 * batch) (tpose_renderer.py:95; configs/sdf_pdf/anisdf_pdf_s9p.yaml:9-12): x->n_pts samples (world
 * points, world view directions; dists is not read: the Laplace density uses the constant 0.005,
 * :330). One call = one reference chunk: the KNN prefilter keeps pnorm < o->norm_th (0.1) plus the
 * argmin of pnorm over the call, and batch['tbounds'] is widened ONCE (tbounds_out, or NULL).
 * world -> pose follows torch's matmul rule for an (n_pts, 3) product (n_pts < 45: its small path).
 *  anr_sdf_network_fwd: evaluation (no observed_gradients), o->precision ANR_FP32 or ANR_BF16X3 as the
 *    sdf render; raw (n,4) zero at dropped samples and outside the widened tbounds, sdf (n) = 10 at
 *    dropped samples. Reads the kept count once (host sync).
 *  anr_sdf_network_counts: device int32 {kept n', 0}; anr_sdf_network_rows: resd (n',3) and gradients
 *    (n',3) of the kept samples, in sample order. */
size_t anr_sdf_network_workspace_bytes(int n_pts, const anr_render_opts* o);
int anr_sdf_network_fwd(const anr_sdf_params* p, const anr_sdf_frame* f, const anr_samples* x, const anr_render_opts* o,
                        float* raw, float* sdf, float* tbounds_out, void* workspace, size_t ws_bytes, void* stream);
const int32_t* anr_sdf_network_counts(const void* workspace, int n_pts);
int anr_sdf_network_rows(const void* workspace, int n_pts, float* resd, float* gradients, void* stream);
/* Under autograd (the reference's training forward, :187-199): the layer-wise exact-fp32 executor of
 * anr_sdf_train_step over the call's samples.
 *  anr_sdf_network_train_fwd: as anr_sdf_network_fwd plus 'observed_gradients' = d sdf(x + resd(x)) / d x
 *    at the kept samples with |sdf| < 0.02 (x = init_bigpose, :140-154). Two host reads (counts).
 *  anr_sdf_network_train_counts: device int32 {kept n', 0, observed rows n_o, 0}.
 *  anr_sdf_network_train_rows: resd (n',3), gradients (n',3), observed_gradients (n_o,3) (any NULL: skipped).
 *  anr_sdf_network_train_bwd: loss.backward() through the call: ACCUMULATES into grads (anr_sdf_params
 *    order; resd_latent may be NULL) the parameter gradients of the upstream adjoints d raw (n,4),
 *    d sdf (n), d resd (n',3), d gradients (n',3), d observed_gradients (n_o,3) (any NULL = 0), with the
 *    second-order terms the reference's create_graph=True input gradients carry. It re-runs the forward
 *    on the same workspace first, so f->tbounds must hold the bounds the forward call was given (before
 *    its widening). */
size_t anr_sdf_network_train_workspace_bytes(int n_pts);
int anr_sdf_network_train_fwd(const anr_sdf_params* p, const anr_sdf_frame* f, const anr_samples* x,
                              const anr_render_opts* o, float* raw, float* sdf, float* tbounds_out, void* workspace,
                              size_t ws_bytes, void* stream);
const int32_t* anr_sdf_network_train_counts(const void* workspace, int n_pts);
int anr_sdf_network_train_rows(const void* workspace, int n_pts, float* resd, float* gradients,
                               float* observed_gradients, void* stream);
int anr_sdf_network_train_bwd(const anr_sdf_params* p, float* const* grads, const anr_sdf_frame* f, const anr_samples* x,
                              const anr_render_opts* o, const float* d_raw, const float* d_sdf, const float* d_resd,
                              const float* d_gradients, const float* d_observed_gradients, void* workspace,
                              size_t ws_bytes, void* stream);

/* ---- sdf_pdf point helpers (the sdf mesh path, lib/networks/renderer/sdf_mesh_renderer.py:16-110) ----
 * anr_sdf_points over n free points x (n,3) in the big-pose (canonical) space, exact fp32 products on the
 * sdf training executor's layers (weight norm formed per call; f needs poses and latent_index only):
 *   ANR_SDFP_NETWORK            tpose_human.sdf_network(x, batch) (anisdf_pdf_network.py:421-437):
 *                               out (n,257) = [sdf || feature vector] (scale 1)
 *   ANR_SDFP_GRADIENT           SDFNetwork.gradient(x) (:441-451): out (n,3) d sdf / d x, out2 (n) sdf (or NULL)
 *   ANR_SDFP_DEFORMED_GRADIENT  Network.gradient_of_deformed_sdf(x, batch) (:140-154): out (n,3) the gradient
 *                               of sdf(x + resd(x)) w.r.t. x (residual MLP included), out2 (n) that sdf (or NULL)
 * The host reads nothing; the call is asynchronous on the stream. */
#define ANR_SDFP_NETWORK 0
#define ANR_SDFP_GRADIENT 1
#define ANR_SDFP_DEFORMED_GRADIENT 2
size_t anr_sdf_points_workspace_bytes(int n);
int anr_sdf_points(const anr_sdf_params* p, const anr_sdf_frame* f, const float* x, int n, int mode, float* out,
                   float* out2, void* workspace, size_t ws_bytes, void* stream);
/* sample_blend_closest_points (lib/utils/sample_utils.py:323-348) of n free points against nv vertices
 * (nv, 3) with their weights (nv, 24): the render front-end's exact 5-NN (lexicographic (d^2, index) ties)
 * and inverse-distance blend. bw (n, 24) the blended weights and / or inside (n) = weighted distance
 * < norm_th (no forced argmin: the sdf mesh path's filter, sdf_mesh_renderer.py:58-60). */
size_t anr_knn_blend_workspace_bytes(int n);
int anr_knn_blend(const float* verts, const float* weights, int nv, const float* pts, int n, float norm_th, float* bw,
                  uint8_t* inside, void* workspace, size_t ws_bytes, void* stream);
/* The sdf mesh path's posed vertices (sdf_mesh_renderer.py:96-101): pose_points_to_tpose_points(pts, bw,
 * big_A), tpose_points_to_pose_points(., bw, A), pose_points_to_world_points(., R, Th) -> out (n, 3). */
int anr_sdf_mesh_pose(const float* pts, const float* bw, int n, const float* big_A, const float* A, const float* R,
                      const float* Th, float* out, void* stream);
/* pts_sample_blend_weights (lib/utils/blend_utils.py:119-149; Network.calculate_bigpose_smpl_bw,
 * anisdf_pdf_network.py:109-112): trilinear grid_sample (align_corners, border padding) of the volume vol
 * (X,Y,Z,C) over bounds (2,3) at pts (n,3) -> out (C, n), the reference's (1, 25, n) without the batch axis,
 * bit-exact in the reference's CPU accumulation order. */
int anr_sample_volume(const float* vol, int X, int Y, int Z, int C, const float* bounds, const float* pts, int n,
                      float* out, void* stream);

/* ---- sdf_pdf training (config 5; lib/train/trainers/tpose_trainer.py:21-73, crit.py:5-19) ---------
 * anr_sdf_train_step: NetworkWrapper.forward + loss.backward() of one batch through the sdf_pdf
 *   network and tpose_renderer (anisdf_pdf_network.py:156-224 in training mode: gradients with
 *   create_graph, observed_gradients at the kept samples with |sdf| < 0.02), then the losses
 *   offset 0.01 mean|resd|, eikonal 0.01 mean(|g|-1)^2 (gradients and observed_gradients), msk_sdf
 *   BCE (alpha 50 doubled past iteration 10k, 20k, ... as crit.sdf_mask_crit) and the image MSE over
 *   mask_at_box (NULL: every ray). ACCUMULATES the gradients of every tensor of anr_sdf_params into
 *   grads (state_dict order; resd_latent, never read, may be NULL). loss (device float[10]) = {loss,
 *   offset_loss, grad_loss, ograd_loss, mask_loss, img_loss, observed rows, msk_sdf entries, kept
 *   samples, 0}.
 *   out: rgb_map / acc_map / depth_map (R), tbounds_out (widened) or NULL; raw / sdf unused.
 *   Perturbation through o->t_rand; o->norm_th = 0.1. Two host reads (kept and observed counts). */
size_t anr_sdf_train_workspace_bytes(int n_rays, const anr_render_opts* o);
int anr_sdf_train_step(const anr_sdf_params* p, float* const* grads, const anr_sdf_frame* f, const float* ray_o,
                       const float* ray_d, const float* near_, const float* far_, int n_rays, const anr_render_opts* o,
                       const float* rgb_gt, const uint8_t* mask_at_box, int iter_step, const anr_sdf_render_out* out,
                       float* loss, void* workspace, size_t ws_bytes, void* stream);
/* anr_sdf_train_step_hooked: anr_sdf_train_step plus a hook for overlapping the gradient all-reduce
 * with the rest of the backward (DDP's buckets, trainer.py:13-18). Once the gradients of tensors 28..43
 * (color_network.*, colour latent included) are final, colour_grads_ready (a hipEvent_t, or NULL) is
 * recorded on the stream and then colour_ready (or NULL) is called on the host with that event and the
 * stream, while the SDF's stacked reverse, the residual backward and the observed-gradient passes
 * (tensors 0..27, 45..62) are still to be issued: the caller issues the colour bucket's collective there
 * (ordered after the event) and it runs beside them. A non-zero return from colour_ready fails the call.
 * struct_size must be sizeof(anr_sdf_train_hooks). hooks == NULL: anr_sdf_train_step. */
typedef int (*anr_ready_fn)(void* user, void* event, void* stream);
typedef struct anr_sdf_train_hooks {
  size_t struct_size;
  void* colour_grads_ready;
  anr_ready_fn colour_ready;
  void* user;
} anr_sdf_train_hooks;
int anr_sdf_train_step_hooked(const anr_sdf_params* p, float* const* grads, const anr_sdf_frame* f,
                              const float* ray_o, const float* ray_d, const float* near_, const float* far_,
                              int n_rays, const anr_render_opts* o, const float* rgb_gt, const uint8_t* mask_at_box,
                              int iter_step, const anr_sdf_render_out* out, float* loss,
                              const anr_sdf_train_hooks* hooks, void* workspace, size_t ws_bytes, void* stream);

/* ---- (f) mesh path (lib/networks/renderer/aninerf_mesh_renderer.py) ----------------------
 * anr_alpha_points: raw alpha (no activation, no bbox mask) of n free world points, zero where the
 *   pbw prefilter drops the point: pnorm < o->norm_th (0.1 in get_alpha) plus the argmin of pnorm
 *   over each chunk of o->chunk_pts points (2048 * 64 in the reference; a multiple of 64). Uses
 *   the pose-space BW MLP (or novel_pose_bw with o->novel_pose), the LBS inverse, the NeRF trunk
 *   and alpha_fc; o->precision ANR_FP32 (exact fp32 MFMA) or ANR_BF16X3. Frame fields read: A, R,
 *   Th, pbw(+dims), pbounds, latent_index (bw_latent_index for novel_pose). No host sync.
 *   anr_alpha_counts: device int32 {kept points} inside the workspace. */
typedef struct anr_alpha_opts {
  int chunk_pts;   /* points per reference chunk (2048 * 64) */
  float norm_th;   /* 0.1 (tpose_nerf_network.py:113) */
  int novel_pose;  /* cfg.test_novel_pose */
  int precision;   /* ANR_FP32 or ANR_BF16X3 */
} anr_alpha_opts;
size_t anr_alpha_workspace_bytes(long n_pts, const anr_alpha_opts* o, const anr_frame* f);
int anr_alpha_points(const anr_params* p, const anr_frame* f, const float* wpts, long n_pts, const anr_alpha_opts* o,
                     float* alpha, void* workspace, size_t ws_bytes, void* stream);
const int32_t* anr_alpha_counts(const void* workspace);
/* Marching cubes over vol (X,Y,Z) f32 padded by `pad` zero voxels on every side (virtually):
 * anr_mc_count writes device int32 {V, T} to counts; anr_mc_emit (same vol / workspace, after the
 * caller sized the outputs) writes vertices (V,3) f64 in padded index coordinates and triangles
 * (T,3) int64. A corner is outside iff value <= iso. One vertex per crossing grid edge, numbered in
 * grid order (C order of the padded grid, then axis x, y, z); triangles per cube in grid order from
 * the case table of tools/gen_mc_table.py, wound with the normal towards the outside. */
size_t anr_mc_workspace_bytes(int X, int Y, int Z, int pad);
int anr_mc_count(const float* vol, int X, int Y, int Z, int pad, double iso, int32_t* counts, void* workspace,
                 size_t ws_bytes, void* stream);
int anr_mc_emit(const float* vol, int X, int Y, int Z, int pad, double iso, double* vertices, int64_t* triangles,
                void* workspace, size_t ws_bytes, void* stream);

/* ---- measurement ----------------------------------------------------------------------
 * When enabled, anr_render_fwd records a hipEvent pair around the fused network kernel (k_mlp)
 * on the caller's stream, and anr_sdf_render_fwd one around each fused sdf_pdf network launch. anr_profile_read waits for the recorded events, returns the summed
 * kernel time (ms) and launch count since the last read, and resets. */
int anr_profile_enable(int on);
int anr_profile_read(double* mlp_ms, int* launches);
/* anr_profile_read plus the median in-kernel shader clock (MHz) over every stamped workgroup of the
 * profiled fused launches (thread 0 stamps s_memtime / s_memrealtime at entry and exit; 0 if none ran
 * long enough): tells a DVFS-throttled box from a slower kernel. */
int anr_profile_read_clock(double* mlp_ms, int* launches, double* clk_mhz);

const char* anr_last_error(void);
int anr_version(void);

#ifdef __cplusplus
}
#endif
#endif
