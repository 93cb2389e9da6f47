// anr_layers.h — the MLP layer program shared by the weight packer (anr_pack) and the fused kernel.
//
// MFMA tiling (v_mfma_f32_16x16x4_f32, exact fp32):  D[i][j] = sum_k A[i][k] B[k][j]
//   i = output neuron (16 per "out-block" ob), j = point (16 per wave), k = 4 inputs per "k-step".
//   A (weights) lane l: A[l&15][l>>4];  B (activations) lane l: B[l>>4][l&15];
//   C/D lane l: point l&15, neurons 4*(l>>4)+r in register r (r = 0..3).
// So a layer's accumulators are directly the next layer's B operand: k-step (ob', r) feeds input
// neurons ob'*16 + 4g + r in k-slot g = l>>4. Gamma features come as k-step s -> feature 4s+g.
//
// Weight image: for every layer, k-steps in program order; per k-step C = ceil(OB/4) chunks of
// [64 lanes][4 floats] (lane reads one float4 per chunk = ds_read_b128, conflict-free), the float
// (ob%4) of chunk ob/4 being W[ob*16 + (l&15)][col(kstep, l>>4)] (0 outside the tensor).
// Layers are grouped into "slices" of 8 k-steps, the unit staged HBM->LDS.
#pragma once

namespace anr {

// SRC_EMB: gamma_10(x) (63); SRC_VEMB: gamma_4(dir) (27); SRC_EMB6: gamma_6(x) (39, the sdf_pdf SDF net);
// SRC_G0 / SRC_G1: columns of a memory row (the sdf_pdf colour net's inputs; anr_mlp_body.h LayerIO)
enum SrcKind { SRC_EMB = 0, SRC_ACT = 1, SRC_VEMB = 2, SRC_EMB6 = 3, SRC_G0 = 4, SRC_G1 = 5 };

// A segment of a layer's K dimension: `ksteps` k-steps from one source; `col0` = first weight column;
// `nact` (ACT segments, 0 = all): input neurons past it are padding (zero weight columns).
struct Seg { int kind; int ksteps; int col0; int nact = 0; };

struct LayerDesc {
  int tensor_w;   // index into anr_params.t of the weight (out, in, 1)
  int tensor_b;   // index of the bias
  int tensor_w2;  // second weight stacked as extra out-blocks (alpha_fc beside feature_fc), or -1
  int tensor_b2;
  int nout;       // output neurons of tensor_w
  int nout2;      // output neurons of tensor_w2 (0 if none)
  int in_ch;      // columns of tensor_w (row stride)
  int ob;         // out-blocks of 16 (incl. the tensor_w2 blocks)
  int nseg;
  Seg seg[2];
  int trans = 0;  // packed as the transpose: element (row i, col k) = W[k * in_ch + i] (in_ch = W's row stride)
};

#define ANR_KSLICE 8  // k-steps per staged slice

// BW MLP (tpose_nerf_network.py:21-29, 55-77): gamma(63) || latent(128) -> 8 x 256 (skip at 4) -> 24.
// Latent columns (63..190 of layers 0 and 5) are folded into a per-frame bias.
// NeRF (TPoseHuman :226-239, 252-275).
#define ANR_NUM_LAYERS 19
#define ANR_BW_LAYERS 9

__host__ __device__ constexpr LayerDesc layer_desc(int i) {
  // clang-format off
  return i == 0  ? LayerDesc{28, 29, -1, -1, 256, 0, 191, 16, 1, {{SRC_EMB, 16, 0}, {0, 0, 0}}}
       : i == 1  ? LayerDesc{30, 31, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 2  ? LayerDesc{32, 33, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 3  ? LayerDesc{34, 35, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 4  ? LayerDesc{36, 37, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 5  ? LayerDesc{38, 39, -1, -1, 256, 0, 447, 16, 2, {{SRC_EMB, 16, 0}, {SRC_ACT, 64, 191}}}
       : i == 6  ? LayerDesc{40, 41, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 7  ? LayerDesc{42, 43, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 8  ? LayerDesc{44, 45, -1, -1, 24, 0, 256, 2, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 9  ? LayerDesc{1, 2, -1, -1, 256, 0, 63, 16, 1, {{SRC_EMB, 16, 0}, {0, 0, 0}}}
       : i == 10 ? LayerDesc{3, 4, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 11 ? LayerDesc{5, 6, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 12 ? LayerDesc{7, 8, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 13 ? LayerDesc{9, 10, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 14 ? LayerDesc{11, 12, -1, -1, 256, 0, 319, 16, 2, {{SRC_EMB, 16, 0}, {SRC_ACT, 64, 63}}}
       : i == 15 ? LayerDesc{13, 14, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == 16 ? LayerDesc{15, 16, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       // feature_fc (16 blocks) + alpha_fc (block 16)
       : i == 17 ? LayerDesc{19, 20, 17, 18, 256, 1, 256, 17, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       // latent_fc: feature part only (cols 0..255); nf_latent part folded into the bias
       : i == 18 ? LayerDesc{21, 22, -1, -1, 256, 0, 384, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : LayerDesc{0, 0, -1, -1, 0, 0, 0, 0, 0, {{0, 0, 0}, {0, 0, 0}}};
  // clang-format on
}
// view_fc (128, 283): latent_fc out (64 ksteps) || gamma(dir) 27 (8 ksteps, padded)
// rgb_fc (3, 128): view out (32 ksteps)
#define ANR_L_VIEW 19
#define ANR_L_RGB 20
// layers 21..29: novel_pose_bw (BackwardBlendWeight), same shapes as 0..8, tensors 46 + (0..18)
#define ANR_L_NOVEL0 21
// layer 30: alpha_fc alone (TPoseHuman.calculate_alpha :241-250, the density-only program of the
// mesh path's get_alpha); the same weights as out-block 16 of layer 17
#define ANR_L_ALPHA 30
#define ANR_NUM_LAYERS_ALL 32  // layers of the fp32 image (0..30 above + the folded head 31 below)
// layer 31: the folded colour head (both images; the render program of either kernel). feature_fc -> [|| nf_latent] latent_fc ->
// [|| gamma(dir)] view_fc has no activation before view_fc's ReLU (tpose_nerf_network.py:260-272), so
// view_fc's pre-activation is (Wv_f Wl_f Wf) net + Wv_d gamma(dir) + c(latent): one 283-input layer
// of 128 outputs, with alpha_fc stacked as output row 128 (out-block 8, no ReLU). Weights: the head
// tensor H (129 x 283) that k_pack_head composes in fp64 inside the packed buffer; per-frame bias
// c = P nf_latent[li] + q (k_prep). Render program V = 2 (anr_mlp_body.h), fp32 and bf16x3 alike.
#define ANR_L_HEAD 31
#define ANR_HEAD_T 65  // PackArgs tensor index of H
#define ANR_NOVEL_T0 46  // tensor index of novel_pose_bw.bw_latent.weight in the packer's list

__host__ __device__ constexpr LayerDesc novel_desc(int i) {
  return LayerDesc{layer_desc(i).tensor_w + 19, layer_desc(i).tensor_b + 19, -1, -1, layer_desc(i).nout, 0,
                   layer_desc(i).in_ch, layer_desc(i).ob, layer_desc(i).nseg,
                   {layer_desc(i).seg[0], layer_desc(i).seg[1]}};
}

// layers 32..40: the sdf_pdf residual deformation MLP (anisdf_pdf_network.py:24-31, 49-73):
// [gamma_10(x) 63 || poses 72] -> 8 x 256 ReLU (skip [features || h] at layer 5, in 391) -> resd_fc 3.
// The poses columns are folded into the layer-0 / layer-5 biases (k_sdf_fold), as the BW MLP's latent.
// Packed into the sdf render's own bf16x3 image (k_pack_resd); tensor indices are those of its
// PackArgs: weight of layer 32 + l at t[l], bias at t[9 + l].
#define ANR_L_RESD0 32
#define ANR_RESD_LAYERS 9
__host__ __device__ constexpr LayerDesc resd_desc(int l) {
  return l == 0   ? LayerDesc{0, 9, -1, -1, 256, 0, 135, 16, 1, {{SRC_EMB, 16, 0}, {0, 0, 0}}}
         : l == 5 ? LayerDesc{5, 14, -1, -1, 256, 0, 391, 16, 2, {{SRC_EMB, 16, 0}, {SRC_ACT, 64, 135}}}
         : l == 8 ? LayerDesc{8, 17, -1, -1, 3, 0, 256, 1, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
                  : LayerDesc{l, 9 + l, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}};
}

// layers 41..49: the sdf_pdf SDF network (anisdf_pdf_network.py:349-440, SDFNetwork: weight-normed
// lin0..lin8, softplus(beta=100) after lin0..lin7, skip at lin4 = [h3 (217) || gamma_6(x) (39)] / sqrt2,
// lin8 -> [sdf || feature 256]) on the effective weights g v / |v| (k_sdf_wnorm). Packed into the sdf
// render's image after the residual MLP (k_pack_seq; lin4's weights pre-scaled by 1/sqrt2); tensor
// indices of its PackArgs: weight of lin l at t[l], bias at t[9 + l].
#define ANR_L_SDF0 41
#define ANR_SDF_LAYERS 9
__host__ __device__ constexpr LayerDesc sdfnet_desc(int l) {
  return l == 0   ? LayerDesc{0, 9, -1, -1, 256, 0, 39, 16, 1, {{SRC_EMB6, 16, 0}, {0, 0, 0}}}
         : l == 3 ? LayerDesc{3, 12, -1, -1, 217, 0, 256, 14, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
         : l == 4 ? LayerDesc{4, 13, -1, -1, 256, 0, 256, 16, 2, {{SRC_ACT, 56, 0, 217}, {SRC_EMB6, 16, 217}}}
         : l == 8 ? LayerDesc{8, 17, -1, -1, 257, 0, 256, 17, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
                  : LayerDesc{l, 9 + l, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}};
}

// layers 50..57: the SDF network's input gradient d sdf / d x (SDFNetwork.gradient, autograd.grad of
// anisdf_pdf_network.py:302-311) in reverse mode: entry r applies lin l = 7 - r transposed, W_l^T dz_l,
// to dz_l = dh_l * sigmoid(100 z_l) (the factor recomputed from the stored h_l). lin4's transpose carries
// the skip's 1/sqrt2 (packed scaled); lin3's has the 217 valid inputs; lin0's gives the 39 gamma_6
// gradients. Same PackArgs as the forward (t[l] = weight of lin l; t[17] NULL: no biases).
#define ANR_L_SREV0 50
#define ANR_SREV_LAYERS 8
__host__ __device__ constexpr LayerDesc sdfrev_desc(int r) {
  return r == 4   ? LayerDesc{3, 17, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 56, 0, 217}, {0, 0, 0}}, 1}
         : r == 7 ? LayerDesc{0, 17, -1, -1, 39, 0, 39, 3, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}, 1}
                  : LayerDesc{7 - r, 17, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}, 1};
}

// layers 58..62: the sdf_pdf colour network (anisdf_pdf_network.py:469-545, ColorNetwork, mode idr):
// lin0 on [points 3 || gamma_4(dir) 27 || normal 3] (a C0 row, SRC_G0) || feature 256 (lin8's, SRC_G1),
// lin1, lin2, lin3 on [h2 || color_latent] (the latent folded into lin3's bias, k_sdf_fold), ReLU after
// each, lin4 -> 3 logits. Weight-normed: t[l] = effective weight of lin l, t[9 + l] its bias.
#define ANR_L_COL0 58
#define ANR_COL_LAYERS 5
__host__ __device__ constexpr LayerDesc color_desc(int l) {
  return l == 0   ? LayerDesc{0, 9, -1, -1, 256, 0, 289, 16, 2, {{SRC_G0, 16, 0, 33}, {SRC_G1, 64, 33}}}
         : l == 3 ? LayerDesc{3, 12, -1, -1, 256, 0, 384, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
         : l == 4 ? LayerDesc{4, 13, -1, -1, 3, 0, 256, 1, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
                  : LayerDesc{l, 9 + l, -1, -1, 256, 0, 256, 16, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}};
}

__host__ __device__ constexpr LayerDesc layer_desc_all(int i) {
  return i >= ANR_L_COL0 ? color_desc(i - ANR_L_COL0)
       : i >= ANR_L_SREV0 ? sdfrev_desc(i - ANR_L_SREV0)
       : i >= ANR_L_SDF0 ? sdfnet_desc(i - ANR_L_SDF0)
       : i >= ANR_L_RESD0 ? resd_desc(i - ANR_L_RESD0)
       : i < ANR_NUM_LAYERS ? layer_desc(i)
       : i == ANR_L_VIEW ? LayerDesc{23, 24, -1, -1, 128, 0, 283, 8, 2, {{SRC_ACT, 64, 0}, {SRC_VEMB, 8, 256}}}
       : i == ANR_L_RGB  ? LayerDesc{25, 26, -1, -1, 3, 0, 128, 1, 1, {{SRC_ACT, 32, 0}, {0, 0, 0}}}
       : i < ANR_L_ALPHA ? novel_desc(i - ANR_L_NOVEL0)
       : i == ANR_L_ALPHA ? LayerDesc{17, 18, -1, -1, 1, 0, 256, 1, 1, {{SRC_ACT, 64, 0}, {0, 0, 0}}}
       : i == ANR_L_HEAD ? LayerDesc{ANR_HEAD_T, -1, -1, -1, 129, 0, 283, 9, 2, {{SRC_ACT, 64, 0}, {SRC_VEMB, 8, 256}}}
       : LayerDesc{0, 0, -1, -1, 0, 0, 0, 0, 0, {{0, 0, 0}, {0, 0, 0}}};
}

__host__ __device__ constexpr int layer_chunks(int i) { return (layer_desc_all(i).ob + 3) / 4; }
__host__ __device__ constexpr int layer_ksteps(int i) {
  return layer_desc_all(i).seg[0].ksteps + (layer_desc_all(i).nseg > 1 ? layer_desc_all(i).seg[1].ksteps : 0);
}
// bytes of a layer's weight image
__host__ __device__ constexpr int layer_bytes(int i) { return layer_ksteps(i) * layer_chunks(i) * 1024; }
__host__ __device__ constexpr int layer_offset(int i) {
  int o = 0;
  for (int k = 0; k < i; ++k) o += layer_bytes(k);
  return o;
}
__host__ __device__ constexpr int weights_bytes() { return layer_offset(ANR_NUM_LAYERS_ALL); }

// bias section (floats), padded to ob*16 per layer, after the weight image
__host__ __device__ constexpr int layer_bias_floats(int i) { return layer_desc_all(i).ob * 16; }
__host__ __device__ constexpr int bias_offset(int i) {
  int o = 0;
  for (int k = 0; k < i; ++k) o += layer_bias_floats(k);
  return o;
}
template <int L> inline constexpr int kBiasOff = bias_offset(L);
// byte / float offsets from a base BW layer to its novel_pose_bw copy
#define ANR_NOVEL_WOFF (layer_offset(ANR_L_NOVEL0) - layer_offset(0))
#define ANR_NOVEL_BOFF (bias_offset(ANR_L_NOVEL0) - bias_offset(0))
__host__ __device__ constexpr int bias_floats() { return bias_offset(ANR_NUM_LAYERS_ALL); }
__host__ __device__ constexpr int packed_bytes() { return weights_bytes() + bias_floats() * 4; }

// weight column fed by k-step t, k-slot g (-1 = padding)
__host__ __device__ inline int layer_col(const LayerDesc& d, int t, int g) {
  int s = 0;
  for (; s < d.nseg; ++s) {
    if (t < d.seg[s].ksteps) break;
    t -= d.seg[s].ksteps;
  }
  const Seg sg = d.seg[s];
  if (sg.kind == SRC_ACT) {
    const int ob = t >> 2, r = t & 3;
    return sg.col0 + ob * 16 + 4 * g + r;
  }
  const int f = 4 * t + g;  // gamma feature
  const int nf = (sg.kind == SRC_EMB) ? 63 : 27;
  return f < nf ? sg.col0 + f : -1;
}

// ------------------------------------------------------------------------------------------
// bf16x3 image (render precision ANR_BF16X3): layers 0..20 again, for v_mfma_f32_16x16x32_bf16.
//   A (weights) lane l: A[row l&15][k = 8(l>>4) + j], j = 0..7;  B (activations) the same k map.
//   Each weight w is stored as hi = bf16(w), lo = bf16(w - hi); a product is accumulated as
//   lo*bh + hi*bl + hi*bh (the dropped lo*bl and rounding terms are ~2^-16 relative).
// k-step s of 32 inputs:
//   ACT segment: previous out-blocks 2s, 2s+1; lane half h element j <-> neuron
//                32s + (j < 4 ? 4h + j : 16 + 4h + j - 4), i.e. the two accumulators of the
//                previous layer as they sit in the lane (no data movement);
//   EMB / VEMB : feature 32s + 8h + j.
// Per k-step, per out-block: [hi: 64 lanes x 16 B][lo: 64 lanes x 16 B] = 2 KiB; a k-step of the
// first 16 out-blocks is the staging slice (<= 32 KiB). A layer wider than 16 out-blocks (feature_fc
// || alpha_fc, 17) stores its extra blocks after the main part, [k-step][tail block], and stages
// them as one more slice after its k-steps, so a ring slot stays 32 KiB.
__host__ __device__ constexpr int ks32(int i) { return layer_ksteps(i) / 8; }
__host__ __device__ constexpr int b16_main_ob(int i) { return layer_desc_all(i).ob < 16 ? layer_desc_all(i).ob : 16; }
__host__ __device__ constexpr int b16_tail_ob(int i) { return layer_desc_all(i).ob - b16_main_ob(i); }
__host__ __device__ constexpr int b16_layer_bytes(int i) { return ks32(i) * layer_desc_all(i).ob * 2048; }
#define ANR_B16_LAYERS 32  // layers 0..31 (incl. the novel_pose_bw copy 21..29, alpha_fc 30, head 31)
__host__ __device__ constexpr int b16_layer_offset(int i) {
  int o = 0;
  for (int k = 0; k < i; ++k) o += b16_layer_bytes(k);
  return o;
}
__host__ __device__ constexpr int b16_bytes() { return b16_layer_offset(ANR_B16_LAYERS); }
#define ANR_B16_NOVEL_WOFF (b16_layer_offset(ANR_L_NOVEL0) - b16_layer_offset(0))
// a packed layer sequence L0 .. L0 + nl - 1 (k_pack_seq): weights from byte 0, biases after
__host__ __device__ constexpr int seq_layer_offset(int L0, int L) { return b16_layer_offset(L) - b16_layer_offset(L0); }
__host__ __device__ constexpr int seq_wbytes(int L0, int nl) { return seq_layer_offset(L0, L0 + nl); }
__host__ __device__ constexpr int seq_bias_off(int L0, int l) {
  int o = 0;
  for (int k = 0; k < l; ++k) o += layer_desc_all(L0 + k).ob * 16;
  return o;
}
__host__ __device__ constexpr int seq_image_bytes(int L0, int nl) { return seq_wbytes(L0, nl) + seq_bias_off(L0, nl) * 4; }
// arithmetic of the pose-space pass in the bf16 kernel: 1 = bf16x3 (default), 2 = bf16x6
#ifndef ANR_POSE_MODE
#define ANR_POSE_MODE 1
#endif
// byte offset of the bf16 image inside the packed buffer (after the fp32 weights and the biases)
__host__ __device__ constexpr int b16_base() { return (packed_bytes() + 255) / 256 * 256; }


// bf16x6 image (render precision ANR_BF16X6, k_mlp_x6 / k_alpha_x6; and the pose-space BW pass of a
// bf16x3 kernel built with ANR_POSE_MODE=2): layers 0..31, each weight as hi/mid/lo bf16 (w = hi +
// mid + lo to 24 bits), the activation likewise; products hl + lh + mm + hm + mh + hh (the dropped
// ml, lm, ll terms are <= ~2^-24 relative: fp32-level). Per k-step, per out-block [hi][mid][lo]
// fragments = 3 KiB; a k-step is staged as groups of <= 8 out-blocks.
#define ANR_X6_LAYERS 32
__host__ __device__ constexpr int x6_layer(int i) { return i; }
__host__ __device__ constexpr int x6_layer_bytes(int i) { return ks32(x6_layer(i)) * layer_desc_all(x6_layer(i)).ob * 3072; }
__host__ __device__ constexpr int x6_layer_offset(int i) {
  int o = 0;
  for (int k = 0; k < i; ++k) o += x6_layer_bytes(k);
  return o;
}
__host__ __device__ constexpr int x6_bytes() { return x6_layer_offset(ANR_X6_LAYERS); }
__host__ __device__ constexpr int x6_base() { return (b16_base() + b16_bytes() + 255) / 256 * 256; }
#define ANR_X6_NOVEL_WOFF (x6_layer_offset(ANR_L_NOVEL0) - x6_layer_offset(0))
// a layer sequence L0 .. L0 + nl - 1 as its own bf16x6 image (k_pack_seq_x6; the sdf render's fused
// programs in render precision ANR_BF16X6): weights [k-step][out-block][hi|mid|lo] from byte 0, then the
// biases laid out as in the bf16x3 sequence image (seq_bias_off)
__host__ __device__ constexpr int x6_any_layer_bytes(int L) { return ks32(L) * layer_desc_all(L).ob * 3072; }
__host__ __device__ constexpr int x6seq_layer_offset(int L0, int L) {
  int o = 0;
  for (int k = L0; k < L; ++k) o += x6_any_layer_bytes(k);
  return o;
}
__host__ __device__ constexpr int x6seq_wbytes(int L0, int nl) { return x6seq_layer_offset(L0, L0 + nl); }
__host__ __device__ constexpr int x6seq_image_bytes(int L0, int nl) { return x6seq_wbytes(L0, nl) + seq_bias_off(L0, nl) * 4; }

// Gamma features in the bf16 image (EMB / VEMB segments of NS k-steps): element pairs (2p, 2p+1) of
// lane half h in k-step t hold (sin, cos) of one argument x[comp] * 2^freq, so a lane evaluates one
// shared-reduction sincos per pair (anr_mlp_body.h embed_b). Pair slot u = 4 NS h + 4 t + p: slots
// 0 and 1 hold x, y, z and a zero pad; slot u >= 2 holds pair P = u - 2 = 3 freq + comp (zero past
// 3 nfreq). Reference feature order (embedder.py:5-54): [x, sin(2^0 x), cos(2^0 x), sin(2^1 x), ...].
__host__ __device__ constexpr int gamma_slot_feature(int ns, int nfreq, int t, int h, int j) {
  const int u = 4 * ns * h + 4 * t + (j >> 1);
  if (u < 2) {
    const int f = 2 * u + (j & 1);
    return f < 3 ? f : -1;
  }
  const int P = u - 2;
  if (P >= 3 * nfreq) return -1;
  const int freq = P / 3, comp = P - 3 * freq;
  return 3 + 6 * freq + 3 * (j & 1) + comp;
}

// weight column for bf16 k-step t, lane half h, element j (-1 = padding)
__host__ __device__ inline int b16_col(const LayerDesc& d, int t, int h, int j) {
  int s = 0;
  for (; s < d.nseg; ++s) {
    if (t < d.seg[s].ksteps / 8) break;
    t -= d.seg[s].ksteps / 8;
  }
  const Seg sg = d.seg[s];
  if (sg.kind == SRC_ACT) {
    const int n = 32 * t + (j < 4 ? 4 * h + j : 16 + 4 * h + j - 4);
    return sg.nact && n >= sg.nact ? -1 : sg.col0 + n;
  }
  if (sg.kind == SRC_G0 || sg.kind == SRC_G1) {  // a memory row, contiguous per lane half
    const int n = 32 * t + 8 * h + j;
    return sg.nact && n >= sg.nact ? -1 : sg.col0 + n;
  }
  const int f = gamma_slot_feature(sg.ksteps / 8, sg.kind == SRC_EMB ? 10 : sg.kind == SRC_EMB6 ? 6 : 4, t, h, j);
  return f >= 0 ? sg.col0 + f : -1;
}

// folded-head region (k_pack_head): H (129 x 283 f32), P = Wv_f Wl_l (128 x 128 f32), q (128 f32),
// then fp64 scratch G = Wv_f Wl_f (128 x 256) and u = Wl_f bf + bl (256)
#define ANR_HEAD_H_FLOATS (129 * 283)
#define ANR_HEAD_P_OFF ANR_HEAD_H_FLOATS
#define ANR_HEAD_Q_OFF (ANR_HEAD_P_OFF + 128 * 128)
#define ANR_HEAD_FLOATS (ANR_HEAD_Q_OFF + 128)
__host__ __device__ constexpr int head_base() { return (x6_base() + x6_bytes() + 255) / 256 * 256; }
__host__ __device__ constexpr int head_scratch_base() { return (head_base() + ANR_HEAD_FLOATS * 4 + 255) / 256 * 256; }
#define ANR_HEAD_SCRATCH_DOUBLES (128 * 256 + 256)
__host__ __device__ constexpr int packed_bytes_all() { return head_scratch_base() + ANR_HEAD_SCRATCH_DOUBLES * 8; }
// per-frame fold buffer (floats): bw0 pose/T, bw5 pose/T, latent_fc (5 x 256), head bias (144)
#define ANR_FOLD_HEAD 1280
#define ANR_FOLD_FLOATS 1536

// LDS of the fused kernel: a ring of staging buffers of the largest slice, the 24 joint transforms
// and the bias table (mlp_bias_floats, every program entry's bias, filled once per launch so no
// global load sits between the staging loads). fp32 kernel: 2 x (8 k-steps x 5 chunks x 1 KiB).
// bf16 kernel: 4 x 32 KiB (a bf16x3 k-step of 16 out-blocks x 2 KiB; bf16x6 k-steps are staged as
// groups of <= 8 out-blocks x 3 KiB = 24 KiB), so three slices are in flight while one is consumed.
template <bool B16>
__host__ __device__ constexpr int mlp_slice_max() { return B16 ? 16 * 2048 : 8 * 5 * 1024; }
template <bool B16>
__host__ __device__ constexpr int mlp_nbuf() { return B16 ? 4 : 3; }
// LDS layout: [bias table][24 joint transforms, T-pose bounds][ring]. The table sits at LDS address 0 so every
// bias read is one base register + an immediate offset (< 64 KiB); the ring starts 256-B aligned.
// bias-table floats of the render program (the larger of the two programs, anr_mlp_body.h)
#define ANR_BIAS_TABLE_FLOATS 6880
__host__ __device__ constexpr int mlp_sa_off() { return ANR_BIAS_TABLE_FLOATS * 4; }
// after the joint transforms: the T-pose bounds (6 floats), read once per tile from LDS
__host__ __device__ constexpr int mlp_ring_off() { return (mlp_sa_off() + 24 * 16 * 4 + 32 + 255) / 256 * 256; }
template <bool B16>
__host__ __device__ constexpr int mlp_lds_bytes() { return mlp_ring_off() + mlp_nbuf<B16>() * mlp_slice_max<B16>(); }

}  // namespace anr
