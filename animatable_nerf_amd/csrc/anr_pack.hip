// anr_pack.hip — weight-image packing (per weight version) and per-frame preparation.
//
//   k_pack_weights  state_dict tensors -> the LDS-image order of anr_layers.h (one float per thread)
//   k_pack_bias     biases padded per layer (feature_fc || alpha_fc stacked like their weights)
//   k_prep          per render call: (X,Y,Z,25) volumes -> 32-channel float4-aligned copies, and the
//                   latent columns of bw_linears.0/.5 and latent_fc folded into per-frame biases
//                   (tpose_nerf_network.py:40-53 feature = [gamma(x), latent]; :264-267)
#include "anr_common.h"
#include "anr_kernels.h"
#include "anr_layers.h"

namespace anr {

__global__ void k_pack_weights(PackArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // float index into the weight image
  if (e >= weights_bytes() / 4) return;
  int L = 0;
  while (L + 1 < ANR_NUM_LAYERS_ALL && e >= layer_offset(L + 1) / 4) ++L;
  const LayerDesc d = layer_desc_all(L);
  const int C = layer_chunks(L);
  const int local = e - layer_offset(L) / 4;
  const int t = local / (C * 256);
  const int rem = local - t * C * 256;
  const int c = rem / 256;
  const int l = (rem & 255) >> 2;
  const int j = rem & 3;
  const int ob = c * 4 + j;
  const int col = layer_col(d, t, l >> 4);
  float v = 0.0f;
  const int main_ob = (d.nout + 15) / 16;
  const bool present = a.t[d.tensor_w] != nullptr;
  if (present && ob < d.ob && col >= 0) {
    if (ob < main_ob) {
      const int i = ob * 16 + (l & 15);
      if (i < d.nout) v = a.t[d.tensor_w][(size_t)i * d.in_ch + col];
    } else if (d.tensor_w2 >= 0) {
      const int i2 = (ob - main_ob) * 16 + (l & 15);
      if (i2 < d.nout2) v = a.t[d.tensor_w2][(size_t)i2 * d.in_ch + col];
    }
  }
  ((float*)a.out)[e] = v;
}

__global__ void k_pack_bias(PackArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= bias_floats()) return;
  int L = 0;
  while (L + 1 < ANR_NUM_LAYERS_ALL && e >= bias_offset(L + 1)) ++L;
  const LayerDesc d = layer_desc_all(L);
  const int n = e - bias_offset(L);
  const int main_n = ((d.nout + 15) / 16) * 16;
  float v = 0.0f;
  if (d.tensor_b < 0 || a.t[d.tensor_b] == nullptr) v = 0.0f;  // the folded head's bias is per frame (k_prep)
  else if (n < d.nout) v = a.t[d.tensor_b][n];
  else if (d.tensor_w2 >= 0 && n >= main_n && n - main_n < d.nout2) v = a.t[d.tensor_b2][n - main_n];
  ((float*)(a.out + weights_bytes()))[e] = v;
}

// bf16x3 image (anr_layers.h): one thread per (layer, k-step, out-block, lane) writes the 8 hi and
// the 8 lo bf16 of its fragment
__device__ __forceinline__ unsigned short bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

__global__ void k_pack_b16(PackArgs a) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= b16_bytes() / 32) return;
  const int byte = u * 32;
  int L = 0;
  while (L + 1 < ANR_B16_LAYERS && byte >= b16_layer_offset(L + 1)) ++L;
  const LayerDesc d = layer_desc_all(L);
  const int local = (byte - b16_layer_offset(L)) / 32;  // (s, ob, lane)
  const int lane = local & 63;
  const int so = local >> 6;
  // main part [k-step][16 out-blocks], then the tail blocks [k-step][tail] (anr_layers.h)
  const int mob = b16_main_ob(L), tob = b16_tail_ob(L), ks = ks32(L);
  const int ob = so < ks * mob ? so % mob : mob + (so - ks * mob) % tob;
  const int t = so < ks * mob ? so / mob : (so - ks * mob) / tob;
  const int row16 = lane & 15, h = lane >> 4;
  const int main_ob = (d.nout + 15) / 16;
  unsigned short hi[8], lo[8];
  for (int j = 0; j < 8; ++j) {
    const int col = b16_col(d, t, h, j);
    float v = 0.0f;
    if (col >= 0 && a.t[d.tensor_w] != nullptr) {
      if (ob < main_ob) {
        const int i = ob * 16 + row16;
        if (i < d.nout) v = a.t[d.tensor_w][(size_t)i * d.in_ch + col];
      } else if (d.tensor_w2 >= 0) {
        const int i2 = (ob - main_ob) * 16 + row16;
        if (i2 < d.nout2) v = a.t[d.tensor_w2][(size_t)i2 * d.in_ch + col];
      }
    }
    hi[j] = bf16_rne(v);
    lo[j] = bf16_rne(v - __uint_as_float((uint32_t)hi[j] << 16));
  }
  unsigned char* base = a.out + b16_base() + b16_layer_offset(L) + (size_t)so * 2048;
  uint4 vh, vl;
  vh.x = hi[0] | ((uint32_t)hi[1] << 16); vh.y = hi[2] | ((uint32_t)hi[3] << 16);
  vh.z = hi[4] | ((uint32_t)hi[5] << 16); vh.w = hi[6] | ((uint32_t)hi[7] << 16);
  vl.x = lo[0] | ((uint32_t)lo[1] << 16); vl.y = lo[2] | ((uint32_t)lo[3] << 16);
  vl.z = lo[4] | ((uint32_t)lo[5] << 16); vl.w = lo[6] | ((uint32_t)lo[7] << 16);
  *(uint4*)(base + lane * 16) = vh;
  *(uint4*)(base + 1024 + lane * 16) = vl;
}

// A layer sequence L0 .. L0 + nl - 1 of the layer table as its own bf16x3 image (the sdf render's
// residual MLP, layers 32..40, and SDF network, 41..49): k_pack_b16's fragments (main out-blocks,
// then tail blocks) from byte 0 of `a.out`, then the biases padded to ob x 16 per layer. Layer
// L0 + sl's weights are multiplied by `sc` (lin4's 1/sqrt2 of its skip concatenation). Layers with
// LayerDesc::trans are packed transposed (the SDF network's input-gradient pass).
__global__ void k_pack_seq(PackArgs a, int L0, int nl, int sl, float sc) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  const int nfrag = seq_wbytes(L0, nl) / 32;
  if (u >= nfrag) {
    const int e = u - nfrag;  // bias float
    if (e >= seq_bias_off(L0, nl)) return;
    int l = 0;
    while (l + 1 < nl && e >= seq_bias_off(L0, l + 1)) ++l;
    const LayerDesc d = layer_desc_all(L0 + l);
    const int i = e - seq_bias_off(L0, l);
    const float* b = a.t[d.tensor_b];
    ((float*)(a.out + seq_wbytes(L0, nl)))[e] = (b && i < d.nout) ? b[i] : 0.0f;
    return;
  }
  const int byte = u * 32;
  int L = L0;
  while (L + 1 < L0 + nl && byte >= seq_layer_offset(L0, L + 1)) ++L;
  const LayerDesc d = layer_desc_all(L);
  const int local = (byte - seq_layer_offset(L0, L)) / 32;  // (s, ob, lane)
  const int lane = local & 63;
  const int so = local >> 6;
  const int mob = b16_main_ob(L), tob = b16_tail_ob(L), ks = ks32(L);
  const int ob = so < ks * mob ? so % mob : mob + (so - ks * mob) % tob;
  const int t = so < ks * mob ? so / mob : (so - ks * mob) / tob;
  const int row = ob * 16 + (lane & 15), h = lane >> 4;
  const float f = L == L0 + sl ? sc : 1.0f;
  unsigned short hi[8], lo[8];
  for (int j = 0; j < 8; ++j) {
    const int col = b16_col(d, t, h, j);
    float v = 0.0f;
    if (col >= 0 && row < d.nout && a.t[d.tensor_w] != nullptr)
      v = a.t[d.tensor_w][d.trans ? (size_t)col * d.in_ch + row : (size_t)row * d.in_ch + col] * f;
    hi[j] = bf16_rne(v);
    lo[j] = bf16_rne(v - __uint_as_float((uint32_t)hi[j] << 16));
  }
  unsigned char* base = a.out + seq_layer_offset(L0, L) + (size_t)so * 2048;
  uint4 vh, vl;
  vh.x = hi[0] | ((uint32_t)hi[1] << 16); vh.y = hi[2] | ((uint32_t)hi[3] << 16);
  vh.z = hi[4] | ((uint32_t)hi[5] << 16); vh.w = hi[6] | ((uint32_t)hi[7] << 16);
  vl.x = lo[0] | ((uint32_t)lo[1] << 16); vl.y = lo[2] | ((uint32_t)lo[3] << 16);
  vl.z = lo[4] | ((uint32_t)lo[5] << 16); vl.w = lo[6] | ((uint32_t)lo[7] << 16);
  *(uint4*)(base + lane * 16) = vh;
  *(uint4*)(base + 1024 + lane * 16) = vl;
}
int seq_pack_threads(int L0, int nl) { return seq_wbytes(L0, nl) / 32 + seq_bias_off(L0, nl); }

// k_pack_seq's layer sequence as a bf16x6 image (anr_layers.h x6seq_*): per (k-step, out-block) the
// hi / mid / lo fragments (3 KiB, k_pack_x6's layout), then the biases as k_pack_seq lays them out.
__global__ void k_pack_seq_x6(PackArgs a, int L0, int nl, int sl, float sc) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  const int nfrag = x6seq_wbytes(L0, nl) / 48;
  if (u >= nfrag) {
    const int e = u - nfrag;  // bias float
    if (e >= seq_bias_off(L0, nl)) return;
    int l = 0;
    while (l + 1 < nl && e >= seq_bias_off(L0, l + 1)) ++l;
    const LayerDesc d = layer_desc_all(L0 + l);
    const int i = e - seq_bias_off(L0, l);
    const float* b = a.t[d.tensor_b];
    ((float*)(a.out + x6seq_wbytes(L0, nl)))[e] = (b && i < d.nout) ? b[i] : 0.0f;
    return;
  }
  const int byte = u * 48;
  int L = L0;
  while (L + 1 < L0 + nl && byte >= x6seq_layer_offset(L0, L + 1)) ++L;
  const LayerDesc d = layer_desc_all(L);
  const int local = (byte - x6seq_layer_offset(L0, L)) / 48;  // (s, ob, lane)
  const int lane = local & 63;
  const int so = local >> 6;
  const int ob = so % d.ob, t = so / d.ob;
  const int row = ob * 16 + (lane & 15), h = lane >> 4;
  const float f = L == L0 + sl ? sc : 1.0f;
  unsigned short q[3][8];
  for (int j = 0; j < 8; ++j) {
    const int col = b16_col(d, t, h, j);
    float v = 0.0f;
    if (col >= 0 && row < d.nout && a.t[d.tensor_w] != nullptr)
      v = a.t[d.tensor_w][d.trans ? (size_t)col * d.in_ch + row : (size_t)row * d.in_ch + col] * f;
    q[0][j] = bf16_rne(v);
    const float r1 = v - __uint_as_float((uint32_t)q[0][j] << 16);
    q[1][j] = bf16_rne(r1);
    q[2][j] = bf16_rne(r1 - __uint_as_float((uint32_t)q[1][j] << 16));
  }
  unsigned char* base = a.out + x6seq_layer_offset(L0, L) + (size_t)so * 3072;
  for (int k = 0; k < 3; ++k) {
    uint4 v;
    v.x = q[k][0] | ((uint32_t)q[k][1] << 16); v.y = q[k][2] | ((uint32_t)q[k][3] << 16);
    v.z = q[k][4] | ((uint32_t)q[k][5] << 16); v.w = q[k][6] | ((uint32_t)q[k][7] << 16);
    *(uint4*)(base + k * 1024 + lane * 16) = v;
  }
}
int seq_x6_pack_threads(int L0, int nl) { return x6seq_wbytes(L0, nl) / 48 + seq_bias_off(L0, nl); }

// bf16x6 image (anr_layers.h): one thread per (layer, k-step, out-block, lane) writes hi, mid, lo fragments
__global__ void k_pack_x6(PackArgs a) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= x6_bytes() / 48) return;
  const int byte = u * 48;
  int X = 0;
  while (X + 1 < ANR_X6_LAYERS && byte >= x6_layer_offset(X + 1)) ++X;
  const LayerDesc d = layer_desc_all(x6_layer(X));
  const int local = (byte - x6_layer_offset(X)) / 48;
  const int lane = local & 63;
  const int so = local >> 6;
  const int ob = so % d.ob, t = so / d.ob;
  const int row16 = lane & 15, h = lane >> 4;
  const int main_ob = (d.nout + 15) / 16;
  unsigned short q[3][8];
  for (int j = 0; j < 8; ++j) {
    const int col = b16_col(d, t, h, j);
    float v = 0.0f;
    if (col >= 0 && a.t[d.tensor_w] != nullptr) {
      if (ob < main_ob) {
        const int i = ob * 16 + row16;
        if (i < d.nout) v = a.t[d.tensor_w][(size_t)i * d.in_ch + col];
      } else if (d.tensor_w2 >= 0) {  // alpha_fc stacked beside feature_fc (layer 17)
        const int i2 = (ob - main_ob) * 16 + row16;
        if (i2 < d.nout2) v = a.t[d.tensor_w2][(size_t)i2 * d.in_ch + col];
      }
    }
    q[0][j] = bf16_rne(v);
    const float r1 = v - __uint_as_float((uint32_t)q[0][j] << 16);
    q[1][j] = bf16_rne(r1);
    q[2][j] = bf16_rne(r1 - __uint_as_float((uint32_t)q[1][j] << 16));
  }
  unsigned char* base = a.out + x6_base() + x6_layer_offset(X) + (size_t)so * 3072;
  for (int k = 0; k < 3; ++k) {
    uint4 v;
    v.x = q[k][0] | ((uint32_t)q[k][1] << 16); v.y = q[k][2] | ((uint32_t)q[k][3] << 16);
    v.z = q[k][4] | ((uint32_t)q[k][5] << 16); v.w = q[k][6] | ((uint32_t)q[k][7] << 16);
    *(uint4*)(base + k * 1024 + lane * 16) = v;
  }
}

// Folded colour head (anr_layers.h ANR_L_HEAD), composed in fp64 from the state_dict tensors
// (feature_fc 19/20, latent_fc 21/22, view_fc 23/24, alpha_fc 17):
//   a: G = Wv[:, :256] Wl[:, :256] (128 x 256), u = Wl[:, :256] bf + bl (256)      (fp64 scratch)
//   b: H[i < 128] = [G Wf | Wv[:, 256:283]], H[128] = [alpha_fc | 0];
//      P = Wv[:, :256] Wl[:, 256:384] (128 x 128); q = Wv[:, :256] u + bv          (f32)
__global__ void k_pack_head_a(PackArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  double* G = (double*)(a.out + head_scratch_base());
  double* u = G + 128 * 256;
  const float *Wf = a.t[19], *bf = a.t[20], *Wl = a.t[21], *bl = a.t[22], *Wv = a.t[23];
  if (e < 128 * 256) {
    const int i = e >> 8, k = e & 255;
    double acc = 0.0;
    for (int m = 0; m < 256; ++m) acc += (double)Wv[i * 283 + m] * (double)Wl[m * 384 + k];
    G[e] = acc;
  } else if (e < 128 * 256 + 256) {
    const int m = e - 128 * 256;
    double acc = bl[m];
    for (int k = 0; k < 256; ++k) acc += (double)Wl[m * 384 + k] * (double)bf[k];
    u[m] = acc;
  }
  (void)Wf;
}

__global__ void k_pack_head_b(PackArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const double* G = (const double*)(a.out + head_scratch_base());
  const double* u = G + 128 * 256;
  float* H = (float*)(a.out + head_base());
  const float *Wf = a.t[19], *Wl = a.t[21], *Wv = a.t[23], *bv = a.t[24], *Wa = a.t[17];
  if (e < ANR_HEAD_H_FLOATS) {
    const int i = e / 283, c = e - i * 283;
    float v;
    if (i == 128) {
      v = c < 256 ? Wa[c] : 0.0f;
    } else if (c >= 256) {
      v = Wv[i * 283 + c];
    } else {
      double acc = 0.0;
      for (int k = 0; k < 256; ++k) acc += G[i * 256 + k] * (double)Wf[k * 256 + c];
      v = (float)acc;
    }
    H[e] = v;
  } else if (e < ANR_HEAD_Q_OFF) {
    const int pe = e - ANR_HEAD_P_OFF, i = pe >> 7, j = pe & 127;
    double acc = 0.0;
    for (int m = 0; m < 256; ++m) acc += (double)Wv[i * 283 + m] * (double)Wl[m * 384 + 256 + j];
    H[e] = (float)acc;
  } else if (e < ANR_HEAD_FLOATS) {
    const int i = e - ANR_HEAD_Q_OFF;
    double acc = bv[i];
    for (int m = 0; m < 256; ++m) acc += (double)Wv[i * 283 + m] * u[m];
    H[e] = (float)acc;
  }
}

// grid (prep_blocks): blocks [0, nvox_blocks) repack volumes; then one wave per folded-bias output
// (5 x 256 of them, a 128-term dot each: lane q sums terms q and q + 64, then a wave reduction), then
// one wave per folded-head entry (fp64 dot over the 128 latent dims)
__global__ __launch_bounds__(256) void k_prep(PrepArgs a) {
  if (blockIdx.x == 0 && a.counts) {  // the front-end's per-call state (k_frontend runs after this launch)
    if (threadIdx.x < 4) a.counts[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < a.nch; i += 256) {
      a.chunk_min[i] = ~0ull;
      a.chunk_max[i] = 0ull;
    }
  }
  const int nvb = (a.np + a.nt + 7) / 8;  // 8 voxels (x 32 channels) per block
  if ((int)blockIdx.x < nvb) {
    const int v = blockIdx.x * 8 + (threadIdx.x >> 5);
    const int c = threadIdx.x & 31;
    if (v < a.np) {
      const float val = c < 25 ? a.pbw[(size_t)v * 25 + c] : 0.0f;
      a.pbw32[(size_t)v * 32 + c] = val;
      if (c == 24 && a.pn24) a.pn24[v] = val;
    } else if (v < a.np + a.nt) {
      const int u = v - a.np;
      a.tbw32[(size_t)u * 32 + c] = c < 25 ? a.tbw[(size_t)u * 25 + c] : 0.0f;
    }
    return;
  }
  const int lane = threadIdx.x & 63;
  const int k = (blockIdx.x - nvb) * 4 + (threadIdx.x >> 6);  // output index (wave-uniform)
  const int li = (int)a.latent_index[0];
  if (k < 5 * 256) {
    // folded biases: which = 0,1 (bw0 pose/tpose), 2,3 (bw5 pose/tpose), 4 (latent_fc)
    const int which = k >> 8, nn = k & 255;
    const float *W, *lat;
    float bias;
    int ld, c0;
    if (which < 4) {
      const bool novel = a.novel && !(which & 1);  // pose pass of a novel-pose render
      const int row = (which & 1) ? 0 : (novel ? (int)a.bw_latent_index[0] : li + 1);
      lat = (novel ? a.n_latent : a.bw_latent) + (size_t)row * 128;
      W = which < 2 ? (novel ? a.nw_bw0 : a.w_bw0) : (novel ? a.nw_bw5 : a.w_bw5);
      ld = which < 2 ? 191 : 447;
      c0 = 63;
      bias = which < 2 ? (novel ? a.nb_bw0 : a.b_bw0)[nn] : (novel ? a.nb_bw5 : a.b_bw5)[nn];
    } else {
      lat = a.nf_latent + (size_t)li * 128;
      W = a.w_lat;
      ld = 384;
      c0 = 256;
      bias = a.b_lat[nn];
    }
    const float* row = W + (size_t)nn * ld + c0;
    float acc = fmaf(row[lane], lat[lane], row[lane + 64] * lat[lane + 64]);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) a.fold[k] = acc + bias;
    return;
  }
  const int i = k - 5 * 256;  // folded-head entry
  if (!a.head_P || i >= ANR_FOLD_FLOATS - ANR_FOLD_HEAD) return;
  float v = 0.0f;
  if (i < 128) {
    const float* lat = a.nf_latent + (size_t)li * 128;
    double acc = (double)a.head_P[i * 128 + lane] * (double)lat[lane] +
                 (double)a.head_P[i * 128 + lane + 64] * (double)lat[lane + 64];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    v = (float)(acc + (double)a.head_q[i]);
  } else if (i == 128) {
    v = a.b_alpha[0];
  }
  if (lane == 0) a.fold[ANR_FOLD_HEAD + i] = v;
}

int prep_blocks(long np, long nt) { return (int)((np + nt + 7) / 8) + (5 * 256 + ANR_FOLD_FLOATS - ANR_FOLD_HEAD + 3) / 4; }

}  // namespace anr
