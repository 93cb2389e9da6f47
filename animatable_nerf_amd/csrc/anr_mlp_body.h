// anr_mlp_body.h — the fused per-kept-sample network kernel (A5, A7-A11), shared by the exact fp32
// (anr_mlp.hip) and the bf16x3 (anr_mlp_b16.hip) instantiations, one per TU so they build in parallel.
//
// One launch processes every kept sample of the render call (persistent grid, 1 workgroup per CU,
// 8 waves x 16 samples = 128 samples per tile). Per sample, entirely on chip:
//   pose-space blend-weight lookup (pbw, 24 ch)            blend_utils.py:119-149
//   gamma(x) -> BW MLP (latent folded into bias) -> softmax tpose_nerf_network.py:40-77
//   LBS inverse warp to the T-pose                          blend_utils.py:41-59
//   T-pose blend-weight lookup + BW MLP (tbw, for the loss) tpose_nerf_network.py:169-174
//   gamma(x_T) -> NeRF 8x256 MLP, alpha/feature/latent/view/rgb heads   :252-275
//   T-pose bbox mask, sigmoid, 1-exp(-relu(sigma) dist)     :186-212
// Activations never leave registers: the MFMA accumulator of one layer is the B operand of the
// next (anr_layers.h). Weights stream through an LDS ring of slices (LDS-DMA, Pipe), one slice
// stream across layers and tiles; biases sit in an LDS table filled once per launch.
#pragma once
#include <type_traits>

#include "anr_common.h"
#include "anr_kernels.h"
#include "anr_layers.h"

namespace anr {


template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

typedef __attribute__((address_space(3))) void lds_void;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// LDS fragment reads in flight ahead of the MFMAs (bf16x3 layers)
#ifndef ANR_FRAG_PF
#define ANR_FRAG_PF 3
#endif
// bf16x3 layers: issue a refill's LDS-DMA pieces one by one between the out-blocks of the slice's
// second half (after its mid() barrier) instead of as one burst right after the barrier, where every
// wave of the workgroup queues its pieces at the texture unit at the same time
#ifndef ANR_DMA_SPREAD
#define ANR_DMA_SPREAD 1
#endif
// bf16x3 kernels: hardware log/exp/rcp in the blend softmax and reciprocal-based lookup coordinates
// bf16x6 layers: read the next out-block's fragments ahead of the current out-block's MFMAs
#ifndef ANR_X6_PF
#define ANR_X6_PF 2
#endif
#ifndef ANR_FAST_MATH
#define ANR_FAST_MATH 1
#endif

// The per-tile layer program, variant V:
//   V = 0 (render): entries 0..8 the pose-space BW MLP, 9..17 the T-pose BW MLP (layers 0..8
//         again), 18..29 the NeRF (layers 9..20);
//   V = 1 (density, get_alpha of the mesh path, tpose_nerf_network.py:105-135): entries 0..8 the
//         pose-space BW MLP, 9..16 the NeRF trunk (layers 9..16), 17 alpha_fc alone (layer 30).
// Arithmetic per entry (anr_layers.h):
//   mode 0 exact fp32 MFMA (k_mlp, every entry);
//   mode 1 bf16x3 (k_mlp_b16; the pose pass too unless built with ANR_POSE_MODE=2);
//   mode 2 bf16x6, fp32-level (the pose pass with ANR_POSE_MODE=2: measured unnecessary, the
//          outputs' error vs the fp32 oracle stays <= 4e-6 with x3, tools/precision_report.py).
//   V = 2 (render, both kernels): entries 0..25 as V = 0, 26 the folded colour head (layer 31:
//         view_fc's pre-activation || alpha_fc, anr_layers.h ANR_L_HEAD), 27 rgb_fc. V = 0 (the
//         reference's unfolded head) sizes the bias table and is no longer run.
//   V = 4 (render, k_mlp_x6, render precision ANR_BF16X6): the V = 2 program with every entry in
//         mode 2 (bf16x6, fp32-level products) and the accurate libm paths of the exact kernel.
//   V = 5 (the sdf_pdf SDF network forward, k_sdfnet_b16): entries 0..8 = layers 41..49
//         (anr_layers.h sdfnet_desc), bf16x3, the image after the residual MLP's.
//   V = 8 (density, k_alpha_x6, render precision ANR_BF16X6): the V = 1 program in mode 2.
//   V = 6 (the sdf_pdf colour network, k_color_b16): entries 0..4 = layers 58..62 (anr_layers.h
//         color_desc), bf16x3, an image of its own; lin0 reads its inputs from memory rows.
//   V = 7 (the sdf_pdf SDF network's input gradient, k_sdfgrad_b16): entries 0..7 = layers 50..57
//         (anr_layers.h sdfrev_desc: lin7 .. lin0 transposed), bf16x3, an image of its own.
//   V = 3 (the sdf_pdf residual deformation MLP, k_resd_b16): entries 0..8 = layers 32..40
//         (anr_layers.h resd_desc), bf16x3, from the sdf render's own image (k_pack_resd).
//   V = 13, 15, 16, 17 (render precision ANR_BF16X6 of the sdf_pdf render): the programs 3, 5, 6, 7
//         with every entry in mode 2 (bf16x6, fp32-level products), from bf16x6 sequence images
//         (k_pack_seq_x6), the softplus and its backward factor at libm accuracy.
template <int V>
__host__ __device__ constexpr int prog_base() { return V >= 10 ? V - 10 : V; }
template <int V>
__host__ __device__ constexpr int prog_len() {
  constexpr int B = prog_base<V>();
  return B == 0 ? 30 : (B == 2 || B == 4) ? 28 : (B == 3 || B == 5) ? 9 : B == 7 ? 8 : B == 6 ? 5 : 18;  // 1, 8: 18
}
// programs whose weights are a packed layer sequence of their own (k_pack_seq), not the render image
template <int V>
__host__ __device__ constexpr bool prog_seq() {
  return prog_base<V>() == 3 || prog_base<V>() == 5 || prog_base<V>() == 6 || prog_base<V>() == 7;
}
template <int V>
__host__ __device__ constexpr int prog_layer(int e) {
  if (V >= 10) return prog_layer<prog_base<V>()>(e);
  return V == 3 ? ANR_L_RESD0 + e
         : V == 5 ? ANR_L_SDF0 + e
         : V == 7 ? ANR_L_SREV0 + e
         : V == 6 ? ANR_L_COL0 + e
         : e < 9 ? e
         : V == 0 ? e - 9
         : (V == 2 || V == 4) ? (e < 26 ? e - 9 : (e == 26 ? ANR_L_HEAD : ANR_L_RGB))
         : V == 8 ? (e < 17 ? e : ANR_L_ALPHA)
                  : (e < 17 ? e : ANR_L_ALPHA);
}
__host__ __device__ constexpr bool prog_pose(int e) { return e < 9; }
template <bool B16, int V>
__host__ __device__ constexpr int prog_mode(int e) {
  return B16 ? ((V == 4 || V == 8 || V >= 10) ? 2 : e < 9 ? ANR_POSE_MODE : 1) : 0;
}
// Slices = the staging unit: mode 0 8 fp32 k-steps; mode 1 one 32-input k-step (OB x 2 KiB);
// mode 2 one 32-input k-step of a group of <= 8 out-blocks (x 3 KiB).
template <int V>
__host__ __device__ constexpr int prog_nobg(int e) { return (layer_desc_all(prog_layer<V>(e)).ob + 7) / 8; }
template <bool B16, int V>
__host__ __device__ constexpr int prog_slices(int e) {
  return prog_mode<B16, V>(e) == 2   ? ks32(prog_layer<V>(e)) * prog_nobg<V>(e)
         : prog_mode<B16, V>(e) == 1 ? ks32(prog_layer<V>(e)) + (b16_tail_ob(prog_layer<V>(e)) > 0 ? 1 : 0)
                                  : layer_ksteps(prog_layer<V>(e)) / ANR_KSLICE;
}
template <int V>
__host__ __device__ constexpr int x6_group_obs(int e, int gidx) {
  return layer_desc_all(prog_layer<V>(e)).ob - 8 * gidx < 8 ? layer_desc_all(prog_layer<V>(e)).ob - 8 * gidx : 8;
}
// bf16x6 layers: fragment G = t * OB + o (k-step t, out-block o) of entry E lives in slice
// x6_slice_of(G) = t * NOBG + o / 8. At iteration F (before its MFMAs) the slices up to
// x6_certified_at(F) may be read: the current one, and the next once the current slice's mid() (after
// the MFMAs of its middle out-block) has certified it. Fragment G is read ANR_X6_PF iterations ahead
// where that is certified, else at the first iteration where it is (never later than G itself).
template <int V>
__host__ __device__ constexpr int x6_slice_of(int e, int G) {
  return (G / layer_desc_all(prog_layer<V>(e)).ob) * prog_nobg<V>(e) + (G % layer_desc_all(prog_layer<V>(e)).ob) / 8;
}
template <int V>
__host__ __device__ constexpr int x6_certified_at(int e, int F) {
  const int o = F % layer_desc_all(prog_layer<V>(e)).ob;
  const int gob = x6_group_obs<V>(e, o / 8);
  return x6_slice_of<V>(e, F) + (o % 8 > (gob - 1) / 2 ? 1 : 0);
}
template <int V>
__host__ __device__ constexpr int x6_issue_at(int e, int G) {
  int F = G - ANR_X6_PF > 0 ? G - ANR_X6_PF : 0;
  while (x6_certified_at<V>(e, F) < x6_slice_of<V>(e, G)) ++F;
  return F;
}
// every fragment read of an x6 layer targets a certified slice, at most one slice ahead, issued
// no later than its use and after the previous occupant of its register set was consumed
template <int V>
__host__ __device__ constexpr bool x6_schedule_ok(int e) {
  const int n = ks32(prog_layer<V>(e)) * layer_desc_all(prog_layer<V>(e)).ob;
  for (int G = 0; G < n; ++G) {
    const int F = x6_issue_at<V>(e, G);
    if (F > G || F < G - ANR_X6_PF) return false;
    if (x6_slice_of<V>(e, G) > x6_certified_at<V>(e, F)) return false;
    if (x6_slice_of<V>(e, G) > x6_slice_of<V>(e, F) + 1 || x6_slice_of<V>(e, G) < x6_slice_of<V>(e, F)) return false;
  }
  return true;
}
template <bool B16, int V>
__host__ __device__ constexpr int prog_slice_kb(int e, int q) {
  return prog_mode<B16, V>(e) == 2 ? x6_group_obs<V>(e, q % prog_nobg<V>(e)) * 3
         : prog_mode<B16, V>(e) == 1
             ? (q < ks32(prog_layer<V>(e)) ? b16_main_ob(prog_layer<V>(e)) * 2
                                          : b16_tail_ob(prog_layer<V>(e)) * ks32(prog_layer<V>(e)) * 2)
             : layer_chunks(prog_layer<V>(e)) * ANR_KSLICE;
}
template <bool B16, int V>
__host__ __device__ constexpr int prog_slice_off(int e, int q) {
  return prog_mode<B16, V>(e) == 2
             ? (prog_seq<V>() ? x6seq_layer_offset(prog_layer<V>(0), prog_layer<V>(e))
                              : x6_base() + x6_layer_offset(prog_layer<V>(e))) +
                   ((q / prog_nobg<V>(e)) * layer_desc_all(prog_layer<V>(e)).ob + 8 * (q % prog_nobg<V>(e))) * 3072
         : prog_mode<B16, V>(e) == 1
             ? (prog_seq<V>() ? seq_layer_offset(prog_layer<V>(0), prog_layer<V>(e))
                              : b16_base() + b16_layer_offset(prog_layer<V>(e))) +
                   q * b16_main_ob(prog_layer<V>(e)) * 2048
             : layer_offset(prog_layer<V>(e)) + q * layer_chunks(prog_layer<V>(e)) * ANR_KSLICE * 1024;
}
// loads per wave for a slice (every wave issues the same count, see Pipe::stage)
template <bool B16, int V>
__host__ __device__ constexpr int prog_slice_loads(int e, int q) { return (prog_slice_kb<B16, V>(e, q) + 7) / 8; }
// the slice d steps after (e, q) in the cyclic program, packed as e * 1024 + q
template <bool B16, int V>
__host__ __device__ constexpr int prog_advance(int e, int q, int d) {
  for (int i = 0; i < d; ++i) {
    if (q + 1 < prog_slices<B16, V>(e)) {
      ++q;
    } else {
      q = 0;
      e = (e + 1) % prog_len<V>();
    }
  }
  return e * 1024 + q;
}
// loads this wave issued after slice (e, q) that may still be in flight when (e, q) is consumed
template <bool B16, int V>
__host__ __device__ constexpr int prog_later_loads(int e, int q) {
  int n = 0;
  for (int d = 1; d <= mlp_nbuf<B16>() - 3; ++d) {
    const int eq = prog_advance<B16, V>(e, q, d);
    n += prog_slice_loads<B16, V>(eq / 1024, eq % 1024);
  }
  return n;
}

// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt out of range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

struct Pipe {
  unsigned char* lds;
  int smax;  // bytes per staging buffer
  int nbuf;  // ring size
  const unsigned char* wimg;
  int cur;   // ring slot of the slice consumed next
  int wave;
  int lane;
  int pose_woff;  // added to slices of the pose-space BW pass (novel_pose_bw weights)
  int pend;       // ring slot of the refill whose pieces are being spread (ANR_DMA_SPREAD)

  // issue the HBM/L2 -> LDS copy of `kb` KiB at byte `off` of the packed image into ring slot `buf`;
  // every wave issues exactly `loads` 1-KiB pieces (pieces past the end repeat the last one: same
  // bytes to the same place), so the per-wave vmcnt bookkeeping is a compile-time constant.
  // The DMA is issued by inline asm, not __builtin_amdgcn_global_load_lds: with the builtin the
  // compiler cannot tell which LDS bytes a pending DMA writes and puts `s_waitcnt vmcnt(0)` before
  // the first ds_read after it, which drains the whole ring (every slice still in flight) once per
  // slice. Hidden from the compiler, the only waits on the stream are ours (wait_vmcnt in next());
  // the compiler's own vmcnt waits stay correct, only stricter (loads return in order).
  __device__ __forceinline__ void stage(int off, int kb, int loads, int buf, int first = 0) {
    const unsigned dst = (unsigned)(uintptr_t)(lds + buf * smax);
    // launder the base so the per-slice addresses are formed here, not hoisted out of the tile
    // loop (hundreds of loop-invariant 64-bit addresses otherwise spill)
    const unsigned char* w = wimg;
    asm volatile("" : "+s"(w));
    for (int i = first; i < loads; ++i) {
      int piece = wave + 8 * i;
      piece = piece < kb ? piece : kb - 1;
      const unsigned m0 = dst + piece * 1024;
      // wave-uniform piece: the whole source offset in the scalar base, the lane's 16 B in a
      // constant VGPR (no per-piece vector address arithmetic)
      const unsigned char* sbase = w + off + piece * 1024;
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(lane * 16), "s"(sbase), "s"(m0)
                   : "memory");
    }
  }

  // wait until this wave's pieces of all but the last N (8-wave count) issued pieces have landed
  template <int N>
  __device__ __forceinline__ void wait_stream() {
    wait_vmcnt<N>();
  }

  template <bool B16, int V, int E, int Q>
  __device__ __forceinline__ void stage_slice(int buf) {
    constexpr int off = prog_slice_off<B16, V>(E, Q);
    stage(off + (prog_pose(E) ? pose_woff : 0), prog_slice_kb<B16, V>(E, Q), prog_slice_loads<B16, V>(E, Q), buf);
  }

  // prologue: slices 0 .. nbuf-2 of the program; slice 0 is certified here
  template <bool B16, int V>
  __device__ __forceinline__ void start() {
    static_for<0, mlp_nbuf<B16>() - 1>([&](auto d) {
      constexpr int eq = prog_advance<B16, V>(0, 0, decltype(d)::value);
      stage_slice<B16, V, eq / 1024, eq % 1024>(decltype(d)::value);
    });
    cur = 0;
    wait_stream<prog_later_loads<B16, V>(0, 0)>();
    __syncthreads();
  }

  // Enter slice Q of program entry E: it was certified by mid() of the previous slice, so no wait
  // and no barrier here and the first MFMAs of a slice follow the last ones of the previous slice
  // without a pipe bubble.
  template <bool B16, int V, int E, int Q>
  __device__ __forceinline__ const unsigned char* enter() {
    return lds + cur * smax;
  }
  // Called halfway through slice (E, Q), while its MFMAs are in flight: certify the next slice (own
  // loads landed + barrier: everyone's landed, and everyone is past the previous slice), then refill
  // the previous slice's slot with the slice nbuf-1 ahead.
  // SPREAD: only certify and pick the slot here; the refill's pieces follow through piece<>().
  template <bool B16, int V, int E, int Q, bool SPREAD = false>
  __device__ __forceinline__ void mid() {
    constexpr int NB = mlp_nbuf<B16>();
    constexpr int e1 = prog_advance<B16, V>(E, Q, 1);
    constexpr int eq = prog_advance<B16, V>(E, Q, NB - 1);
    wait_stream<prog_later_loads<B16, V>(e1 / 1024, e1 % 1024)>();
    __syncthreads();
    int slot = cur + NB - 1;
    slot = slot >= NB ? slot - NB : slot;
    if constexpr (SPREAD) pend = slot;
    else stage_slice<B16, V, eq / 1024, eq % 1024>(slot);
  }
  // pieces [I0, I1) of this wave's share of the refill picked by mid<..., true>() of slice (E, Q)
  template <bool B16, int V, int E, int Q, int I0, int I1>
  __device__ __forceinline__ void piece() {
    constexpr int NB = mlp_nbuf<B16>();
    constexpr int eq = prog_advance<B16, V>(E, Q, NB - 1);
    constexpr int EE = eq / 1024, QQ = eq % 1024;
    constexpr int off = prog_slice_off<B16, V>(EE, QQ);
    constexpr int loads = prog_slice_loads<B16, V>(EE, QQ);
    constexpr int i1 = I1 < loads ? I1 : loads;
    if constexpr (I0 < i1) stage(off + (prog_pose(EE) ? pose_woff : 0), prog_slice_kb<B16, V>(EE, QQ), i1, pend, I0);
  }
  __device__ __forceinline__ void leave() { cur = cur + 1 >= nbuf ? 0 : cur + 1; }
};

// x -> hi = bf16(x), lo = bf16(x - hi)   (RNE both)
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)x[j];
    hi[j] = h;
    lo[j] = (__bf16)(x[j] - (float)h);
  }
}

// x -> hi + mid + lo, each bf16 (RNE), x == hi + mid + lo to 24 bits
__device__ __forceinline__ void split8x3(const float (&x)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)x[j];
    const float r1 = x[j] - (float)h;
    const __bf16 m = (__bf16)r1;
    hi[j] = h;
    mid[j] = m;
    lo[j] = (__bf16)(r1 - (float)m);
  }
}

// LDS bias table: program entry e's biases (ob x 16 floats) at float offset prog_bias_off<V>(e)
template <int V>
__host__ __device__ constexpr int prog_bias_off(int e) {
  int o = 0;
  for (int k = 0; k < e; ++k) o += layer_desc_all(prog_layer<V>(k)).ob * 16;
  return o;
}
static_assert(prog_bias_off<0>(prog_len<0>()) == ANR_BIAS_TABLE_FLOATS, "bias table size (anr_layers.h)");
static_assert(prog_bias_off<1>(prog_len<1>()) <= ANR_BIAS_TABLE_FLOATS, "bias table size (anr_layers.h)");
static_assert(prog_bias_off<2>(prog_len<2>()) <= ANR_BIAS_TABLE_FLOATS, "bias table size (anr_layers.h)");
static_assert(prog_bias_off<4>(prog_len<4>()) <= ANR_BIAS_TABLE_FLOATS, "bias table size (anr_layers.h)");
static_assert(prog_bias_off<8>(prog_len<8>()) <= ANR_BIAS_TABLE_FLOATS, "bias table size (anr_layers.h)");
static_assert(prog_bias_off<3>(prog_len<3>()) == seq_bias_off(ANR_L_RESD0, ANR_RESD_LAYERS), "resd bias section");
static_assert(prog_bias_off<5>(prog_len<5>()) == seq_bias_off(ANR_L_SDF0, ANR_SDF_LAYERS), "sdf bias section");
static_assert(prog_bias_off<5>(prog_len<5>()) <= ANR_BIAS_TABLE_FLOATS, "bias table size (anr_layers.h)");
static_assert(prog_bias_off<7>(prog_len<7>()) == seq_bias_off(ANR_L_SREV0, ANR_SREV_LAYERS), "sdf grad bias section");
static_assert(prog_bias_off<6>(prog_len<6>()) == seq_bias_off(ANR_L_COL0, ANR_COL_LAYERS), "colour bias section");
static_assert(prog_bias_off<7>(prog_len<7>()) + 256 <= ANR_BIAS_TABLE_FLOATS, "bias table + W8 row (anr_layers.h)");

// Fill the bias table once per launch (before the first barrier of the slice stream). Sources:
// the packed bias section, the novel_pose_bw copy for the pose pass (pose_boff), and the per-frame
// folds (bw0/bw5 pose and T-pose, latent_fc) for the entries whose latent columns were folded.
template <int V>
__device__ __forceinline__ void fill_bias_table(const MlpArgs& a, float* __restrict__ sb, int tid) {
  static_for<0, prog_len<V>()>([&](auto ee) {
    constexpr int e = decltype(ee)::value;
    constexpr int L = prog_layer<V>(e);
    constexpr int n = layer_desc_all(L).ob * 16;
    constexpr int boff = bias_offset(L);  // constexpr: evaluated by the compiler, not per launch
    constexpr int toff = prog_bias_off<V>(e);
    const float* src;
    constexpr int VB = prog_base<V>();
    if constexpr (VB == 3) {  // sdf residual MLP: poses folded into layers 0 / 5 (k_sdf_fold)
      src = e == 0 ? a.fold : e == 5 ? a.fold + 256 : a.bias + toff;
    } else if constexpr (VB == 5 || VB == 7) {  // sdf network (forward / gradient): the image's bias section
      src = a.bias + toff;
    } else if constexpr (VB == 6) {  // colour network: color_latent folded into lin3 (k_sdf_fold)
      src = e == 3 ? a.fold + 512 : a.bias + toff;
    } else if constexpr (e < 9) {
      src = L == 0 ? a.fold + 0 : L == 5 ? a.fold + 512 : a.bias + a.pose_boff + boff;
    } else if constexpr (V != 1 && V != 8 && e < 18) {
      src = L == 0 ? a.fold + 256 : L == 5 ? a.fold + 768 : a.bias + boff;
    } else {
      src = L == 18 ? a.fold + 1024 : L == ANR_L_HEAD ? a.fold + ANR_FOLD_HEAD : a.bias + boff;
    }
    for (int i = tid; i < n; i += 512) sb[toff + i] = src[i];
  });
}

// One MLP layer (program entry E): out = W * src + bias (acc layout), k-steps from its segments.
// bf16x3 layers as one continuous MFMA stream (ANR_X3_STREAM): the B fragment of k-step t+1 is split
// while k-step t's MFMAs run, A fragments are read ANR_FRAG_PF out-blocks ahead across k-step (slice)
// boundaries, and the ReLU of the previous layer is applied in this layer's split (RELU_IN) instead
// of as a pass over the previous layer's outputs.
#ifndef ANR_X3_STREAM
#define ANR_X3_STREAM 1
#endif
template <int L>
__host__ __device__ constexpr bool x3_stream_layer() {
  return ANR_X3_STREAM && b16_tail_ob(L) == 0;
}

// iteration (k-step * MOB + out-block) at which fragment G is read; < 0: the layer's prologue
template <int MOB, int PF>
__host__ __device__ constexpr int x3_issue_at(int G) {
  const int t = G / MOB;
  const int a = G - PF;
  if (t == 0) return a;
  const int m = (t - 1) * MOB + (MOB - 1) / 2;
  return a > m ? a : m;
}

// Per-call memory operands of a streamed layer (the sdf programs): spst (SP_IN stores), fst / fscale
// (FAC_IN factors), g0 / g1 (the rows that SRC_G0 / SRC_G1 segments read, k-step t lane half h taking
// columns 32 t + 8 h .. + 7 of the segment).
struct LayerIO {
  float* spst = nullptr;
  const float* fst = nullptr;
  float fscale = 1.0f;
  const float* g0 = nullptr;
  const float* g1 = nullptr;
};

// the sdf programs' stored softplus outputs h (8 KiB per sample, written once, read once) bypass
// the weight stream's L2 lines: non-temporal stores (k_sdfnet_b16) and loads (k_sdfgrad_b16)
#ifndef ANR_SDF_NT
#define ANR_SDF_NT 1
#endif

// softplus(beta = 100, threshold = 20) as log2(1 + 2^(100 x log2 e)) ln2 / 100 on the hardware exp2 /
// log2 (~1 ulp each): 2 transcendentals + 5 VALU instead of the ~25 of k_lgemm's libm-grade epilogue
// (fast_exp / fast_log1p). Its h feeds a hi/lo bf16 split (~2^-16 relative) and the reverse pass's
// factor 1 - exp(-100 h); where 1 + e rounds (e < ~1e-3), h and that factor are < 1e-5 and their
// absolute error < 1e-9. The SDF outputs stay within tests/test_gpu_sdf.py's 1e-4 / 2e-4.
__device__ __forceinline__ float softplus100(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 144.269504f);
  const float h = __builtin_amdgcn_logf(1.0f + e) * 0.00693147181f;
  return x * 100.f > 20.f ? x : h;
}

// the fp32-level programs (V >= 10): torch's softplus(beta = 100, threshold = 20) = log1p(exp(100 x)) /
// 100 and its backward factor sigmoid(100 x) = e / (1 + e) (torch's softplus_backward: z / (z + 1),
// z = exp(100 x)) from ONE exp and ONE log, both within ~2 ulp of fp64 over the whole range (numpy
// emulation with correctly rounded exp2 / log2: <= 4.3 units of 2^-24 relative; torch's own fp32
// evaluation is off by up to 65 there, its RN(100 x) amplified by the exp):
//   e = 2^(x C) with C = 100 log2(e) as C_hi + C_lo and the residual of x C_hi exact by FMA, so the
//       hardware exp2 sees the argument to ~2^-48 and e = 2^a (1 + a_lo ln2);
//   log1p(e) = log(u) + (e - (u - 1)) / u with u = RN(1 + e): e - (u - 1) is the exact rounding error
//       of 1 + e (Sterbenz), so where 1 + e rounds the correction restores log1p's relative precision.
// Above torch's threshold (100 x > 20) softplus returns x and passes the gradient: here the argument
// is clamped to 0.4 (no overflow: e <= e^40) and h = max(h, x), which is x wherever log1p(exp(-100 x))
// / 100 < x's half ulp (from 100 x ~ 17 on, within ~1 ulp of torch's x between 20 and 40), and the
// factor e / (1 + e) is 1 within an ulp there. No compare masks: 15 VALU + 3 transcendentals for the
// pair, against ~27 + 3 for the libm-grade fast_exp / fast_log1p softplus alone and ~15 + 1 more for
// the factor recomputed from h (1 - exp(-100 h), with a series) in the reverse pass: the bf16x6 SDF
// forward stores the factor itself, its input gradient multiplies.
__device__ __forceinline__ float softplus100_fac(float x, float& fac) {
  constexpr float C_HI = 144.26950073242188f, C_LO = 3.356474508109386e-06f;
  constexpr float LN2 = 0.6931471824645996f;
  const float xc = fminf(x, 0.4f);
  const float a = xc * C_HI;
  const float a_lo = __builtin_fmaf(xc, C_LO, __builtin_fmaf(xc, C_HI, -a));
  const float E = __builtin_amdgcn_exp2f(a);
  const float e = __builtin_fmaf(E, a_lo * LN2, E);
  const float u = 1.f + e;
  const float err = e - (u - 1.f);
  const float ru = __builtin_amdgcn_rcpf(u);
  fac = e * ru;
  return fmaxf(__builtin_fmaf(__builtin_amdgcn_logf(u), LN2, err * ru) * 0.01f, x);
}
template <int V>
__device__ __forceinline__ float sp_fwd(float x) {
  static_assert(V < 10, "the fp32-level programs use softplus100_fac");
  return softplus100(x);
}

// SP_IN (the sdf network, V = 5): the previous layer's softplus(beta = 100) is applied in this layer's
// split like RELU_IN (its VALU work beside this layer's MFMAs), and the softplus outputs h of the
// k-step's 8 input neurons are stored to spst (the row's base; nothing when NULL): SP_IN 1 as h,
// SP_IN 2 as h / sqrt2 for input neurons < 217 (lin3's outputs into X4).
// FAC_IN (the SDF network's input gradient, V = 7): the input gradient dh of this layer's k-step is
// multiplied by the softplus-backward factor 1 - exp(-100 h) (softplus_factor_h) of the forward's
// stored outputs h (row fst, times fscale: lin3's X4 holds h / sqrt2), loaded two k-steps ahead so
// the loads' waits never reach the newest weight-slice DMA; FAC_IN 2 zeroes inputs >= 217 (lin3).
template <bool B16, int V, int E, bool RELU_IN, int SP_IN, int FAC_IN, int NIN, int NOUT>
__device__ __forceinline__ void layer_x3(Pipe& p, const f32x4 (&in)[NIN], const float (&emb)[16], const float (&vemb)[8],
                                         f32x4 (&out)[NOUT], const float* __restrict__ sbias, int g, int lane,
                                         const LayerIO& io) {
  float* __restrict__ spst = io.spst;
  const float* __restrict__ fst = io.fst;
  const float fscale = io.fscale;
  constexpr int L = prog_layer<V>(E);
  constexpr LayerDesc D = layer_desc_all(L);
  constexpr int KS = ks32(L);
  constexpr int K0 = D.seg[0].ksteps / 8;
  constexpr int MOB = b16_main_ob(L);
  constexpr int PF = ANR_FRAG_PF;
  constexpr int NF = PF + 1;
  constexpr int MID = (MOB - 1) / 2;
  constexpr int BOFF = prog_bias_off<V>(E);
  static_assert(b16_tail_ob(L) == 0, "streamed x3 layers have no tail slice");
  // the B operand of k-step t: 8 inputs (ReLU of the previous layer applied here), hi/lo split
  f32x4 hv[2][2];  // FAC_IN: stored h of k-steps t (slot t & 1), two k-steps ahead
  auto load_h = [&](auto tc) {
    constexpr int t = decltype(tc)::value;
    if constexpr (FAC_IN != 0 && t < KS) {
#if ANR_SDF_NT
      hv[t & 1][0] = __builtin_nontemporal_load((const f32x4*)(fst + 32 * t + 4 * g));
      hv[t & 1][1] = __builtin_nontemporal_load((const f32x4*)(fst + 32 * t + 16 + 4 * g));
#else
      hv[t & 1][0] = *(const f32x4*)(fst + 32 * t + 4 * g);
      hv[t & 1][1] = *(const f32x4*)(fst + 32 * t + 16 + 4 * g);
#endif
    }
  };
  auto split_k = [&](auto tc, bf16x8& bh, bf16x8& bl) {
    constexpr int t = decltype(tc)::value;
    constexpr int seg = t < K0 ? 0 : 1;
    constexpr int ts = t < K0 ? t : t - K0;
    constexpr int kind = D.seg[seg].kind;
    float x[8];
    if constexpr (kind == SRC_EMB || kind == SRC_EMB6) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = emb[8 * ts + j];
    } else if constexpr (kind == SRC_VEMB) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = vemb[j];
    } else if constexpr (kind == SRC_G0 || kind == SRC_G1) {
      // 8 consecutive columns of a memory row (the colour net's inputs); past nact: zero, not loaded
      constexpr int NA = D.seg[seg].nact;
      const int c0 = 32 * ts + 8 * g;
      const float* gp = (kind == SRC_G0 ? io.g0 : io.g1) + c0;
      f32x4 u = {0.f, 0.f, 0.f, 0.f}, w = {0.f, 0.f, 0.f, 0.f};
      if (NA == 0 || c0 < NA) {
        u = *(const f32x4*)gp;
        w = *(const f32x4*)(gp + 4);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = NA == 0 || c0 + j < NA ? u[j] : 0.0f;
        x[4 + j] = NA == 0 || c0 + 4 + j < NA ? w[j] : 0.0f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = RELU_IN ? fmaxf(in[2 * ts][j], 0.0f) : in[2 * ts][j];
        x[4 + j] = RELU_IN ? fmaxf(in[2 * ts + 1][j], 0.0f) : in[2 * ts + 1][j];
      }
      if constexpr (FAC_IN != 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x[j] = x[j] * softplus_factor_h(hv[t & 1][0][j] * fscale);
          x[4 + j] = x[4 + j] * softplus_factor_h(hv[t & 1][1][j] * fscale);
          if constexpr (FAC_IN == 2) {  // lin3: 217 inputs; the rest are gamma gradients (and X4's padding)
            x[j] = 32 * ts + 4 * g + j < 217 ? x[j] : 0.0f;
            x[4 + j] = 32 * ts + 16 + 4 * g + j < 217 ? x[4 + j] : 0.0f;
          }
        }
        load_h(std::integral_constant<int, t + 2>{});
      }
      if constexpr (SP_IN != 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = softplus100(x[j]);
        if (spst) {  // neurons 32 ts + 4 g + (0..3) and 32 ts + 16 + 4 g + (0..3)
          float* d = spst + 32 * ts + 4 * g;
          if constexpr (SP_IN == 1) {  // streamed once to HBM, read once by the gradient pass: non-temporal
#if ANR_SDF_NT
            __builtin_nontemporal_store(f32x4{x[0], x[1], x[2], x[3]}, (f32x4*)d);
            __builtin_nontemporal_store(f32x4{x[4], x[5], x[6], x[7]}, (f32x4*)(d + 16));
#else
            *(f32x4*)d = f32x4{x[0], x[1], x[2], x[3]};
            *(f32x4*)(d + 16) = f32x4{x[4], x[5], x[6], x[7]};
#endif
          } else {
            const float sqrt2 = 1.41421356237309515f, rs2 = 0.707106769084930420f;  // RN(1 / RN(sqrt2))
            const int c = 32 * ts + 4 * g;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (c + j < 217) d[j] = div_const(x[j], sqrt2, rs2);
              if (c + 16 + j < 217) d[16 + j] = div_const(x[4 + j], sqrt2, rs2);
            }
          }
        }
      }
    }
    split8(x, bh, bl);
  };
  // fragment G = t * MOB + o (k-step t, out-block o) lives in register set G % NF. Same-slice
  // fragments are read PF out-blocks ahead; a fragment of slice t >= 1 read from slice t - 1 waits
  // for that slice's mid() (which certifies slice t), i.e. no earlier than out-block MID.
  bf16x8 fh[NF], fl[NF];
  bf16x8 bh[2], bl[2];
  const unsigned char* buf = p.template enter<B16, V, E, 0>();
  __builtin_amdgcn_sched_barrier(0);
  static_for<0, D.ob>([&](auto ob) {
    constexpr int o = decltype(ob)::value;
    out[o] = *(const f32x4*)(sbias + BOFF + o * 16 + 4 * g);
  });
  load_h(std::integral_constant<int, 0>{});
  load_h(std::integral_constant<int, 1>{});
  split_k(std::integral_constant<int, 0>{}, bh[0], bl[0]);
  static_for<0, PF>([&](auto gg) {
    constexpr int G = decltype(gg)::value;
    if constexpr (G < MOB && x3_issue_at<MOB, PF>(G) < 0) {
      fh[G % NF] = *(const bf16x8*)(buf + G * 2048 + lane * 16);
      fl[G % NF] = *(const bf16x8*)(buf + G * 2048 + 1024 + lane * 16);
    }
  });
  static_for<0, KS>([&](auto t) {
    constexpr int tt = decltype(t)::value;
    if constexpr (tt > 0) buf = p.template enter<B16, V, E, tt>();
    const unsigned char* nbuf = p.lds + (p.cur + 1 >= p.nbuf ? 0 : p.cur + 1) * p.smax;
    static_for<0, MOB>([&](auto ob) {
      constexpr int o = decltype(ob)::value;
      constexpr int F = tt * MOB + o;
      // fragments due at this out-block: same slice, or the next one once it is certified (o > MID)
      static_for<1, PF + 1>([&](auto dd) {
        constexpr int G = F + decltype(dd)::value;
        if constexpr (G / MOB == tt && x3_issue_at<MOB, PF>(G) == F) {
          fh[G % NF] = *(const bf16x8*)(buf + (G % MOB) * 2048 + lane * 16);
          fl[G % NF] = *(const bf16x8*)(buf + (G % MOB) * 2048 + 1024 + lane * 16);
        } else if constexpr (o > MID && tt + 1 < KS && G / MOB == tt + 1 && x3_issue_at<MOB, PF>(G) == F) {
          fh[G % NF] = *(const bf16x8*)(nbuf + (G % MOB) * 2048 + lane * 16);
          fl[G % NF] = *(const bf16x8*)(nbuf + (G % MOB) * 2048 + 1024 + lane * 16);
        }
      });
      __builtin_amdgcn_sched_barrier(0);
      constexpr int r = F % NF, c = tt & 1;
      out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl[r], bh[c], out[o], 0, 0, 0);
      out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[r], bl[c], out[o], 0, 0, 0);
      out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[r], bh[c], out[o], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      // the next k-step's B fragment, early in this k-step
      if constexpr (o == (MOB > 1 ? 1 : 0) && tt + 1 < KS)
        split_k(std::integral_constant<int, tt + 1>{}, bh[c ^ 1], bl[c ^ 1]);
      if constexpr (!ANR_DMA_SPREAD) {
        if constexpr (o == MID) p.template mid<B16, V, E, tt>();
      } else {
        constexpr int eqr = prog_advance<B16, V>(E, tt, mlp_nbuf<B16>() - 1);
        constexpr int NL = prog_slice_loads<B16, V>(eqr / 1024, eqr % 1024);
        constexpr int SPAN = MOB - 1 - MID;
        if constexpr (o == MID) p.template mid<B16, V, E, tt, true>();
        if constexpr (SPAN == 0) {
          if constexpr (o == MID) p.template piece<B16, V, E, tt, 0, NL>();
        } else if constexpr (o > MID) {
          constexpr int lo = ((o - MID - 1) * NL + SPAN - 1) / SPAN;
          constexpr int hi = o == MOB - 1 ? NL : ((o - MID) * NL + SPAN - 1) / SPAN;
          p.template piece<B16, V, E, tt, lo, hi>();
        }
      }
      // next-slice fragments due at out-block MID: after mid(), which certifies the next slice
      if constexpr (tt + 1 < KS && o == MID) {
        static_for<1, PF + 1>([&](auto dd) {
          constexpr int G = F + decltype(dd)::value;
          if constexpr (G / MOB == tt + 1 && x3_issue_at<MOB, PF>(G) == F) {
            fh[G % NF] = *(const bf16x8*)(nbuf + (G % MOB) * 2048 + lane * 16);
            fl[G % NF] = *(const bf16x8*)(nbuf + (G % MOB) * 2048 + 1024 + lane * 16);
          }
        });
      }
    });
    p.leave();
  });
}

template <bool B16, int V, int E, bool RELU, bool RELU_IN = false, int SP_IN = 0, int FAC_IN = 0, int NIN, int NOUT>
__device__ __forceinline__ void layer(Pipe& p, const f32x4 (&in)[NIN], const float (&emb)[16], const float (&vemb)[8],
                                      f32x4 (&out)[NOUT], const float* __restrict__ sbias, int g, int lane,
                                      const LayerIO& io = LayerIO{}) {
  constexpr int L = prog_layer<V>(E);
  constexpr LayerDesc D = layer_desc_all(L);
  static_assert(NOUT >= D.ob, "output array too small");
  static_assert((SP_IN == 0 && FAC_IN == 0) || prog_mode<B16, V>(E) == 2 ||
                    (prog_mode<B16, V>(E) == 1 && x3_stream_layer<L>()),
                "SP_IN / FAC_IN on streamed bf16x3 or on bf16x6 layers only");
  if constexpr (prog_mode<B16, V>(E) == 1 && x3_stream_layer<L>()) {
    // output ReLU deferred to the consumer's split (RELU_IN of the next layer)
    layer_x3<B16, V, E, RELU_IN, SP_IN, FAC_IN>(p, in, emb, vemb, out, sbias, g, lane, io);
    return;
  }
  // accumulators start at the bias; read right after the layer's first slice barrier, so the
  // compiler cannot hoist the reads (64 registers) into the previous layer
  constexpr int BOFF = prog_bias_off<V>(E);
  auto init_bias = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, D.ob>([&](auto ob) {
      constexpr int o = decltype(ob)::value;
      out[o] = *(const f32x4*)(sbias + BOFF + o * 16 + 4 * g);
    });
  };
  if constexpr (prog_mode<B16, V>(E) == 2) {
    // bf16x6 (mode 2): per k-step of 32 one hi/mid/lo split of the B fragment, per out-block 3 A
    // reads and 6 MFMAs (smallest terms first). The A fragments are read ANR_X6_PF out-blocks ahead
    // (x6_issue_at), across out-block groups and k-steps, into ANR_X6_PF + 1 register sets, but
    // never from a slice its ring slot does not certifiably hold yet (x6_schedule_ok).
    static_assert(x6_schedule_ok<V>(E), "bf16x6 fragment schedule reads an uncertified slice");
    constexpr int KS = ks32(L);
    constexpr int K0 = D.seg[0].ksteps / 8;
    constexpr int OB = D.ob;
    constexpr int NOBG = prog_nobg<V>(E);
    constexpr int NS = ANR_X6_PF + 1;
    bf16x8 fr[NS][3];
    const unsigned char* buf = nullptr;
    // FAC_IN: the stored h of the k-step's 8 input neurons, loaded one k-step ahead
    f32x4 hv[2][2];
    auto load_h = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (FAC_IN != 0 && t < KS) {
        hv[t & 1][0] = *(const f32x4*)(io.fst + 32 * t + 4 * g);
        hv[t & 1][1] = *(const f32x4*)(io.fst + 32 * t + 16 + 4 * g);
      }
    };
    load_h(std::integral_constant<int, 0>{});
    static_for<0, KS>([&](auto t) {
      constexpr int tt = decltype(t)::value;
      constexpr int seg = tt < K0 ? 0 : 1;
      constexpr int ts = tt < K0 ? tt : tt - K0;
      constexpr int kind = D.seg[seg].kind;
      float x[8];
      if constexpr (kind == SRC_EMB || kind == SRC_EMB6) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = emb[8 * ts + j];
      } else if constexpr (kind == SRC_VEMB) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = vemb[j];
      } else if constexpr (kind == SRC_G0 || kind == SRC_G1) {
        // 8 consecutive columns of a memory row (the colour net's inputs); past nact: zero, not loaded
        constexpr int NA = D.seg[seg].nact;
        const int c0 = 32 * ts + 8 * g;
        const float* gp = (kind == SRC_G0 ? io.g0 : io.g1) + c0;
        f32x4 u = {0.f, 0.f, 0.f, 0.f}, w = {0.f, 0.f, 0.f, 0.f};
        if (NA == 0 || c0 < NA) {
          u = *(const f32x4*)gp;
          w = *(const f32x4*)(gp + 4);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x[j] = NA == 0 || c0 + j < NA ? u[j] : 0.0f;
          x[4 + j] = NA == 0 || c0 + 4 + j < NA ? w[j] : 0.0f;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x[j] = RELU_IN ? fmaxf(in[2 * ts][j], 0.0f) : in[2 * ts][j];
          x[4 + j] = RELU_IN ? fmaxf(in[2 * ts + 1][j], 0.0f) : in[2 * ts + 1][j];
        }
        if constexpr (FAC_IN != 0) {  // the forward stored the softplus factors themselves (softplus100_fac)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            x[j] = x[j] * hv[tt & 1][0][j];
            x[4 + j] = x[4 + j] * hv[tt & 1][1][j];
            if constexpr (FAC_IN == 2) {  // lin3: 217 inputs; the rest are gamma gradients (and X4's padding)
              x[j] = 32 * ts + 4 * g + j < 217 ? x[j] : 0.0f;
              x[4 + j] = 32 * ts + 16 + 4 * g + j < 217 ? x[4 + j] : 0.0f;
            }
          }
          load_h(std::integral_constant<int, tt + 1>{});
        }
        if constexpr (SP_IN != 0) {  // h for this split, the backward factors to spst for the reverse pass
          // neurons 32 ts + 4 g + (0..3) and 32 ts + 16 + 4 g + (0..3), each half stored as it is done
          float* d = io.spst ? io.spst + 32 * ts + 4 * g : nullptr;
          const int c = 32 * ts + 4 * g;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            float f[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[4 * q + j] = softplus100_fac(x[4 * q + j], f[j]);
            if (d) {
              if constexpr (SP_IN == 1) {
                __builtin_nontemporal_store(f32x4{f[0], f[1], f[2], f[3]}, (f32x4*)(d + 16 * q));
              } else {  // lin3: 217 neurons (X4's columns past them are the skip's gamma inputs)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  if (c + 16 * q + j < 217) d[16 * q + j] = f[j];
              }
            }
          }
        }
      }
      bf16x8 bh, bm, bl;
      split8x3(x, bh, bm, bl);
      static_for<0, OB>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
        constexpr int F = tt * OB + o;
        constexpr int SQ = tt * NOBG + o / 8;  // the slice of this out-block group
        if constexpr (o % 8 == 0) buf = p.template enter<B16, V, E, SQ>();
        if constexpr (tt == 0 && o == 0) init_bias();
        static_for<0, NS>([&](auto dd) {
          constexpr int G = F + decltype(dd)::value;
          if constexpr (G < KS * OB && x6_issue_at<V>(E, G) == F) {
            constexpr int og = G % OB;
            const unsigned char* src =
                x6_slice_of<V>(E, G) == SQ ? buf : p.lds + (p.cur + 1 >= p.nbuf ? 0 : p.cur + 1) * p.smax;
            fr[G % NS][0] = *(const bf16x8*)(src + (og % 8) * 3072 + lane * 16);
            fr[G % NS][1] = *(const bf16x8*)(src + (og % 8) * 3072 + 1024 + lane * 16);
            fr[G % NS][2] = *(const bf16x8*)(src + (og % 8) * 3072 + 2048 + lane * 16);
          }
        });
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 ah = fr[F % NS][0], am = fr[F % NS][1], al = fr[F % NS][2];
        out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, out[o], 0, 0, 0);
        out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, out[o], 0, 0, 0);
        out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, out[o], 0, 0, 0);
        out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, out[o], 0, 0, 0);
        out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, out[o], 0, 0, 0);
        out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, out[o], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        constexpr int GOB = x6_group_obs<V>(E, o / 8);
        if constexpr (o % 8 == (GOB - 1) / 2) p.template mid<B16, V, E, SQ>();
        if constexpr (o % 8 == GOB - 1) p.leave();
      });
    });
  } else if constexpr (prog_mode<B16, V>(E) != 0) {
    // bf16x3 (mode 1): per k-step of 32 one hi/lo split of the B fragment, per out-block 2 A reads,
    // 3 MFMAs
    constexpr int KS = ks32(L);
    constexpr int K0 = D.seg[0].ksteps / 8;
    static_for<0, KS>([&](auto t) {
      constexpr int tt = decltype(t)::value;
      const unsigned char* buf = p.template enter<B16, V, E, tt>();
      if constexpr (tt == 0) init_bias();
      constexpr int seg = tt < K0 ? 0 : 1;
      constexpr int ts = tt < K0 ? tt : tt - K0;
      constexpr int kind = D.seg[seg].kind;
      float x[8];
      if constexpr (kind == SRC_EMB || kind == SRC_EMB6) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = emb[8 * ts + j];
      } else if constexpr (kind == SRC_VEMB) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = vemb[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x[j] = in[2 * ts][j];
          x[4 + j] = in[2 * ts + 1][j];
        }
      }
      {
        bf16x8 bh, bl;
        split8(x, bh, bl);
        // fragments of out-block o+PF are read while the MFMAs of o run (register double buffer),
        // pinned by scheduling barriers: left alone the compiler reads each pair right before its
        // MFMAs and the LDS latency (> the 48 MFMA cycles of one out-block) is exposed
        constexpr int MOB = b16_main_ob(L);
        constexpr int PF = ANR_FRAG_PF;
        bf16x8 fh[PF + 1], fl[PF + 1];
        static_for<0, PF>([&](auto pp) {
          constexpr int o = decltype(pp)::value;
          if constexpr (o < MOB) {
            fh[o] = *(const bf16x8*)(buf + o * 2048 + lane * 16);
            fl[o] = *(const bf16x8*)(buf + o * 2048 + 1024 + lane * 16);
          }
        });
        static_for<0, MOB>([&](auto ob) {
          constexpr int o = decltype(ob)::value;
          constexpr int r = o % (PF + 1), rn = (o + PF) % (PF + 1);
          if constexpr (o + PF < MOB) {
            fh[rn] = *(const bf16x8*)(buf + (o + PF) * 2048 + lane * 16);
            fl[rn] = *(const bf16x8*)(buf + (o + PF) * 2048 + 1024 + lane * 16);
          }
          __builtin_amdgcn_sched_barrier(0);
          out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl[r], bh, out[o], 0, 0, 0);
          out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[r], bl, out[o], 0, 0, 0);
          out[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[r], bh, out[o], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          constexpr int MID = (MOB - 1) / 2;
          if constexpr (!ANR_DMA_SPREAD) {
            if constexpr (o == MID) p.template mid<B16, V, E, tt>();
          } else {
            // refill pieces i at out-block MID + 1 + i * (MOB - 1 - MID) / NL (all at MID when the
            // slice has no second half); every piece is out before the next slice's mid()
            constexpr int eqr = prog_advance<B16, V>(E, tt, mlp_nbuf<B16>() - 1);
            constexpr int NL = prog_slice_loads<B16, V>(eqr / 1024, eqr % 1024);
            constexpr int SPAN = MOB - 1 - MID;
            if constexpr (o == MID) p.template mid<B16, V, E, tt, true>();
            if constexpr (SPAN == 0) {
              if constexpr (o == MID) p.template piece<B16, V, E, tt, 0, NL>();
            } else if constexpr (o > MID) {
              // pieces whose slot is this out-block: i with MID + 1 + i * SPAN / NL == o
              constexpr int lo = ((o - MID - 1) * NL + SPAN - 1) / SPAN;
              constexpr int hi = o == MOB - 1 ? NL : ((o - MID) * NL + SPAN - 1) / SPAN;
              p.template piece<B16, V, E, tt, lo, hi>();
            }
          }
        });
        p.leave();
      }
    });
    if constexpr (b16_tail_ob(L) > 0) {
      // the out-blocks past 16 (alpha_fc beside feature_fc): one slice [k-step][tail block]
      constexpr int TOB = b16_tail_ob(L);
      const unsigned char* buf = p.template enter<B16, V, E, KS>();
      static_for<0, KS>([&](auto t) {
        constexpr int tt = decltype(t)::value;
        static_assert(D.nseg == 1 && D.seg[0].kind == SRC_ACT, "tail blocks only on activation-input layers");
        float x[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x[j] = in[2 * tt][j];
          x[4 + j] = in[2 * tt + 1][j];
        }
        bf16x8 bh, bl;
        split8(x, bh, bl);
        static_for<0, TOB>([&](auto ob) {
          constexpr int o = decltype(ob)::value;
          const unsigned char* f = buf + (tt * TOB + o) * 2048 + lane * 16;
          const bf16x8 ah = *(const bf16x8*)f;
          const bf16x8 al = *(const bf16x8*)(f + 1024);
          out[16 + o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, out[16 + o], 0, 0, 0);
          out[16 + o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, out[16 + o], 0, 0, 0);
          out[16 + o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, out[16 + o], 0, 0, 0);
        });
        if constexpr (tt == (KS - 1) / 2) p.template mid<B16, V, E, KS>();
      });
      p.leave();
    }
  } else {
    constexpr int C = layer_chunks(L);
    constexpr int K = layer_ksteps(L);
    constexpr int K0 = D.seg[0].ksteps;
    const unsigned char* buf = nullptr;
    static_for<0, K>([&](auto t) {
      constexpr int tt = decltype(t)::value;
      if constexpr (tt % ANR_KSLICE == 0) buf = p.template enter<B16, V, E, tt / ANR_KSLICE>();
      if constexpr (tt == 0) init_bias();
      f32x4 w[C];
      static_for<0, C>([&](auto c) {
        constexpr int cc = decltype(c)::value;
        w[cc] = *(const f32x4*)(buf + (((tt % ANR_KSLICE) * C + cc) * 64 + lane) * 16);
      });
      constexpr int seg = tt < K0 ? 0 : 1;
      constexpr int ts = tt < K0 ? tt : tt - K0;
      constexpr int kind = D.seg[seg].kind;
      float b;
      if constexpr (kind == SRC_EMB) b = emb[ts];
      else if constexpr (kind == SRC_VEMB) b = vemb[ts];
      else b = in[ts >> 2][ts & 3];
      static_for<0, D.ob>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
        out[o] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[o >> 2][o & 3], b, out[o], 0, 0, 0);
      });
      if constexpr (tt % ANR_KSLICE == ANR_KSLICE / 2 - 1) p.template mid<B16, V, E, tt / ANR_KSLICE>();
      if constexpr (tt % ANR_KSLICE == ANR_KSLICE - 1) p.leave();
    });
  }
  if constexpr (RELU) {
    static_for<0, D.ob>([&](auto ob) {
      constexpr int o = decltype(ob)::value;
#pragma unroll
      for (int r = 0; r < 4; ++r) out[o][r] = fmaxf(out[o][r], 0.0f);
    });
  }
}

// sin and cos of x sharing one Cody-Waite reduction (three-constant FMA split of pi/2, accurate for
// |x| <= 1e5) and cephes' minimax polynomials on [-pi/4, pi/4]: <= 1.5 ulp, 7e-8 absolute (checked
// against float64 over |x| <= 5e4). Branch-free; embed_b keeps larger arguments on the library path.
__device__ __forceinline__ void sincos_fast(float x, float& s, float& c) {
  const float k = __builtin_rintf(x * 0.636619772367581343f);
  float r = __builtin_fmaf(-k, 1.57079601287841796875f, x);      // 0x1.921fb0p+0
  r = __builtin_fmaf(-k, 3.1391647326017846e-07f, r);             // 0x1.5110b4p-22
  r = __builtin_fmaf(-k, 5.3903025299577648e-15f, r);             // 0x1.846988p-48
  const float z = r * r;
  float ps = __builtin_fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
  ps = __builtin_fmaf(ps, z, -1.6666654611e-1f);
  const float sn = __builtin_fmaf(ps * z, r, r);
  float pc = __builtin_fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = __builtin_fmaf(pc, z, 4.166664568298827e-2f);
  pc = __builtin_fmaf(pc, z, -0.5f);
  const float cs = __builtin_fmaf(pc, z, 1.0f);
  const int q = (int)k;
  const float s0 = (q & 1) ? cs : sn, c0 = (q & 1) ? sn : cs;
  s = (q & 2) ? -s0 : s0;
  c = ((q + 1) & 2) ? -c0 : c0;
}

// gamma(x) in the bf16 fragment layout (anr_layers.h gamma_slot_feature): e[8s + 2p], e[8s + 2p + 1]
// = sin, cos of pair P = 4 NS h + 4 s + p - 2 (x, y, z, 0 in the first two slots of lane half 0)
template <int NS>
__device__ __forceinline__ void embed_b(const float x[3], int h, int nfreq, float (&e)[8 * NS]) {
  // launder the lane half: otherwise the per-lane pair indices of all slots are hoisted out of the
  // tile loop and pin registers for the whole kernel
  asm volatile("" : "+v"(h));
  const float m = fmaxf(fabsf(x[0]), fmaxf(fabsf(x[1]), fabsf(x[2])));
  // any lane with arguments past the fast reduction's range takes the library sincos (wave-uniform)
  const bool slow = __builtin_amdgcn_ballot_w64(!(m * (float)(1 << (nfreq - 1)) <= 65536.0f)) != 0;
  const int hb = 4 * NS * h - 2;
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int P = hb + 4 * s + p;        // pair index (< 0: the raw slots of lane half 0)
      const int freq = (P * 11) >> 5;      // P / 3 for 0 <= P < 30
      const int comp = P - 3 * freq;
      const float xc = comp == 0 ? x[0] : (comp == 1 ? x[1] : x[2]);
      const float arg = __builtin_ldexpf(xc, freq);
      float sv, cv;
      if (!slow) sincos_fast(arg, sv, cv);
      else sincosf(arg, &sv, &cv);
      const bool valid = (unsigned)P < (unsigned)(3 * nfreq);
      float v0 = valid ? sv : 0.0f, v1 = valid ? cv : 0.0f;
      if (s == 0 && p < 2) {  // lane half 0: x, y | z, 0
        const bool raw = h == 0;
        v0 = raw ? x[2 * p] : v0;
        v1 = raw ? (p == 0 ? x[1] : 0.0f) : v1;
      }
      e[8 * s + 2 * p] = v0;
      e[8 * s + 2 * p + 1] = v1;
    }
}

// gamma(x) features 4s+g, s = 0..NS-1 (embedder.py:5-54); sincos once per feature
template <int NS>
__device__ __forceinline__ void embed(const float x[3], int g, int nfreq, float (&e)[NS]) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int f = 4 * s + g;
    float v;
    if (f < 3) {
      v = x[f == 0 ? 0 : (f == 1 ? 1 : 2)];
    } else {
      const int q = f - 3;
      const int freq = q / 6;
      const int w = q - freq * 6;
      const int comp = w >= 3 ? w - 3 : w;
      const float xc = comp == 0 ? x[0] : (comp == 1 ? x[1] : x[2]);
      const float arg = xc * (float)(1 << (freq < 15 ? freq : 0));
      float sv, cv;
      sincosf(arg, &sv, &cv);
      v = freq >= nfreq ? 0.0f : (w >= 3 ? cv : sv);
    }
    e[s] = v;
  }
}

// 24-channel lookup from the 32-channel repacked volume, reference accumulation order.
// block 0 -> channels 4g..4g+3, block 1 -> 16+4g..16+4g+3
// FAST (bf16x3 kernels, whose outputs are held to the 1e-4 tolerance, not to the bits of init_pbw):
// the normalised coordinate from one reciprocal per axis instead of an IEEE division.
template <bool FAST = false>
__device__ __forceinline__ void lookup24(const float* __restrict__ vol32, const float p[3], const float* __restrict__ bounds,
                                         int X, int Y, int Z, int g, f32x4 (&out)[2]) {
#pragma clang fp contract(off)
  // formed per call (see embed_b): the float dims and bounds are not worth a register per tile
  asm volatile("" : "+s"(X), "+s"(Y), "+s"(Z), "+s"(bounds));
  float lo[3], hi[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) { lo[c] = bounds[c]; hi[c] = bounds[3 + c]; }
  TriCell t;
  if constexpr (FAST) {
    // (p - lo) / ext as (p - lo) * rcp(ext): within 1-2 ulp of the division
    float gq[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) gq[c] = (p[c] - lo[c]) * __builtin_amdgcn_rcpf(hi[c] - lo[c]) * 2.0f - 1.0f;
    const float ix = grid_src(gq[2], Z), iy = grid_src(gq[1], Y), iz = grid_src(gq[0], X);
    tri_cell_src(ix, iy, iz, X, Y, Z, t);
  } else {
    tri_cell(p, lo, hi, X, Y, Z, t);
  }
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (t.base[k] >= 0) {
      const f32x4 v0 = *(const f32x4*)(vol32 + (size_t)t.base[k] * 32 + 4 * g);
      const f32x4 v1 = *(const f32x4*)(vol32 + (size_t)t.base[k] * 32 + 16 + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a0[r] = a0[r] + v0[r] * t.w[k];
        a1[r] = a1[r] + v1[r] * t.w[k];
      }
    }
  }
  out[0] = a0;
  out[1] = a1;
}

// softmax over 24 channels of log(init + 1e-9) + fc (tpose_nerf_network.py:74-76); lanes
// l, l^16, l^32, l^48 hold one point's channels.
// FAST (bf16x3 kernels): hardware log2/exp2 and one reciprocal instead of the library logf/expf and
// eight divisions (relative error ~1e-6 on the weights, inside the 1e-4 output tolerance).
template <bool FAST = false>
__device__ __forceinline__ void blend_softmax(const f32x4 (&fc)[2], const f32x4 (&init)[2], int g, f32x4 (&bw)[2]) {
  float lg[2][4];
  float m = -INFINITY;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool valid = b == 0 || g < 2;
      const float v = (FAST ? __logf(init[b][r] + 1e-9f) : logf(init[b][r] + 1e-9f)) + fc[b][r];
      lg[b][r] = valid ? v : -INFINITY;
      m = fmaxf(m, lg[b][r]);
    }
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  float s = 0.f;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      lg[b][r] = FAST ? __expf(lg[b][r] - m) : expf(lg[b][r] - m);
      s += lg[b][r];
    }
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) bw[b][r] = FAST ? lg[b][r] * __builtin_amdgcn_rcpf(s) : lg[b][r] / s;
}

// LBS inverse warp: A_b = sum_j bw_j A_j; x_T = inv(A_b[:3,:3]) (x - A_b[:3,3])
__device__ __forceinline__ void lbs_inverse(const f32x4 (&bw)[2], const float* __restrict__ sA, int g, const float x[3],
                                            float xt[3]) {
  float Ab[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) Ab[m] = 0.f;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = b * 16 + 4 * g + r;
      if (j < 24) {
        const float wj = bw[b][r];
#pragma unroll
        for (int m = 0; m < 16; ++m) Ab[m] += wj * sA[j * 16 + m];
      }
    }
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    Ab[m] += __shfl_xor(Ab[m], 16);
    Ab[m] += __shfl_xor(Ab[m], 32);
  }
  const float a = Ab[0], b = Ab[1], c = Ab[2], d = Ab[4], e = Ab[5], f = Ab[6], gg = Ab[8], h = Ab[9], i = Ab[10];
  const float c00 = e * i - f * h, c01 = c * h - b * i, c02 = b * f - c * e;
  const float c10 = f * gg - d * i, c11 = a * i - c * gg, c12 = c * d - a * f;
  const float c20 = d * h - e * gg, c21 = b * gg - a * h, c22 = a * e - b * d;
  const float det = a * c00 + b * c10 + c * c20;
  const float rd = 1.0f / det;
  const float y0 = x[0] - Ab[3], y1 = x[1] - Ab[7], y2 = x[2] - Ab[11];
  xt[0] = (c00 * rd) * y0 + (c01 * rd) * y1 + (c02 * rd) * y2;
  xt[1] = (c10 * rd) * y0 + (c11 * rd) * y1 + (c12 * rd) * y2;
  xt[2] = (c20 * rd) * y0 + (c21 * rd) * y1 + (c22 * rd) * y2;
}

__device__ __forceinline__ void store_rows(float* __restrict__ rows, int idx, const f32x4 (&bw)[2], int g, bool valid) {
  if (!valid) return;
  *(f32x4*)(rows + (size_t)idx * 24 + 4 * g) = bw[0];
  if (g < 2) *(f32x4*)(rows + (size_t)idx * 24 + 16 + 4 * g) = bw[1];
}

// BW MLP pass starting at program entry E0 (0: pose pass; 9: T-pose pass). The pose pass may read
// the novel_pose_bw copy of the weights (p.pose_woff); its biases are in the LDS table (fill_bias_table).
template <bool B16, int V, int E0>
__device__ __forceinline__ void bw_mlp(Pipe& p, const float (&emb)[16], const float (&vemb)[8], const float* __restrict__ sb,
                                       f32x4 (&A)[17], f32x4 (&B)[17], f32x4 (&fc)[2], int g, int lane) {
  f32x4 dummy[1];
  layer<B16, V, E0 + 0, true>(p, dummy, emb, vemb, A, sb, g, lane);
  layer<B16, V, E0 + 1, true, true>(p, A, emb, vemb, B, sb, g, lane);
  layer<B16, V, E0 + 2, true, true>(p, B, emb, vemb, A, sb, g, lane);
  layer<B16, V, E0 + 3, true, true>(p, A, emb, vemb, B, sb, g, lane);
  layer<B16, V, E0 + 4, true, true>(p, B, emb, vemb, A, sb, g, lane);
  layer<B16, V, E0 + 5, true, true>(p, A, emb, vemb, B, sb, g, lane);
  layer<B16, V, E0 + 6, true, true>(p, B, emb, vemb, A, sb, g, lane);
  layer<B16, V, E0 + 7, true, true>(p, A, emb, vemb, B, sb, g, lane);
  layer<B16, V, E0 + 8, false, true>(p, B, emb, vemb, fc, sb, g, lane);
}

template <bool B16, int V = 2>
__device__ __forceinline__ void mlp_body(const MlpArgs& a) {
  // every kernel runs the folded colour head (anr_layers.h ANR_L_HEAD): 131,072 fewer MACs per sample
  static_assert(V == 2 || V == 4, "render programs");
  // hardware log/exp/rcp and reciprocal lookup coordinates only in the bf16x3 kernel
  constexpr bool FAST = B16 && ANR_FAST_MATH && V == 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int pl = lane & 15;
  float* sb = (float*)smem;  // bias table (anr_layers.h LDS layout)
  float* sA = (float*)(smem + mlp_sa_off());
  for (int i = tid; i < 384; i += 512) sA[i] = a.A[i];
  fill_bias_table<V>(a, sb, tid);

  float* sT = sA + 384;  // T-pose bounds
  if (tid < 6) sT[tid] = a.tbounds[tid];
  const int n = *a.n_kept;
  const int ntiles = (n + 127) / 128;
  if ((int)blockIdx.x >= ntiles) return;  // uniform per workgroup, before any LDS-DMA

  Pipe p{smem + mlp_ring_off(), mlp_slice_max<B16>(), mlp_nbuf<B16>(), a.wimg, 0, wave, lane, a.pose_woff};
  p.template start<B16, V>();

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int idx = tile * 128 + wave * 16 + pl;
    const bool valid = idx < n;
    const int pid = a.list[valid ? idx : n - 1];
    float dist, pose[3], dir[3];
    if (a.dists) {  // free samples (Network.forward): the caller's world point, view direction, dist
      world_to_pose_pt(a.wpts, pid, a.n_pts, a.chunk_pts, a.R, a.Th, pose);
      dist = a.dists[pid];
#pragma unroll
      for (int c = 0; c < 3; ++c) dir[c] = a.vdir[3 * (size_t)pid + c];
    } else {
      const int ray = pid >> 6, s = pid & 63;
      float z, pts[3];
      sample_point(a.ray_o, a.ray_d, a.near_, a.far_, a.t_rand, ray, s, 64, z, dist, pts);
      world_to_pose(pts, a.R, a.Th, pose);
#pragma unroll
      for (int c = 0; c < 3; ++c) dir[c] = a.ray_d[3 * ray + c];
    }

    float emb[16], vemb[8];
    f32x4 A[17], B[17], fc[2], init[2], bw[2];

    // ---- pose space: pbw lookup, BW MLP (latent_index + 1), softmax, LBS
    if constexpr (B16) embed_b<2>(pose, g, 10, emb);
    else embed<16>(pose, g, 10, emb);
    lookup24<FAST>(a.pbw32, pose, a.pbounds, a.pX, a.pY, a.pZ, g, init);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) vemb[s8] = 0.f;
    bw_mlp<B16, V, 0>(p, emb, vemb, sb, A, B, fc, g, lane);
    blend_softmax<FAST>(fc, init, g, bw);
    store_rows(a.pbw_rows, idx, bw, g, valid);
    float xt[3];
    lbs_inverse(bw, sA, g, pose, xt);

    // ---- T-pose: tbw lookup, BW MLP (latent 0) -> tbw rows (training loss only)
    if constexpr (B16) embed_b<2>(xt, g, 10, emb);
    else embed<16>(xt, g, 10, emb);
    lookup24<FAST>(a.tbw32, xt, a.tbounds, a.tX, a.tY, a.tZ, g, init);
    bw_mlp<B16, V, 9>(p, emb, vemb, sb, A, B, fc, g, lane);
    blend_softmax<FAST>(fc, init, g, bw);
    store_rows(a.tbw_rows, idx, bw, g, valid);

    // ---- canonical NeRF (TPoseHuman.calculate_alpha_rgb)
    f32x4 dummy[1];
    layer<B16, V, 18, true>(p, dummy, emb, vemb, A, sb, g, lane);
    layer<B16, V, 19, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<B16, V, 20, true, true>(p, B, emb, vemb, A, sb, g, lane);
    layer<B16, V, 21, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<B16, V, 22, true, true>(p, B, emb, vemb, A, sb, g, lane);
    layer<B16, V, 23, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<B16, V, 24, true, true>(p, B, emb, vemb, A, sb, g, lane);
    layer<B16, V, 25, true, true>(p, A, emb, vemb, B, sb, g, lane);
    float sigma_raw;
    if constexpr (B16) embed_b<1>(dir, g, 4, vemb);
    else embed<8>(dir, g, 4, vemb);
    layer<B16, V, 26, false, true>(p, B, emb, vemb, A, sb, g, lane);  // view_fc pre-activation || alpha
    sigma_raw = __shfl(A[8][0], pl);
    if constexpr (!(prog_mode<B16, V>(27) == 1 && x3_stream_layer<ANR_L_RGB>())) {  // else rgb_fc applies view_fc's ReLU in its split
      static_for<0, 8>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
#pragma unroll
        for (int r = 0; r < 4; ++r) A[o][r] = fmaxf(A[o][r], 0.0f);
      });
    }
    layer<B16, V, 27, false, true>(p, A, emb, vemb, B, sb, g, lane);  // rgb_fc

    // ---- bbox mask, activations, outputs
    bool inside = true;
#pragma unroll
    for (int c = 0; c < 3; ++c) inside = inside && (xt[c] > sT[c]) && (xt[c] < sT[3 + c]);
    const float sig = inside ? sigma_raw : 0.0f;
    if (valid && g == 0) {
      float4 r;
      r.x = 1.0f / (1.0f + expf(-B[0][0]));
      r.y = 1.0f / (1.0f + expf(-B[0][1]));
      r.z = 1.0f / (1.0f + expf(-B[0][2]));
      r.w = 1.0f - expf(-fmaxf(sig, 0.0f) * dist);
      a.raw[pid] = r;
      a.sigma[idx] = sig;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the last (unused) prefetch
}

// Density program (V = 1): Network.calculate_alpha (tpose_nerf_network.py:105-135) per kept free
// point — pose-space blend-weight lookup + BW MLP (latent_index + 1, or novel_pose_bw), softmax,
// LBS inverse, then TPoseHuman.calculate_alpha (:241-250): NeRF trunk + alpha_fc. The T-pose BW MLP
// the reference also evaluates there does not reach the returned alpha and is not run; no bbox
// mask, no activation: alpha_out[id] = the raw alpha_fc output.
template <bool B16, int V = 1>
__device__ __forceinline__ void alpha_body(const MlpArgs& a) {
  static_assert(V == 1 || V == 8, "density programs");
  constexpr bool FAST = B16 && ANR_FAST_MATH && V == 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int pl = lane & 15;
  float* sb = (float*)smem;  // bias table (anr_layers.h LDS layout)
  float* sA = (float*)(smem + mlp_sa_off());
  for (int i = tid; i < 384; i += 512) sA[i] = a.A[i];
  fill_bias_table<V>(a, sb, tid);

  const int n = *a.n_kept;
  const int ntiles = (n + 127) / 128;
  if ((int)blockIdx.x >= ntiles) return;  // uniform per workgroup, before any LDS-DMA

  Pipe p{smem + mlp_ring_off(), mlp_slice_max<B16>(), mlp_nbuf<B16>(), a.wimg, 0, wave, lane, a.pose_woff};
  p.template start<B16, V>();

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int idx = tile * 128 + wave * 16 + pl;
    const bool valid = idx < n;
    const int pid = a.list[valid ? idx : n - 1];
    float pose[3];
    world_to_pose_pt(a.wpts, pid, a.n_pts, a.chunk_pts, a.R, a.Th, pose);

    float emb[16], vemb[8];
    f32x4 A[17], B[17], fc[2], init[2], bw[2];
    if constexpr (B16) embed_b<2>(pose, g, 10, emb);
    else embed<16>(pose, g, 10, emb);
    lookup24<FAST>(a.pbw32, pose, a.pbounds, a.pX, a.pY, a.pZ, g, init);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) vemb[s8] = 0.f;
    bw_mlp<B16, V, 0>(p, emb, vemb, sb, A, B, fc, g, lane);
    blend_softmax<FAST>(fc, init, g, bw);
    float xt[3];
    lbs_inverse(bw, sA, g, pose, xt);

    if constexpr (B16) embed_b<2>(xt, g, 10, emb);
    else embed<16>(xt, g, 10, emb);
    f32x4 dummy[1];
    layer<B16, V, 9, true>(p, dummy, emb, vemb, A, sb, g, lane);
    layer<B16, V, 10, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<B16, V, 11, true, true>(p, B, emb, vemb, A, sb, g, lane);
    layer<B16, V, 12, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<B16, V, 13, true, true>(p, B, emb, vemb, A, sb, g, lane);
    layer<B16, V, 14, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<B16, V, 15, true, true>(p, B, emb, vemb, A, sb, g, lane);
    layer<B16, V, 16, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<B16, V, 17, false, true>(p, B, emb, vemb, A, sb, g, lane);  // alpha_fc
    if (valid && g == 0) a.alpha_out[pid] = A[0][0];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the last (unused) prefetch
}

// sdf_pdf residual deformation program (V = 3): Network.calculate_residual_deformation
// (anisdf_pdf_network.py:49-73) per kept sample of one batch, all on chip — gamma_10 of the big-pose
// point, 8 x 256 ReLU layers (poses folded into the layer-0 / layer-5 biases), resd_fc. Writes the
// resd_fc output; k_sdf_mid applies 0.05 tanh. Replaces 8 layer GEMMs over HBM-resident activations.
template <bool X6>
__device__ __forceinline__ void resd_body(const MlpArgs& a) {
  constexpr int V = 3 + (X6 ? 10 : 0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int pl = lane & 15;
  float* sb = (float*)smem;  // bias table (anr_layers.h LDS layout)
  fill_bias_table<V>(a, sb, tid);
  const int n = a.n_rows;
  const int ntiles = (n + 127) / 128;
  if ((int)blockIdx.x >= ntiles) return;  // uniform per workgroup, before any LDS-DMA

  Pipe p{smem + mlp_ring_off(), mlp_slice_max<true>(), mlp_nbuf<true>(), a.wimg, 0, wave, lane, 0};
  p.template start<true, V>();

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int idx = tile * 128 + wave * 16 + pl;
    const bool valid = idx < n;
    const float* pt = a.ptb + (size_t)(valid ? idx : n - 1) * a.ptb_ld;
    const float x[3] = {pt[0], pt[1], pt[2]};
    float emb[16], vemb[8];
    f32x4 A[17], B[17], fc[2];
    embed_b<2>(x, g, 10, emb);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) vemb[s8] = 0.f;
    bw_mlp<true, V, 0>(p, emb, vemb, sb, A, B, fc, g, lane);
    if (valid && g == 0) {
      float* y = a.yr + (size_t)idx * 4;
      y[0] = fc[0][0];
      y[1] = fc[0][1];
      y[2] = fc[0][2];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the last (unused) prefetch
}

// softplus(beta = 100, threshold = 20) of the accumulators in place
template <int NOB, int V>
__device__ __forceinline__ void softplus_regs(f32x4 (&v)[17]) {
  static_for<0, NOB>([&](auto ob) {
    constexpr int o = decltype(ob)::value;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[o][r] = sp_fwd<V>(v[o][r]);
  });
}

// sdf_pdf SDF network forward (V = 5): SDFNetwork.forward (anisdf_pdf_network.py:421-437) per kept
// sample of one batch, on chip — gamma_6 of the canonical point, lin0..lin7 with softplus, the skip
// [h3 || gamma_6] / sqrt2 at lin4 (the 1/sqrt2 is in lin4's packed weights), lin8. What the reverse
// pass (the input gradient) and the colour net read is written once: every softplus output h (lin3's
// as h / sqrt2 in X4, the layout of the layer-GEMM path) and lin8's sdf (Y8 column 0) and feature
// (Y8 columns 8..263: 16-B aligned for k_color_b16's row loads). bf16x6 (V = 15) writes the backward
// factors sigmoid(100 z) in those slots instead (lin3's unscaled in X4[:, :217]): softplus100_fac
// gives them beside h, and the reverse pass then multiplies without recomputing them.
template <bool X6>
__device__ __forceinline__ void sdfnet_body(const MlpArgs& a) {
  constexpr int V = 5 + (X6 ? 10 : 0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int pl = lane & 15;
  float* sb = (float*)smem;  // bias table (anr_layers.h LDS layout)
  fill_bias_table<V>(a, sb, tid);
  const int n = a.n_rows;
  const int ntiles = (n + 127) / 128;
  if ((int)blockIdx.x >= ntiles) return;  // uniform per workgroup, before any LDS-DMA

  Pipe p{smem + mlp_ring_off(), mlp_slice_max<true>(), mlp_nbuf<true>(), a.wimg, 0, wave, lane, 0};
  p.template start<true, V>();

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int idx = tile * 128 + wave * 16 + pl;
    const bool valid = idx < n;
    const size_t row = (size_t)(valid ? idx : n - 1);
    const float* pt = a.ptb + row * a.ptb_ld;
    const float x[3] = {pt[0], pt[1], pt[2]};
    float emb[16], vemb[8];
    f32x4 A[17], B[17];
    embed_b<2>(x, g, 6, emb);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) vemb[s8] = 0.f;
    // h of a 256-wide softplus layer -> sdf_h[l] (16 B per lane and out-block)
    auto store_h = [&](const f32x4(&v)[17], float* __restrict__ dst) {
      if (!valid) return;
      float* d = dst + row * 256 + 4 * g;
      static_for<0, 16>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
        *(f32x4*)(d + 16 * o) = v[o];
      });
    };
    // each layer's softplus runs in the next layer's split (SP_IN), which also stores its h
    // store targets formed at each call (a per-tile array of row pointers costs 16 VGPRs for the tile)
    auto st = [&](int i) { return LayerIO{valid ? (i == 3 ? a.x4 : a.sdf_h[i]) + row * 256 : nullptr}; };
    f32x4 dummy[1];
    layer<true, V, 0, false>(p, dummy, emb, vemb, A, sb, g, lane);
    layer<true, V, 1, false, false, 1>(p, A, emb, vemb, B, sb, g, lane, st(0));
    layer<true, V, 2, false, false, 1>(p, B, emb, vemb, A, sb, g, lane, st(1));
    layer<true, V, 3, false, false, 1>(p, A, emb, vemb, B, sb, g, lane, st(2));  // 217 outputs (14 out-blocks)
    // [h3 || gamma_6] (1/sqrt2 in the weights); h3 / sqrt2 -> X4[:, :217]
    layer<true, V, 4, false, false, 2>(p, B, emb, vemb, A, sb, g, lane, st(3));
    layer<true, V, 5, false, false, 1>(p, A, emb, vemb, B, sb, g, lane, st(4));
    layer<true, V, 6, false, false, 1>(p, B, emb, vemb, A, sb, g, lane, st(5));
    layer<true, V, 7, false, false, 1>(p, A, emb, vemb, B, sb, g, lane, st(6));
    if constexpr (X6) {  // h7 in place for lin8, its backward factors to sdf_h[7]
      float* d = a.sdf_h[7] + row * 256 + 4 * g;
      static_for<0, 16>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
        float f[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) B[o][r] = softplus100_fac(B[o][r], f[r]);
        if (valid) *(f32x4*)(d + 16 * o) = f32x4{f[0], f[1], f[2], f[3]};
      });
    } else {
      softplus_regs<16, V>(B);  // lin8 (a tail-slice layer, not streamed) reads h7 as is
      store_h(B, a.sdf_h[7]);
    }
    layer<true, V, 8, false>(p, B, emb, vemb, A, sb, g, lane);  // [sdf || feature], no activation
    if (valid) {  // sdf (neuron 0) to column 0, the feature (neurons 1..256) to columns 8..263
      float* d = a.y8 + row * 264;
      // lane holds neurons 16 o + 4 g + r: neuron m > 0 -> column m + 7
      static_for<0, 17>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * o + 4 * g + r;
          if (m == 0) d[0] = A[o][r];
          else if (m <= 256) d[m + 7] = A[o][r];
        }
      });
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the last (unused) prefetch
}

// sdf_pdf SDF network input gradient (V = 7): d sdf / d x (the autograd.grad of anisdf_pdf_network.py
// :302-311 through SDFNetwork.forward) per kept sample of one batch, on chip. The gradient vector is the
// MFMA B operand, lin7^T .. lin0^T the weights; each layer's input is multiplied by the softplus-backward
// factor recomputed from the forward's stored h (FAC_IN; bf16x6: the stored factor itself). Writes the gamma_6 gradients (lin0's, and
// the skip part of lin4's) for k_sdf_gamma_bwd. Replaces 8 reverse layer GEMMs over HBM activations.
template <bool X6>
__device__ __forceinline__ void sdfgrad_body(const MlpArgs& a) {
  constexpr int V = 7 + (X6 ? 10 : 0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int pl = lane & 15;
  float* sb = (float*)smem;  // bias table (zeros), then lin8's row 0
  fill_bias_table<V>(a, sb, tid);
  float* sw8 = sb + prog_bias_off<V>(prog_len<V>());
  for (int i = tid; i < 256; i += 512) sw8[i] = a.w8row[i];
  const int n = a.n_rows;
  const int ntiles = (n + 127) / 128;
  if ((int)blockIdx.x >= ntiles) return;  // uniform per workgroup, before any LDS-DMA

  Pipe p{smem + mlp_ring_off(), mlp_slice_max<true>(), mlp_nbuf<true>(), a.wimg, 0, wave, lane, 0};
  p.template start<true, V>();  // its barrier also publishes sw8

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int idx = tile * 128 + wave * 16 + pl;
    const bool valid = idx < n;
    const size_t row = (size_t)(valid ? idx : n - 1);
    float emb[16], vemb[8];
#pragma unroll
    for (int i = 0; i < 16; ++i) emb[i] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) vemb[i] = 0.f;
    f32x4 A[17], B[17];
    // dz7 = W8[0] * sigmoid(100 z7) (lin8's sdf row; the softplus factor from h7)
    {
      const float* h7 = a.sdf_h[7] + row * 256 + 4 * g;
      static_for<0, 16>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
        const f32x4 hv = *(const f32x4*)(h7 + 16 * o);
        const f32x4 wv = *(const f32x4*)(sw8 + 16 * o + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) A[o][r] = wv[r] * (X6 ? hv[r] : softplus_factor_h(hv[r]));  // X6: stored factors
      });
    }
    const float sqrt2 = 1.41421356237309515f;
    layer<true, V, 0, false>(p, A, emb, vemb, B, sb, g, lane);  // dh6 = W7^T dz7
    layer<true, V, 1, false, false, 0, 1>(p, B, emb, vemb, A, sb, g, lane, LayerIO{nullptr, a.sdf_h[6] + row * 256});
    layer<true, V, 2, false, false, 0, 1>(p, A, emb, vemb, B, sb, g, lane, LayerIO{nullptr, a.sdf_h[5] + row * 256});
    // d [h3 || gamma_6] = W4^T dz4 / sqrt2 (the 1/sqrt2 packed into the weights)
    layer<true, V, 3, false, false, 0, 1>(p, B, emb, vemb, A, sb, g, lane, LayerIO{nullptr, a.sdf_h[4] + row * 256});
    if (valid) {  // the skip's gamma_6 gradients: neurons 217..255
      float* d = a.gc + row * 256;
      static_for<13, 16>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 16 * o + 4 * g + r;
          if (c >= 217) d[c] = A[o][r];
        }
      });
    }
    // lin3's inputs < 217, factor from X4 = h3 / sqrt2
    layer<true, V, 4, false, false, 0, 2>(p, A, emb, vemb, B, sb, g, lane, LayerIO{nullptr, a.x4 + row * 256, sqrt2});
    layer<true, V, 5, false, false, 0, 1>(p, B, emb, vemb, A, sb, g, lane, LayerIO{nullptr, a.sdf_h[2] + row * 256});
    layer<true, V, 6, false, false, 0, 1>(p, A, emb, vemb, B, sb, g, lane, LayerIO{nullptr, a.sdf_h[1] + row * 256});
    layer<true, V, 7, false, false, 0, 1>(p, B, emb, vemb, A, sb, g, lane, LayerIO{nullptr, a.sdf_h[0] + row * 256});
    if (valid) {  // lin0's gamma_6 gradients (39)
      float* d = a.gb + row * 40;
      static_for<0, 3>([&](auto ob) {
        constexpr int o = decltype(ob)::value;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 16 * o + 4 * g + r;
          if (c < 39) d[c] = A[o][r];
        }
      });
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the last (unused) prefetch
}

// sdf_pdf colour network (V = 6): ColorNetwork.forward (anisdf_pdf_network.py:516-545) per kept sample
// of one batch, on chip: lin0 reads [points, gamma_4(dir), normal] from the sample's C0 row and the
// SDF net's feature from its Y8 row (columns 8..263, written there by k_sdfnet_b16), then
// lin1..lin3 (ReLU deferred into the next split, the colour latent folded into lin3's bias), lin4's
// three logits to yr ([n][4]); k_sdf_raw applies the sigmoid.
template <bool X6>
__device__ __forceinline__ void color_body(const MlpArgs& a) {
  constexpr int V = 6 + (X6 ? 10 : 0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int pl = lane & 15;
  float* sb = (float*)smem;
  fill_bias_table<V>(a, sb, tid);
  const int n = a.n_rows;
  const int ntiles = (n + 127) / 128;
  if ((int)blockIdx.x >= ntiles) return;  // uniform per workgroup, before any LDS-DMA

  Pipe p{smem + mlp_ring_off(), mlp_slice_max<true>(), mlp_nbuf<true>(), a.wimg, 0, wave, lane, 0};
  p.template start<true, V>();

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int idx = tile * 128 + wave * 16 + pl;
    const bool valid = idx < n;
    const size_t row = (size_t)(valid ? idx : n - 1);
    float emb[16], vemb[8];
#pragma unroll
    for (int i = 0; i < 16; ++i) emb[i] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) vemb[i] = 0.f;
    f32x4 A[17], B[17];
    LayerIO io{};
    io.g0 = a.ptb + row * a.ptb_ld;
    io.g1 = a.y8 + row * 264 + 8;
    f32x4 dummy[1];
    layer<true, V, 0, true>(p, dummy, emb, vemb, A, sb, g, lane, io);
    layer<true, V, 1, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<true, V, 2, true, true>(p, B, emb, vemb, A, sb, g, lane);
    layer<true, V, 3, true, true>(p, A, emb, vemb, B, sb, g, lane);
    layer<true, V, 4, false, true>(p, B, emb, vemb, A, sb, g, lane);
    if (valid && g == 0) {
      float* y = a.yr + row * 4;
      y[0] = A[0][0];
      y[1] = A[0][1];
      y[2] = A[0][2];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the last (unused) prefetch
}

}  // namespace anr
