// anr_tgemm.hip — the bf16 row GEMM of the training executor (precision 'bf16', config 3) for the two
// products whose B operand is a layer's weight:
//   forward  Y  = act(X W^T + b)          rows of W   (k = input column)
//   backward dX = (dY W) * (H > 0)        rows of W^T (k = output neuron)
// Weights are converted once per training call into bf16 images (k_wimg_pack) whose rows are
// k-contiguous and padded to whole 64-wide K chunks (segments of a concatenated input start on a
// chunk), so both products read B the same way. One workgroup (4 waves) owns 64 rows x up to 256
// output columns; every K chunk of 64 is brought in by LDS-DMA — the activations as fp32 (16 KiB),
// the weight rows as bf16 (32 KiB) — into a 3-slot ring with two chunks in flight behind counted
// vmcnt waits, and each wave runs 4 x 4 v_mfma_f32_16x16x32_bf16 per 32-deep k-step (fp32
// accumulation; the activations rounded to bf16 RNE as their fragments are read, as the generic
// kernel rounds them at staging). LDS images are XOR-swizzled through the DMA source addresses.
// Epilogue order as anr_gemm.hip: bias, accumulate, ReLU, mask.
#include <algorithm>
#include <vector>

#include "anr_common.h"
#include "anr_train.h"

namespace anr {

// ------------------------------------------------------------------------------------------
// weight images
// ------------------------------------------------------------------------------------------
struct WDesc {
  int t, n, in_ch, nseg, c0[2], k[2];
};
// the Conv1d weights the training GEMMs read (tensor index, out, in, used column segments)
static const WDesc kWDesc[] = {
    {28, 256, 191, 1, {0, 0}, {63, 0}},    {30, 256, 256, 1, {0, 0}, {256, 0}}, {32, 256, 256, 1, {0, 0}, {256, 0}},
    {34, 256, 256, 1, {0, 0}, {256, 0}},   {36, 256, 256, 1, {0, 0}, {256, 0}}, {38, 256, 447, 2, {0, 191}, {63, 256}},
    {40, 256, 256, 1, {0, 0}, {256, 0}},   {42, 256, 256, 1, {0, 0}, {256, 0}}, {44, 24, 256, 1, {0, 0}, {256, 0}},
    {1, 256, 63, 1, {0, 0}, {63, 0}},      {3, 256, 256, 1, {0, 0}, {256, 0}},  {5, 256, 256, 1, {0, 0}, {256, 0}},
    {7, 256, 256, 1, {0, 0}, {256, 0}},    {9, 256, 256, 1, {0, 0}, {256, 0}},  {11, 256, 319, 2, {0, 63}, {63, 256}},
    {13, 256, 256, 1, {0, 0}, {256, 0}},   {15, 256, 256, 1, {0, 0}, {256, 0}}, {17, 1, 256, 1, {0, 0}, {256, 0}},
    {19, 256, 256, 1, {0, 0}, {256, 0}},   {21, 256, 384, 1, {0, 0}, {256, 0}}, {23, 128, 283, 2, {0, 256}, {256, 27}},
    {25, 3, 128, 1, {0, 0}, {128, 0}},
    // novel_pose_bw (animation stage; index ANR_NUM_TENSORS + its state_dict position, kept last so
    // a call without it packs only the entries above)
    {46 + 1, 256, 191, 1, {0, 0}, {63, 0}},  {46 + 3, 256, 256, 1, {0, 0}, {256, 0}},
    {46 + 5, 256, 256, 1, {0, 0}, {256, 0}},  {46 + 7, 256, 256, 1, {0, 0}, {256, 0}},
    {46 + 9, 256, 256, 1, {0, 0}, {256, 0}},  {46 + 11, 256, 447, 2, {0, 191}, {63, 256}},
    {46 + 13, 256, 256, 1, {0, 0}, {256, 0}}, {46 + 15, 256, 256, 1, {0, 0}, {256, 0}},
    {46 + 17, 24, 256, 1, {0, 0}, {256, 0}},
};
constexpr int kNWBase = 22;  // entries of the network's own tensors (the rest: novel_pose_bw)
constexpr int kNW = sizeof(kWDesc) / sizeof(kWDesc[0]);
static_assert(kNW - kNWBase <= kNWBase, "WPackArgs holds one range");
static_assert(WG_MAX_Z % 8 == 0, "k_wgrad XCD order");

static int rup64(int v) { return (v + 63) / 64 * 64; }

struct WPackJob {
  const float* W;
  int n, in_ch, ld, bwd;  // bwd: transposed image (rows = input columns)
  int c0[2], k[2], col[2], nseg;
  long start, dst;        // first element (flat) and destination offset (elements)
};
struct WPackArgs {
  WPackJob job[2 * 22];  // one launch per descriptor range (kernel arguments stay < 4 KiB)
  int njob;
  long total, first, packed;  // image elements (hi); this launch's element range [first, packed)
  unsigned short* out;
};

__device__ __forceinline__ unsigned short f2bf_rne(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

__global__ void k_wimg_pack(WPackArgs a) {
  const long e = a.first + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.packed) return;
  int j = 0;
  while (j + 1 < a.njob && e >= a.job[j + 1].start) ++j;
  const WPackJob& J = a.job[j];
  const long local = e - J.start;
  const int row = (int)(local / J.ld), col = (int)(local - (long)row * J.ld);
  float v = 0.0f;
  if (J.bwd) {
    // row = input column c, col = output neuron
    if (col < J.n) v = J.W[(long)col * J.in_ch + row];
  } else {
    for (int s = 0; s < J.nseg; ++s)
      if (col >= J.col[s] && col < J.col[s] + J.k[s]) v = J.W[(long)row * J.in_ch + J.c0[s] + col - J.col[s]];
  }
  const unsigned short hi = f2bf_rne(v);
  a.out[J.dst + local] = hi;
  a.out[a.total + J.dst + local] = f2bf_rne(v - __uint_as_float((uint32_t)hi << 16));  // lo image
}

// layout of the images: per descriptor a forward image (n rows x sum of 64-padded segments) and a
// backward image (in_ch rows x 64-padded n)
static long wimg_layout(std::vector<WPackJob>* jobs) {
  long off = 0, start = 0;
  for (int i = 0; i < kNW; ++i) {
    const WDesc& d = kWDesc[i];
    WPackJob f{};
    f.n = d.n; f.in_ch = d.in_ch; f.nseg = d.nseg; f.bwd = 0;
    int ld = 0;
    for (int s = 0; s < d.nseg; ++s) {
      f.c0[s] = d.c0[s]; f.k[s] = d.k[s]; f.col[s] = ld;
      ld += rup64(d.k[s]);
    }
    f.ld = ld;
    f.dst = off; f.start = start;
    off += (long)d.n * ld; start += (long)d.n * ld;
    WPackJob b = f;
    b.bwd = 1; b.ld = rup64(d.n);
    b.dst = off; b.start = start;
    off += (long)d.in_ch * b.ld; start += (long)d.in_ch * b.ld;
    if (jobs) { jobs->push_back(f); jobs->push_back(b); }
  }
  return off;
}

// hi images, then the lo images (w - hi, for the split-bf16 products) at the same offsets + total
size_t wimg_bytes() { return (size_t)wimg_layout(nullptr) * 2 * 2; }

int wimg_pack(const float* const* t, void* dst, hipStream_t s) {
  std::vector<WPackJob> jobs;
  const long total = wimg_layout(&jobs);
  // the network's own images, then (when given) the novel_pose_bw images: one launch per range
  const bool novel = t[kWDesc[kNWBase].t] != nullptr;
  const int ranges[3] = {0, 2 * kNWBase, 2 * kNW};
  for (int r = 0; r < (novel ? 2 : 1); ++r) {
    WPackArgs a{};
    a.njob = ranges[r + 1] - ranges[r];
    for (int j = 0; j < a.njob; ++j) {
      a.job[j] = jobs[ranges[r] + j];
      a.job[j].W = t[kWDesc[(ranges[r] + j) / 2].t];
    }
    a.total = total;
    a.first = jobs[ranges[r]].start;
    a.packed = ranges[r + 1] < 2 * kNW ? jobs[ranges[r + 1]].start : total;
    a.out = (unsigned short*)dst;
    hipLaunchKernelGGL(k_wimg_pack, dim3((unsigned)((a.packed - a.first + 255) / 256)), dim3(256), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

bool wimg_view(const void* base, const float* const* t, const float* W, int c0, int K, bool bwd, WView* v) {
  long off = 0;
  const int nw = t[kWDesc[kNWBase].t] != nullptr ? kNW : kNWBase;
  for (int i = 0; i < nw; ++i) {
    const WDesc& d = kWDesc[i];
    int fld = 0, col[2] = {0, 0};
    for (int s = 0; s < d.nseg; ++s) { col[s] = fld; fld += rup64(d.k[s]); }
    const long foff = off, boff = off + (long)d.n * fld;
    const int bld = rup64(d.n);
    off = boff + (long)d.in_ch * bld;
    if (t[d.t] != W) continue;
    const long lo_off = wimg_layout(nullptr);
    v->lo_off = lo_off;
    if (bwd) {
      // rows c0 .. c0 + (output columns) of the transposed image, K = d.n
      if (K != d.n) return false;
      v->B = (const unsigned short*)base + boff + (long)c0 * bld;
      v->ldb = bld;
      v->bcol = 0;
      v->rows = d.in_ch - c0;
      return true;
    }
    for (int s = 0; s < d.nseg; ++s)
      if (d.c0[s] == c0 && K <= d.k[s]) {
        v->B = (const unsigned short*)base + foff;
        v->ldb = fld;
        v->bcol = col[s];
        v->rows = d.n;
        return true;
      }
    return false;
  }
  return false;
}

// ------------------------------------------------------------------------------------------
// the row GEMM
// ------------------------------------------------------------------------------------------
// 128 rows per workgroup (8 waves = 2 row groups x 4 column groups of 64), 2-slot ring, so the
// weight image each workgroup streams serves 128 rows. bf16: 64-deep K chunks. X3 (split-bf16,
// fp32-level: lo*h + h*lo + h*h, the weight rows' lo image riding in the same slot): 32-deep chunks
// so that three 128-row operand images fit two slots.
// (Measured alternatives, tools/gemm_probe at 24,893 rows: three slots 13.5 vs 12.9 us; 64-row
// workgroups (4 waves, 2-4 slots) 21.5 us; 32-deep chunks in a 3-slot 72 KiB ring, two workgroups per
// CU, 14.9 us alone and 11.6 vs 9.9 us per launch with two streams. The workgroup's time is its load
// burst, four chunks and a store burst that runs at the HBM write rate (phase clocks).)
template <bool X3, bool ABF = false> struct RgCfg {
  static constexpr int BM = 128;
  static constexpr int WAVES = BM / 16;
  static constexpr int KC = X3 ? 32 : 64;                              // K chunk
  static constexpr int AE = ABF ? 2 : 4;                               // bytes per activation element
  static constexpr int A_BYTES = BM * KC * AE;                         // activations, BM rows x KC
  static constexpr int B_BYTES = 256 * KC * 2;                         // bf16 weight rows, 256 x KC
  static constexpr int NIMG = X3 ? 2 : 1;                              // weight images per slot
  static constexpr int NS = 2;                                         // ring slots
  static constexpr int SLOT = A_BYTES + B_BYTES * NIMG;                // bytes per slot
  static constexpr int PIECES_A = A_BYTES / 1024 / WAVES;              // per wave
  static constexpr int PIECES_B = B_BYTES / 1024 / WAVES;
  static constexpr int OPS = PIECES_A + PIECES_B * NIMG;               // vmem ops per wave per chunk
  static constexpr int CHA = KC * AE / 16, CHB = KC / 8;              // 16-B chunks per A / B row
  // XOR swizzle of a row's 16-B chunks, chosen so the 16 rows of one fragment read hit distinct banks
  static __device__ __forceinline__ int swa(int r) { return X3 ? ((r >> 1) & 7) : ABF ? (r & 7) : (r & 15); }
  static __device__ __forceinline__ int swb(int r) { return X3 ? ((r >> 2) & 3) : (r & 7); }
};

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

template <int N>
__device__ __forceinline__ void rg_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void rg_dma(const void* src, unsigned m0) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory");
}

// issue chunk c (segment-relative K offset kk) into ring slot `slot`
template <bool X3, bool ABF>
__device__ __forceinline__ void rg_issue(const RGemm& g, int seg, int kk, int m0, int M, int N, unsigned slot_lds, int w,
                                         int lane) {
  using C = RgCfg<X3, ABF>;
  const unsigned char* A = (const unsigned char*)(seg ? g.seg[1].A : g.seg[0].A);
  const long lda = seg ? g.seg[1].lda : g.seg[0].lda;
  const unsigned short* B = seg ? g.seg[1].B : g.seg[0].B;
  const long ldb = seg ? g.seg[1].ldb : g.seg[0].ldb;
  const int bcol = seg ? g.seg[1].bcol : g.seg[0].bcol;
  const int brows = seg ? g.seg[1].rows : g.seg[0].rows;
  // A: BM rows x CHA chunks; a 1 KiB piece holds 64 / CHA rows; LDS chunk q of row r holds source
  // chunk q ^ swa(r)
  constexpr int RPA = 64 / C::CHA, RPB = 64 / C::CHB;
#pragma unroll
  for (int i = 0; i < C::PIECES_A; ++i) {
    const int p = w + C::WAVES * i;
    const int r = RPA * p + lane / C::CHA;
    const int gr = min(m0 + r, M - 1);
    const int ch = (lane % C::CHA) ^ C::swa(r);
    rg_dma(A + ((long)gr * lda + kk) * C::AE + ch * 16, slot_lds + p * 1024);
  }
  // B: 256 rows x CHB chunks, chunk q of row r holds source chunk q ^ swb(r)
#pragma unroll
  for (int i = 0; i < C::PIECES_B; ++i) {
    const int p = w + C::WAVES * i;
    const int r = RPB * p + lane / C::CHB;
    const int br = min(r, brows - 1);
    const int ch = (lane % C::CHB) ^ C::swb(r);
    rg_dma(B + (long)br * ldb + bcol + kk + ch * 8, slot_lds + C::A_BYTES + p * 1024);
  }
  if constexpr (X3) {
    const long lo = seg ? g.seg[1].lo_off : g.seg[0].lo_off;
#pragma unroll
    for (int i = 0; i < C::PIECES_B; ++i) {
      const int p = w + C::WAVES * i;
      const int r = RPB * p + lane / C::CHB;
      const int br = min(r, brows - 1);
      const int ch = (lane % C::CHB) ^ C::swb(r);
      rg_dma(B + lo + (long)br * ldb + bcol + kk + ch * 8, slot_lds + C::A_BYTES + C::B_BYTES + p * 1024);
    }
  }
  (void)N;
}

// MBF: the mask rows are bf16 (a template parameter, so every epilogue load stays one straight-line
// batch ahead of its use; a runtime branch around them would drain the loads one by one)
// RG_TIMING (tools/gemm_probe's own build of this file only): wave 0 of every workgroup records the
// shader clock at the phase boundaries (start, prologue issued, each chunk's data ready, loop end,
// epilogue done) into rg_tbuf[block][16]
#ifdef RG_TIMING
__device__ unsigned long long* rg_tbuf;
#define RG_T(i)                                                                                \
  do {                                                                                         \
    if (threadIdx.x < 64) {                                                                    \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                              \
      if (threadIdx.x == 0 && rg_tbuf) rg_tbuf[(long)blockIdx.x * 16 + (i)] = t_;              \
    }                                                                                          \
  } while (0)
void rg_timing_buffer(unsigned long long* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(rg_tbuf), &p, sizeof(p)); }
#else
#define RG_T(i) \
  do {          \
  } while (0)
#endif

template <bool X3, bool ABF, bool MBF>
__global__ __launch_bounds__(RgCfg<X3>::WAVES * 64) void k_rgemm(RGemm g) {
  using CF = RgCfg<X3, ABF>;
  constexpr int RG_NS = CF::NS, RG_SLOT = CF::SLOT, RG_OPS = CF::OPS;
  constexpr int RG_BM = CF::BM, RG_A_BYTES = CF::A_BYTES;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int M = g.M_dev ? *g.M_dev : g.M;
  const int N = g.N;
  const int m0 = blockIdx.x * RG_BM;
  if (m0 >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned base = (unsigned)(uintptr_t)lds;
  constexpr int KC = CF::KC;
  const int nc0 = (g.seg[0].K + KC - 1) / KC;
  const int nch = nc0 + (g.nseg > 1 ? (g.seg[1].K + KC - 1) / KC : 0);
  auto issue = [&](int c) {
    const int seg = c < nc0 ? 0 : 1;
    const int kk = (c - (seg ? nc0 : 0)) * KC;
    rg_issue<X3, ABF>(g, seg, kk, m0, M, N, base + (c % RG_NS) * RG_SLOT, w, lane);
  };
  RG_T(0);
  const int wr = (w >> 2) * 64;   // this wave's 64 rows of the tile
  const int wc = (w & 3) * 64;    // and 64 output columns
  const bool active = wc < N;     // which hold some of the N
  // the epilogue's bias columns load now, ahead of the ring (older than every DMA, so the counted
  // vmcnt waits below retire them first); the bf16 mask rows load at the last chunk (below): the
  // epilogue then finds its operands in registers (tools/gemm_probe phase clocks: the epilogue was
  // 4.1 us of an 11 us workgroup, 7.2 us with the mask)
  f32x4 bj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = min(wc + 16 * j + 4 * (lane >> 4), N - 4);
    bj[j] = (g.vec_out && g.bias && active) ? *(const f32x4*)(g.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int pro = nch < RG_NS ? nch : RG_NS;
  for (int c = 0; c < pro; ++c) issue(c);
  RG_T(1);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint2 mk16[4][4];  // MBF vec_out: the mask's bf16 quads in the accumulator layout
  const bool early_mask = MBF && g.vec_out && g.mask != nullptr && active;

  for (int c = 0; c < nch; ++c) {
    // chunks issued after c: min(nch, c + RG_NS) - c - 1 (the refill of c - 1's slot went out last iteration)
    const int later = (nch < c + RG_NS ? nch : c + RG_NS) - c - 1;
    if (later >= 2) rg_wait<(RG_NS > 2 ? 2 * RG_OPS : 0)>();
    else if (later == 1) rg_wait<RG_OPS>();
    else rg_wait<0>();
    __builtin_amdgcn_s_barrier();
    RG_T(2 + (c < 9 ? c : 9));
    if (early_mask && c == nch - 1) {  // every DMA has landed (wait 0 above): these are the youngest loads
      const unsigned short* mask16 = (const unsigned short*)g.mask;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long m = min(m0 + wr + 16 * i + (lane & 15), M - 1);
          const int n = min(wc + 16 * j + 4 * (lane >> 4), N - 4);
          mk16[i][j] = *(const uint2*)(mask16 + m * g.ldm + n);
        }
    }
    const int seg = c < nc0 ? 0 : 1;
    const int kk = (c - (seg ? nc0 : 0)) * KC;
    const int K = seg ? g.seg[1].K : g.seg[0].K;
    const unsigned char* sA = lds + (c % RG_NS) * RG_SLOT;
    const unsigned char* sB = sA + RG_A_BYTES;
    if (active) {
#pragma unroll
      for (int ks = 0; ks < KC / 32; ++ks) {
        bf16x8_t af[4], bfr[4], al[4], bl[4];
        const int kc = 4 * ks + (lane >> 4);  // 8-element k group of this lane
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wr + 16 * i + (lane & 15);
          if constexpr (ABF) {
            // bf16 row r, k = 8 kc .. 8 kc + 7: one 16-B chunk kc (swizzled by swa(r))
            af[i] = *(const bf16x8_t*)(sA + r * (KC * 2) + ((kc ^ CF::swa(r)) * 16));
            if (kk + KC > K) {  // the last, partial chunk of a segment: columns past K read as zero
#pragma unroll
              for (int e = 0; e < 8; ++e) af[i][e] = (kk + 8 * kc + e < K) ? af[i][e] : (__bf16)0.0f;
            }
            continue;
          }
          // fp32 row r, k = 8 kc .. 8 kc + 7: 16-B chunks 2 kc, 2 kc + 1 (swizzled by swa(r))
          const int sa = CF::swa(r);
          const f32x4 x0 = *(const f32x4*)(sA + r * (KC * 4) + (((2 * kc) ^ sa) * 16));
          const f32x4 x1 = *(const f32x4*)(sA + r * (KC * 4) + (((2 * kc + 1) ^ sa) * 16));
          float x[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
          if (kk + KC > K) {  // the last, partial chunk of a segment: columns past K read as zero
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = (kk + 8 * kc + e < K) ? x[e] : 0.0f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            af[i][e] = (__bf16)x[e];
            if constexpr (X3) al[i][e] = (__bf16)(x[e] - (float)af[i][e]);
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = wc + 16 * j + (lane & 15);
          const int sb = CF::swb(r);
          bfr[j] = *(const bf16x8_t*)(sB + r * (KC * 2) + ((kc ^ sb) * 16));
          if constexpr (X3) bl[j] = *(const bf16x8_t*)(sB + CF::B_BYTES + r * (KC * 2) + ((kc ^ sb) * 16));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if constexpr (X3) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], af[i], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], al[i], acc[i][j], 0, 0, 0);
            }
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
          }
      }
    }
    // everyone is past this slot's reads (lgkmcnt drained by the barrier's wait) before it is refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (c + RG_NS < nch) issue(c + RG_NS);
  }
  rg_wait<0>();
  RG_T(12);
  if (!active) return;
  // weights are the MFMA A operand, so lane l holds C[16 i + (l & 15)][64 w + 16 j + 4 (l >> 4) + r],
  // r = 0..3: four consecutive columns of one row, stored as one 16-B store (vec_out). Every
  // operand load of the epilogue is issued before the first use.
  const unsigned short* mask16 = (const unsigned short*)g.mask;
  unsigned short* C16 = (unsigned short*)g.C;
  auto bf2f = [](unsigned short b) { return __uint_as_float((uint32_t)b << 16); };
  if (g.vec_out) {
    f32x4 cv[4][4], mk[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long m = min(m0 + wr + 16 * i + (lane & 15), M - 1);
        const int n = min(wc + 16 * j + 4 * (lane >> 4), N - 4);
        if (g.accumulate) cv[i][j] = *(const f32x4*)(g.C + m * g.ldc + n);
        if (g.mask) {
          if constexpr (MBF) {
            const uint2 q = mk16[i][j];  // loaded at the last chunk (early_mask holds here)
            mk[i][j] = f32x4{bf2f(q.x & 0xffffu), bf2f(q.x >> 16), bf2f(q.y & 0xffffu), bf2f(q.y >> 16)};
          } else {
            mk[i][j] = *(const f32x4*)(g.mask + m * g.ldm + n);
          }
        }
      }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 v = acc[i][j];
        if (g.bias) v += bj[j];
        if (g.accumulate) v += cv[i][j];
        if (g.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (g.mask) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = mk[i][j][e] > 0.f ? v[e] : 0.f;
        }
        acc[i][j] = v;
      }
    auto pack4 = [](const f32x4& v) {
      return make_uint2((uint32_t)f2bf_rne(v[0]) | ((uint32_t)f2bf_rne(v[1]) << 16),
                        (uint32_t)f2bf_rne(v[2]) | ((uint32_t)f2bf_rne(v[3]) << 16));
    };
    if (g.cbf && g.vec16) {
      // bf16 rows as 16-B stores: lanes l and l ^ 16 hold columns 4q..4q+3 and 4q+4..4q+7 of one row
      // in each 16-column block, so a pair of blocks (j0, j1) swaps one quad per lane and each lane
      // stores 8 consecutive columns of one block: 8 stores per lane instead of 16 (the store issue
      // was the epilogue's cost: tools/gemm_probe phase clocks, 3.7 of an 11 us workgroup)
      const bool odd = (lane >> 4) & 1;
      const int m = m0 + wr + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int pj = 0; pj < 2; ++pj) {
          const uint2 a = pack4(acc[i][2 * pj]), b = pack4(acc[i][2 * pj + 1]);
          const uint2 snd = odd ? a : b;
          const uint2 rcv = make_uint2((uint32_t)__shfl_xor((int)snd.x, 16), (uint32_t)__shfl_xor((int)snd.y, 16));
          const uint4 o = odd ? make_uint4(rcv.x, rcv.y, b.x, b.y) : make_uint4(a.x, a.y, rcv.x, rcv.y);
          const int n = wc + 16 * (2 * pj + (odd ? 1 : 0)) + 8 * ((lane >> 5) & 1);
          const int mm = m + 16 * i;
          if (mm < M) {
            unsigned short* dst = C16 + (long)mm * g.ldc + n;
            if (n + 8 <= N) {
              *(uint4*)dst = o;
            } else if (n < N) {  // N % 4 == 0: the first quad only
              *(uint2*)dst = make_uint2(o.x, o.y);
            }
          }
        }
      RG_T(13);
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wr + 16 * i + (lane & 15);
        const int n = wc + 16 * j + 4 * (lane >> 4);
        const f32x4 v = acc[i][j];
        if (m < M && n < N) {
          if (g.cbf)
            *(uint2*)(C16 + (long)m * g.ldc + n) = pack4(v);
          else
            *(f32x4*)(g.C + (long)m * g.ldc + n) = v;
        }
      }
    RG_T(13);
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr + 16 * i + (lane & 15);
        const int n = wc + 16 * j + 4 * (lane >> 4) + r;
        if (m >= M || n >= N) continue;
        float v = acc[i][j][r];
        float* cp = g.C + (long)m * g.ldc + n;
        if (g.bias) v += g.bias[n];
        if (g.accumulate) v += *cp;
        if (g.relu) v = fmaxf(v, 0.f);
        if (g.mask) {
          const float mv = MBF ? bf2f(mask16[(long)m * g.ldm + n]) : g.mask[(long)m * g.ldm + n];
          if (!(mv > 0.f)) v = 0.f;
        }
        if (g.cbf) C16[(long)m * g.ldc + n] = f2bf_rne(v);
        else *cp = v;
      }
}

template <bool X3, bool ABF>
size_t rgemm_lds_bytes() { return (size_t)RgCfg<X3, ABF>::NS * RgCfg<X3, ABF>::SLOT; }

void launch_rgemm(const RGemm& g0, int M_host, hipStream_t s) {
  RGemm g = g0;
  const size_t ce = g.cbf ? 2 : 4, me = g.mbf ? 2 : 4;  // C / mask element bytes
  g.vec_out = (g.N % 4 == 0) && (g.ldc % 4 == 0) && ((uintptr_t)g.C % (4 * ce) == 0) &&
              (!g.mask || ((g.ldm % 4 == 0) && ((uintptr_t)g.mask % (4 * me) == 0))) && ((uintptr_t)g.bias % 16 == 0);
  g.vec16 = g.vec_out && g.cbf && g.ldc % 8 == 0 && (uintptr_t)g.C % 16 == 0;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_rgemm<false, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)rgemm_lds_bytes<false, false>());
    (void)hipFuncSetAttribute((const void*)k_rgemm<false, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)rgemm_lds_bytes<false, false>());
    (void)hipFuncSetAttribute((const void*)k_rgemm<false, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)rgemm_lds_bytes<false, true>());
    (void)hipFuncSetAttribute((const void*)k_rgemm<false, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)rgemm_lds_bytes<false, true>());
    (void)hipFuncSetAttribute((const void*)k_rgemm<true, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)rgemm_lds_bytes<true, false>());
    attr = true;
  }
  constexpr int BM = RgCfg<false>::BM;
  const dim3 grid((M_host + BM - 1) / BM), block(RgCfg<false>::WAVES * 64);
  const bool mbf = g.mbf && g.mask;
  if (g.x3)
    hipLaunchKernelGGL((k_rgemm<true, false, false>), grid, block, (rgemm_lds_bytes<true, false>()), s, g);
  else if (g.abf && mbf)
    hipLaunchKernelGGL((k_rgemm<false, true, true>), grid, block, (rgemm_lds_bytes<false, true>()), s, g);
  else if (g.abf)
    hipLaunchKernelGGL((k_rgemm<false, true, false>), grid, block, (rgemm_lds_bytes<false, true>()), s, g);
  else if (mbf)
    hipLaunchKernelGGL((k_rgemm<false, false, true>), grid, block, (rgemm_lds_bytes<false, false>()), s, g);
  else
    hipLaunchKernelGGL((k_rgemm<false, false, false>), grid, block, (rgemm_lds_bytes<false, false>()), s, g);
}

}  // namespace anr

namespace anr {

// ------------------------------------------------------------------------------------------
// weight gradient dW[:, c0:c0+K] += dY^T X (+ column sums of dY into bsum / bsum2), bf16 operands,
// fp32 accumulation: the reduction runs over the kept samples. Each workgroup (4 waves, 2 x 2 of
// 64 x 64) owns a 128 (outputs) x 128 (inputs) tile and a contiguous range of samples; it stages
// 32 samples per step through registers (fp32 -> bf16 RNE) into [sample][column] LDS images read
// with ds_read_b64_tr_b16 (8 consecutive samples per MFMA fragment), double-buffered, and writes its
// partial tile to a slab in the accumulator's own layout (16 B per lane, coalesced). k_wgrad_reduce
// sums the slabs in sample-range order and adds them into dW: no atomics, deterministic.
// ------------------------------------------------------------------------------------------
#define WG_T 128        // tile edge
#define WG_S 32         // samples per step
#define WG_LD 136       // LDS row stride (bf16 elements)
#define WG_TILE_FLOATS (WG_T * WG_T)

typedef short wv4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8_t wg_frag(const unsigned short* S, int cb, int lane) {
  // 16-lane group g: rows 8g + q (q = 0..3, then 4..7), lane 4q + p supplies columns cb + 4p .. +3;
  // lane i receives column cb + i, element q = row q (anr_gemm.hip frag16)
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) wv4s lds_v4s;
  const unsigned short* a0 = S + (8 * g + q) * WG_LD + cb + 4 * p;
  const wv4s x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(uintptr_t)(unsigned)(uintptr_t)a0);
  const wv4s x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(uintptr_t)(unsigned)(uintptr_t)(a0 + 4 * WG_LD));
  bf16x8_t f;
  const short e[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  __builtin_memcpy(&f, e, 16);
  return f;
}

// X3: also the lo image (x - hi) into SL
template <bool X3>
__device__ __forceinline__ void wg_store(unsigned short* S, unsigned short* SL, int tid, const f32x4 (&v)[4]) {
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int row = 8 * h + (tid >> 5), col = 4 * (tid & 31);
    unsigned short e[4], l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[k] = f2bf_rne(v[h][k]);
      if constexpr (X3) l[k] = f2bf_rne(v[h][k] - __uint_as_float((uint32_t)e[k] << 16));
    }
    *(uint2*)(S + row * WG_LD + col) = make_uint2((uint32_t)e[0] | ((uint32_t)e[1] << 16), (uint32_t)e[2] | ((uint32_t)e[3] << 16));
    if constexpr (X3)
      *(uint2*)(SL + row * WG_LD + col) = make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
  }
}

// The operand loads run WG_D steps ahead: each step's rows are held raw (bf16 pairs or fp32 quads,
// exactly as loaded) in a register ring of WG_D steps and widened / split only at their LDS store
// (tools/gemm_probe, 24,893 rows: 26.6 us per launch with its reduction against 28.4 us for loads one
// step ahead; 35.7 against 37.8 us split-bf16).
// YBF / XBF: dY / X rows hold bf16 (template parameters: the prefetch must stay branch-free)
template <bool BF>
struct WgRaw {
  typedef f32x4 T;
};
template <>
struct WgRaw<true> {
  typedef uint2 T;
};

template <bool BF>
__device__ __forceinline__ void wg_load_raw(const float* P, long ld, int ncol, int c0, int s, int s1, int srow, int tid,
                                            typename WgRaw<BF>::T (&r)[4]) {
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int ss = s + 8 * h + (tid >> 5);
    const int c = c0 + 4 * (tid & 31);
    const bool ok = ss < s1 && c < ncol;
    const long at = (long)(ok ? ss : srow) * ld + (ok ? c : 0);  // a valid row either way (no branch)
    if constexpr (BF) r[h] = *(const uint2*)((const unsigned short*)P + at);
    else r[h] = *(const f32x4*)(P + at);
  }
}

template <bool BF>
__device__ __forceinline__ void wg_widen(const typename WgRaw<BF>::T (&r)[4], int ncol, int c0, int s, int s1, int tid,
                                         f32x4 (&v)[4]) {
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int ss = s + 8 * h + (tid >> 5);
    const int c = c0 + 4 * (tid & 31);
    const bool ok = ss < s1 && c < ncol;
    f32x4 x;
    if constexpr (BF)
      x = f32x4{__uint_as_float(r[h].x << 16), __uint_as_float(r[h].x & 0xffff0000u), __uint_as_float(r[h].y << 16),
                __uint_as_float(r[h].y & 0xffff0000u)};
    else
      x = r[h];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[h][e] = (ok && c + e < ncol) ? x[e] : 0.0f;
  }
}

#define WG_D 4
// bf16 rows straight into the [sample][column] image: samples past the range and columns past ncol
// read as zero (the f2bf round trip of the fp32 path would return the same bits)
__device__ __forceinline__ void wg_put_bf(unsigned short* S, const uint2 (&r)[4], int ncol, int c0, int s, int s1,
                                          int tid) {
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int ss = s + 8 * h + (tid >> 5);
    const int c = c0 + 4 * (tid & 31);
    uint2 v = (ss < s1 && c < ncol) ? r[h] : make_uint2(0u, 0u);
    if (c + 4 > ncol) {  // a partial 4-column group (the last of a narrow operand)
      const int k = ncol - c;  // valid columns in the group, < 4
      v.x &= k >= 2 ? 0xffffffffu : k == 1 ? 0x0000ffffu : 0u;
      v.y &= k >= 4 ? 0xffffffffu : k == 3 ? 0x0000ffffu : 0u;
    }
    *(uint2*)(S + (8 * h + (tid >> 5)) * WG_LD + 4 * (tid & 31)) = v;
  }
}

// the LDS of one weight-gradient workgroup: per buffer two 32-sample images (hi and lo under X3, two
// sample halves otherwise), double-buffered, and the column-sum exchange
struct WgLds {
  unsigned short sY[2][2 * WG_S * WG_LD];
  unsigned short sX[2][2 * WG_S * WG_LD];
  float srs[8][WG_T];
};

// one (output tile, sample range) of dW: (ti, tj) the 128 x 128 tile of dW, z the sample range
template <bool X3, bool YBF, bool XBF>
__device__ __forceinline__ void wgrad_tile(const WGrad& g, int ti, int tj, int z, WgLds& sm) {
  constexpr int D = WG_D;
  constexpr int NI = X3 ? 2 : 1;
  constexpr int NH = X3 ? 1 : 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = g.M_dev ? *g.M_dev : g.n;
  const int spb = g.spb ? g.spb : ((n + g.nz - 1) / g.nz + 2 * WG_S - 1) / (2 * WG_S) * (2 * WG_S);
  const int s0 = z * spb, s1 = min(n, s0 + spb);
  const int i0 = ti * WG_T, j0 = tj * WG_T;
  const int wi = (w >> 1) * 64, wj = (w & 1) * 64;
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 rsum = {0.f, 0.f, 0.f, 0.f};
  const bool do_rs = g.rs_slab != nullptr && tj == 0;
  constexpr int STEP = NH * WG_S;
  typename WgRaw<YBF>::T ry[D][NH][4];
  typename WgRaw<XBF>::T rx[D][NH][4];
  auto load = [&](int d, int s) {
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      wg_load_raw<YBF>(g.dY, g.ldY, g.nout, i0, s + h * WG_S, s1, s0, tid, ry[d][h]);
      wg_load_raw<XBF>(g.X, g.ldX, g.K, j0, s + h * WG_S, s1, s0, tid, rx[d][h]);
    }
  };
  if (s0 < s1) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (s0 + d * STEP < s1) load(d, s0 + d * STEP);
  }
  int buf = 0;
  for (int base = s0; base < s1; base += D * STEP) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = base + d * STEP;
      if (s >= s1) break;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        // bf16 rows go to LDS as loaded (masked); fp32 rows are rounded (and split under X3)
        if constexpr (YBF) {
          wg_put_bf((sm.sY[buf] + h * WG_S * WG_LD), ry[d][h], g.nout, i0, s + h * WG_S, s1, tid);
          if (do_rs) {
            f32x4 vy[4];
            wg_widen<true>(ry[d][h], g.nout, i0, s + h * WG_S, s1, tid, vy);
#pragma unroll
            for (int q = 0; q < 4; ++q) rsum += vy[q];
          }
        } else {
          f32x4 vy[4];
          wg_widen<false>(ry[d][h], g.nout, i0, s + h * WG_S, s1, tid, vy);
          if (do_rs) {
#pragma unroll
            for (int q = 0; q < 4; ++q) rsum += vy[q];
          }
          wg_store<X3>((sm.sY[buf] + h * WG_S * WG_LD), (sm.sY[buf] + (NI - 1 + h) * WG_S * WG_LD), tid, vy);
        }
        if constexpr (XBF) {
          wg_put_bf((sm.sX[buf] + h * WG_S * WG_LD), rx[d][h], g.K, j0, s + h * WG_S, s1, tid);
        } else {
          f32x4 vx[4];
          wg_widen<false>(rx[d][h], g.K, j0, s + h * WG_S, s1, tid, vx);
          wg_store<X3>((sm.sX[buf] + h * WG_S * WG_LD), (sm.sX[buf] + (NI - 1 + h) * WG_S * WG_LD), tid, vx);
        }
      }
      __syncthreads();
      if (s + D * STEP < s1) load(d, s + D * STEP);  // this ring entry is free again: refill D steps ahead
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        bf16x8_t fa[4], fb[4], la[4], lb[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          fa[a] = wg_frag((sm.sY[buf] + h * WG_S * WG_LD), wi + 16 * a, lane);
          if constexpr (X3) la[a] = wg_frag((sm.sY[buf] + (NI - 1 + h) * WG_S * WG_LD), wi + 16 * a, lane);
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          fb[b] = wg_frag((sm.sX[buf] + h * WG_S * WG_LD), wj + 16 * b, lane);
          if constexpr (X3) lb[b] = wg_frag((sm.sX[buf] + (NI - 1 + h) * WG_S * WG_LD), wj + 16 * b, lane);
        }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            if constexpr (X3) {
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(la[a], fb[b], acc[a][b], 0, 0, 0);
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], lb[b], acc[a][b], 0, 0, 0);
            }
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
          }
      }
      buf ^= 1;
    }
  }
  float* slab = g.slab + ((long)(z * g.tiles + ti * g.tj + tj) * 4 + w) * 16 * 256;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) *(f32x4*)(slab + (a * 4 + b) * 256 + lane * 4) = acc[a][b];
  if (do_rs) {
    *(f32x4*)&sm.srs[tid >> 5][4 * (tid & 31)] = rsum;
    __syncthreads();
    if (tid < WG_T) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) t += sm.srs[k][tid];
      g.rs_slab[(long)z * 256 + i0 + tid] = t;
    }
  }
}

template <bool X3, bool YBF, bool XBF>
__global__ __launch_bounds__(256) void k_wgrad(WGrad g) {
  __shared__ __attribute__((aligned(16))) WgLds sm;
  // XCD-aware order: workgroups are dealt to the 8 XCDs round-robin by linear id, so the tiles of
  // one sample range (which read the same dY and X rows) get ids on one XCD and share its L2
  // (launch_wgrad makes the range count a multiple of 8)
  const int tiles = gridDim.x * gridDim.y;
  const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int slot = L >> 3, tile = slot % tiles;
  const int z = (slot / tiles) * 8 + (L & 7);
  wgrad_tile<X3, YBF, XBF>(g, tile % gridDim.x, tile / gridDim.x, z, sm);
}

// several weight gradients of one operand format in one launch (the layers of an MLP's backward):
// workgroup b belongs to descriptor k with start[k] <= b < start[k+1] and is placed within it as in
// k_wgrad. One format per launch: a run-time switch would size the registers for the widest variant
// (measured: 256 VGPRs + 123 AGPRs, occupancy 1, where the bf16 variant takes 190 + 64)
template <bool X3, bool YBF, bool XBF>
__device__ __forceinline__ void wgrad_group_body(const WGradGroup& G) {
  __shared__ __attribute__((aligned(16))) WgLds sm;
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < G.n && b >= G.start[k + 1]) ++k;
  const WGrad& g = G.d[k];
  const int L = b - G.start[k];
  const int slot = L >> 3, tile = slot % g.tiles;
  const int z = (slot / g.tiles) * 8 + (L & 7);
  const int nti = g.tiles / g.tj;
  wgrad_tile<X3, YBF, XBF>(g, tile % nti, tile / nti, z, sm);
}
template <bool X3, bool YBF, bool XBF>
__global__ __launch_bounds__(256) void k_wgrad_group(WGradGroup G) {
  wgrad_group_body<X3, YBF, XBF>(G);
}
// bf16 rows both ways (the bulk of the bf16 training backward): held to two waves per SIMD, as k_wgrad's
template <>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_wgrad_group<false, true, true>(WGradGroup G) {
  wgrad_group_body<false, true, true>(G);
}

// dW[i][c0 + j] += sum_z slab; bsum[i] (+ bsum2[i]) += sum_z rs_slab[z][i]. One thread per 4 rows of
// one column (a slab lane's float4) and per group of WG_ZG consecutive slabs; the groups' sums meet
// in fp32 atomics (as the generic kernel's split-K does).
#define WG_ZG 8
__device__ __forceinline__ void wgrad_reduce_at(const WGrad& g, int u) {  // u: (z group, tile, w, a, b, lane)
  const int per_tile = 4 * 16 * 64;
  const int nu = g.tiles * per_tile;
  const int zg = u / nu, v = u - zg * nu;
  const int z0 = zg * WG_ZG, z1 = min(g.nz, z0 + WG_ZG);
  if (z0 < g.nz) {
    const int t = v / per_tile, rem = v - t * per_tile;
    const int w = rem / (16 * 64), ab = (rem / 64) & 15, lane = rem & 63;
    const int a = ab >> 2, b = ab & 3;
    const int ti = t / g.tj, tj = t - ti * g.tj;
    const int i = ti * WG_T + (w >> 1) * 64 + 16 * a + 4 * (lane >> 4);
    const int j = tj * WG_T + (w & 1) * 64 + 16 * b + (lane & 15);
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < WG_ZG; ++k)
      if (z0 + k < z1) s += *(const f32x4*)(g.slab + ((long)((z0 + k) * g.tiles + t) * 4 + w) * 16 * 256 + ab * 256 + lane * 4);
    if (j < g.K && j >= g.j0) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (i + r < g.nout) atomicAdd(g.dW + (long)(i + r) * g.ldw + j, s[r]);
    }
  }
  // column sums: thread (z group, column) for the first nout * z-groups threads
  if (g.rs_slab && u < g.nout * ((g.nz + WG_ZG - 1) / WG_ZG)) {
    const int c = u % g.nout, q0 = (u / g.nout) * WG_ZG;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < WG_ZG; ++k)
      if (q0 + k < g.nz) t += g.rs_slab[(long)(q0 + k) * 256 + c];
    if (g.bsum) atomicAdd(g.bsum + c, t);
    if (g.bsum2) atomicAdd(g.bsum2 + c, t);
  }
}

__global__ void k_wgrad_reduce(WGrad g) { wgrad_reduce_at(g, blockIdx.x * blockDim.x + threadIdx.x); }

__global__ void k_wgrad_reduce_group(WGradGroup G) {
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < G.n && b >= G.rstart[k + 1]) ++k;
  wgrad_reduce_at(G.d[k], (b - G.rstart[k]) * blockDim.x + threadIdx.x);
}

// ------------------------------------------------------------------------------------------
// k_wgrad_dma: the bf16 x bf16 weight gradients of a group (the bulk of the bf16 training backward),
// one workgroup per (product, sample range) owning the whole <= 256 x 256 dW: 8 waves of 64 outputs x
// 128 inputs (4 x 8 MFMA blocks, 128 accumulator registers). dY and X rows stream through a 4-slot LDS
// ring of 32-sample stages by LDS-DMA (global_load_lds_dwordx4; no staging registers, 3 stages in
// flight, counted vmcnt waits — the loop stores nothing), each image [sample][256 columns] with its
// 16-B chunks XOR-swizzled per row so the ds_read_b64_tr_b16 fragment reads are conflict-free
// (rows 8g + q of a 32-lane half land in 16 distinct chunk positions). The column sums of dY (bias /
// latent-row gradients) are one more MFMA per out-block against a ones fragment. Partial tiles go to
// k_wgrad_group's slab layout (its 128 x 128 tiles, 64 x 64 quadrants), so k_wgrad_reduce_group sums
// them unchanged. The register-staged k_wgrad_group kept 128 registers of prefetch for 4 steps and ran
// the groups at ~150 TFLOP/s (profiles/r6a, r6b).
// ------------------------------------------------------------------------------------------
#define WD_ST 32                 // samples per stage
#define WD_NB 4                  // ring slots
#define WD_IMG (WD_ST * 512)     // one image: 32 rows x 256 bf16
#define WD_SLOT (2 * WD_IMG)     // dY image, X image

__device__ __forceinline__ int wd_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

// fragment (16 columns c0 .. c0 + 15 of the image, rows 0..31 as k): lane i gets column c0 + (i & 15),
// rows 8 (i >> 4) + 0..7 (wg_frag's tr16 pattern on the swizzled image)
__device__ __forceinline__ bf16x8_t wd_frag(const unsigned char* img, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) wv4s lds_v4s;
  const int c = c0 + 4 * p;
  const int r0 = 8 * g + q, r1 = r0 + 4;
  const unsigned a0 = (unsigned)(uintptr_t)(img + r0 * 512 + (((c >> 3) ^ wd_swz(r0)) << 4) + (c & 7) * 2);
  const unsigned a1 = (unsigned)(uintptr_t)(img + r1 * 512 + (((c >> 3) ^ wd_swz(r1)) << 4) + (c & 7) * 2);
  const wv4s x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(uintptr_t)a0);
  const wv4s x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(uintptr_t)a1);
  bf16x8_t f;
  const short e[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  __builtin_memcpy(&f, e, 16);
  return f;
}

template <int N>
__device__ __forceinline__ void wd_wait() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__global__ __launch_bounds__(512) void k_wgrad_dma(WGradGroup G) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < G.n && b >= G.start[k + 1]) ++k;
  const WGrad& g = G.d[k];
  const int z = b - G.start[k];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = g.M_dev ? *g.M_dev : g.n;
  const int spb = g.spb ? g.spb : ((n + g.nz - 1) / g.nz + 2 * WG_S - 1) / (2 * WG_S) * (2 * WG_S);
  const int s0 = z * spb, s1 = min(n, s0 + spb);
  const int nst = s1 > s0 ? (s1 - s0 + WD_ST - 1) / WD_ST : 0;
  const int i0 = (wave & 3) * 64, j0 = (wave >> 2) * 128;
  const bool rs = g.rs_slab != nullptr && j0 == 0;
  const unsigned short* Y = (const unsigned short*)g.dY;
  const unsigned short* X = (const unsigned short*)g.X;
  // this wave's 4 pieces of a stage: images 0 (dY) / 1 (X), pieces 2 wave, 2 wave + 1 (rows 4 wave ..
  // 4 wave + 3); lane: row 2 piece + (lane >> 5), physical chunk lane & 31
  auto issue = [&](int st) {
    const unsigned char* slot = smem + (st % WD_NB) * WD_SLOT;
#pragma unroll
    for (int im = 0; im < 2; ++im) {
      const unsigned short* base = im ? X : Y;
      const long ld = im ? g.ldX : g.ldY;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int piece = 2 * wave + h;
        const int r = 2 * piece + (lane >> 5);
        int c = (lane & 31) ^ wd_swz(r);
        c = 8 * c + 8 <= ld ? c : 0;                          // chunks past the row: any in-bounds bytes
        const int srow = min(s0 + st * WD_ST + r, s1 - 1);   // rows past the range: zeroed in LDS
        const unsigned short* src = base + (size_t)srow * ld + 8 * c;
        const unsigned m0 = (unsigned)(uintptr_t)(slot + im * WD_IMG + piece * 1024);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory");
      }
    }
  };
  f32x4 acc[4][8], rsum[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    rsum[a] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  bf16x8_t ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
  for (int st = 0; st < WD_NB - 1 && st < nst; ++st) issue(st);
  for (int st = 0; st < nst; ++st) {
    // certify stage st: this wave's pieces of the stages after it may stay in flight, then the barrier
    const int after = min(st + WD_NB - 2, nst - 1) - st;
    if (after >= 2) wd_wait<8>();
    else if (after == 1) wd_wait<4>();
    else wd_wait<0>();
    __syncthreads();
    unsigned char* slot = smem + (st % WD_NB) * WD_SLOT;
    const int vr = s1 - (s0 + st * WD_ST);  // valid rows of this stage
    if (vr < WD_ST) {  // the range's last stage: rows past it read as zero (uniform branch)
      for (int e = tid; e < 2 * (WD_ST - vr) * 32; e += 512) {
        const int im = e / ((WD_ST - vr) * 32), rem = e % ((WD_ST - vr) * 32);
        *(uint4*)(slot + im * WD_IMG + (vr + rem / 32) * 512 + (rem % 32) * 16) = make_uint4(0u, 0u, 0u, 0u);
      }
      __syncthreads();
    }
    if (st + WD_NB - 1 < nst) issue(st + WD_NB - 1);  // the slot of stage st - 1: every wave is past it
    bf16x8_t fa[4], fb[8];
#pragma unroll
    for (int a = 0; a < 4; ++a) fa[a] = wd_frag(slot, i0 + 16 * a, lane);
#pragma unroll
    for (int c = 0; c < 8; ++c) fb[c] = wd_frag(slot + WD_IMG, j0 + 16 * c, lane);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[c], acc[a][c], 0, 0, 0);
      if (rs) rsum[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], ones, rsum[a], 0, 0, 0);
    }
  }
  // partial tiles in k_wgrad_group's slab layout: 128 x 128 tile (ti, tj), quadrant w' = 2 wr + wc
  const int nti = (g.nout + WG_T - 1) / WG_T;
  const int ti = i0 / WG_T, wr = (i0 % WG_T) / 64;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int jc = j0 + 64 * (c / 4);
    const int tj = jc / WG_T, wc = (jc % WG_T) / 64;
    if (ti >= nti || tj >= g.tj) continue;
    const int t = ti * g.tj + tj;
    float* slab = g.slab + ((long)(z * g.tiles + t) * 4 + (2 * wr + wc)) * 16 * 256;
#pragma unroll
    for (int a = 0; a < 4; ++a) *(f32x4*)(slab + (a * 4 + (c % 4)) * 256 + lane * 4) = acc[a][c];
  }
  if (rs && (lane & 15) == 0) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) g.rs_slab[(long)z * 256 + i0 + 16 * a + 4 * (lane >> 4) + r] = rsum[a][r];
  }
}

// ------------------------------------------------------------------------------------------
// k_wgrad_f32: exact-fp32 weight gradients dW += dY^T X (+ column sums of dY) for the exact-fp32
// executors (the sdf_pdf training step's 'fp32' precision), v_mfma_f32_16x16x4_f32 with fp32 operands
// as stored — the products k_gemm_t's atomic split-K computes, without its register staging (8 VALU
// instructions per MFMA, profiles/r4q_sq_k_gemm_t) or its 4.7 M atomics per 36k-row product.
// Workgroup = one 128 x 128 tile of dW (8 waves of 32 x 64) over one sample range; dY and X rows of the
// tile stream through a 4-slot LDS ring of 16-sample stages by LDS-DMA (8 KiB each, [sample][128 cols],
// 16-B chunks XOR-swizzled by 4 on odd rows so the ds_read_b32 fragment reads — rows 4 ks + (lane >> 4),
// 16 consecutive columns — are conflict-free). Partial tiles go to the slab layout of k_wgrad (reduce
// unchanged); column sums are MFMAs of the dY fragments against ones.
// ------------------------------------------------------------------------------------------
#define WF_ST 32                   // samples per stage
#define WF_NB 4                    // ring slots
#define WF_IMG (WF_ST * WG_T * 4)  // one image: 32 rows x 128 fp32
#define WF_SLOT (2 * WF_IMG)

__device__ __forceinline__ float wf_read(const unsigned char* img, int row, int col) {
  const int ch = (col >> 2) ^ ((row & 1) << 2);
  return *(const float*)(img + row * (WG_T * 4) + ch * 16 + (col & 3) * 4);
}

__global__ __launch_bounds__(512) void k_wgrad_f32(WGrad g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tiles = g.tiles;
  const int b = blockIdx.x;
  const int t = b % tiles, z = b / tiles;
  const int ti = t / g.tj, tj = t - ti * g.tj;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = g.M_dev ? *g.M_dev : g.n;
  const int spb = ((n + g.nz - 1) / g.nz + WF_ST - 1) / WF_ST * WF_ST;
  const int s0 = z * spb, s1 = min(n, s0 + spb);
  const int nst = s1 > s0 ? (s1 - s0 + WF_ST - 1) / WF_ST : 0;
  const int i0 = ti * WG_T, j0 = tj * WG_T;
  // 8 waves of 32 x 64 (two waves per SIMD: the fragment reads of one hide behind the other's MFMAs)
  const int wi = (wave >> 1) * 32, wj = (wave & 1) * 64;
  const bool rs = g.rs_slab != nullptr && tj == 0;
  // a wave's pieces of a stage: image im (0 dY, 1 X), 1 KiB pieces p = wave, wave + 8: rows 2 p, 2 p + 1
  // (32 chunks of 16 B each), LDS chunk q of row r holds source chunk q ^ 4 (r & 1)
  auto issue = [&](int st) {
    const unsigned char* slot = smem + (st % WF_NB) * WF_SLOT;
#pragma unroll
    for (int im = 0; im < 2; ++im)
#pragma unroll
    for (int h = 0; h < WF_ST / 16; ++h) {
      const float* base = im ? g.X : g.dY;
      const long ld = im ? g.ldX : g.ldY;
      const int c0 = im ? j0 : i0, cn = im ? g.K : g.nout;
      const int p = wave + 8 * h;
      const int r = 2 * p + (lane >> 5);
      const int q = (lane & 31) ^ ((r & 1) << 2);
      int c = c0 + 4 * q;
      c = (c < cn && c + 4 <= ld) ? c : 0;  // chunks past the columns: any in-bounds bytes (discarded)
      const int srow = min(s0 + st * WF_ST + r, s1 - 1);
      const float* src = base + (size_t)srow * ld + c;
      const unsigned m0 = (unsigned)(uintptr_t)(slot + im * WF_IMG + p * 1024);
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory");
    }
  };
  f32x4 acc[2][4], rsum[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    rsum[a] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int st = 0; st < WF_NB - 1 && st < nst; ++st) issue(st);
  for (int st = 0; st < nst; ++st) {
    const int after = min(st + WF_NB - 2, nst - 1) - st;  // stages issued after st: WF_OPS pieces each
    constexpr int WF_OPS = 2 * (WF_ST / 16);
    if (after >= 2) wd_wait<2 * WF_OPS>();
    else if (after == 1) wd_wait<WF_OPS>();
    else wd_wait<0>();
    __syncthreads();
    unsigned char* slot = smem + (st % WF_NB) * WF_SLOT;
    const int vr = s1 - (s0 + st * WF_ST);
    if (vr < WF_ST) {  // the range's last stage: rows past it read as zero (uniform branch)
      for (int e = tid; e < 2 * (WF_ST - vr) * 32; e += 512) {
        const int im = e / ((WF_ST - vr) * 32), rem = e % ((WF_ST - vr) * 32);
        *(uint4*)(slot + im * WF_IMG + (vr + rem / 32) * (WG_T * 4) + (rem % 32) * 16) = make_uint4(0u, 0u, 0u, 0u);
      }
      __syncthreads();
    }
    if (st + WF_NB - 1 < nst) issue(st + WF_NB - 1);  // the slot of stage st - 1: every wave is past it
    float fa[WF_ST / 4][2], fb[WF_ST / 4][4];
#pragma unroll
    for (int ks = 0; ks < WF_ST / 4; ++ks) {
      const int row = 4 * ks + (lane >> 4);
#pragma unroll
      for (int a = 0; a < 2; ++a) fa[ks][a] = wf_read(slot, row, wi + 16 * a + (lane & 15));
#pragma unroll
      for (int c = 0; c < 4; ++c) fb[ks][c] = wf_read(slot + WF_IMG, row, wj + 16 * c + (lane & 15));
    }
#pragma unroll
    for (int ks = 0; ks < WF_ST / 4; ++ks) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[ks][a], fb[ks][c], acc[a][c], 0, 0, 0);
      // the column sums of the wave pair's 32 dY columns, one block per wave (even: a = 0, odd: a = 1), so
      // both waves of a pair issue the same MFMA count between barriers
      if (rs) rsum[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[ks][wave & 1], 1.0f, rsum[0], 0, 0, 0);
    }
  }
  // partial tile in k_wgrad's slab layout: quadrant q = 2 (wi / 64) + wj / 64 (64 x 64, blocks (a', c) of
  // 16 x 16, a' = (wi % 64) / 16 + a), the lane's float4
  const int qd = 2 * (wi / 64) + wj / 64, a0 = (wi % 64) / 16;
  float* slab = g.slab + ((long)(z * tiles + t) * 4 + qd) * 16 * 256;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) *(f32x4*)(slab + ((a0 + a) * 4 + c) * 256 + lane * 4) = acc[a][c];
  if (rs && (lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) g.rs_slab[(long)z * 256 + i0 + wi + 16 * (wave & 1) + 4 * (lane >> 4) + r] = rsum[0][r];
  }
}

// can k_wgrad_f32 take this product (16-B addressable rows, whole 16-B chunks of columns)
bool wgrad_f32_fits(const WGrad& g) {
  return !g.x3 && !g.ybf && !g.xbf && g.nout >= 1 && g.nout <= 256 && g.K >= 1 && g.K <= 256 && g.ldY >= 4 &&
         g.ldX >= 4 && g.ldY % 4 == 0 && g.ldX % 4 == 0 && ((uintptr_t)g.dY & 15) == 0 && ((uintptr_t)g.X & 15) == 0;
}

static int wgrad_reduce_blocks(const WGrad& g);

int launch_wgrad_f32(WGrad g, int n_host, hipStream_t s) {
  if (n_host <= 0) return 0;
  if (!wgrad_f32_fits(g)) return -1;
  const int ti = (g.nout + WG_T - 1) / WG_T, tj = (g.K + WG_T - 1) / WG_T;
  g.tj = tj;
  g.tiles = ti * tj;
  // sample ranges: about two workgroups per CU, within the slab region (tiles x nz <= 4 WG_MAX_Z)
  int nz = (512 + g.tiles - 1) / g.tiles;
  nz = std::min(nz, std::max(1, (n_host + 4 * WF_ST - 1) / (4 * WF_ST)));  // at least 4 stages per range
  nz = std::max(1, std::min(nz, std::min(WG_MAX_Z, 4 * WG_MAX_Z / g.tiles)));
  g.nz = nz;
  g.n = n_host;
  g.rs_slab = (g.bsum || g.bsum2) ? g.slab + (size_t)WG_MAX_Z * 4 * WG_TILE_FLOATS : nullptr;
  static bool attr[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64 || !attr[dev]) {
    if (hipFuncSetAttribute((const void*)k_wgrad_f32, hipFuncAttributeMaxDynamicSharedMemorySize, WF_NB * WF_SLOT) !=
        hipSuccess)
      return -1;
    if (dev >= 0 && dev < 64) attr[dev] = true;
  }
  hipLaunchKernelGGL(k_wgrad_f32, dim3(g.tiles * g.nz), dim3(512), WF_NB * WF_SLOT, s, g);
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(wgrad_reduce_blocks(g)), dim3(256), 0, s, g);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

static int wgrad_reduce_blocks(const WGrad& g) {
  const int nred = g.tiles * 4 * 16 * 64 * ((g.nz + WG_ZG - 1) / WG_ZG);
  return ((nred > 256 ? nred : 256) + 255) / 256;
}

size_t wgrad_slab_floats() { return (size_t)WG_MAX_Z * 4 * WG_TILE_FLOATS + (size_t)WG_MAX_Z * 256; }

int launch_wgrad(WGrad g, int n_host, hipStream_t s) {
  if (n_host <= 0) return 0;
  const int ti = (g.nout + WG_T - 1) / WG_T, tj = (g.K + WG_T - 1) / WG_T;
  g.tj = tj;
  g.tiles = ti * tj;
  // samples per workgroup: enough workgroups to cover the CUs, at most WG_MAX_Z slabs
  int nz = (n_host + 383) / 384;
  nz = nz < 1 ? 1 : (nz > WG_MAX_Z ? WG_MAX_Z : nz);
  nz = (nz + 7) / 8 * 8;  // a multiple of 8 for the XCD-aware order (trailing ranges may be empty)
  // whole 64-sample steps; with a device count (n_host = its capacity) the kernel derives them
  g.spb = g.M_dev ? 0 : ((n_host + nz - 1) / nz + 2 * WG_S - 1) / (2 * WG_S) * (2 * WG_S);
  g.nz = nz;
  g.n = n_host;
  g.rs_slab = (g.bsum || g.bsum2) ? g.slab + (size_t)WG_MAX_Z * 4 * WG_TILE_FLOATS : nullptr;
  const dim3 grid(ti, tj, g.nz);
  if (g.x3) hipLaunchKernelGGL((k_wgrad<true, false, false>), grid, dim3(256), 0, s, g);
  else if (g.ybf && g.xbf) hipLaunchKernelGGL((k_wgrad<false, true, true>), grid, dim3(256), 0, s, g);
  else if (g.ybf) hipLaunchKernelGGL((k_wgrad<false, true, false>), grid, dim3(256), 0, s, g);
  else if (g.xbf) hipLaunchKernelGGL((k_wgrad<false, false, true>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((k_wgrad<false, false, false>), grid, dim3(256), 0, s, g);
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(wgrad_reduce_blocks(g)), dim3(256), 0, s, g);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ANR_WG_DMA (read per call, default 1): the bf16 x bf16 products of a group on k_wgrad_dma. Measured
// (tools/gemm_probe grouptime, 16 products of 256 x 256 at 24,893 rows, 16 sample ranges): 111 us per
// group vs 188 us for k_wgrad_group, identical sums; bf16_all step 1.160 -> 1.064 ms (profiles/r7a)
static bool wgrad_dma_on() {
  const char* v = getenv("ANR_WG_DMA");
  return !(v && v[0] == '0');
}
// what k_wgrad_dma assumes of a product: one workgroup covers <= 256 x 256 outputs, rows of >= 8 bf16
// (chunk 0 stands in for the chunks past a row) in 16-B aligned rows (global_load_lds_dwordx4)
static bool wgrad_dma_fits(const WGrad& g) {
  return g.nout <= 256 && g.K <= 256 && g.ldY >= 8 && g.ldX >= 8 && g.ldY % 8 == 0 && g.ldX % 8 == 0 &&
         ((uintptr_t)g.dY & 15) == 0 && ((uintptr_t)g.X & 15) == 0;
}

int launch_wgrad_group(const WGrad* d, int nd, int n_host, int nz, float* slab, size_t slab_floats, hipStream_t s) {
  if (n_host <= 0 || nd <= 0) return 0;
  nz = nz < 8 ? 8 : (nz > WG_MAX_Z ? WG_MAX_Z : (nz + 7) / 8 * 8);
  WGradGroup G{};
  size_t used = 0;
  // formats: 0 split fp32, 1 bf16 x bf16 on k_wgrad_dma, 2 / 3 / 4 mixed / fp32 rows, 5 bf16 x bf16 on
  // k_wgrad_group (switched off, or a product k_wgrad_dma does not take)
  const bool dma = wgrad_dma_on();
  auto fmt = [dma](const WGrad& g) {
    return g.x3 ? 0 : (g.ybf && g.xbf) ? (dma && wgrad_dma_fits(g) ? 1 : 5) : g.ybf ? 2 : g.xbf ? 3 : 4;
  };
  auto issue = [&]() {
    if (G.n == 0) return;
    for (int v = 0; v < 6; ++v) {  // one product launch per operand format present, one reduce for all
      WGradGroup H{};
      for (int k = 0; k < G.n; ++k)
        if (fmt(G.d[k]) == v) {
          H.d[H.n] = G.d[k];
          H.start[H.n + 1] = H.start[H.n] + G.start[k + 1] - G.start[k];
          ++H.n;
        }
      if (!H.n) continue;
      const dim3 grid(H.start[H.n]);
      if (v == 1) {
        // one workgroup per (product, sample range): the whole <= 256 x 256 dW of the range
        WGradGroup D = H;
        for (int q = 0; q < H.n; ++q) D.start[q + 1] = D.start[q] + H.d[q].nz;
        static bool attr[64] = {};  // the dynamic-LDS attribute, once per device
        int dev = 0;
        (void)hipGetDevice(&dev);
        bool ok = dev >= 0 && dev < 64 && attr[dev];
        if (!ok) {
          ok = hipFuncSetAttribute((const void*)k_wgrad_dma, hipFuncAttributeMaxDynamicSharedMemorySize, WD_NB * WD_SLOT) == hipSuccess;
          if (ok && dev >= 0 && dev < 64) attr[dev] = true;
        }
        if (ok) {
          hipLaunchKernelGGL(k_wgrad_dma, dim3(D.start[D.n]), dim3(512), WD_NB * WD_SLOT, s, D);
          continue;
        }
        (void)hipGetLastError();  // the attribute failed: the register-staged kernel below
      }
      if (v == 0) hipLaunchKernelGGL((k_wgrad_group<true, false, false>), grid, dim3(256), 0, s, H);
      else if (v == 1 || v == 5) hipLaunchKernelGGL((k_wgrad_group<false, true, true>), grid, dim3(256), 0, s, H);
      else if (v == 2) hipLaunchKernelGGL((k_wgrad_group<false, true, false>), grid, dim3(256), 0, s, H);
      else if (v == 3) hipLaunchKernelGGL((k_wgrad_group<false, false, true>), grid, dim3(256), 0, s, H);
      else hipLaunchKernelGGL((k_wgrad_group<false, false, false>), grid, dim3(256), 0, s, H);
    }
    hipLaunchKernelGGL(k_wgrad_reduce_group, dim3(G.rstart[G.n]), dim3(256), 0, s, G);
    G = WGradGroup{};
    used = 0;
  };
  // sample ranges per format: each format's launch should fill the chip on its own (the launches of a
  // flush run one after another), so a format with little work — the few small fp32-row products of the
  // NeRF heads (rgb_fc 3 x 128, view_fc 128 x 283: 1 - 3 tiles), or a short tail of k_wgrad_dma products
  // (one 512-thread workgroup per product and range) — gets more, shorter ranges: workgroups per range
  // summed over the format's products, ranges up to WG_MAX_Z (k_wgrad_dma: 32, its partial slabs are
  // whole 256 x 256 tiles). ANR_WG_FILL=0: every product at nz (ANR_WG_GROUP_NZ).
  int fz[6] = {nz, nz, nz, nz, nz, nz};
  {
    const char* fe = getenv("ANR_WG_FILL");
    if (!(fe && fe[0] == '0')) {
      int per[6] = {0, 0, 0, 0, 0, 0};  // workgroups per sample range
      for (int k = 0; k < nd; ++k) {
        const int v = fmt(d[k]);
        per[v] += v == 1 ? 1 : ((d[k].nout + WG_T - 1) / WG_T) * ((d[k].K + WG_T - 1) / WG_T);
      }
      for (int v = 0; v < 6; ++v) {
        if (!per[v]) continue;
        const int want = v == 1 ? 256 : 512, cap = v == 1 ? 32 : WG_MAX_Z;
        const int z = ((want + per[v] - 1) / per[v] + 7) / 8 * 8;
        fz[v] = z < nz ? nz : (z > cap ? (cap > nz ? cap : nz) : z);
      }
    }
  }
  for (int k = 0; k < nd; ++k) {
    WGrad g = d[k];
    g.tj = (g.K + WG_T - 1) / WG_T;
    g.tiles = ((g.nout + WG_T - 1) / WG_T) * g.tj;
    // a descriptor's slabs are (nz, tile) partial tiles, then (nz, 256) column sums; nz halves (not below 8)
    // until the descriptor fits the region on its own
    int z = fz[fmt(g)];
    auto need = [&](int zz) { return (size_t)zz * g.tiles * WG_TILE_FLOATS + ((g.bsum || g.bsum2) ? (size_t)zz * 256 : 0); };
    while (z > 8 && need(z) > slab_floats) z = z / 16 * 8 > 8 ? z / 16 * 8 : 8;
    if (need(z) > slab_floats) return -1;
    if (G.n == WG_GROUP_MAX || used + need(z) > slab_floats) issue();  // the region is reused in stream order
    g.nz = z;
    g.n = n_host;
    g.spb = g.M_dev ? 0 : ((n_host + z - 1) / z + 2 * WG_S - 1) / (2 * WG_S) * (2 * WG_S);
    g.slab = slab + used;
    g.rs_slab = (g.bsum || g.bsum2) ? g.slab + (size_t)z * g.tiles * WG_TILE_FLOATS : nullptr;
    used += need(z);
    G.d[G.n] = g;
    G.start[G.n + 1] = G.start[G.n] + g.tiles * z;
    G.rstart[G.n + 1] = G.rstart[G.n] + wgrad_reduce_blocks(g);
    ++G.n;
  }
  issue();
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace anr
