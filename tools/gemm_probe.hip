// gemm_probe.hip — times the training executor's layer GEMM kernels in isolation on one stream
// (hipEvents around R back-to-back launches -> mean us per launch, the launch gap included as the
// step sees it) for a range of row counts M at one 256 x 256 layer, next to an HBM copy of the same
// activation bytes and an empty kernel. Built by `make probe` (links the library's objects); run on
// the GPU box: tools/gemm_probe [M ...]. One JSON line per (kernel, M).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <functional>
#include <string>
#include <vector>

#include "../animatable_nerf_amd/csrc/anr_common.h"
#include "../animatable_nerf_amd/csrc/anr_kernels.h"
#include "../animatable_nerf_amd/csrc/anr_train.h"

using namespace anr;
namespace anr {
// the library's profiling slots (anr_capi.hip) are not linked into the probe: profiling off
ProfSlot* prof_begin(hipStream_t, int) { return nullptr; }
int prof_end(ProfSlot*, hipStream_t) { return 0; }
}  // namespace anr
namespace anr {
void rg_timing_buffer(unsigned long long* p);  // the probe's RG_TIMING build of anr_tgemm.hip
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_probe_empty() {}

// bf16 rows copy: the activation traffic of one bf16 layer (M x 256 in, M x 256 out)
__global__ void k_probe_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, long n16) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) dst[i] = src[i];
}

// LDS-DMA stream rate: every workgroup (one per CU: a 128 KiB LDS ring) streams `bytes` from src (shared
// != 0: the same addresses for every workgroup, as a weight image; else its own region) in 1 KiB
// pieces, each wave issuing every W-th piece and keeping at most DEPTH of its pieces in flight
template <int W, int DEPTH>
__global__ __launch_bounds__(W * 64) void k_probe_dma(const unsigned char* src, long bytes, int shared) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const unsigned char* base = src + (shared ? 0 : (long)blockIdx.x * bytes);
  const int pieces = (int)(bytes / 1024);
  const unsigned lbase = (unsigned)(uintptr_t)lds;
  for (int p = w; p < pieces; p += W) {
    const unsigned dst = lbase + (unsigned)(p & 127) * 1024u;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(base + (long)p * 1024 + lane * 16),
                 "s"(dst)
                 : "memory");
    __builtin_amdgcn_s_waitcnt((DEPTH & 15) | (7 << 4) | (15 << 8) | ((DEPTH >> 4) << 14));
  }
  __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
}

// the same stream into registers (global_load_dwordx4), DEPTH loads in flight per wave
template <int W, int DEPTH>
__global__ __launch_bounds__(W * 64) void k_probe_vload(const unsigned char* src, long bytes, int shared, uint4* sink) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const unsigned char* base = src + (shared ? 0 : (long)blockIdx.x * bytes);
  const int pieces = (int)(bytes / 1024);
  uint4 acc = {0, 0, 0, 0};
  uint4 r[DEPTH];
  int p = w;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) r[d] = p + d * W < pieces ? *(const uint4*)(base + (long)(p + d * W) * 1024 + lane * 16) : uint4{0, 0, 0, 0};
  for (; p < pieces; p += DEPTH * W) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      acc.x ^= r[d].x; acc.y ^= r[d].y; acc.z ^= r[d].z; acc.w ^= r[d].w;
      const int q = p + (d + DEPTH) * W;
      if (q < pieces) r[d] = *(const uint4*)(base + (long)q * 1024 + lane * 16);
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}

__global__ void k_probe_fill(float* p, long n, unsigned seed, float scale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u + seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  p[i] = scale * ((float)(x & 0xffffff) / 16777216.0f - 0.5f);
}

// bytes of two device buffers equal (row-GEMM geometry variants compute each output in the same order)
static bool same_bytes(const void* a, const void* b, size_t n) {
  std::vector<unsigned char> x(n), y(n);
  CK(hipMemcpy(x.data(), a, n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), b, n, hipMemcpyDeviceToHost));
  return x == y;
}

static double max_rel_diff(const float* a, const float* b, size_t n) {
  std::vector<float> x(n), y(n);
  CK(hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost));
  double m = 0, sc = 0;
  for (size_t i = 0; i < n; ++i) {
    m = std::max(m, (double)std::fabs(x[i] - y[i]));
    sc = std::max(sc, (double)std::fabs(y[i]));
  }
  return sc > 0 ? m / sc : m;
}

static float time_us(hipStream_t s, int reps, const std::function<void()>& f) {
  for (int i = 0; i < 3; ++i) f();
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  CK(hipGetLastError());
  return ms * 1000.f / reps;
}

__global__ void k_probe_fill16(unsigned short* p, long n, unsigned seed, float scale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u + seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  const float v = scale * ((float)(x & 0xffffff) / 16777216.0f - 0.5f);
  p[i] = (unsigned short)(__float_as_uint(v) >> 16);
}

// grouped weight gradients against one launch per product: 16 products of mixed shapes and operand
// formats (bf16 / fp32 rows, K 63 / 256, nout 24 / 256, column sums into bsum / bsum2), the sample
// count on the device as in the training executor; every dW must be finite and match to 1e-5
static int group_check(hipStream_t s, int M) {
  const int NP = 16, cap = (M + 1023) / 1024 * 1024 + 4096;
  unsigned short *Y16, *X16;
  float *Y32, *X32, *dWr, *dWg, *bs, *slab, *slabg;
  int* Mdev;
  const long rows = (long)cap * 256;
  CK(hipMalloc(&Y16, NP * rows * 2));
  CK(hipMalloc(&X16, NP * rows * 2));
  CK(hipMalloc(&Y32, NP * rows * 4));
  CK(hipMalloc(&X32, NP * rows * 4));
  CK(hipMalloc(&dWr, NP * 256L * 256 * 4));
  CK(hipMalloc(&dWg, NP * 256L * 256 * 4));
  CK(hipMalloc(&bs, NP * 4 * 256 * 4));
  CK(hipMalloc(&slab, wgrad_slab_floats() * 4));
  CK(hipMalloc(&slabg, 4 * wgrad_slab_floats() * 4));
  CK(hipMalloc(&Mdev, 4));
  CK(hipMemcpy(Mdev, &M, 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_probe_fill16, dim3((unsigned)((NP * rows + 255) / 256)), dim3(256), 0, s, Y16, NP * rows, 11u, 0.02f);
  hipLaunchKernelGGL(k_probe_fill16, dim3((unsigned)((NP * rows + 255) / 256)), dim3(256), 0, s, X16, NP * rows, 12u, 2.f);
  hipLaunchKernelGGL(k_probe_fill, dim3((unsigned)((NP * rows + 255) / 256)), dim3(256), 0, s, Y32, NP * rows, 13u, 0.02f);
  hipLaunchKernelGGL(k_probe_fill, dim3((unsigned)((NP * rows + 255) / 256)), dim3(256), 0, s, X32, NP * rows, 14u, 2.f);
  // stale slabs full of NaN: a partial slab the group forgets to write shows up
  CK(hipMemsetAsync(slabg, 0xff, 4 * wgrad_slab_floats() * 4, s));
  std::vector<WGrad> d(NP);
  for (int k = 0; k < NP; ++k) {
    WGrad& w = d[k];
    const int f = k % 4;  // 0 bf16 both, 1 fp32 dY + bf16 X, 2 fp32 both, 3 bf16 dY K=63 with two sums
    w.ybf = (f == 0 || f == 3);
    w.xbf = (f == 0 || f == 1 || f == 3);
    w.nout = (k % 5 == 4) ? 24 : 256;
    w.K = f == 3 ? 63 : 256;
    w.ldY = 256;
    w.ldX = f == 3 ? 64 : 256;
    w.dY = w.ybf ? (const float*)(Y16 + k * rows) : Y32 + k * rows;
    w.X = w.xbf ? (const float*)(X16 + k * rows) : X32 + k * rows;
    w.dW = dWr + k * 65536L; w.ldw = 256;
    w.bsum = (k % 2) ? bs + k * 1024 : nullptr;
    w.bsum2 = f == 3 ? bs + k * 1024 + 256 : nullptr;
    w.M_dev = Mdev;
  }
  CK(hipMemsetAsync(dWr, 0, NP * 256L * 256 * 4, s));
  CK(hipMemsetAsync(bs, 0, NP * 4 * 256 * 4, s));
  for (int k = 0; k < NP; ++k) {
    WGrad w = d[k];
    w.slab = slab;
    if (launch_wgrad(w, cap, s) != 0) return 1;
  }
  std::vector<float> ref(NP * 65536L), bref(NP * 1024L);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(ref.data(), dWr, ref.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(bref.data(), bs, bref.size() * 4, hipMemcpyDeviceToHost));
  for (int k = 0; k < NP; ++k) d[k].dW = dWg + k * 65536L;
  for (int nz : {16, 32, 64}) {
    CK(hipMemsetAsync(dWg, 0, NP * 256L * 256 * 4, s));
    CK(hipMemsetAsync(bs, 0, NP * 4 * 256 * 4, s));
    if (launch_wgrad_group(d.data(), NP, cap, nz, slabg, 4 * wgrad_slab_floats(), s) != 0) return 1;
    std::vector<float> got(NP * 65536L), bgot(NP * 1024L);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got.data(), dWg, got.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(bgot.data(), bs, bgot.size() * 4, hipMemcpyDeviceToHost));
    for (int k = 0; k < NP; ++k) {
      double m = 0, sc = 0, mb = 0, sb = 0;
      bool fin = true;
      for (long i = 0; i < 65536; ++i) {
        const float a = got[k * 65536L + i], r = ref[k * 65536L + i];
        fin = fin && std::isfinite(a);
        m = std::max(m, (double)std::fabs(a - r));
        sc = std::max(sc, (double)std::fabs(r));
      }
      for (long i = 0; i < 1024; ++i) {
        const float a = bgot[k * 1024L + i], r = bref[k * 1024L + i];
        fin = fin && std::isfinite(a);
        mb = std::max(mb, (double)std::fabs(a - r));
        sb = std::max(sb, (double)std::fabs(r));
      }
      printf("{\"group_check\": %d, \"nz\": %d, \"finite\": %d, \"dW_rel\": %.3g, \"bsum_rel\": %.3g, \"ybf\": %d, "
             "\"xbf\": %d, \"nout\": %d, \"K\": %d}\n", k, nz, fin ? 1 : 0, sc > 0 ? m / sc : m, sb > 0 ? mb / sb : mb,
             d[k].ybf, d[k].xbf, d[k].nout, d[k].K);
    }
  }
  fflush(stdout);
  return 0;
}

// one flushed group of NP bf16 x bf16 products (256 x 256, the step's bulk; column sums on every other)
// timed with the register-staged k_wgrad_group and with k_wgrad_dma (ANR_WG_DMA, read per call), at
// several sample-range counts; the two results compared (fixed inputs, relative to the max |dW|)
static int group_time(hipStream_t s, int M, int NP) {
  const int cap = (M + 1023) / 1024 * 1024 + 4096;
  const long rows = (long)cap * 256;
  unsigned short *Y16, *X16;
  float *dW, *dW2, *bs, *slab;
  int* Mdev;
  CK(hipMalloc(&Y16, NP * rows * 2));
  CK(hipMalloc(&X16, NP * rows * 2));
  CK(hipMalloc(&dW, NP * 65536L * 4));
  CK(hipMalloc(&dW2, NP * 65536L * 4));
  CK(hipMalloc(&bs, NP * 256L * 4));
  CK(hipMalloc(&slab, 4 * wgrad_slab_floats() * 4));
  CK(hipMalloc(&Mdev, 4));
  CK(hipMemcpy(Mdev, &M, 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_probe_fill16, dim3((unsigned)((NP * rows + 255) / 256)), dim3(256), 0, s, Y16, NP * rows, 21u, 0.02f);
  hipLaunchKernelGGL(k_probe_fill16, dim3((unsigned)((NP * rows + 255) / 256)), dim3(256), 0, s, X16, NP * rows, 22u, 2.f);
  std::vector<WGrad> d(NP);
  for (int k = 0; k < NP; ++k) {
    WGrad& w = d[k];
    w.ybf = 1; w.xbf = 1; w.nout = 256; w.K = 256; w.ldY = 256; w.ldX = 256;
    w.dY = (const float*)(Y16 + k * rows);
    w.X = (const float*)(X16 + k * rows);
    w.dW = dW + k * 65536L; w.ldw = 256;
    w.bsum = (k % 2) ? bs + k * 256 : nullptr;
    w.M_dev = Mdev;
  }
  const double fl = 2.0 * NP * M * 256.0 * 256.0, by = 2.0 * NP * M * 256.0 * 2.0;
  for (int nz : {8, 16, 32}) {
    for (int dma = 0; dma < 2; ++dma) {
      setenv("ANR_WG_DMA", dma ? "1" : "0", 1);
      for (int k = 0; k < NP; ++k) d[k].dW = (dma ? dW2 : dW) + k * 65536L;
      const float us = time_us(s, 20, [&] { launch_wgrad_group(d.data(), NP, cap, nz, slab, 4 * wgrad_slab_floats(), s); });
      printf("{\"group_time\": \"%s\", \"M\": %d, \"products\": %d, \"nz\": %d, \"us\": %.2f, \"TFLOPs\": %.1f, \"GBps\": %.1f}\n",
             dma ? "k_wgrad_dma" : "k_wgrad_group", M, NP, nz, us, fl / us * 1e-6, by / us * 1e-3);
      fflush(stdout);
    }
    // one clean accumulation each, compared
    CK(hipMemsetAsync(dW, 0, NP * 65536L * 4, s));
    CK(hipMemsetAsync(dW2, 0, NP * 65536L * 4, s));
    setenv("ANR_WG_DMA", "0", 1);
    for (int k = 0; k < NP; ++k) d[k].dW = dW + k * 65536L;
    launch_wgrad_group(d.data(), NP, cap, nz, slab, 4 * wgrad_slab_floats(), s);
    setenv("ANR_WG_DMA", "1", 1);
    for (int k = 0; k < NP; ++k) d[k].dW = dW2 + k * 65536L;
    launch_wgrad_group(d.data(), NP, cap, nz, slab, 4 * wgrad_slab_floats(), s);
    CK(hipStreamSynchronize(s));
    printf("{\"group_time_diff\": %.3g, \"nz\": %d}\n", max_rel_diff(dW2, dW, NP * 65536L), nz);
  }
  unsetenv("ANR_WG_DMA");
  fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "grouptime") {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return group_time(s, argc > 2 ? atoi(argv[2]) : 24893, argc > 3 ? atoi(argv[3]) : 16);
  }
  if (argc > 1 && std::string(argv[1]) == "groupcheck") {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return group_check(s, argc > 2 ? atoi(argv[2]) : 24893);
  }
  std::vector<int> Ms;
  for (int i = 1; i < argc; ++i) Ms.push_back(atoi(argv[i]));
  if (Ms.empty()) Ms = {6223, 12446, 24893, 49786, 99572};
  int Mmax = 0;
  for (int m : Ms) Mmax = m > Mmax ? m : Mmax;
  const int K = 256, N = 256, reps = 50;
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const long rowsz = (long)Mmax * 256;
  float *A, *C, *C2, *Mk, *W, *bias, *dW, *dW2, *bsum, *slab, *img_l = nullptr;
  unsigned short* Bimg;
  CK(hipMalloc(&A, rowsz * 4));
  CK(hipMalloc(&C, rowsz * 4));
  CK(hipMalloc(&C2, rowsz * 4));
  CK(hipMalloc(&dW2, 256 * 256 * 4));
  CK(hipMalloc(&Mk, rowsz * 4));
  CK(hipMalloc(&W, 256 * 256 * 4));
  CK(hipMalloc(&bias, 256 * 4));
  CK(hipMalloc(&dW, 256 * 256 * 4));
  CK(hipMalloc(&bsum, 256 * 4));
  CK(hipMalloc(&slab, wgrad_slab_floats() * 4));
  CK(hipMalloc(&Bimg, 2 * 256 * 256 * 2));
  hipLaunchKernelGGL(k_probe_fill, dim3((rowsz + 255) / 256), dim3(256), 0, s, A, rowsz, 1u, 2.f);
  hipLaunchKernelGGL(k_probe_fill, dim3((rowsz + 255) / 256), dim3(256), 0, s, Mk, rowsz, 2u, 2.f);
  hipLaunchKernelGGL(k_probe_fill, dim3(256), dim3(256), 0, s, W, 256L * 256, 3u, 0.1f);
  hipLaunchKernelGGL(k_probe_fill, dim3(1), dim3(256), 0, s, bias, 256L, 4u, 0.1f);
  // a bf16 image of random bits in the exponent range of the weights (values are irrelevant to timing)
  CK(hipMemsetAsync(Bimg, 0x3c, 2 * 256 * 256 * 2, s));
  CK(hipStreamSynchronize(s));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

  for (int M : Ms) {
    auto out = [&](const char* name, double us, double bytes, double flop) {
      printf("{\"kernel\": \"%s\", \"M\": %d, \"us\": %.2f, \"GBps\": %.1f, \"TFLOPs\": %.1f}\n", name, M, us,
             bytes / us * 1e-3, flop / us * 1e-6);
      fflush(stdout);
    };
    const double fl = 2.0 * M * K * N;
    // row GEMM, bf16 storage (training precision bf16: forward with bias+ReLU, backward with mask)
    for (int mode = 0; mode < 4; ++mode) {
      RGemm r{};
      r.N = N; r.nseg = 1;
      r.seg[0] = RGemmSeg{A, 256, K, Bimg, 256, 0, 256, 256L * 256};
      r.C = C; r.ldc = 256;
      const char* name = "";
      if (mode == 0) { r.abf = 1; r.cbf = 1; r.bias = bias; r.relu = 1; name = "rgemm_bf16_fwd"; }
      if (mode == 1) { r.abf = 1; r.cbf = 1; r.mask = Mk; r.ldm = 256; r.mbf = 1; name = "rgemm_bf16_bwd_mask"; }
      if (mode == 2) { r.bias = bias; r.relu = 1; name = "rgemm_f32io_bf16"; }
      if (mode == 3) { r.x3 = 1; r.bias = bias; r.relu = 1; name = "rgemm_x3_fwd"; }
      r.M = M;
      const double eb = (r.abf ? 2 : 4) + (r.cbf ? 2 : 4) + (r.mask ? (r.mbf ? 2 : 4) : 0);
      out(name, time_us(s, reps, [&] { launch_rgemm(r, M, s); }), (double)M * 256 * eb, fl);
      if (!r.x3) {
        // two streams, each with its own launches (the step's s / s2 chains): time per launch
        {  // independent pairs: s and s2 each run their own launches
          RGemm c1 = r, c2 = r;
          c2.C = C2;
          for (int i = 0; i < 3; ++i) { launch_rgemm(c1, M, s); launch_rgemm(c2, M, s2); }
          CK(hipDeviceSynchronize());
          hipEvent_t a0, a1;
          CK(hipEventCreate(&a0));
          CK(hipEventCreate(&a1));
          CK(hipEventRecord(a0, s));
          CK(hipStreamWaitEvent(s2, a0, 0));
          for (int i = 0; i < reps; ++i) { launch_rgemm(c1, M, s); launch_rgemm(c2, M, s2); }
          CK(hipEventRecord(a1, s2));
          CK(hipStreamWaitEvent(s, a1, 0));
          CK(hipEventRecord(a1, s));
          CK(hipEventSynchronize(a1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, a0, a1));
          const std::string v2 = std::string(name) + "_2streams_per_launch";
          out(v2.c_str(), ms * 1000.0 / (2 * reps), (double)M * 256 * eb, fl);
          CK(hipEventDestroy(a0));
          CK(hipEventDestroy(a1));
        }
      }
      {  // phase clocks of one launch (wave 0 of each workgroup; shader clock ticks, 100 MHz memtime
         // on gfx950 -> converted with the measured ratio below)
        const int nb = (M + 127) / 128;
        unsigned long long* tb;
        CK(hipMalloc(&tb, (size_t)nb * 16 * 8));
        CK(hipMemset(tb, 0, (size_t)nb * 16 * 8));
        rg_timing_buffer(tb);
        launch_rgemm(r, M, s);
        CK(hipStreamSynchronize(s));
        rg_timing_buffer(nullptr);
        std::vector<unsigned long long> h((size_t)nb * 16);
        CK(hipMemcpy(h.data(), tb, h.size() * 8, hipMemcpyDeviceToHost));
        CK(hipFree(tb));
        unsigned long long t0 = ~0ull, t1 = 0;
        double ph[16] = {};
        int cnt = 0;
        for (int b = 0; b < nb; ++b) {
          const unsigned long long* q = &h[(size_t)b * 16];
          if (!q[0] || !q[13]) continue;
          t0 = std::min(t0, q[0]);
          t1 = std::max(t1, q[13]);
          unsigned long long prev = q[0];
          for (int i = 1; i < 14; ++i) {
            if (!q[i]) continue;
            ph[i] += (double)(q[i] - prev);
            prev = q[i];
          }
          ++cnt;
        }
        printf("{\"phases\": \"%s\", \"M\": %d, \"wgs\": %d, \"span_ticks\": %llu", name, M, cnt, t1 - t0);
        for (int i = 1; i < 14; ++i)
          if (ph[i] > 0) printf(", \"t%d\": %.0f", i, ph[i] / cnt);
        printf("}\n");
      }
    }
    // generic fp32 / bf16x3 tile GEMMs (anr_gemm.hip), forward layout
    for (int mode = 0; mode < 2; ++mode) {
      GemmArgs g{};
      g.N = N; g.nseg = 1;
      g.seg[0] = GemmSeg{A, 256, 1, W, 1, 256, K};
      g.C = C; g.ldc = 256; g.bias = bias; g.relu = 1; g.ksplit = 1; g.M = M;
      g.x3 = mode;
      out(mode ? "gemm_b_x3_fwd" : "gemm_t_f32_fwd",
          time_us(s, reps, [&] { launch_gemm(g, dim3((N + 63) / 64, (M + 63) / 64, 1), s); }), (double)M * 256 * 8, fl);
      if (mode == 1 && lgemm_supported(g)) {
        if (!img_l) CK(hipMalloc(&img_l, lgemm_image_bytes(g)));
        if (lgemm_pack(g, img_l, s) != 0) { fprintf(stderr, "lgemm_pack failed\n"); return 1; }
        out("lgemm_x3_fwd", time_us(s, reps, [&] { lgemm_run(g, img_l, cus, s); }), (double)M * 256 * 8, fl);
      }
      if (mode == 0 && lgemm_supported(g)) {  // exact fp32 on k_lgemm's F32 kernel, checked against k_gemm_t
        if (!img_l) CK(hipMalloc(&img_l, lgemm_image_bytes(g)));
        if (lgemm_pack(g, img_l, s) != 0) { fprintf(stderr, "lgemm_pack failed\n"); return 1; }
        GemmArgs h = g;
        h.C = C2;
        out("lgemm_f32_fwd", time_us(s, reps, [&] { lgemm_run(h, img_l, cus, s); }), (double)M * 256 * 8, fl);
        launch_gemm(g, dim3((N + 63) / 64, (M + 63) / 64, 1), s);
        CK(hipStreamSynchronize(s));
        printf("{\"check\": \"lgemm_f32_fwd vs gemm_t_f32_fwd\", \"M\": %d, \"max_rel\": %.3g}\n", M,
               max_rel_diff(C2, C, (size_t)M * 256));
        // masked input-gradient shape (dX = (dY W) * (H > 0)): the mask rows of Mk
        GemmArgs x{};
        x.N = 256; x.nseg = 1; x.M = M;
        x.seg[0] = GemmSeg{A, 256, 1, W, 256, 1, 256};
        x.C = C; x.ldc = 256; x.mask = Mk; x.ldm = 256; x.ksplit = 1;
        if (lgemm_supported(x)) {
          void* img_x;
          CK(hipMalloc(&img_x, lgemm_image_bytes(x)));
          if (lgemm_pack(x, img_x, s) != 0) { fprintf(stderr, "lgemm_pack failed\n"); return 1; }
          GemmArgs y = x;
          y.C = C2;
          out("lgemm_f32_xgrad_mask", time_us(s, reps, [&] { lgemm_run(y, img_x, cus, s); }), (double)M * 256 * 12, fl);
          out("gemm_t_f32_xgrad_mask", time_us(s, reps, [&] { launch_gemm(x, dim3(4, (M + 63) / 64, 1), s); }),
              (double)M * 256 * 12, fl);
          CK(hipStreamSynchronize(s));
          printf("{\"check\": \"lgemm_f32_xgrad_mask vs gemm_t\", \"M\": %d, \"max_rel\": %.3g}\n", M,
                 max_rel_diff(C2, C, (size_t)M * 256));
          CK(hipFree(img_x));
        }
      }
    }
    // weight gradients dW += dY^T X over the M rows (+ bias column sums)
    for (int mode = 0; mode < 3; ++mode) {
      WGrad w{};
      w.dY = A; w.ldY = 256; w.nout = 256; w.X = Mk; w.ldX = 256; w.K = 256;
      w.dW = dW; w.ldw = 256; w.bsum = bsum; w.slab = slab;
      const char* name = mode == 0 ? "wgrad_bf16" : mode == 1 ? "wgrad_x3" : "wgrad_f32io_bf16";
      if (mode == 0) { w.ybf = 1; w.xbf = 1; }
      if (mode == 1) w.x3 = 1;
      const double eb = mode == 0 ? 4 : 8;
      out(name, time_us(s, reps, [&] { launch_wgrad(w, M, s); }), (double)M * 256 * eb, fl);
    }
    {
      GemmArgs g{};
      g.rowsum = bsum; g.N = 256; g.nseg = 1;
      g.seg[0] = GemmSeg{A, 1, 256, Mk, 256, 1, M};
      g.C = dW; g.ldc = 256; g.atomic = 1; g.ksplit = (M + 511) / 512; g.kper = 512; g.M = 256;
      out("wgrad_gemm_t_f32", time_us(s, reps, [&] { launch_gemm(g, dim3(4, 4, g.ksplit), s); }), (double)M * 256 * 8, fl);
      // the exact slab kernel on the same operands, checked against one clean split-K accumulation
      WGrad w{};
      w.dY = A; w.ldY = 256; w.nout = 256; w.X = Mk; w.ldX = 256; w.K = 256;
      w.dW = dW2; w.ldw = 256; w.bsum = bsum; w.slab = slab;
      out("wgrad_f32_slab", time_us(s, reps, [&] { launch_wgrad_f32(w, M, s); }), (double)M * 256 * 8, fl);
      CK(hipMemsetAsync(dW, 0, 256 * 256 * 4, s));
      CK(hipMemsetAsync(dW2, 0, 256 * 256 * 4, s));
      launch_gemm(g, dim3(4, 4, g.ksplit), s);
      if (launch_wgrad_f32(w, M, s) != 0) { fprintf(stderr, "launch_wgrad_f32 failed\n"); return 1; }
      CK(hipStreamSynchronize(s));
      printf("{\"check\": \"wgrad_f32_slab vs gemm_t split-K\", \"M\": %d, \"max_rel\": %.3g}\n", M,
             max_rel_diff(dW2, dW, 256 * 256));
      // a K = 63 / ld 64 product with column sums (the gamma columns of a first layer)
      WGrad v = w;
      v.K = 63; v.ldX = 64; v.X = Mk;
      GemmArgs h{};
      h.rowsum = bsum; h.N = 63; h.nseg = 1;
      h.seg[0] = GemmSeg{A, 1, 256, Mk, 64, 1, M};
      h.C = dW; h.ldc = 256; h.atomic = 1; h.ksplit = (M + 511) / 512; h.kper = 512; h.M = 256;
      CK(hipMemsetAsync(dW, 0, 256 * 256 * 4, s));
      CK(hipMemsetAsync(dW2, 0, 256 * 256 * 4, s));
      CK(hipMemsetAsync(bsum, 0, 256 * 4, s));
      launch_gemm(h, dim3(1, 4, h.ksplit), s);
      std::vector<float> b1(256), b2(256);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(b1.data(), bsum, 1024, hipMemcpyDeviceToHost));
      CK(hipMemsetAsync(bsum, 0, 256 * 4, s));
      v.ldw = 256; v.dW = dW2;
      if (launch_wgrad_f32(v, M, s) != 0) { fprintf(stderr, "launch_wgrad_f32 (K 63) failed\n"); return 1; }
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(b2.data(), bsum, 1024, hipMemcpyDeviceToHost));
      double mb = 0, sb = 0;
      for (int i = 0; i < 256; ++i) { mb = std::max(mb, (double)std::fabs(b1[i] - b2[i])); sb = std::max(sb, (double)std::fabs(b1[i])); }
      printf("{\"check\": \"wgrad_f32_slab K=63 vs gemm_t\", \"M\": %d, \"max_rel\": %.3g, \"bsum_rel\": %.3g}\n", M,
             max_rel_diff(dW2, dW, 256 * 256), sb > 0 ? mb / sb : mb);
    }
    const long n16 = (long)M * 256 * 2 / 16;
    out("copy_bf16_rows", time_us(s, reps, [&] {
          hipLaunchKernelGGL(k_probe_copy, dim3(cus * 4), dim3(256), 0, s, (const uint4*)A, (uint4*)C, n16);
        }), (double)M * 256 * 4, 0);
  }
  {  // LDS-DMA and register stream rates per CU (1 MiB per workgroup, 256 workgroups)
    const long per = 1 << 20;
    unsigned char* big;
    CK(hipMalloc(&big, per * 256));
    CK(hipMemset(big, 1, per * 256));
    uint4* sink;
    CK(hipMalloc(&sink, 1024 * 16));
    auto dma = [&](const char* name, auto kern, int W, int shared) {
      CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
      const float us = time_us(s, 20, [&] { hipLaunchKernelGGL(kern, dim3(256), dim3(W * 64), 128 * 1024, s, (const unsigned char*)big, per, shared); });
      printf("{\"stream\": \"%s\", \"shared\": %d, \"us\": %.2f, \"GBps_per_CU\": %.1f, \"TBps\": %.2f}\n", name, shared, us,
             per / us * 1e-3, 256.0 * per / us * 1e-6);
    };
    auto vld = [&](const char* name, auto kern, int W, int shared) {
      const float us = time_us(s, 20, [&] { hipLaunchKernelGGL(kern, dim3(256), dim3(W * 64), 0, s, (const unsigned char*)big, per, shared, sink); });
      printf("{\"stream\": \"%s\", \"shared\": %d, \"us\": %.2f, \"GBps_per_CU\": %.1f, \"TBps\": %.2f}\n", name, shared, us,
             per / us * 1e-3, 256.0 * per / us * 1e-6);
    };
    for (int sh = 0; sh < 2; ++sh) {
      dma("dma_w4_d1", k_probe_dma<4, 1>, 4, sh);
      dma("dma_w4_d4", k_probe_dma<4, 4>, 4, sh);
      dma("dma_w4_d16", k_probe_dma<4, 16>, 4, sh);
      dma("dma_w8_d2", k_probe_dma<8, 2>, 8, sh);
      dma("dma_w8_d8", k_probe_dma<8, 8>, 8, sh);
      dma("dma_w16_d4", k_probe_dma<16, 4>, 16, sh);
      vld("vload_w4_d4", k_probe_vload<4, 4>, 4, sh);
      vld("vload_w8_d8", k_probe_vload<8, 8>, 8, sh);
      vld("vload_w16_d8", k_probe_vload<16, 8>, 16, sh);
    }
  }
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  printf("{\"stream_priority_range\": [%d, %d]}\n", least, greatest);
  printf("{\"kernel\": \"empty\", \"M\": 0, \"us\": %.2f}\n",
         time_us(s, 200, [&] { hipLaunchKernelGGL(k_probe_empty, dim3(1), dim3(64), 0, s); }));
  return 0;
}
