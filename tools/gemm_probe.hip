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
#include "../animatable_nerf_amd/csrc/anr_train.h"

using namespace anr;

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

int main(int argc, char** argv) {
  std::vector<int> Ms;
  for (int i = 1; i < argc; ++i) Ms.push_back(atoi(argv[i]));
  if (Ms.empty()) Ms = {6223, 12446, 24893, 49786, 99572};
  int Mmax = 0;
  for (int m : Ms) Mmax = m > Mmax ? m : Mmax;
  const int K = 256, N = 256, reps = 50;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
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
      {  // the LDS-staged epilogue: same bytes, timed
        RGemm a = r, b = r;
        a.stage = -1;
        b.stage = 1;
        b.C = C2;
        launch_rgemm(a, M, s);
        launch_rgemm(b, M, s);
        CK(hipStreamSynchronize(s));
        const size_t bytes = (size_t)M * 256 * (r.cbf ? 2 : 4);
        if (!same_bytes(C, C2, bytes)) printf("{\"kernel\": \"%s_stage\", \"M\": %d, \"error\": \"MISMATCH\"}\n", name, M);
        const std::string v = std::string(name) + "_stage";
        out(v.c_str(), time_us(s, reps, [&] { launch_rgemm(b, M, s); }), (double)M * 256 * eb, fl);
      }
      if (mode == 2) continue;
      const int geo[4][2] = {{128, 3}, {64, 2}, {64, 3}, {64, 4}};
      for (auto& gm : geo) {
        if (launch_rgemm_variant(r, M, s, gm[0], gm[1]) != 0) {
          (void)hipGetLastError();
          printf("{\"kernel\": \"%s_bm%d_ns%d\", \"M\": %d, \"error\": \"launch\"}\n", name, gm[0], gm[1], M);
          continue;
        }
        CK(hipStreamSynchronize(s));
        {  // the variant's output equals the default kernel's, byte for byte
          RGemm r2 = r;
          r2.C = C2;
          launch_rgemm(r2, M, s);
          launch_rgemm(r, M, s);
          CK(hipStreamSynchronize(s));
          if (launch_rgemm_variant(r2, M, s, gm[0], gm[1]) != 0) return 1;
          CK(hipStreamSynchronize(s));
          const size_t bytes = (size_t)M * 256 * (r.cbf ? 2 : 4);
          if (!same_bytes(C, C2, bytes)) printf("{\"kernel\": \"%s_bm%d_ns%d\", \"M\": %d, \"error\": \"MISMATCH\"}\n", name, gm[0], gm[1], M);
        }
        const std::string v = std::string(name) + "_bm" + std::to_string(gm[0]) + "_ns" + std::to_string(gm[1]);
        out(v.c_str(), time_us(s, reps, [&] { launch_rgemm_variant(r, M, s, gm[0], gm[1]); }), (double)M * 256 * eb, fl);
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
      for (int d : {2, 4}) {
        {  // the deep kernel's dW against k_wgrad's (slab groups meet in fp32 atomics: order may differ)
          WGrad a = w, b = w;
          a.deep = 0; a.bsum = nullptr;
          b.deep = d; b.bsum = nullptr; b.dW = dW2;
          CK(hipMemsetAsync(dW, 0, 256 * 256 * 4, s));
          CK(hipMemsetAsync(dW2, 0, 256 * 256 * 4, s));
          launch_wgrad(a, M, s);
          CK(hipStreamSynchronize(s));
          launch_wgrad(b, M, s);
          CK(hipStreamSynchronize(s));
          const double e = max_rel_diff(dW2, dW, 256 * 256);
          if (!(e < 1e-5)) printf("{\"kernel\": \"%s_deep%d\", \"M\": %d, \"error\": \"MISMATCH %g\"}\n", name, d, M, e);
        }
        w.deep = d;
        const std::string v = std::string(name) + "_deep" + std::to_string(d);
        out(v.c_str(), time_us(s, reps, [&] { launch_wgrad(w, M, s); }), (double)M * 256 * eb, fl);
      }
      w.deep = 0;
    }
    {
      GemmArgs g{};
      g.rowsum = bsum; g.N = 256; g.nseg = 1;
      g.seg[0] = GemmSeg{A, 1, 256, Mk, 256, 1, M};
      g.C = dW; g.ldc = 256; g.atomic = 1; g.ksplit = (M + 511) / 512; g.kper = 512; g.M = 256;
      out("wgrad_gemm_t_f32", time_us(s, reps, [&] { launch_gemm(g, dim3(4, 4, g.ksplit), s); }), (double)M * 256 * 8, fl);
    }
    const long n16 = (long)M * 256 * 2 / 16;
    out("copy_bf16_rows", time_us(s, reps, [&] {
          hipLaunchKernelGGL(k_probe_copy, dim3(cus * 4), dim3(256), 0, s, (const uint4*)A, (uint4*)C, n16);
        }), (double)M * 256 * 4, 0);
  }
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  printf("{\"stream_priority_range\": [%d, %d]}\n", least, greatest);
  printf("{\"kernel\": \"empty\", \"M\": 0, \"us\": %.2f}\n",
         time_us(s, 200, [&] { hipLaunchKernelGGL(k_probe_empty, dim3(1), dim3(64), 0, s); }));
  return 0;
}
