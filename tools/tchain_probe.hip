// tchain_probe — times one fused-chain program (anr_tchain.hip) alone on the GPU, on synthetic weights
// and rows: tools/tchain_probe PROG ROWS [REPS] [CUS]
//   PROG 0 BW forward, 1 NeRF forward, 2 BW input gradients, 3 NeRF input gradients
// Prints the average launch time (HIP events over REPS back-to-back launches) and the MFMA rate.
// Built by `make tchain-probe` (links the chain kernels directly, so -D variants build alongside).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../animatable_nerf_amd/csrc/anr_kernels.h"
#include "../animatable_nerf_amd/csrc/anr_train.h"

namespace anr {
// the library's profiling slots (anr_capi.hip) are not linked into the probe: profiling off
ProfSlot* prof_begin(hipStream_t, int) { return nullptr; }
int prof_end(ProfSlot*, hipStream_t) { return 0; }
}  // namespace anr

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void k_fill_bf16(unsigned short* p, size_t n, unsigned seed, float scale) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned h = (unsigned)i * 2654435761u ^ seed;
  h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
  const float v = ((h & 0xffff) / 65535.f - 0.5f) * scale;
  p[i] = (unsigned short)(__float_as_uint(v) >> 16);
}
__global__ void k_fill_f32(float* p, size_t n, unsigned seed, float scale) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned h = (unsigned)i * 2654435761u ^ seed;
  h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
  p[i] = ((h & 0xffff) / 65535.f - 0.5f) * scale;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s PROG ROWS [REPS] [CUS]\n", argv[0]);
    return 2;
  }
  const int prog = atoi(argv[1]), rows = atoi(argv[2]);
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  int cus = argc > 4 ? atoi(argv[4]) : 0;
  if (prog < 0 || prog > 3 || rows <= 0 || rows > (1 << 20)) return 2;
  if (cus <= 0) {
    int d = 0;
    CK(hipGetDevice(&d));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d));
  }
  const size_t pad = (size_t)(rows + 127) / 128 * 128;
  const size_t img = anr::tchain_image_bytes(prog);
  unsigned char* dimg;
  CK(hipMalloc(&dimg, img));
  k_fill_bf16<<<(unsigned)((img / 2 + 255) / 256), 256>>>((unsigned short*)dimg, img / 2, 7u, 0.2f);
  // per layer: an output region of pad x 256 fp32, a bits region of pad x 32 B
  std::vector<void*> outs(12), bits(12);
  for (int l = 0; l < 12; ++l) {
    CK(hipMalloc(&outs[l], pad * 256 * 4));
    CK(hipMalloc(&bits[l], (pad + 128) * 32));
    k_fill_bf16<<<(unsigned)(((pad + 128) * 16 + 255) / 256), 256>>>((unsigned short*)bits[l], (pad + 128) * 16, 11u + l, 2.f);
  }
  float *mem, *mem2, *aux, *bias;
  CK(hipMalloc(&mem, pad * 64 * 4));
  CK(hipMalloc(&mem2, pad * 64 * 4));
  CK(hipMalloc(&aux, pad * 64 * 4));
  CK(hipMalloc(&bias, 512 * 4));
  k_fill_f32<<<(unsigned)((pad * 64 + 255) / 256), 256>>>(mem, pad * 64, 3u, 1.f);
  k_fill_f32<<<(unsigned)((pad * 64 + 255) / 256), 256>>>(mem2, pad * 64, 5u, 1.f);
  CK(hipMemset(aux, 0, pad * 64 * 4));
  CK(hipMemset(bias, 0, 512 * 4));
  int* Mdev;
  CK(hipMalloc(&Mdev, 4));
  CK(hipMemcpy(Mdev, &rows, 4, hipMemcpyHostToDevice));

  anr::TcArgs a{};
  a.img = dimg;
  const bool bwd = prog >= 2;
  for (int l = 0; l < 12; ++l) {
    a.bias[l] = bias;
    a.nout[l] = 256;
    a.out[l] = outs[l];
    a.ldo[l] = 256;
    a.bits[l] = bits[l];
  }
  a.bias2 = bias;
  a.out2 = (float*)outs[11];
  if (prog == 0) { a.nout[8] = 24; a.ldo[8] = 32; }
  if (prog == 1) { a.nout[10] = 128; a.ldo[10] = 128; a.nout[11] = 3; a.ldo[11] = 4; }
  if (prog == 3) { a.nout[0] = 128; a.ldo[0] = 128; }
  // forward: gamma rows bf16 (ld 64, 63 cols), gamma(dir) bf16 (27 cols); backward: d logits / d rgb fp32
  a.mem = (const unsigned short*)mem;
  a.ld_mem = bwd ? (prog == 2 ? 64 : 4) : 64;
  a.kmem_cols = bwd ? (prog == 2 ? 24 : 3) : 63;
  a.mem_f32 = bwd ? 1 : 0;
  a.mem2 = (const unsigned short*)mem2;
  a.ld_mem2 = 64;
  a.kmem2_cols = prog == 1 ? 27 : 1;
  a.aux = bwd ? aux : nullptr;
  a.ld_aux = 64;
  a.aux_cols = 63;
  a.M_dev = Mdev;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (int i = 0; i < 3; ++i)
    if (anr::tchain_run(prog, a, rows, cus, s) != 0) return 1;
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i)
    if (anr::tchain_run(prog, a, rows, cus, s) != 0) return 1;
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / reps;
  // MACs per row: every 1-KiB fragment of the image is 16 outputs x 32 inputs
  const double macs = (double)(img / 1024) * 512;
  const double tflops = 2.0 * macs * rows / (us * 1e-6) / 1e12;
  const int tiles = (rows + 111) / 112;
  printf("prog %d rows %d tiles %d grid %d: %.2f us per launch, %.1f TFLOP/s (padded MFMA work)\n", prog, rows, tiles,
         tiles < cus ? tiles : cus, us, tflops);
  return 0;
}
