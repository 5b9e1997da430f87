// Standalone timing of libmathocr's bf16 / bf16x3 GEMM for one shape (HIP events) with an
// output checksum, for fast iteration and PMC runs on the encoder GEMM shapes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/gemm_bench.hip
//        -L handwritten-math-ocr-api_amd/lib -lmathocr -Wl,-rpath,<repo>/handwritten-math-ocr-api_amd/lib
// Run:   tools/gemm_bench M N K passes epi iters [data [kernel]]   (epi 0 store, 1 gelu, 2 resadd;
//        data 0: hi and lo planes U(+-0.05), 1: lo planes U(+-0.05/256) as real splits, 2: zeros;
//        kernel: GemmParams::force_kernel, 0 = the dispatch's choice)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../handwritten-math-ocr-api_amd/csrc/kernels.h"

using namespace mocr;

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

__global__ void fill_bf16(uint16_t* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    const float f = ((h & 0xffff) / 32768.0f - 1.0f) * scale;  // uniform +-scale
    p[i] = (uint16_t)(__float_as_uint(f) >> 16);
  }
}

int main(int argc, char** argv) {
  if (argc < 7) {
    printf("usage: gemm_bench M N K passes epi iters\n");
    return 1;
  }
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]), passes = atoi(argv[4]), epi = atoi(argv[5]);
  const int iters = atoi(argv[6]);
  uint16_t *A, *Al, *W, *Wl, *Ch, *Cl;
  float *C, *bias;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&Al, (size_t)M * K * 2));
  CK(hipMalloc(&W, (size_t)N * K * 2));
  CK(hipMalloc(&Wl, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 4));
  CK(hipMalloc(&Ch, (size_t)M * N * 2));
  CK(hipMalloc(&Cl, (size_t)M * N * 2));
  CK(hipMalloc(&bias, (size_t)N * 4));
  const int data = argc > 7 ? atoi(argv[7]) : 0;
  const float hs = data == 2 ? 0.f : 0.05f, ls = data == 0 ? 0.05f : (data == 1 ? 0.05f / 256 : 0.f);
  fill_bf16<<<1024, 256>>>(A, (size_t)M * K, 1, hs);
  fill_bf16<<<1024, 256>>>(Al, (size_t)M * K, 2, ls);
  fill_bf16<<<1024, 256>>>(W, (size_t)N * K, 3, hs);
  fill_bf16<<<1024, 256>>>(Wl, (size_t)N * K, 4, ls);
  CK(hipMemset(C, 0, (size_t)M * N * 4));
  CK(hipMemset(bias, 0, (size_t)N * 4));
  GemmParams p{};
  p.A = A;
  p.W = W;
  p.A_lo = passes == 3 ? Al : nullptr;
  p.W_lo = passes == 3 ? Wl : nullptr;
  p.bias = bias;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = K;
  p.ldw = K;
  p.ldc = N;
  p.epi = epi;
  p.force_kernel = argc > 8 ? atoi(argv[8]) : 0;
  if (epi == EPI_RESADD) {
    p.C = C;
  } else {
    p.C16 = Ch;
    p.C16lo = passes == 3 ? Cl : nullptr;
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int i = 0; i < 3; ++i) launch_gemm_bf16(p, s);
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) launch_gemm_bf16(p, s);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / iters;
  const double tf = 2.0 * M * N * K / (us * 1e-6) / 1e12;
  // checksum of the output (bitwise comparison of kernel variants across processes)
  unsigned long long h = 1469598103934665603ull;
  if (epi == EPI_RESADD) {
    std::vector<uint32_t> c((size_t)M * N);
    CK(hipMemcpy(c.data(), C, c.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t v : c) h = (h ^ v) * 1099511628211ull;
  } else {
    std::vector<uint16_t> c((size_t)M * N);
    CK(hipMemcpy(c.data(), Ch, c.size() * 2, hipMemcpyDeviceToHost));
    for (uint16_t v : c) h = (h ^ v) * 1099511628211ull;
    if (passes == 3) {
      CK(hipMemcpy(c.data(), Cl, c.size() * 2, hipMemcpyDeviceToHost));
      for (uint16_t v : c) h = (h ^ v) * 1099511628211ull;
    }
  }
  printf("M %d N %d K %d passes %d epi %d : %.1f us  %.1f TF/s (x%d MFMA: %.1f TF/s raw)  sum %016llx\n", M, N, K,
         passes, epi, us, tf, passes, tf * passes, h);
  return 0;
}
