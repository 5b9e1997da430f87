// Microbenchmark: per-kernel cost of a dependent chain of small kernels replayed from a
// hipGraph (the decode step's structure).  Variants: empty kernel; one dependent
// load+store per thread; a 64 KB read per workgroup; grid sizes 64 / 256 / 1024 WGs.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__global__ void k_empty(float* p) {}

__global__ void k_dep(const float* __restrict__ in, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  out[i] = in[i] * 1.0001f + 1.0f;
}

__global__ void k_read64k(const float* __restrict__ in, float* __restrict__ out, const float* __restrict__ w) {
  // each workgroup reads 64 KB of "weights" (16 float4 per thread) plus one activation
  const int tid = threadIdx.x;
  const float4* w4 = reinterpret_cast<const float4*>(w) + (size_t)blockIdx.x * 4096;
  float s = in[blockIdx.x * blockDim.x + tid];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float4 v = w4[tid + i * 256];
    s += v.x + v.y + v.z + v.w;
  }
  out[blockIdx.x * blockDim.x + tid] = s;
}

int main() {
  const int chain = 400;
  const int grids[] = {64, 256, 1024};
  float *a, *b, *w;
  CK(hipMalloc(&a, 1024 * 256 * 4));
  CK(hipMalloc(&b, 1024 * 256 * 4));
  CK(hipMalloc(&w, 1024ull * 65536));
  CK(hipMemset(a, 0, 1024 * 256 * 4));
  CK(hipMemset(b, 0, 1024 * 256 * 4));
  CK(hipMemset(w, 0, 1024ull * 65536));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int variant = 0; variant < 3; ++variant) {
    for (int g : grids) {
      hipGraph_t graph;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < chain; ++i) {
        float* in = (i & 1) ? b : a;
        float* out = (i & 1) ? a : b;
        if (variant == 0) k_empty<<<g, 256, 0, s>>>(out);
        if (variant == 1) k_dep<<<g, 256, 0, s>>>(in, out);
        if (variant == 2) k_read64k<<<g, 256, 0, s>>>(in, out, w);
      }
      CK(hipStreamEndCapture(s, &graph));
      hipGraphExec_t exec;
      CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
      CK(hipGraphLaunch(exec, s));
      CK(hipStreamSynchronize(s));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(exec, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const char* names[] = {"empty", "dep-load-store", "64KB-read/WG"};
      printf("%-16s grid %5d : %.2f us per kernel\n", names[variant], g, ms * 1000.f / (5 * chain));
      CK(hipGraphExecDestroy(exec));
      CK(hipGraphDestroy(graph));
    }
  }
  return 0;
}
