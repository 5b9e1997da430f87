// Aggregate throughput of S concurrent streams, each replaying a hipGraph of a
// dependent chain of small kernels (the decode step's structure; bench.py pipelines
// up to 3-4 engine replicas, one stream each).  Reports µs per kernel aggregated over
// the streams: if it falls as 1/S, dispatch is not a shared bottleneck.
// Build: hipcc --offload-arch=gfx950 -O3 tools/launch_floor_mt.hip -o tools/launch_floor_mt
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

__global__ void k_dep(const float* __restrict__ in, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  out[i] = in[i] * 1.0001f + 1.0f;
}

// a decode-like kernel: each workgroup streams 16 KB of "weights" from L2 and one row
__global__ void k_rowlike(const float* __restrict__ in, float* __restrict__ out, const float* __restrict__ w) {
  const int tid = threadIdx.x;
  const float4* w4 = reinterpret_cast<const float4*>(w) + (size_t)(blockIdx.x & 255) * 1024;
  float s = in[blockIdx.x * blockDim.x + tid];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 v = w4[tid + i * 256];
    s += v.x + v.y + v.z + v.w;
  }
  out[blockIdx.x * blockDim.x + tid] = s;
}

int main() {
  const int chain = 400, reps = 5;
  const int grids[] = {64, 512};
  float* w;
  CK(hipMalloc(&w, 256ull * 16384));
  CK(hipMemset(w, 0, 256ull * 16384));
  for (int variant = 0; variant < 2; ++variant)
    for (int g : grids)
      for (int S : {1, 2, 3, 4, 6}) {
        std::vector<hipStream_t> st(S);
        std::vector<hipGraphExec_t> ex(S);
        std::vector<float*> a(S), b(S);
        for (int s = 0; s < S; ++s) {
          CK(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
          CK(hipMalloc(&a[s], 512 * 256 * 4));
          CK(hipMalloc(&b[s], 512 * 256 * 4));
          CK(hipMemset(a[s], 0, 512 * 256 * 4));
          hipGraph_t graph;
          CK(hipStreamBeginCapture(st[s], hipStreamCaptureModeThreadLocal));
          for (int i = 0; i < chain; ++i) {
            float* in = (i & 1) ? b[s] : a[s];
            float* out = (i & 1) ? a[s] : b[s];
            if (variant == 0) k_dep<<<g, 256, 0, st[s]>>>(in, out);
            else k_rowlike<<<g, 256, 0, st[s]>>>(in, out, w);
          }
          CK(hipStreamEndCapture(st[s], &graph));
          CK(hipGraphInstantiate(&ex[s], graph, nullptr, nullptr, 0));
          CK(hipGraphDestroy(graph));
          CK(hipGraphLaunch(ex[s], st[s]));
        }
        CK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, nullptr));
        CK(hipDeviceSynchronize());
        for (int r = 0; r < reps; ++r)
          for (int s = 0; s < S; ++s) CK(hipGraphLaunch(ex[s], st[s]));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-10s grid %4d streams %d : %.2f us per kernel aggregate, %.2f us per kernel per stream\n",
               variant ? "rowlike" : "dep", g, S, ms * 1000.f / (reps * chain * S), ms * 1000.f / (reps * chain));
        for (int s = 0; s < S; ++s) {
          CK(hipGraphExecDestroy(ex[s]));
          CK(hipStreamDestroy(st[s]));
          CK(hipFree(a[s]));
          CK(hipFree(b[s]));
        }
      }
  return 0;
}
