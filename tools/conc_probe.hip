// Concurrency probe: does a chain of small dependent kernels (the decode step's shape:
// 128-512 workgroups of 256 threads, a few KB of LDS, ~3 us each) run beside a large
// encoder-shaped kernel (512-thread workgroups holding 128 KB of LDS, grid >> CUs) that
// another stream is dispatching?  Compared: the large kernel as one workgroup per tile
// (grid = tiles) and as a persistent grid (one workgroup per CU looping over the tiles).
//
//   hipcc -O3 --offload-arch=gfx950 tools/conc_probe.hip -o tools/conc_probe && tools/conc_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__device__ __forceinline__ void spin_us(unsigned us) {
  const unsigned long long t0 = wall_clock64();  // 100 MHz
  while (wall_clock64() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(2);
}

// "encoder" tile: 128 KB LDS touched, `us` microseconds of residency per tile
__global__ void __launch_bounds__(512) big_kernel(float* out, int tiles, unsigned us) {
  __shared__ float lds[32 * 1024];
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    for (int i = threadIdx.x; i < 32 * 1024; i += 512) lds[i] = (float)(i + t);
    __syncthreads();
    spin_us(us);
    if (threadIdx.x == 0) out[t] = lds[(t * 7) & 32767];
    __syncthreads();
  }
}

// "decode" kernel: 4 KB LDS, `us` microseconds
__global__ void __launch_bounds__(256) small_kernel(float* out, unsigned us) {
  __shared__ float lds[1024];
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  spin_us(us);
  if (threadIdx.x == 0) out[blockIdx.x] += lds[(blockIdx.x * 3) & 1023];
}

// memory streamers: each workgroup walks its slice of a large buffer `passes` times
__global__ void __launch_bounds__(256) write_stream(float4* buf, size_t n, int passes) {
  for (int p = 0; p < passes; ++p)
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
      buf[i] = make_float4((float)p, 0.f, 0.f, 0.f);
}
__global__ void __launch_bounds__(256) read_stream(const float4* buf, size_t n, int passes, float* out) {
  float acc = 0.f;
  for (int p = 0; p < passes; ++p)
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += buf[i].x;
  if (acc == 12345.f) out[0] = acc;
}

int main(int argc, char** argv) {
  const int tiles = 864;        // s3.fc1's 256x256 tiles
  const unsigned big_us = 80;   // per tile
  const int big_launches = 6;
  const int small_n = 400;      // dependent small kernels (~10 decode steps)
  const unsigned small_us = 3;
  const int small_grid = 256;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  float *ob, *os;
  CK(hipMalloc(&ob, tiles * sizeof(float)));
  CK(hipMalloc(&os, small_grid * sizeof(float)));
  CK(hipMemset(os, 0, small_grid * sizeof(float)));
  hipStream_t sb, ss;
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
  // the small chain as one graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(ss, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < small_n; ++i) small_kernel<<<small_grid, 256, 0, ss>>>(os, small_us);
  CK(hipStreamEndCapture(ss, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));

  auto run = [&](bool big, bool small, int big_grid) {
    hipEvent_t b0, b1, s0, s1;
    CK(hipEventCreate(&b0)); CK(hipEventCreate(&b1)); CK(hipEventCreate(&s0)); CK(hipEventCreate(&s1));
    CK(hipDeviceSynchronize());
    auto w0 = std::chrono::steady_clock::now();
    if (big) {
      CK(hipEventRecord(b0, sb));
      for (int i = 0; i < big_launches; ++i) big_kernel<<<big_grid, 512, 0, sb>>>(ob, tiles, big_us);
      CK(hipEventRecord(b1, sb));
    }
    if (small) {
      CK(hipEventRecord(s0, ss));
      CK(hipGraphLaunch(ge, ss));
      CK(hipEventRecord(s1, ss));
    }
    CK(hipDeviceSynchronize());
    const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    float tb = 0, ts = 0;
    if (big) CK(hipEventElapsedTime(&tb, b0, b1));
    if (small) CK(hipEventElapsedTime(&ts, s0, s1));
    printf("big=%d(grid %4d) small=%d | big %.3f ms  small chain %.3f ms  wall %.3f ms\n", big, big ? big_grid : 0, small,
           tb, ts, wall);
  };
  for (int rep = 0; rep < 2; ++rep) {
    printf("-- rep %d (CUs %d)\n", rep, ncu);
    run(false, true, 0);
    run(true, false, tiles);
    run(true, true, tiles);
    run(true, false, ncu);
    run(true, true, ncu);
  }
  // the small chain beside a memory streamer (writes dirty the L2s; reads do not)
  {
    const size_t n = (size_t)64 << 20;  // 1 GiB of float4
    float4* buf;
    CK(hipMalloc(&buf, n * sizeof(float4)));
    CK(hipMemset(buf, 0, n * sizeof(float4)));
    hipStream_t sm;
    CK(hipStreamCreateWithFlags(&sm, hipStreamNonBlocking));
    for (int mode = 0; mode < 5; ++mode) {
      hipEvent_t s0, s1, m0, m1;
      CK(hipEventCreate(&s0)); CK(hipEventCreate(&s1)); CK(hipEventCreate(&m0)); CK(hipEventCreate(&m1));
      CK(hipDeviceSynchronize());
      if (mode) {
        CK(hipEventRecord(m0, sm));
        // modes 3 / 4: a 2 MiB buffer (L2-resident) written / read 3000 times: dirty L2 lines
        // (or clean hits) without HBM bandwidth
        if (mode == 1) write_stream<<<2048, 256, 0, sm>>>(buf, n, 3);
        else if (mode == 2) read_stream<<<2048, 256, 0, sm>>>(buf, n, 3, ob);
        else if (mode == 3) write_stream<<<2048, 256, 0, sm>>>(buf, (size_t)1 << 17, 3000);
        else read_stream<<<2048, 256, 0, sm>>>(buf, (size_t)1 << 17, 3000, ob);
        CK(hipEventRecord(m1, sm));
      }
      CK(hipEventRecord(s0, ss));
      CK(hipGraphLaunch(ge, ss));
      CK(hipEventRecord(s1, ss));
      CK(hipDeviceSynchronize());
      float ts = 0, tm = 0;
      CK(hipEventElapsedTime(&ts, s0, s1));
      if (mode) CK(hipEventElapsedTime(&tm, m0, m1));
      const char* nm[] = {"alone", "|| HBM write streamer", "|| HBM read streamer", "|| L2-resident writer",
                          "|| L2-resident reader"};
      printf("small chain %s: %.3f ms (streamer %.3f ms)\n", nm[mode], ts, tm);
    }
  }
  // N independent small chains on N streams: does the aggregate launch rate scale?
  for (int n = 1; n <= 8; n *= 2) {
    hipStream_t st[8];
    hipEvent_t e0[8], e1[8];
    for (int i = 0; i < n; ++i) {
      CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
      CK(hipEventCreate(&e0[i]));
      CK(hipEventCreate(&e1[i]));
    }
    CK(hipDeviceSynchronize());
    auto w0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
      CK(hipEventRecord(e0[i], st[i]));
      CK(hipGraphLaunch(ge, st[i]));
      CK(hipEventRecord(e1[i], st[i]));
    }
    CK(hipDeviceSynchronize());
    const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    printf("%d concurrent small chains (%d kernels each, %u us): wall %.3f ms, chain ms:", n, small_n, small_us, wall);
    for (int i = 0; i < n; ++i) {
      float t = 0;
      CK(hipEventElapsedTime(&t, e0[i], e1[i]));
      printf(" %.3f", t);
    }
    printf("\n");
  }
  return 0;
}
