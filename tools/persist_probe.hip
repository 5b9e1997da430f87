// Persistent-vs-launch probe for the decode step's structure: P dependent phases, each a
// small all-to-all exchange (every workgroup reads 16 KB that the other workgroups wrote in
// the previous phase and writes 1 KB).  (A) one kernel per phase, captured in a graph;
// (B) one persistent launch with a counter barrier between phases: payload stored
// write-through (sc1), each storing wave drained, one relaxed agent-scope add per workgroup,
// one lane polls relaxed with s_sleep (bounded: a timeout word, then every wave exits),
// payload read with sc1 loads (MI355X guide, Guideline 16 R1).  Each is timed alone, three
// at once on three streams, and beside an HBM streamer.
//   hipcc -O3 --offload-arch=gfx950 tools/persist_probe.hip -o tools/persist_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

constexpr int G = 256;        // workgroups (one per CU)
constexpr int T = 256;        // threads
constexpr int SLOT = 256;     // floats each workgroup writes per phase (1 KB)
constexpr int READS = 16;     // floats each thread reads per phase (16 KB per workgroup)

typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load((const unsigned*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((unsigned*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one phase's work: read READS floats of other workgroups' slots (buffer `in`), write own slot of `out`
__device__ __forceinline__ void phase_work(const float* in, float* out, int ph, bool sc1) {
  const int b = blockIdx.x, t = threadIdx.x;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < READS; ++i) {
    const int src = (b + 1 + i * 13 + t / 16) % G;  // other workgroups' slots
    const float* p = in + (size_t)src * SLOT + (t * 7 + i) % SLOT;
    acc += sc1 ? ld_sc1(p) : *p;
  }
  const float v = acc * 0.5f + (float)ph;
  if (sc1)
    st_sc1(out + (size_t)b * SLOT + t, v);
  else
    out[(size_t)b * SLOT + t] = v;
}

__global__ void __launch_bounds__(T) phase_kernel(const float* in, float* out, int ph) { phase_work(in, out, ph, false); }

__global__ void __launch_bounds__(T) persistent_kernel(float* buf0, float* buf1, int phases, unsigned* counter,
                                                       unsigned* timeout) {
  __shared__ int quit;
  for (int ph = 0; ph < phases; ++ph) {
    float* in = (ph & 1) ? buf1 : buf0;
    float* out = (ph & 1) ? buf0 : buf1;
    phase_work(in, out, ph, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)G * (ph + 1);
      unsigned spins = 0;
      int q = 0;
      while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {  // give up: some workgroup is not resident
          __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          q = 1;
          break;
        }
        if (__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          q = 1;
          break;
        }
      }
      quit = q;
    }
    __syncthreads();
    if (quit) return;
  }
}

__global__ void __launch_bounds__(256) read_stream(const float4* buf, size_t n, int passes, float* out) {
  float acc = 0.f;
  for (int p = 0; p < passes; ++p)
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += buf[i].x;
  if (acc == 12345.f) out[0] = acc;
}

int main() {
  const int P = 336;  // 8 decode steps x 42 kernels
  const int NI = 3;   // concurrent instances
  std::vector<float*> b0(NI), b1(NI);
  std::vector<unsigned*> cnt(NI), tmo(NI);
  std::vector<hipStream_t> st(NI);
  std::vector<hipGraphExec_t> ge(NI);
  for (int i = 0; i < NI; ++i) {
    CK(hipMalloc(&b0[i], (size_t)G * SLOT * 4));
    CK(hipMalloc(&b1[i], (size_t)G * SLOT * 4));
    CK(hipMemset(b0[i], 0, (size_t)G * SLOT * 4));
    CK(hipMemset(b1[i], 0, (size_t)G * SLOT * 4));
    CK(hipMalloc(&cnt[i], 16));
    CK(hipMalloc(&tmo[i], 16));
    CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    hipGraph_t g;
    CK(hipStreamBeginCapture(st[i], hipStreamCaptureModeThreadLocal));
    for (int ph = 0; ph < P; ++ph) phase_kernel<<<G, T, 0, st[i]>>>((ph & 1) ? b1[i] : b0[i], (ph & 1) ? b0[i] : b1[i], ph);
    CK(hipStreamEndCapture(st[i], &g));
    CK(hipGraphInstantiate(&ge[i], g, nullptr, nullptr, 0));
  }
  const size_t ns = (size_t)64 << 20;
  float4* sbuf;
  float* sout;
  CK(hipMalloc(&sbuf, ns * 16));
  CK(hipMemset(sbuf, 0, ns * 16));
  CK(hipMalloc(&sout, 16));
  hipStream_t ss;
  CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));

  auto run = [&](bool persistent, int ninst, bool streamer) {
    std::vector<hipEvent_t> e0(ninst), e1(ninst);
    for (int i = 0; i < ninst; ++i) {
      CK(hipEventCreate(&e0[i]));
      CK(hipEventCreate(&e1[i]));
      CK(hipMemsetAsync(cnt[i], 0, 16, st[i]));
      CK(hipMemsetAsync(tmo[i], 0, 16, st[i]));
    }
    CK(hipDeviceSynchronize());
    if (streamer) read_stream<<<2048, 256, 0, ss>>>(sbuf, ns, 6, sout);
    for (int i = 0; i < ninst; ++i) {
      CK(hipEventRecord(e0[i], st[i]));
      if (persistent)
        persistent_kernel<<<G, T, 0, st[i]>>>(b0[i], b1[i], P, cnt[i], tmo[i]);
      else
        CK(hipGraphLaunch(ge[i], st[i]));
      CK(hipEventRecord(e1[i], st[i]));
    }
    CK(hipDeviceSynchronize());
    float worst = 0.f;
    unsigned to = 0;
    for (int i = 0; i < ninst; ++i) {
      float ms;
      CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      worst = ms > worst ? ms : worst;
      unsigned h = 0;
      CK(hipMemcpy(&h, tmo[i], 4, hipMemcpyDeviceToHost));
      to |= h;
    }
    printf("%-11s x%d%s: %.2f us per phase%s\n", persistent ? "persistent" : "launches", ninst,
           streamer ? " + HBM streamer" : "", worst * 1000.f / P, to ? "  (TIMED OUT)" : "");
  };
  for (int rep = 0; rep < 2; ++rep) {
    run(false, 1, false);
    run(true, 1, false);
    run(false, NI, false);
    run(true, NI, false);
    run(false, 1, true);
    run(true, 1, true);
  }
  return 0;
}
