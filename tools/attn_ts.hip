// Where a decode attention kernel's time goes: per-workgroup phase clocks of
// dec_foldattn_kernel (thread 0 of each (row, head) workgroup) in a 100-long graph chain.
// Library built with -DMOCR_FOLD_TS (tools/build_variant.sh lib_var/ts -DMOCR_FOLD_TS);
// build as tools/fold_ts.hip.   attn_ts [cross|self] [R] [t]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../handwritten-math-ocr-api_amd/csrc/kernels.h"

using namespace mocr;
extern "C" int mocr_debug_attn_ts(unsigned long long* out, int n);

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

template <typename T>
T* alloc(size_t n) {
  void* p;
  CK(hipMalloc(&p, n * sizeof(T)));
  CK(hipMemset(p, 0, n * sizeof(T)));
  return (T*)p;
}

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
}

int main(int argc, char** argv) {
  const bool self = argc > 1 && !strcmp(argv[1], "self");
  const int R = argc > 2 ? atoi(argv[2]) : 256;
  const int t = argc > 3 ? atoi(argv[3]) : 100;
  const int waves = argc > 4 ? atoi(argv[4]) : 0;
  const int d = 256, P = 150, M = 144;
  float* z = alloc<float>((size_t)R * 3 * d);
  float* st = alloc<float>((size_t)R * 32);
  float* vec = alloc<float>(4 * d);
  float* out = alloc<float>((size_t)R * d);
  uint8_t* kc = alloc<uint8_t>((size_t)R * P * d * 3);
  uint8_t* vc = alloc<uint8_t>((size_t)R * P * d * 3);
  float* kcf = alloc<float>(16);
  int16_t* kv16 = alloc<int16_t>((size_t)R * M * 2 * d);
  float* scale = alloc<float>((size_t)R * 2 * d);
  {
    std::vector<float> h((size_t)R * 32);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (i % 2) ? 16.f : 0.5f;
    CK(hipMemcpy(st, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> one((size_t)R * 2 * d, 1e-4f);
    CK(hipMemcpy(scale, one.data(), one.size() * 4, hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int chain = 100;
  hipGraph_t graph;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < chain; ++i) {
    FoldAttnParams a{};
    a.waves = waves;
    a.t = t; a.B = R; a.out = out; a.z = z; a.z_stats = st; a.s = vec; a.c = vec;
    if (self) {
      a.z_ld = 3 * d; a.K = kcf; a.V = kcf; a.kcache = kcf; a.vcache = kcf; a.kv_b_stride = (size_t)P * d;
      a.kv_row_stride = d; a.n = t + 1;
      a.K24 = a.kc24 = kc; a.V24 = a.vc24 = vc;
      a.f24_b = (size_t)8 * P * 32; a.f24_h = (size_t)P * 32;
    } else {
      a.z_ld = d; a.K = kcf; a.V = kcf; a.kv_b_stride = (size_t)M * 2 * d; a.kv_row_stride = 2 * d; a.n = M;
      a.K16 = kv16; a.V16 = kv16 + (size_t)8 * M * 32; a.Ks = scale; a.Vs = scale + d; a.s_b = 2 * d;
      a.f24_b = (size_t)2 * 8 * M * 32; a.f24_h = (size_t)M * 32;
    }
    launch_dec_foldattn(a, self, s);
  }
  CK(hipStreamEndCapture(s, &graph));
  hipGraphExec_t exec;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(exec, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  CK(hipGraphLaunch(exec, s));
  CK(hipEventRecord(e1, s));
  CK(hipStreamSynchronize(s));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> ts((size_t)8192 * 8);
  if (mocr_debug_attn_ts(ts.data(), 8192 * 8)) { printf("no timestamps (library built without MOCR_FOLD_TS?)\n"); return 1; }
  unsigned long long rt_min = ~0ull, rt_max = 0;
  int n = 0;
  for (int b = 0; b < 8192; ++b)
    if (ts[b * 8]) { ++n; rt_min = std::min(rt_min, ts[b * 8]); rt_max = std::max(rt_max, ts[b * 8 + 6]); }
  std::vector<double> start, end, span, ph[4];
  for (int b = 0; b < 8192; ++b) {
    const unsigned long long* q = &ts[b * 8];
    if (!q[0]) continue;
    start.push_back((q[0] - rt_min) * 0.01);
    end.push_back((q[6] - rt_min) * 0.01);
    span.push_back((q[6] - q[0]) * 0.01);
    for (int k = 0; k < 4; ++k) ph[k].push_back((double)(q[2 + k] - q[1 + k]));
  }
  printf("%s attention R=%d t=%d waves=%d: %.2f us per kernel in the chain; %d workgroups timed\n", self ? "self" : "cross", R, t, waves,
         ms * 1000.0 / chain, n);
  printf("last kernel: first start -> last exit %.2f us\n", (rt_max - rt_min) * 0.01);
  printf("workgroup start offset us: p0 %.2f p50 %.2f p90 %.2f p100 %.2f\n", pct(start, 0), pct(start, .5),
         pct(start, .9), pct(start, 1));
  printf("workgroup exit offset  us: p0 %.2f p50 %.2f p90 %.2f p100 %.2f\n", pct(end, 0), pct(end, .5), pct(end, .9),
         pct(end, 1));
  printf("workgroup span us:         p0 %.2f p50 %.2f p90 %.2f p100 %.2f\n", pct(span, 0), pct(span, .5),
         pct(span, .9), pct(span, 1));
  const char* names[4] = {"issue + wait loads", "scores/softmax/PV", "LDS partials + barrier", "merge + store"};
  for (int k = 0; k < 4; ++k)
    printf("  %-22s cycles p10 %7.0f p50 %7.0f p90 %7.0f\n", names[k], pct(ph[k], .1), pct(ph[k], .5), pct(ph[k], .9));
  return 0;
}
