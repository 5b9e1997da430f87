// Where a fold GEMM's time goes: per-workgroup phase clocks of foldwide_kernel in a
// 100-long dependent graph chain (each launch reads the previous launch's y as its A2,
// as in the decode step).  Needs a library built with -DMOCR_FOLD_TS:
//   tools/build_variant.sh lib_var/ts -DMOCR_FOLD_TS
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/fold_ts.hip \
//     -L handwritten-math-ocr-api_amd/lib_var/ts -lmathocr -Wl,-rpath,$PWD/handwritten-math-ocr-api_amd/lib_var/ts
//   fold_ts [R] [K1] [NZ]      (default 256 256 256: the y_sa + z_q GEMM)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../handwritten-math-ocr-api_amd/csrc/kernels.h"

using namespace mocr;
extern "C" int mocr_debug_fold_ts(unsigned long long* out, int n);

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
  const int R = argc > 1 ? atoi(argv[1]) : 256;
  const int K1 = argc > 2 ? atoi(argv[2]) : 256;
  const int NZ = argc > 3 ? atoi(argv[3]) : 256;
  const int d = 256;
  const bool s1 = K1 == 512;
  float* a1 = alloc<float>((size_t)R * 512);
  float* yb[2] = {alloc<float>((size_t)R * d), alloc<float>((size_t)R * d)};
  float* sb[2] = {alloc<float>((size_t)R * 32), alloc<float>((size_t)R * 32)};
  float* vec = alloc<float>(2048);
  float* z = alloc<float>((size_t)R * 1024);
  float* bias = alloc<float>(2048);
  uint16_t* Wh = alloc<uint16_t>((size_t)1024 * 768);
  {  // statistics (mean, M2) per slice with a positive M2, unit vectors
    std::vector<float> h((size_t)R * 32);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (i % 2) ? 16.f : 0.5f;
    for (int k = 0; k < 2; ++k) CK(hipMemcpy(sb[k], h.data(), h.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> one(2048, 1.f);
    CK(hipMemcpy(vec, one.data(), one.size() * 4, hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int chain = 100;
  hipGraph_t graph;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < chain; ++i) {
    FoldGemmParams p{};
    p.B = R; p.t = 10; p.A1 = a1; p.K1 = K1; p.A2 = yb[i & 1];
    p.a2_stats = sb[i & 1]; p.a2_g = vec; p.a2_b = vec;
    if (s1) { p.a1_stats = sb[i & 1]; p.a1_s = vec; p.a1_c = vec; }
    p.Wy = vec; p.by = bias; p.y = yb[(i + 1) & 1]; p.y_stats = sb[(i + 1) & 1];
    p.Wz = vec; p.bz = bias; p.z = z; p.NZ = NZ; p.NY = d;
    p.Fy_hi = Wh; p.Fy_lo = Wh; p.Fz_hi = Wh; p.Fz_lo = Wh;
    launch_foldwide(p, s);
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
  const int nblk = (d + NZ) / 16 * ((R + 31) / 32);  // 32 x 16 tiles at R > 64 when N/32 tiles < 256
  std::vector<unsigned long long> ts((size_t)8192 * 8);
  if (mocr_debug_fold_ts(ts.data(), 8192 * 8)) { printf("no timestamps (library built without MOCR_FOLD_TS?)\n"); return 1; }
  int n = 0;
  unsigned long long rt_min = ~0ull, rt_max = 0;
  for (int b = 0; b < 8192; ++b)
    if (ts[b * 8]) { ++n; rt_min = std::min(rt_min, ts[b * 8]); rt_max = std::max(rt_max, ts[b * 8 + 6]); }
  std::vector<double> start, span, ph[4], end;
  for (int b = 0; b < 8192; ++b) {
    const unsigned long long* t = &ts[b * 8];
    if (!t[0]) continue;
    start.push_back((t[0] - rt_min) * 0.01);  // 100 MHz -> us
    end.push_back((t[6] - rt_min) * 0.01);
    span.push_back((t[6] - t[0]) * 0.01);
    for (int k = 0; k < 4; ++k) ph[k].push_back((double)(t[2 + k] - t[1 + k]));
  }
  const double clk_per_us = (ts[0 * 8 + 5] - ts[0 * 8 + 1]) / std::max(0.01, (ts[6] - ts[0]) * 0.01);
  printf("R=%d K1=%d NZ=%d: %.2f us per kernel in the chain; %d workgroups timed (expected %d)\n", R, K1, NZ,
         ms * 1000.0 / chain, n, nblk);
  printf("last kernel: first start -> last exit %.2f us; shader clock ~%.0f per us\n", (rt_max - rt_min) * 0.01,
         clk_per_us);
  printf("workgroup start offset us: p0 %.2f p50 %.2f p90 %.2f p100 %.2f\n", pct(start, 0), pct(start, .5),
         pct(start, .9), pct(start, 1));
  printf("workgroup exit offset  us: p0 %.2f p50 %.2f p90 %.2f p100 %.2f\n", pct(end, 0), pct(end, .5), pct(end, .9),
         pct(end, 1));
  printf("workgroup span us:         p0 %.2f p50 %.2f p90 %.2f p100 %.2f\n", pct(span, 0), pct(span, .5),
         pct(span, .9), pct(span, 1));
  const char* names[4] = {"issue + wait loads", "LN/split + MFMA loop", "reduce barrier", "epilogue + stores"};
  for (int k = 0; k < 4; ++k)
    printf("  %-22s cycles p10 %7.0f p50 %7.0f p90 %7.0f\n", names[k], pct(ph[k], .1), pct(ph[k], .5), pct(ph[k], .9));
  return 0;
}
