// Decode-step kernels at R rows in 100-long graph-captured chains (per-kernel chain time,
// launch gap included): the narrow 16x16-tile fold GEMMs (decfold.hip) against the wide
// tiles (decwide.hip), the logits, and the fold attention kernels.
//   wide_bench [R ...]     (default 64 256)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/wide_bench.hip
//        -L handwritten-math-ocr-api_amd/lib -lmathocr -Wl,-rpath,$PWD/handwritten-math-ocr-api_amd/lib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../handwritten-math-ocr-api_amd/csrc/kernels.h"

using namespace mocr;

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

template <typename T>
T* alloc(size_t n) {
  void* p;
  CK(hipMalloc(&p, n * sizeof(T)));
  CK(hipMemset(p, 0, n * sizeof(T)));
  return (T*)p;
}

// small deterministic values (statistics must give a finite rstd)
__global__ void fill_kernel(float* p, size_t n, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = scale * (float)((i * 2654435761u) % 1000) / 1000.f;
}
void fill(float* p, size_t n, float scale) {
  fill_kernel<<<1024, 256>>>(p, n, scale);
  CK(hipDeviceSynchronize());
}

double run_chain(hipStream_t s, const std::function<void(hipStream_t)>& f, int chain = 100) {
  hipGraph_t graph;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < chain; ++i) f(s);
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
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  return ms * 1000.0 / (5 * chain);
}

int main(int argc, char** argv) {
  std::vector<int> Rs;
  for (int i = 1; i < argc; ++i) Rs.push_back(atoi(argv[i]));
  if (Rs.empty()) Rs = {64, 256};
  const int d = 256, P = 150, M = 144, Vp = 5120, V = 5075, t = 100;
  const int Rmax = 512;
  float* a1 = alloc<float>((size_t)Rmax * 512);
  float* a2 = alloc<float>((size_t)Rmax * d);
  float* st1 = alloc<float>((size_t)Rmax * 32);
  float* st2 = alloc<float>((size_t)Rmax * 32);
  float* ystats = alloc<float>((size_t)Rmax * 32);
  float* vec = alloc<float>(1024);
  float* W = alloc<float>((size_t)Vp * 768);
  uint16_t* Wh = alloc<uint16_t>((size_t)Vp * 768);
  float* bias = alloc<float>(Vp);
  float* y = alloc<float>((size_t)Rmax * d);
  float* z = alloc<float>((size_t)Rmax * Vp);
  float* part = alloc<float>((size_t)Rmax * Vp / 4);
  float* kc = alloc<float>((size_t)Rmax * P * d);
  float* vc = alloc<float>((size_t)Rmax * P * d);
  float* memkv = alloc<float>((size_t)Rmax * M * 2 * d);
  float* att = alloc<float>((size_t)Rmax * d);
  fill(a1, (size_t)Rmax * 512, 1.f);
  fill(a2, (size_t)Rmax * d, 1.f);
  fill(W, (size_t)Vp * 768, 0.01f);
  fill(vec, 1024, 1.f);
  fill(kc, (size_t)Rmax * P * d, 0.1f);
  fill(vc, (size_t)Rmax * P * d, 0.1f);
  fill(memkv, (size_t)Rmax * M * 2 * d, 0.1f);
  {  // statistics: (mean, M2) per slice -> positive M2
    std::vector<float> h((size_t)Rmax * 32);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (i % 2) ? 16.f : 0.5f;
    CK(hipMemcpy(st1, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(st2, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int R : Rs) {
    auto fg = [&](int K1, int NZ, bool s1, bool s2, bool wide, bool x3, int nw = 0) {
      return [=](hipStream_t ss) {
        FoldGemmParams p{};
        p.waves = nw;
        p.B = R; p.t = t; p.A1 = a1; p.K1 = K1; p.A2 = a2;
        if (s2) { p.a2_stats = st2; p.a2_g = vec; p.a2_b = vec; }
        if (s1) { p.a1_stats = st1; p.a1_s = vec; p.a1_c = vec; }
        p.Wy = W; p.by = bias; p.y = y; p.y_stats = ystats; p.Wz = W; p.bz = bias; p.z = z; p.NZ = NZ;
        if (x3) { p.Wy_hi = Wh; p.Wy_lo = Wh; p.Wz_hi = Wh; p.Wz_lo = Wh; p.Fy_hi = Wh; p.Fy_lo = Wh; p.Fz_hi = Wh; p.Fz_lo = Wh; }
        p.Fy = W; p.Fz = W;  // timing only: fragment-major buffers of the same size
        p.NY = d;
        if (wide) launch_foldwide(p, ss); else launch_foldgemm(p, ss);
      };
    };
    auto lg = [&](bool wide, bool x3, int nw = 0, int bm = 0) {
      return [=](hipStream_t ss) {
        if (wide) {
          FoldGemmParams p{};
          p.waves = nw;
          p.tile_cols = bm;
          p.B = R; p.t = t; p.K1 = 0; p.NY = 0; p.A2 = a2; p.a2_stats = st2; p.a2_g = vec; p.a2_b = vec;
          p.Wz = W; p.bz = bias; p.z = z; p.NZ = Vp; p.n_valid = V; p.part = part;
          if (x3) { p.Fz_hi = Wh; p.Fz_lo = Wh; }
          p.Fz = W;
          launch_foldwide(p, ss);
        } else {
          RowGemmParams p{};
          p.A = a2; p.W = W; p.bias = bias; p.out = z; p.B = R; p.N = Vp; p.K = d; p.ldo = Vp; p.d = d;
          p.max_pos = P; p.n_valid = V; p.epi = DEC_LOGITS; p.t = t; p.a_ln_g = vec; p.a_ln_b = vec;
          p.a_stats = st2; p.part = part;
          launch_rowgemm(p, ss);
        }
      };
    };
    auto fa = [&](bool self) {
      return [=](hipStream_t ss) {
        FoldAttnParams a{};
        a.t = t; a.B = R; a.out = att; a.z = z; a.z_stats = st2; a.s = vec; a.c = vec;
        if (self) {
          a.z_ld = 3 * d; a.K = kc; a.V = vc; a.kcache = kc; a.vcache = vc; a.kv_b_stride = (size_t)P * d;
          a.kv_row_stride = d; a.n = t + 1;
        } else {
          a.z_ld = d; a.K = memkv; a.V = memkv + d; a.kv_b_stride = (size_t)M * 2 * d; a.kv_row_stride = 2 * d;
          a.n = M;
        }
        launch_dec_foldattn(a, self, ss);
      };
    };
    std::vector<std::pair<std::string, std::function<void(hipStream_t)>>> cases = {
        {"narrow y256+z256 K1=256 LN x3", fg(256, 256, false, true, false, true)},
        {"wide4  y256+z256 K1=256 LN x3", fg(256, 256, false, true, true, true, 4)},
        {"wide8  y256+z256 K1=256 LN x3", fg(256, 256, false, true, true, true, 8)},
        {"narrow y256+z512 K1=256 LN x3", fg(256, 512, false, true, false, true)},
        {"wide4  y256+z512 K1=256 LN x3", fg(256, 512, false, true, true, true, 4)},
        {"wide8  y256+z512 K1=256 LN x3", fg(256, 512, false, true, true, true, 8)},
        {"narrow y256+z768 K1=512 unf x3", fg(512, 768, true, true, false, true)},
        {"wide4  y256+z768 K1=512 unf x3", fg(512, 768, true, true, true, true, 4)},
        {"wide8  y256+z768 K1=512 unf x3", fg(512, 768, true, true, true, true, 8)},
        {"wide8  y256+z768 K1=512 unf f32", fg(512, 768, true, true, true, false, 8)},
        {"narrow logits f32", lg(false, false)},
        {"wide4  logits x3", lg(true, true, 4)},
        {"wide8  logits x3", lg(true, true, 8)},
        {"wide4  logits x3 64-col tiles", lg(true, true, 4, 64)},
        {"wide4  logits x3 128-col tiles", lg(true, true, 4, 128)},
        {"wide8  logits x3 128-col tiles", lg(true, true, 8, 128)},
        {"wide8  logits f32", lg(true, false, 8)},
        {"fold cross-attn M=144", fa(false)},
        {"fold self-attn t=100", fa(true)},
    };
    for (auto& c : cases) printf("R=%3d %-36s %7.2f us per kernel\n", R, c.first.c_str(), run_chain(s, c.second));
    fflush(stdout);
  }
  return 0;
}
