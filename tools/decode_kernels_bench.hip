// Per-kernel cost of each decode kernel of libmathocr.so, in a 200-long chain replayed
// from a hipGraph (B = 64 rows, d = 256, max_pos = 150, M = 144, V = 5075, step t = 100);
// `decode_kernels_bench N` replays each chain on N streams at once (replica contention).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/decode_kernels_bench.hip
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
      return 1;                                                         \
    }                                                                   \
  } while (0)

template <typename T>
T* alloc(size_t n) {
  void* p;
  if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) return nullptr;
  hipMemset(p, 0, n * sizeof(T));
  return (T*)p;
}

int main(int argc, char** argv) {
  const int NS = argc > 1 ? atoi(argv[1]) : 1;  // concurrent streams replaying each chain
  const int B = 64, d = 256, P = 150, M = 144, V = 5075, Vp = 5088, t = 100, L = 8;
  float* x = alloc<float>(B * 512);
  float* y = alloc<float>(B * 512);
  float* q = alloc<float>(B * d);
  float* att = alloc<float>(B * d);
  float* W = alloc<float>((size_t)Vp * 512);
  float* bias = alloc<float>(Vp);
  float* g = alloc<float>(1024);
  float* kc = alloc<float>((size_t)B * P * d);
  float* vc = alloc<float>((size_t)B * P * d);
  float* memkv = alloc<float>((size_t)L * B * M * 2 * d);
  float* logits = alloc<float>((size_t)B * Vp);
  int32_t* ids = alloc<int32_t>(B * 151);
  int32_t* feed = alloc<int32_t>(B * 151);
  int32_t* fin = alloc<int32_t>(B);
  float* logp = alloc<float>(B * 150);
  DecodeState* st = alloc<DecodeState>(1);
  float* stats = alloc<float>(B * 32);
  float* stats2 = alloc<float>(B * 32);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  auto rg = [&](int epi, int N, int K, bool aln, bool rln) {
    return [=](hipStream_t ss) {
      RowGemmParams p{};
      p.A = x; p.W = W; p.bias = bias; p.out = y; p.resid = q; p.kcache = kc; p.vcache = vc;
      p.B = B; p.N = N; p.K = K; p.ldo = (epi == DEC_LOGITS) ? Vp : (epi == DEC_RELU ? 512 : d);
      p.d = d; p.max_pos = P; p.n_valid = epi == DEC_LOGITS ? V : N; p.epi = epi; p.t = t; p.st = nullptr;
      if (epi == DEC_LOGITS) p.out = logits;
      if (aln) { p.a_ln_g = g; p.a_ln_b = g; p.a_stats = stats; }
      if (rln) { p.r_ln_g = g; p.r_ln_b = g; p.r_stats = stats; }
      p.out_stats = stats2;
      launch_rowgemm(p, ss);
    };
  };
  float* zb = alloc<float>(B * 768);
  float* part = alloc<float>(B * Vp / 4);
  float* wz = alloc<float>((size_t)768 * 768);
  uint16_t* w16 = alloc<uint16_t>((size_t)768 * 768);
  auto fg = [&](int K1, int NZ, bool s1, bool x3 = false) {
    return [=](hipStream_t ss) {
      FoldGemmParams p{};
      if (x3) { p.Wy_hi = w16; p.Wy_lo = w16; p.Wz_hi = w16; p.Wz_lo = w16; }
      p.B = B; p.t = t; p.A1 = x; p.K1 = K1; p.A2 = q; p.a2_stats = stats; p.a2_g = g; p.a2_b = g;
      if (s1) { p.a1_stats = stats; p.a1_s = g; p.a1_c = g; }
      p.Wy = W; p.by = bias; p.y = y; p.y_stats = stats2; p.Wz = wz; p.bz = bias; p.z = zb; p.NZ = NZ;
      launch_foldgemm(p, ss);
    };
  };
  auto sel = [=](const float* pt) {
    SelectArgs a{};
    a.st = st; a.t = t; a.logits = logits; a.ldl = Vp; a.V = V; a.ids = ids; a.feed = feed; a.ld_ids = 151;
    a.logp = logp; a.finished = fin; a.eos = 2; a.part = pt; a.nparts = Vp / 16;
    return a;
  };
  std::vector<std::pair<std::string, std::function<void(hipStream_t)>>> cases = {
      {"qkv N768 K256 +LN(A)", rg(DEC_QKV, 768, 256, true, false)},
      {"oproj N256 K256 +LN(res)", rg(DEC_RESADD, 256, 256, false, true)},
      {"qproj N256 K256 +LN(A)", rg(DEC_STORE, 256, 256, true, false)},
      {"ffn1 N512 K256 +LN(A)", rg(DEC_RELU, 512, 256, true, false)},
      {"ffn2 N256 K512 +LN(res)", rg(DEC_RESADD, 256, 512, false, true)},
      {"plain N256 K256", rg(DEC_STORE, 256, 256, false, false)},
      {"logits N5088 K256 +LN(A)", rg(DEC_LOGITS, Vp, 256, true, false)},
      {"self-attn t=100", [=](hipStream_t ss) {
         launch_dec_attn(nullptr, t, q, kc, vc, (size_t)P * d, d, t + 1, t + 1, att, B, d, 8, ss);
       }},
      {"cross-attn M=144", [=](hipStream_t ss) {
         launch_dec_attn(nullptr, t, q, memkv, memkv + d, (size_t)M * 2 * d, 2 * d, M, M, att, B, d, 8, ss);
       }},
      {"argmax+embed", [=](hipStream_t ss) {
         launch_dec_argmax(sel(nullptr), 0, B, W, W, x, d, ss);
       }},
      {"logits + tile partials", [=](hipStream_t ss) {
         RowGemmParams p{};
         p.A = x; p.W = W; p.bias = bias; p.out = logits; p.B = B; p.N = Vp; p.K = d; p.ldo = Vp; p.d = d;
         p.max_pos = P; p.n_valid = V; p.epi = DEC_LOGITS; p.t = t; p.a_ln_g = g; p.a_ln_b = g; p.a_stats = stats;
         p.part = part;
         launch_rowgemm(p, ss);
       }},
      {"argmax (tile partials)+qkv", [=](hipStream_t ss) {
         launch_dec_argmax(sel(part), 0, B, W, W, x, d, ss, W, W, zb);
       }},
      {"argmax+embed+qkv table", [=](hipStream_t ss) {
         launch_dec_argmax(sel(nullptr), 0, B, W, W, x, d, ss, W, W, zb);
       }},
      {"fold self-attn t=100 + select of t-1 (tile partials)", [=](hipStream_t ss) {
         FoldAttnParams a{};
         a.t = t; a.B = B; a.out = att; a.z = zb; a.z_ld = 3 * d;
         a.K = kc; a.V = vc; a.kcache = kc; a.vcache = vc; a.kv_b_stride = (size_t)P * d; a.kv_row_stride = d;
         a.n = t + 1;
         a.sel_on = 1; a.sel = sel(part); a.sel.t = t - 1; a.qtab = W; a.qpos = W; a.emb = W; a.pos = W; a.x = x;
         launch_dec_foldattn(a, true, ss);
       }},
      {"fold self-attn t=100", [=](hipStream_t ss) {
         FoldAttnParams a{};
         a.t = t; a.B = B; a.out = att; a.z = zb; a.z_ld = 3 * d; a.z_stats = stats; a.s = g; a.c = g;
         a.K = kc; a.V = vc; a.kcache = kc; a.vcache = vc; a.kv_b_stride = (size_t)P * d; a.kv_row_stride = d;
         a.n = t + 1;
         launch_dec_foldattn(a, true, ss);
       }},
      {"fold self-attn t=100 plain z", [=](hipStream_t ss) {
         FoldAttnParams a{};
         a.t = t; a.B = B; a.out = att; a.z = zb; a.z_ld = 3 * d;
         a.K = kc; a.V = vc; a.kcache = kc; a.vcache = vc; a.kv_b_stride = (size_t)P * d; a.kv_row_stride = d;
         a.n = t + 1;
         launch_dec_foldattn(a, true, ss);
       }},
      {"fold cross-attn M=144", [=](hipStream_t ss) {
         FoldAttnParams a{};
         a.t = t; a.B = B; a.out = att; a.z = zb; a.z_ld = d; a.z_stats = stats; a.s = g; a.c = g;
         a.K = memkv; a.V = memkv + d; a.kv_b_stride = (size_t)M * 2 * d; a.kv_row_stride = 2 * d; a.n = M;
         launch_dec_foldattn(a, false, ss);
       }},
      {"foldgemm y256+z256 K1=256 +LN", fg(256, 256, false)},
      {"foldgemm y256+z512 K1=256 +LN", fg(256, 512, false)},
      {"foldgemm y256+z768 K1=512 +unf", fg(512, 768, true)},
      {"foldgemm y256+z256 K1=256 +LN bf16x3", fg(256, 256, false, true)},
      {"foldgemm y256+z512 K1=256 +LN bf16x3", fg(256, 512, false, true)},
      {"foldgemm y256+z768 K1=512 +unf bf16x3", fg(512, 768, true, true)},
  };
  const int chain = 200;
  for (auto& c : cases) {
    hipGraph_t graph;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < chain; ++i) c.second(s);
    CK(hipStreamEndCapture(s, &graph));
    hipGraphExec_t exec;
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    CK(hipGraphLaunch(exec, s));
    CK(hipStreamSynchronize(s));
    std::vector<hipStream_t> sts(NS);
    std::vector<hipEvent_t> e0(NS), e1(NS);
    for (int i = 0; i < NS; ++i) {
      CK(hipStreamCreateWithFlags(&sts[i], hipStreamNonBlocking));
      CK(hipEventCreate(&e0[i]));
      CK(hipEventCreate(&e1[i]));
    }
    for (int i = 0; i < NS; ++i) {
      CK(hipEventRecord(e0[i], sts[i]));
      for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(exec, sts[i]));
      CK(hipEventRecord(e1[i], sts[i]));
    }
    float worst = 0.f;
    for (int i = 0; i < NS; ++i) {
      CK(hipEventSynchronize(e1[i]));
      float ms;
      CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      worst = ms > worst ? ms : worst;
    }
    printf("%-34s %.2f us per kernel (%d concurrent stream%s)\n", c.first.c_str(), worst * 1000.f / (5 * chain), NS,
           NS > 1 ? "s" : "");
    for (int i = 0; i < NS; ++i) CK(hipStreamDestroy(sts[i]));
    CK(hipGraphExecDestroy(exec));
    CK(hipGraphDestroy(graph));
  }
  return 0;
}
