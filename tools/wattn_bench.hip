// Standalone timing of the fused Swin attention-half kernel (wattn.hip) on synthetic data
// of the stage-1 / stage-2 shapes of a 64-image 384x384 batch, with per-phase s_memtime
// stamps (A: norm1 -> LDS, B: k/v/q GEMMs, C: attention, D: proj + residual).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/wattn_bench.hip -o tools/wattn_bench
#define WATTN_STAMPS
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <random>
#include <vector>

#include "../handwritten-math-ocr-api_amd/csrc/wattn.hip"

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
T* upload(const std::vector<T>& h) {
  void* p;
  CK(hipMalloc(&p, h.size() * sizeof(T)));
  CK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return (T*)p;
}

static uint16_t bf16_bits(float x) {  // round to nearest even
  uint32_t u;
  memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf16_val(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static void run(int C, int H, int shift, bool x3, int reps) {
  const int B = 64, heads = C / 32;
  WinGeom wg{};
  wg.H = wg.W = H;
  wg.pH = wg.pW = (H + 6) / 7 * 7;
  wg.sh = wg.sw = (7 >= wg.pH) ? 0 : shift;
  wg.nWx = wg.pW / 7;
  wg.nWin = wg.nWx * (wg.pH / 7);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> X((size_t)B * H * H * C), g(C), b(C), bq(3 * C), bp(C), table((size_t)4 * heads * 64 * 64);
  for (auto& v : X) v = nd(rng);
  for (auto& v : g) v = 1.f + 0.1f * nd(rng);
  for (auto& v : b) v = 0.1f * nd(rng);
  for (auto& v : bq) v = 0.1f * nd(rng);
  for (auto& v : bp) v = 0.1f * nd(rng);
  for (size_t i = 0; i < table.size(); ++i) table[i] = (i % 64) < 49 ? 0.5f * nd(rng) : -INFINITY;
  auto planes = [&](int n, std::vector<uint16_t>& hi, std::vector<uint16_t>& lo) {
    hi.resize(n);
    lo.resize(n);
    for (int i = 0; i < n; ++i) {
      const float w = 0.05f * nd(rng);
      hi[i] = bf16_bits(w);
      lo[i] = bf16_bits(w - bf16_val(hi[i]));
    }
  };
  std::vector<uint16_t> wqh, wql, wph, wpl;
  planes(3 * C * C, wqh, wql);
  planes(C * C, wph, wpl);
  SwinAttnParams p{};
  p.X = upload(X);
  p.ln_g = upload(g);
  p.ln_b = upload(b);
  p.wqkv = upload(wqh);
  p.wqkv_lo = x3 ? upload(wql) : nullptr;
  p.bqkv = upload(bq);
  p.wproj = upload(wph);
  p.wproj_lo = x3 ? upload(wpl) : nullptr;
  p.bproj = upload(bp);
  p.table = upload(table);
  p.B = B;
  p.C = C;
  p.heads = heads;
  p.wg = wg;
  const size_t nw = (size_t)B * wg.nWin * heads;
  CK(hipMalloc(&p.stamps, nw * 8 * sizeof(unsigned long long)));
  CK(hipMemset(p.stamps, 0, nw * 8 * sizeof(unsigned long long)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  SwinAttnParams q = p;
  q.stamps = nullptr;
  for (int i = 0; i < 3; ++i) launch_swin_attn_fused(q, 0);
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch_swin_attn_fused(q, 0);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1000.0 * ms / reps;
  launch_swin_attn_fused(p, 0);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> st(nw * 8);
  CK(hipMemcpy(st.data(), p.stamps, st.size() * 8, hipMemcpyDeviceToHost));
  double ph[7] = {0};
  unsigned long long t0 = ~0ull, t1 = 0;
  size_t used = 0;
  for (size_t w = 0; w < nw; ++w) {
    if (st[w * 8] == 0 || st[w * 8 + 7] == 0) continue;  // persistent grid: fewer workgroups than windows
    ++used;
    for (int i = 0; i < 7; ++i) ph[i] += (double)(st[w * 8 + i + 1] - st[w * 8 + i]);
    t0 = std::min(t0, st[w * 8]);
    t1 = std::max(t1, st[w * 8 + 7]);
  }
  const double life = (ph[0] + ph[1] + ph[2] + ph[3] + ph[4] + ph[5] + ph[6]) / used;
  printf("C=%d H=%d shift=%d %s: %.1f us/launch; per wave (memtime ticks): A %.0f | barA %.0f | B %.0f | barB %.0f | "
         "C %.0f | barC %.0f | D %.0f | life %.0f; span %llu ticks\n",
         C, H, wg.sh, x3 ? "bf16x3" : "bf16", us, ph[0] / used, ph[1] / used, ph[2] / used, ph[3] / used, ph[4] / used,
         ph[5] / used, ph[6] / used, life, t1 - t0);
}

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;  // one configuration (PMC runs)
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  if (only < 0 || only == 0) run(96, 96, 3, true, reps);
  if (only < 0 || only == 1) run(96, 96, 0, true, reps);
  if (only < 0 || only == 2) run(192, 48, 3, true, reps);
  if (only < 0 || only == 3) run(96, 96, 3, false, reps);
  return 0;
}
