// Swin-T encoder kernels other than the GEMMs (torchvision swin_t().features, SURVEY.md
// Appendix A; the 1-channel stem is src/model_swin.py:19-34).
//
// Activations are NHWC fp32 [B, H, W, C].  The shifted-window geometry (zero pad to a
// multiple of 7 after norm1, roll(-s), window partition, region mask on the padded
// map, window reverse, roll(+s), crop) is index arithmetic inside the kernels: the
// padded/rolled map is never materialised.  Padded tokens enter the window as zero
// rows after LayerNorm, so their k/v equal the qkv bias and they stay unmasked keys,
// exactly as in torchvision.
#include "kernels.h"
#include "lanes.h"

namespace mocr {

namespace {

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Row outputs: fp32 and/or bf16 hi plane and/or lo plane (x - bf16(x)), as the
// consuming GEMM's precision needs.
struct RowOut {
  float* f32;
  uint16_t* hi;
  uint16_t* lo;
};

__device__ __forceinline__ void store_val(const RowOut& o, size_t off, float v) {
  if (o.f32) o.f32[off] = v;
  if (o.hi) {
    const uint16_t h = f32_to_bf16_rne(v);
    o.hi[off] = h;
    if (o.lo) o.lo[off] = f32_to_bf16_rne(v - __uint_as_float((uint32_t)h << 16));
  }
}

// ---------------------------------------------------------------- row-group LayerNorm
// LPR lanes per row, F floats per lane (C = LPR*F: 96 -> 8 lanes, 192 -> 16, 384 -> 32,
// 768 -> 64 with F = 12; 1536 -> 64 with F = 24), 16-B loads and stores, statistics
// reduced over the row's lanes with shuffles (mean, then Σ(x - mean)², two passes).
//   MODE_ROWS:  Y[r] = LN(X[r]);
//   MODE_WIN:   row r of the shifted-window partition (ln_partition_kernel's mapping;
//               padded tokens are zero rows);
//   MODE_MERGE: PatchMerging's [x(0,0), x(1,0), x(0,1), x(1,1)] gather (merge_ln_kernel).
enum { MODE_ROWS = 0, MODE_WIN = 1, MODE_MERGE = 2 };

struct LnGeom {
  long rows;
  int C;         // row length (4C for MODE_MERGE)
  int B, H, W;   // MODE_MERGE: input map; MODE_WIN: via win
  int Cin;       // MODE_MERGE: input channels
  WinGeom win;
};

// bf16 planes leave through LDS as whole 16-B lanes (merge2 / merge3 norms 408 / 276 ->
// 304 / 180 us per 512 images, profiles/r05/r07r/)
template <int LPR, int F, int MODE>
__global__ void __launch_bounds__(256) ln_group_kernel(const float* __restrict__ X, const float* __restrict__ g,
                                                       const float* __restrict__ b, RowOut out, LnGeom geo) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int gi = lane % LPR;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool live = row < geo.rows;
  const int c0 = gi * F;
  float v[F];
#pragma unroll
  for (int e = 0; e < F; ++e) v[e] = 0.f;
  bool zero_row = !live;
  const float* src = nullptr;
  if (live) {
    if constexpr (MODE == MODE_ROWS) {
      src = X + (size_t)row * geo.C + c0;
    } else if constexpr (MODE == MODE_WIN) {
      const WinGeom& wg = geo.win;
      const int per_img = wg.nWin * kWinTok;
      const int bi = (int)(row / per_img);
      const int rem = (int)(row - (long)bi * per_img);
      const int win = rem / kWinTok;
      const int tk = rem - win * kWinTok;
      const int wy = win / wg.nWx;
      const int wx = win - wy * wg.nWx;
      int y = wy * kWin + tk / kWin + wg.sh;
      int x = wx * kWin + tk % kWin + wg.sw;
      if (y >= wg.pH) y -= wg.pH;
      if (x >= wg.pW) x -= wg.pW;
      if (y < wg.H && x < wg.W) src = X + ((size_t)(bi * wg.H + y) * wg.W + x) * geo.C + c0;
      else zero_row = true;  // F.pad after norm1: zero token, LayerNorm not applied
    } else {
      const int Ho = (geo.H + 1) / 2, Wo = (geo.W + 1) / 2;
      const int bi = (int)(row / ((long)Ho * Wo));
      const int rem = (int)(row - (long)bi * Ho * Wo);
      const int oy = rem / Wo;
      const int ox = rem - oy * Wo;
      const int q = c0 / geo.Cin;  // cat order (dy,dx) = (0,0), (1,0), (0,1), (1,1)
      const int y = 2 * oy + (q & 1);
      const int x = 2 * ox + (q >> 1);
      if (y < geo.H && x < geo.W) src = X + ((size_t)(bi * geo.H + y) * geo.W + x) * geo.Cin + (c0 - q * geo.Cin);
    }
  }
  if (src) {
#pragma unroll
    for (int e = 0; e < F; e += 4) {
      const floatx4 t = *reinterpret_cast<const floatx4*>(src + e);
      v[e] = t[0];
      v[e + 1] = t[1];
      v[e + 2] = t[2];
      v[e + 3] = t[3];
    }
  }
  if (!zero_row) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < F; ++e) s += v[e];
    s = row_sum<LPR>(s);  // the row's LPR lanes, by DPP / permlane (lanes.h; the butterfly's pairs)
    const float mean = s / (float)geo.C;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < F; ++e) {
      const float d = v[e] - mean;
      q += d * d;
    }
    q = row_sum<LPR>(q);
    const float rstd = 1.0f / sqrtf(q / (float)geo.C + 1e-5f);
#pragma unroll
    for (int e = 0; e < F; e += 4) {
      const floatx4 gg = *reinterpret_cast<const floatx4*>(g + c0 + e);
      const floatx4 bb = *reinterpret_cast<const floatx4*>(b + c0 + e);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[e + k] = (v[e + k] - mean) * rstd * gg[k] + bb[k];
    }
  }
  if (!out.f32 && out.hi) {
    // the wave's RPW rows are 64 F contiguous outputs: each plane goes through the wave's
    // LDS slice and leaves as whole 16-B lanes (8 bf16), not F / 4 8-B stores per lane
    __shared__ __attribute__((aligned(16))) uint32_t st[4][32 * F];
    uint32_t* ws = st[threadIdx.x >> 6];
    const long row0 = row - lane / LPR;  // the wave's first row
    const size_t base = (size_t)row0 * geo.C;
    uint32_t hp[F / 2], lp[F / 2];
#pragma unroll
    for (int e = 0; e < F; e += 2) split2_bf16(v[e], v[e + 1], hp[e / 2], lp[e / 2]);
#pragma unroll
    for (int plane = 0; plane < 2; ++plane) {
      uint16_t* dst = plane ? out.lo : out.hi;
      if (!dst) break;  // wave-uniform
#pragma unroll
      for (int e = 0; e < F / 2; e += 2)
        *reinterpret_cast<uint2*>(ws + lane * (F / 2) + e) = plane ? make_uint2(lp[e], lp[e + 1]) : make_uint2(hp[e], hp[e + 1]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < (8 * F + 63) / 64; ++k) {
        const int f = lane + 64 * k;  // 16-B chunk of the wave's 128 F bytes
        if ((8 * F) % 64 == 0 || f < 8 * F)
          if (row0 + (8 * f) / geo.C < geo.rows)
            *reinterpret_cast<uint4*>(dst + base + 8 * f) = *reinterpret_cast<const uint4*>(ws + 4 * f);
      }
      __builtin_amdgcn_wave_barrier();
    }
    return;
  }
  if (!live) return;
  const size_t off = (size_t)row * geo.C + c0;
#pragma unroll
  for (int e = 0; e < F; e += 4) {
    if (out.f32) *reinterpret_cast<floatx4*>(out.f32 + off + e) = floatx4{v[e], v[e + 1], v[e + 2], v[e + 3]};
    if (out.hi) {
      uint32_t h0, l0, h1, l1;
      split2_bf16(v[e], v[e + 1], h0, l0);
      split2_bf16(v[e + 2], v[e + 3], h1, l1);
      *reinterpret_cast<uint2*>(out.hi + off + e) = make_uint2(h0, h1);
      if (out.lo) *reinterpret_cast<uint2*>(out.lo + off + e) = make_uint2(l0, l1);
    }
  }
}

template <int MODE>
void launch_ln_group(const float* X, const float* g, const float* b, const RowOut& o, const LnGeom& geo,
                     hipStream_t s) {
  auto blocks = [&](int lpr) { return (unsigned)((geo.rows + 4 * (64 / lpr) - 1) / (4 * (64 / lpr))); };
  switch (geo.C) {
    case 96: ln_group_kernel<8, 12, MODE><<<blocks(8), 256, 0, s>>>(X, g, b, o, geo); break;
    case 192: ln_group_kernel<16, 12, MODE><<<blocks(16), 256, 0, s>>>(X, g, b, o, geo); break;
    case 384: ln_group_kernel<32, 12, MODE><<<blocks(32), 256, 0, s>>>(X, g, b, o, geo); break;
    case 768: ln_group_kernel<64, 12, MODE><<<blocks(64), 256, 0, s>>>(X, g, b, o, geo); break;
    case 1536: ln_group_kernel<64, 24, MODE><<<blocks(64), 256, 0, s>>>(X, g, b, o, geo); break;
    default: throw std::runtime_error("layernorm: unsupported row length " + std::to_string(geo.C));
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- stem (vectorised)
// Conv2d(1, 96, 4, 4) + LayerNorm(96): 16 lanes per token, 6 channels per lane whose
// 6x16 weights stay in registers over a grid-stride loop of tokens; LayerNorm over the 16
// lanes.
// The same per-token arithmetic with the patch loads spread over the wave: each lane loads
// one float4 (a patch row) of 16 consecutive tokens, one sweep ahead, and the four 16-lane
// groups read their tokens' patches back from the wave's 1 KB LDS slice. The 4-float4-per-
// lane form keeps one wave's 4 patches (256 B) in flight per HBM round trip; this one 16
// patches plus the next sweep's 16.
// X leaves through an LDS slice as whole 16-B lanes (596 -> 457 us per 512 images against
// three 8-B stores per lane, profiles/r05/r07q/).
template <int DEPTH>
__global__ void __launch_bounds__(256) stem16w_kernel(const float* __restrict__ img, const float* __restrict__ w,
                                                      const float* __restrict__ bias, const float* __restrict__ g,
                                                      const float* __restrict__ beta, float* __restrict__ X, long ntok,
                                                      int H, int W, int Hs, int Ws) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int gi = lane & 15;
  const int grp = lane >> 4;
  const int c0 = gi * 6;
  __shared__ floatx4 patch[4][64];  // per wave: 16 tokens x 4 patch rows
  __shared__ __attribute__((aligned(16))) float xout[4][16 * 96];  // per wave: 16 tokens of X
  float wr[6][16], br[6], gr[6], be[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      const floatx4 t = *reinterpret_cast<const floatx4*>(w + (c0 + c) * 16 + 4 * k4);
#pragma unroll
      for (int e = 0; e < 4; ++e) wr[c][4 * k4 + e] = t[e];
    }
    br[c] = bias[c0 + c];
    gr[c] = g[c0 + c];
    be[c] = beta[c0 + c];
  }
  const long hw = (long)Hs * Ws;
  auto load_row = [&](long t0) -> floatx4 {  // row lane % 4 of token t0 + lane / 4 (clamped)
    long tok = t0 + (lane >> 2);
    tok = tok < ntok ? tok : ntok - 1;
    const int b = (int)(tok / hw);
    const int rem = (int)(tok - (long)b * hw);
    const int y = rem / Ws;
    const int x = rem - y * Ws;
    return *reinterpret_cast<const floatx4*>(img + ((size_t)b * H + 4 * y + (lane & 3)) * W + 4 * x);
  };
  const long sweep = (long)gridDim.x * 64;  // tokens per sweep of all waves
  long t0 = ((long)blockIdx.x * 4 + wave) * 16;
  if (t0 >= ntok) return;  // wave-uniform
  floatx4 next[DEPTH];  // the patch rows of the next DEPTH sweeps
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d == 0 || t0 + d * sweep < ntok) next[d] = load_row(t0 + d * sweep);
  for (; t0 < ntok; t0 += sweep) {
    patch[wave][lane] = next[0];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int d = 0; d + 1 < DEPTH; ++d) next[d] = next[d + 1];
    if (t0 + DEPTH * sweep < ntok) next[DEPTH - 1] = load_row(t0 + DEPTH * sweep);
#pragma unroll 1
    for (int j = 0; j < 4; ++j) {
      const int tw = 4 * j + grp;  // token within the wave's 16
      float px[16];
#pragma unroll
      for (int ky = 0; ky < 4; ++ky) {
        const floatx4 t = patch[wave][4 * tw + ky];
        px[4 * ky] = t[0];
        px[4 * ky + 1] = t[1];
        px[4 * ky + 2] = t[2];
        px[4 * ky + 3] = t[3];
      }
      float v[6];
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = fmaf(wr[c][k], px[k], acc);
        v[c] = acc + br[c];
        s += v[c];
      }
      s = row_sum<16>(s);
      const float mean = s / 96.f;
      float q = 0.f;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const float d = v[c] - mean;
        q += d * d;
      }
      q = row_sum<16>(q);
      const float rstd = 1.0f / sqrtf(q / 96.f + 1e-5f);
      float o[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) o[c] = (v[c] - mean) * rstd * gr[c] + be[c];
      float* os = xout[wave] + tw * 96 + c0;
#pragma unroll
      for (int e = 0; e < 3; ++e) *reinterpret_cast<float2*>(os + 2 * e) = make_float2(o[2 * e], o[2 * e + 1]);
    }
    {  // the 16 tokens' 6 KB of X as whole 1 KB store instructions
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 2
      for (int k = 0; k < 6; ++k) {
        const int f = lane + 64 * k;  // float4 index among the 16 tokens' 384
        if (t0 + f / 24 < ntok)
          *reinterpret_cast<floatx4*>(X + (size_t)t0 * 96 + 4 * f) = *reinterpret_cast<const floatx4*>(xout[wave] + 4 * f);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the slices are rewritten by the next sweep
  }
}

// ---------------------------------------------------------------- window attention
// One workgroup (4 waves) per (window, head) on v_mfma_f32_32x32x2_f32:
//   S = (q * 32^-0.5) kᵀ  (49x49 padded to 64x64; wave w owns S block (w>>1, w&1)),
//   + relative-position bias, + -100 where the shift-mask regions differ;
//   row softmax through LDS (one wave per row, wave max/sum reduce);
//   O = P V  (wave w owns row block w>>1 and key half w&1; the two halves are summed
//   through LDS in a fixed order).
// q/k fragments are read straight from the qkv rows (16 contiguous floats per lane:
// lane half h feeds k = 16h + s at MFMA step s); V is staged transposed in LDS so the
// P·V B-operand is also 16 contiguous floats per lane.  q is scaled before the matmul
// and the mask added after the bias, as in torchvision.
constexpr int SP = 68;  // padded LDS row stride (floats): 16-B aligned, 17 slots per row

__global__ void __launch_bounds__(256) window_attention_kernel(const float* __restrict__ QKV,
                                                               const float* __restrict__ relbias,
                                                               RowOut out, int C, WinGeom wg) {
  __shared__ float S[64 * SP];
  __shared__ float Vt[kHeadDim * SP];
  __shared__ int region[64];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int l32 = lane & 31;
  const int half = lane >> 5;
  const long wg_idx = blockIdx.x;  // global window index (b * nWin + win)
  const int h = blockIdx.y;
  const int C3 = 3 * C;
  const size_t base = (size_t)wg_idx * kWinTok;
  const float scale = 0.17677669529663687f;  // 32 ** -0.5

  // V^T into LDS (zero for padded keys 49..63)
  for (int idx = tid; idx < 64 * kHeadDim; idx += 256) {
    const int t = idx >> 5;
    const int dd = idx & 31;
    Vt[dd * SP + t] = t < kWinTok ? QKV[(base + t) * C3 + 2 * C + h * kHeadDim + dd] : 0.f;
  }
  const bool masked = (wg.sh + wg.sw) > 0;
  if (masked && tid < kWinTok) {
    const int win = (int)(wg_idx % wg.nWin);
    const int wy = win / wg.nWx;
    const int wx = win - wy * wg.nWx;
    region[tid] = 3 * shift_region(wy * kWin + tid / kWin, wg.pH, wg.sh) +
                  shift_region(wx * kWin + tid % kWin, wg.pW, wg.sw);
  }

  // ---- S block (bi, bj)
  const int bi = wave >> 1, bj = wave & 1;
  {
    const int qi = bi * 32 + l32;
    const int kj = bj * 32 + l32;
    float qa[16], kb[16];
    if (qi < kWinTok) {
      const float* src = QKV + (base + qi) * C3 + h * kHeadDim + 16 * half;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(src + 4 * i);
#pragma unroll
        for (int e = 0; e < 4; ++e) qa[4 * i + e] = v[e] * scale;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) qa[i] = 0.f;
    }
    if (kj < kWinTok) {
      const float* src = QKV + (base + kj) * C3 + C + h * kHeadDim + 16 * half;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(src + 4 * i);
#pragma unroll
        for (int e = 0; e < 4; ++e) kb[4 * i + e] = v[e];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) kb[i] = 0.f;
    }
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qa[s], kb[s], acc, 0, 0, 0);
    __syncthreads();  // region[] ready
    const float* rb = relbias + (size_t)h * kWinTok * kWinTok;
    const int col = bj * 32 + l32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = bi * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
      if (row < kWinTok && col < kWinTok) {
        float v = acc[r] + rb[row * kWinTok + col];
        if (masked && region[row] != region[col]) v = v + (-100.0f);
        S[row * SP + col] = v;
      }
    }
  }
  __syncthreads();

  // ---- softmax over the 49 keys of each row; padded keys get P = 0
  for (int i = wave; i < kWinTok; i += 4) {
    const float x = lane < kWinTok ? S[i * SP + lane] : -INFINITY;
    const float m = wave_max(x);
    const float e = lane < kWinTok ? expf(x - m) : 0.f;
    const float sum = wave_sum(e);
    S[i * SP + lane] = e / sum;  // lanes 49..63 write 0
  }
  __syncthreads();

  // ---- O = P V: row block bi, key half kh
  const int kh = wave & 1;
  floatx16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
  {
    const int pi = bi * 32 + l32;  // rows >= 49 read stale LDS rows: results discarded
    const float* prow = &S[pi * SP + 32 * kh + 16 * half];
    const float* vrow = &Vt[l32 * SP + 32 * kh + 16 * half];
    float pa[16], vb[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const floatx4 p4 = *reinterpret_cast<const floatx4*>(prow + 4 * i);
      const floatx4 v4 = *reinterpret_cast<const floatx4*>(vrow + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pa[4 * i + e] = p4[e];
        vb[4 * i + e] = v4[e];
      }
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) o = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[s], vb[s], o, 0, 0, 0);
  }
  __syncthreads();  // everyone is done reading S; reuse it for the key-half exchange
  float* red = S;   // [2 row blocks][16 regs][64 lanes]
  if (kh == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(bi * 16 + r) * 64 + lane] = o[r];
  }
  __syncthreads();
  if (kh == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = bi * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
      if (row < kWinTok) {
        const float v = o[r] + red[(bi * 16 + r) * 64 + lane];
        store_val(out, (base + row) * C + h * kHeadDim + l32, v);
      }
    }
  }
}

// ---------------------------------------------------------------- window attention on bf16 MFMA
// One wave per (window, head), no LDS, no block barrier (bf16 / bf16x3 precision modes).
//   S^T = K Q^T   v_mfma_f32_16x16x32_bf16, tile (key tile kt, query tile qt), k = head dim:
//                 A = K[key 16kt + l%16][8(l/16) .. +7], B = Q[q 16qt + l%16][same] -- both
//                 are 8 contiguous floats of one QKV row, loaded straight from HBM.
//   softmax over the keys of a query column: 16 values per lane (kt, r) + 4 lane groups.
//   O^T = V^T P^T with k = keys permuted so that the B operand of k-step s is exactly the
//                 P^T accumulators of key tiles 2s, 2s+1 (lane keys 4(l/16) + r, r = 0..3):
//                 A = V[keys 32s + {0,16} + 4(l/16) + r][d 16dt + l%16].
// `table` = [type][head][64 q][64 key] fp32: relative-position bias + shift mask for the
// window type (last window row / column), -inf on the padded keys 49..63 (host-built,
// engine.hip build_relmask).  PASSES = 3: hi*hi + hi*lo + lo*hi (bf16x3), 1: hi*hi.
typedef __bf16 abf16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t au16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split8(const float (&x)[8], abf16x8& hi, abf16x8& lo) {
  uint4 h, l;
  split2_bf16(x[0], x[1], h.x, l.x);
  split2_bf16(x[2], x[3], h.y, l.y);
  split2_bf16(x[4], x[5], h.z, l.z);
  split2_bf16(x[6], x[7], h.w, l.w);
  hi = __builtin_bit_cast(abf16x8, h);
  lo = __builtin_bit_cast(abf16x8, l);
}

template <int PASSES>
__device__ __forceinline__ floatx4 mfma3(const abf16x8& ah, const abf16x8& al, const abf16x8& bh,
                                         const abf16x8& bl, floatx4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
  if constexpr (PASSES == 3) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  }
  return c;
}

// One wave per (window, head).  Window-token mode (bqkv == nullptr): QKV rows are the
// window tokens (the partition LayerNorm's order, padded tokens included) and O goes to
// the same rows.  Pixel mode (bqkv != nullptr): QKV and O rows are the image's tokens in
// X's order; a window slot maps to its pixel through the shift roll, and a padded token's
// k / v are the qkv bias (its LayerNorm'd input is zero, so W . 0 + b, bitwise), its
// query is never written.  Both modes give the same bits for every real token.
//
// Operands come in through buffer loads (a 32-bit byte offset per lane against a
// wave-uniform descriptor of the launch's QKV rows, qkv_bytes): a slot's row offset is
// computed once per lane and shuffled, with no 64-bit address arithmetic, and the slots
// without a row (>= 49, padded tokens) carry an offset past the end of the buffer, which
// the hardware's range check turns into zeros -- no branch around any load.  A padded
// token's k / v then take the bias (selected, bitwise the old path's value) in the
// windows that have one (a wave-uniform ballot).  The launcher splits the batch into
// image chunks of < 2 GiB of QKV rows.
// the O planes as 16-B stores, lane pairs trading halves (s4.wattn 614 -> 558 us per 512
// images against 8-B stores, profiles/r05/r07x/)
template <int PASSES>
__global__ void __launch_bounds__(256) window_attention_mfma_kernel(const float* __restrict__ QKV,
                                                                    const float* __restrict__ table, RowOut out,
                                                                    int C, int heads, long npairs, WinGeom wg,
                                                                    const float* __restrict__ bqkv, int qkv_bytes) {
  const int lane = threadIdx.x & 63;
  const long pair = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= npairs) return;  // whole wave; nothing below synchronises across waves
  const long win_g = pair / heads;
  const int h = (int)(pair - win_g * heads);
  const int l15 = lane & 15;
  const int g = lane >> 4;
  const int C3 = 3 * C;
  const float scale = 0.17677669529663687f;  // 32 ** -0.5
  const int win = (int)(win_g % wg.nWin);
  const int wy = win / wg.nWx;
  const int wx = win - wy * wg.nWx;
  const bool pix = bqkv != nullptr;
  // row of window slot `lane` (>= 0 real token, -1 padded token, -2 slot >= 49), and its
  // byte offset: past the end of the buffer for the slots without a row (loads give 0),
  // further past it for the padded tokens (flagged by the offset itself)
  const unsigned oob = (unsigned)qkv_bytes, oob_pad = (unsigned)qkv_bytes + (1u << 20);
  int slot_row;
  {
    const int ty = lane / kWin;
    int y = wy * kWin + ty + wg.sh;
    int x = wx * kWin + (lane - ty * kWin) + wg.sw;
    if (y >= wg.pH) y -= wg.pH;
    if (x >= wg.pW) x -= wg.pW;
    const long b = win_g / wg.nWin;
    slot_row = lane >= kWinTok ? -2 : (y < wg.H && x < wg.W ? (int)((b * wg.H + y) * wg.W + x) : -1);
    if (!pix) slot_row = lane < kWinTok ? (int)(win_g * kWinTok + lane) : -2;
  }
  const unsigned slot_off = slot_row >= 0 ? (unsigned)slot_row * (unsigned)(C3 * 4) : (slot_row == -1 ? oob_pad : oob);
  const bool any_pad = __builtin_amdgcn_ballot_w64(slot_row == -1) != 0;  // wave-uniform
  auto off_of = [&](int slot) { return (unsigned)__shfl((int)slot_off, slot); };
  const __amdgpu_buffer_rsrc_t qkv = __builtin_amdgcn_make_buffer_rsrc((void*)QKV, (short)0, qkv_bytes, 0x00020000);
  const unsigned kcol = (unsigned)(C + h * kHeadDim + 8 * g) * 4u;
  const unsigned vcol = (unsigned)(2 * C + h * kHeadDim + l15) * 4u;
  const unsigned qcol = (unsigned)(h * kHeadDim + 8 * g) * 4u;
  auto ld4 = [&](unsigned off) { return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(qkv, off, 0, 0)); };
  auto ld1 = [&](unsigned off) { return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(qkv, off, 0, 0)); };

  // the bias operands of padded tokens (read only in windows that have one)
  floatx4 kb0 = {0.f, 0.f, 0.f, 0.f}, kb1 = kb0;
  float vb[2] = {0.f, 0.f};
  if (any_pad) {
    kb0 = *reinterpret_cast<const floatx4*>(bqkv + C + h * kHeadDim + 8 * g);
    kb1 = *reinterpret_cast<const floatx4*>(bqkv + C + h * kHeadDim + 8 * g + 4);
    vb[0] = bqkv[2 * C + h * kHeadDim + l15];
    vb[1] = bqkv[2 * C + h * kHeadDim + 16 + l15];
  }
  abf16x8 kh[4], kl[4];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    const unsigned o = off_of(16 * kt + l15);
    const floatx4 a = ld4(o + kcol);
    const floatx4 b = ld4(o + kcol + 16);
    float x[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[e] = a[e];
      x[4 + e] = b[e];
    }
    if (any_pad && o >= oob_pad) {  // a padded token's key is the qkv bias
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = kb0[e];
        x[4 + e] = kb1[e];
      }
    }
    split8(x, kh[kt], kl[kt]);
  }
  // V^T fragments by scalar gathers (a transpose through a per-wave LDS slab, 8 vector
  // loads instead of 32 scalar ones, measured slower: s3.wattn 1964 -> 2123 us per encode)
  abf16x8 vh[2][2], vl[2][2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned o = off_of(32 * s + (j >> 2) * 16 + 4 * g + (j & 3));
        x[j] = ld1(o + vcol + 64 * dt);
        if (any_pad) x[j] = o >= oob_pad ? vb[dt] : x[j];  // a padded token's value is the qkv bias
      }
      split8(x, vh[dt][s], vl[dt][s]);
    }

  int type = 0;
  if (wg.sh + wg.sw > 0) type = 2 * (wy == wg.nWin / wg.nWx - 1) + (wx == wg.nWx - 1);
  const __amdgpu_buffer_rsrc_t tbr =
      __builtin_amdgcn_make_buffer_rsrc((void*)table, (short)0, 4 * heads * 64 * 64 * 4, 0x00020000);
  const unsigned tbo = (unsigned)(((type * heads + h) * 64 + l15) * 64 + 4 * g) * 4u;

#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    const int q = 16 * qt + l15;
    const int qr = __shfl(slot_row, q);
    abf16x8 qh, ql;
    {
      const unsigned o = off_of(q) + qcol;  // rows >= 49 and padded tokens read zeros (never written)
      const floatx4 a = ld4(o);
      const floatx4 b = ld4(o + 16);
      float x[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = a[e] * scale;
        x[4 + e] = b[e] * scale;
      }
      split8(x, qh, ql);
    }
    floatx4 st[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) st[kt] = mfma3<PASSES>(kh[kt], kl[kt], qh, ql, floatx4{0.f, 0.f, 0.f, 0.f});
    // bias + mask (+ -inf on padded keys), then softmax over the query's 64 key slots.  Key
    // tile 3 holds keys 48 + 4 g + r: only key 48 (g = 0, r = 0) exists and keys 49..63 are
    // -inf for every real query, so r = 1..3 of that tile are skipped (exp = 0 exactly, max
    // and sum unchanged); the padded queries' rows are never written.
    const unsigned to = tbo + (unsigned)qt * 16u * 64u * 4u;
    floatx4 bt[3];
#pragma unroll
    for (int kt = 0; kt < 3; ++kt)
      bt[kt] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(tbr, to + 64 * kt, 0, 0));
    const float bt3 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(tbr, to + 192, 0, 0));
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 3; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[kt][r] = st[kt][r] + bt[kt][r];
        m = fmaxf(m, st[kt][r]);
      }
    }
    st[3][0] = st[3][0] + bt3;
    m = fmaxf(m, st[3][0]);
    m = xmax16_32(m);
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 3; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[kt][r] = __expf(st[kt][r] - m);  // v_exp_f32 (libm expf: ~10 VALU each, 64 per lane)
        sum += st[kt][r];
      }
    st[3][0] = __expf(st[3][0] - m);
    sum += st[3][0];
    st[3][1] = st[3][2] = st[3][3] = 0.f;
    sum = xsum16_32(sum);
    const float rs = __builtin_amdgcn_rcpf(sum);  // one rcp instead of 16 IEEE divisions
    abf16x8 ph[2], pl[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = st[2 * s + (j >> 2)][j & 3] * rs;
      split8(x, ph[s], pl[s]);
    }
    floatx4 od[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      floatx4 o = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) o = mfma3<PASSES>(vh[dt][s], vl[dt][s], ph[s], pl[s], o);
      if (!out.f32) {
        od[dt] = o;
        continue;
      }
      if (qr >= 0) {
        const size_t off = (size_t)qr * C + h * kHeadDim + 16 * dt + 4 * g;
        if (out.f32) *reinterpret_cast<floatx4*>(out.f32 + off) = o;
        if (out.hi) {
          uint32_t h0, l0, h1, l1;
          split2_bf16(o[0], o[1], h0, l0);
          split2_bf16(o[2], o[3], h1, l1);
          *reinterpret_cast<uint2*>(out.hi + off) = make_uint2(h0, h1);
          if (out.lo) *reinterpret_cast<uint2*>(out.lo + off) = make_uint2(l0, l1);
        }
      }
    }
    if (!out.f32 && out.hi && qr >= 0) {
      // lanes g and g ^ 1 (16 apart, the same query row) trade halves: 8 consecutive
      // channels per lane, one 16-B store per plane (attend_to_planes in wattn.hip)
      const bool odd = g & 1;
      const size_t off = (size_t)qr * C + h * kHeadDim + (odd ? 16 + 4 * (g - 1) : 4 * g);
#pragma unroll
      for (int plane = 0; plane < 2; ++plane) {
        uint16_t* dst = plane ? out.lo : out.hi;
        if (!dst) break;
        uint32_t v[2][2], t;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            if (plane) split2_bf16(od[dt][2 * e], od[dt][2 * e + 1], t, v[dt][e]);
            else split2_bf16(od[dt][2 * e], od[dt][2 * e + 1], v[dt][e], t);
          }
        const uint32_t r0 = __shfl_xor(odd ? v[0][0] : v[1][0], 16);
        const uint32_t r1 = __shfl_xor(odd ? v[0][1] : v[1][1], 16);
        *reinterpret_cast<uint4*>(dst + off) = odd ? make_uint4(r0, r1, v[1][0], v[1][1]) : make_uint4(v[0][0], v[0][1], r0, r1);
      }
    }
  }
}

__global__ void split_bf16_kernel(const float* __restrict__ x, RowOut out, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) store_val(out, i, x[i]);
}

// the same split, 4 values per lane per iteration (float4 in, two 8-B stores out)
__global__ void split4_bf16_kernel(const floatx4* __restrict__ x, uint2* __restrict__ hi, uint2* __restrict__ lo,
                                   size_t n4) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n4; i += stride) {
    const floatx4 v = x[i];
    uint32_t h0, l0, h1, l1;
    split2_bf16(v[0], v[1], h0, l0);
    split2_bf16(v[2], v[3], h1, l1);
    hi[i] = make_uint2(h0, h1);
    if (lo) lo[i] = make_uint2(l0, l1);
  }
}

// cross K/V fp32 [B * M][512] -> fp24 head-major planes [B][2][8][M][32], 4 columns per thread
__global__ void split_kv_fp24_kernel(const float* __restrict__ kv, uint8_t* __restrict__ kv24, int M, size_t n4) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n4; i += stride) {
    const size_t row = i >> 7;           // 128 groups of 4 columns per 512-column row
    const int col = (int)(i & 127) * 4;  // k: 0..255, v: 256..511
    const size_t b = row / M;
    const int m = (int)(row - b * M);
    const size_t o = ((b * 2 + (col >> 8)) * 8 + ((col >> 5) & 7)) * (size_t)M * 32 + (size_t)m * 32 + (col & 31);
    st_fp24x4(kv24, o, reinterpret_cast<const floatx4*>(kv)[i]);
  }
}

// cross K/V fp32 [B * M][512] -> int16 head-major [B][2][8][M][32] with one scale per (b,
// column) over the M keys; one workgroup per (b, layer), 2 columns per thread
__global__ void __launch_bounds__(256) quant_kv_i16_kernel(const float* __restrict__ kv, int16_t* __restrict__ q,
                                                           float* __restrict__ scale, int M, size_t layer_stride,
                                                           size_t scale_stride) {
  const int b = blockIdx.x;
  const int c = threadIdx.x * 2;
  const float* src = kv + blockIdx.y * layer_stride + (size_t)b * M * 512 + c;
  float a0 = 0.f, a1 = 0.f;
  bool n0 = false, n1 = false;  // fmaxf drops NaN operands: tracked apart
#pragma unroll 8
  for (int m = 0; m < M; ++m) {
    const float2 v = *reinterpret_cast<const float2*>(src + (size_t)m * 512);
    a0 = fmaxf(a0, fabsf(v.x));
    a1 = fmaxf(a1, fabsf(v.y));
    n0 |= v.x != v.x;
    n1 |= v.y != v.y;
  }
  const float i0 = a0 > 0.f ? 32767.f / a0 : 0.f, i1 = a1 > 0.f ? 32767.f / a1 : 0.f;
  // a NaN in a column makes its scale NaN (it reaches the logits and the engine's non-finite
  // check, as on the fp32 / fp24 paths); an inf gives an inf scale
  *reinterpret_cast<float2*>(scale + blockIdx.y * scale_stride + (size_t)b * 512 + c) =
      float2{n0 ? __builtin_nanf("") : (a0 > 0.f ? a0 / 32767.f : 1.f),
             n1 ? __builtin_nanf("") : (a1 > 0.f ? a1 / 32767.f : 1.f)};
  int16_t* dst = q + blockIdx.y * layer_stride + ((size_t)(b * 2 + (c >> 8)) * 8 + ((c >> 5) & 7)) * M * 32 + (c & 31);
#pragma unroll 8
  for (int m = 0; m < M; ++m) {
    const float2 v = *reinterpret_cast<const float2*>(src + (size_t)m * 512);
    // clamp in float first: (int) of a NaN or out-of-range float is undefined
    const int r0 = (int)rintf(fminf(fmaxf(v.x * i0, -32767.f), 32767.f));
    const int r1 = (int)rintf(fminf(fmaxf(v.y * i1, -32767.f), 32767.f));
    *reinterpret_cast<uint32_t*>(dst + (size_t)m * 32) = ((uint32_t)r0 & 0xffffu) | ((uint32_t)r1 << 16);
  }
}

inline unsigned blocks_for_rows(long rows) { return (unsigned)((rows + 3) / 4); }

}  // namespace

void launch_stem(const float* img, const float* w, const float* b, const float* ln_w, const float* ln_b, float* X,
                 int B, int H, int W, hipStream_t s) {
  const int Hs = H / 4, Ws = W / 4;
  if (W % 4 != 0) throw std::runtime_error("stem: image width must be a multiple of 4");
  const long ntok = (long)B * Hs * Ws;
  // One resident round: 768 workgroups = 256 CUs x 3 waves per SIMD (150 VGPRs). 4096 paid
  // the weight prologue for 2-3 tokens per wave (profiles/r02/ab_stem_grid.log); 1024 left a
  // quarter-full second round: 829 -> 748 us per 512-image encode (profiles/r05/r07k/)
  constexpr long kStemBlocks = 768;
  const unsigned blocks = (unsigned)std::min<long>((ntok + 63) / 64, kStemBlocks);
  stem16w_kernel<1><<<blocks, 256, 0, s>>>(img, w, b, ln_w, ln_b, X, ntok, H, W, Hs, Ws);  // one sweep ahead
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_ln_partition(const float* X, const float* g, const float* b, float* XW, uint16_t* XWh, uint16_t* XWl,
                         int B, int C, const WinGeom& wg, hipStream_t s) {
  LnGeom geo{};
  geo.rows = (long)B * wg.nWin * kWinTok;
  geo.C = C;
  geo.win = wg;
  launch_ln_group<MODE_WIN>(X, g, b, RowOut{XW, XWh, XWl}, geo, s);
}

void launch_layernorm(const float* X, const float* g, const float* b, float* Y, uint16_t* Yh, uint16_t* Yl,
                      int rows, int C, hipStream_t s) {
  LnGeom geo{};
  geo.rows = rows;
  geo.C = C;
  launch_ln_group<MODE_ROWS>(X, g, b, RowOut{Y, Yh, Yl}, geo, s);
}

void launch_merge_ln(const float* X, const float* g, const float* b, float* Y, uint16_t* Yh, uint16_t* Yl, int B,
                     int H, int W, int C, hipStream_t s) {
  LnGeom geo{};
  geo.rows = (long)B * ((H + 1) / 2) * ((W + 1) / 2);
  geo.C = 4 * C;
  geo.B = B;
  geo.H = H;
  geo.W = W;
  geo.Cin = C;
  launch_ln_group<MODE_MERGE>(X, g, b, RowOut{Y, Yh, Yl}, geo, s);
}

void launch_window_attention(const float* QKV, const float* relbias, const float* relmask, float* O, uint16_t* Oh,
                             uint16_t* Ol, int B, int C, int heads, const WinGeom& wg, int passes, hipStream_t s,
                             const float* bqkv) {
  if (bqkv && passes == 0) throw std::runtime_error("window_attention: pixel-order rows need the MFMA kernel");
  if (passes == 0) {
    dim3 grid((unsigned)((long)B * wg.nWin), (unsigned)heads);
    window_attention_kernel<<<grid, 256, 0, s>>>(QKV, relbias, RowOut{O, Oh, Ol}, C, wg);
  } else {
    if (passes != 1 && passes != 3) throw std::runtime_error("window_attention: passes must be 0, 1 or 3");
    // the kernel addresses QKV through a buffer descriptor with 32-bit offsets: image chunks
    // of < 2 GiB - 2 MiB of QKV rows (one chunk at every batch the bench runs)
    const size_t rows_img = bqkv ? (size_t)wg.H * wg.W : (size_t)wg.nWin * kWinTok;
    const size_t bytes_img = rows_img * 3 * C * sizeof(float);
    const size_t limit = ((size_t)1 << 31) - ((size_t)2 << 20);
    if (bytes_img > limit) throw std::runtime_error("window_attention: one image's QKV rows exceed 2 GiB");
    const int chunk = (int)std::min<size_t>((size_t)B, limit / bytes_img);
    for (int b0 = 0; b0 < B; b0 += chunk) {
      const int nb = std::min(chunk, B - b0);
      const size_t r0 = (size_t)b0 * rows_img;
      const float* q = QKV + r0 * 3 * C;
      const RowOut o{O ? O + r0 * C : nullptr, Oh ? Oh + r0 * C : nullptr, Ol ? Ol + r0 * C : nullptr};
      const int nbytes = (int)((size_t)nb * bytes_img);
      const long npairs = (long)nb * wg.nWin * heads;
      const unsigned blocks = (unsigned)((npairs + 3) / 4);
      if (passes == 3)
        window_attention_mfma_kernel<3><<<blocks, 256, 0, s>>>(q, relmask, o, C, heads, npairs, wg, bqkv, nbytes);
      else
        window_attention_mfma_kernel<1><<<blocks, 256, 0, s>>>(q, relmask, o, C, heads, npairs, wg, bqkv, nbytes);
    }
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_split_kv_fp24(const float* kv, uint8_t* kv24, int B, int M, hipStream_t s) {
  const size_t n4 = (size_t)B * M * 128;
  if (n4 == 0) return;
  const unsigned blocks = (unsigned)std::min<size_t>((n4 + 255) / 256, 65536);
  split_kv_fp24_kernel<<<blocks, 256, 0, s>>>(kv, kv24, M, n4);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_quant_kv_i16(const float* kv, int16_t* q, float* scale, int B, int M, int L, size_t layer_stride,
                         size_t scale_stride, hipStream_t s) {
  if (B <= 0 || L <= 0) return;
  if (M <= 0 || scale_stride < (size_t)B * 512 || layer_stride < (size_t)B * M * 512)
    throw std::runtime_error("quant_kv_i16: bad strides");
  quant_kv_i16_kernel<<<dim3(B, L), 256, 0, s>>>(kv, q, scale, M, layer_stride, scale_stride);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_split_bf16(const float* x, uint16_t* hi, uint16_t* lo, size_t n, hipStream_t s) {
  if (n == 0) return;
  const auto al = [](const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
  if (n % 4 == 0 && al(x, 16) && al(hi, 8) && al(lo, 8)) {  // split(memory): 158 -> ~90 us per 512 images
    const size_t n4 = n / 4;
    const unsigned blocks = (unsigned)std::min<size_t>((n4 + 255) / 256, 65536);
    split4_bf16_kernel<<<blocks, 256, 0, s>>>(reinterpret_cast<const floatx4*>(x), reinterpret_cast<uint2*>(hi),
                                              reinterpret_cast<uint2*>(lo), n4);
  } else {
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 65536);
    split_bf16_kernel<<<blocks, 256, 0, s>>>(x, RowOut{nullptr, hi, lo}, n);
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
