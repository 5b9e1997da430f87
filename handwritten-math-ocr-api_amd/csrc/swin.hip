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

namespace mocr {

namespace {

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// LayerNorm of one row held as NPER values per lane (element c = lane + 64*i), C valid.
template <int NPER>
__device__ __forceinline__ void ln_regs(float (&v)[NPER], int C, int lane, const float* g, const float* b) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPER; ++i)
    if (lane + 64 * i < C) s += v[i];
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NPER; ++i)
    if (lane + 64 * i < C) {
      const float d = v[i] - mean;
      q += d * d;
    }
  const float var = wave_sum(q) / (float)C;
  const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
  for (int i = 0; i < NPER; ++i) {
    const int c = lane + 64 * i;
    if (c < C) v[i] = (v[i] - mean) * rstd * g[c] + b[c];
  }
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

template <int NPER>
__device__ __forceinline__ void store_row(float (&v)[NPER], int C, int lane, const RowOut& o, size_t row_off) {
#pragma unroll
  for (int i = 0; i < NPER; ++i) {
    const int c = lane + 64 * i;
    if (c < C) store_val(o, row_off + c, v[i]);
  }
}

// ---------------------------------------------------------------------------- stem
// Conv2d(1, 96, k=4, s=4, bias) -> Permute -> LayerNorm(96).  One wave per output token.
__global__ void __launch_bounds__(256) stem_kernel(const float* __restrict__ img, const float* __restrict__ w,
                                                   const float* __restrict__ bias, const float* __restrict__ g,
                                                   const float* __restrict__ beta, float* __restrict__ X, int B,
                                                   int H, int W, int Hs, int Ws) {
  const int lane = threadIdx.x & 63;
  const long tok = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= (long)B * Hs * Ws) return;
  const int b = (int)(tok / (Hs * Ws));
  const int rem = (int)(tok - (long)b * Hs * Ws);
  const int y = rem / Ws;
  const int x = rem - y * Ws;
  float px[16];
  const float* src = img + ((size_t)b * H + 4 * y) * W + 4 * x;
#pragma unroll
  for (int ky = 0; ky < 4; ++ky)
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) px[ky * 4 + kx] = src[(size_t)ky * W + kx];
  float v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i;
    float acc = 0.f;
    if (c < 96) {
      const float* wc = w + c * 16;
#pragma unroll
      for (int k = 0; k < 16; ++k) acc = fmaf(wc[k], px[k], acc);
      acc += bias[c];
    }
    v[i] = acc;
  }
  ln_regs<2>(v, 96, lane, g, beta);
  store_row<2>(v, 96, lane, RowOut{X, nullptr, nullptr}, (size_t)tok * 96);
}

// ---------------------------------------------------------------- LN + window partition
template <int NPER>
__global__ void __launch_bounds__(256) ln_partition_kernel(const float* __restrict__ X, const float* __restrict__ g,
                                                           const float* __restrict__ b, RowOut out, int B, int C,
                                                           WinGeom wg) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int per_img = wg.nWin * kWinTok;
  if (row >= (long)B * per_img) return;
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
  float v[NPER];
  if (y < wg.H && x < wg.W) {
    const float* src = X + ((size_t)(bi * wg.H + y) * wg.W + x) * C;
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
      const int c = lane + 64 * i;
      v[i] = c < C ? src[c] : 0.f;
    }
    ln_regs<NPER>(v, C, lane, g, b);
  } else {
#pragma unroll
    for (int i = 0; i < NPER; ++i) v[i] = 0.f;  // F.pad after norm1: zero tokens
  }
  store_row<NPER>(v, C, lane, out, (size_t)row * C);
}

template <int NPER>
__global__ void __launch_bounds__(256) layernorm_kernel(const float* __restrict__ X, const float* __restrict__ g,
                                                        const float* __restrict__ b, RowOut out, long rows, int C) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* src = X + (size_t)row * C;
  float v[NPER];
#pragma unroll
  for (int i = 0; i < NPER; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C ? src[c] : 0.f;
  }
  ln_regs<NPER>(v, C, lane, g, b);
  store_row<NPER>(v, C, lane, out, (size_t)row * C);
}

// ---------------------------------------------------------------- PatchMerging + LN(4C)
template <int NPER>
__global__ void __launch_bounds__(256) merge_ln_kernel(const float* __restrict__ X, const float* __restrict__ g,
                                                       const float* __restrict__ b, RowOut out, int B, int H, int W,
                                                       int C) {
  const int lane = threadIdx.x & 63;
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)B * Ho * Wo) return;
  const int bi = (int)(row / (Ho * Wo));
  const int rem = (int)(row - (long)bi * Ho * Wo);
  const int oy = rem / Wo;
  const int ox = rem - oy * Wo;
  const int C4 = 4 * C;
  float v[NPER];
#pragma unroll
  for (int i = 0; i < NPER; ++i) {
    const int c4 = lane + 64 * i;
    float val = 0.f;
    if (c4 < C4) {
      const int q = c4 / C;          // cat order x0=(0,0), x1=(1,0), x2=(0,1), x3=(1,1) as (dy,dx)
      const int c = c4 - q * C;
      const int y = 2 * oy + (q & 1);
      const int x = 2 * ox + (q >> 1);
      if (y < H && x < W) val = X[((size_t)(bi * H + y) * W + x) * C + c];
    }
    v[i] = val;
  }
  ln_regs<NPER>(v, C4, lane, g, b);
  store_row<NPER>(v, C4, lane, out, (size_t)row * C4);
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
  au16x8 h, l;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h[e] = f32_to_bf16_rne(x[e]);
    l[e] = f32_to_bf16_rne(x[e] - __uint_as_float((uint32_t)h[e] << 16));
  }
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

template <int PASSES>
__global__ void __launch_bounds__(256) window_attention_mfma_kernel(const float* __restrict__ QKV,
                                                                    const float* __restrict__ table, RowOut out,
                                                                    int C, int heads, long npairs, WinGeom wg) {
  const int lane = threadIdx.x & 63;
  const long pair = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= npairs) return;  // whole wave; nothing below synchronises across waves
  const long win_g = pair / heads;
  const int h = (int)(pair - win_g * heads);
  const int l15 = lane & 15;
  const int g = lane >> 4;
  const int C3 = 3 * C;
  const float* base = QKV + (size_t)win_g * kWinTok * C3 + h * kHeadDim;
  const float scale = 0.17677669529663687f;  // 32 ** -0.5

  abf16x8 kh[4], kl[4];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    const int key = 16 * kt + l15;
    float x[8];
    if (key < kWinTok) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(base + (size_t)key * C3 + C + 8 * g);
      const floatx4 b = *reinterpret_cast<const floatx4*>(base + (size_t)key * C3 + C + 8 * g + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = a[e];
        x[4 + e] = b[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = 0.f;
    }
    split8(x, kh[kt], kl[kt]);
  }
  abf16x8 vh[2][2], vl[2][2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int key = 32 * s + (j >> 2) * 16 + 4 * g + (j & 3);
        x[j] = key < kWinTok ? base[(size_t)key * C3 + 2 * C + 16 * dt + l15] : 0.f;
      }
      split8(x, vh[dt][s], vl[dt][s]);
    }

  int type = 0;
  if (wg.sh + wg.sw > 0) {
    const int win = (int)(win_g % wg.nWin);
    const int wy = win / wg.nWx;
    const int wx = win - wy * wg.nWx;
    type = 2 * (wy == wg.nWin / wg.nWx - 1) + (wx == wg.nWx - 1);
  }
  const float* tb = table + ((size_t)type * heads + h) * 64 * 64;

#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    const int q = 16 * qt + l15;
    abf16x8 qh, ql;
    {
      float x[8];
      if (q < kWinTok) {
        const floatx4 a = *reinterpret_cast<const floatx4*>(base + (size_t)q * C3 + 8 * g);
        const floatx4 b = *reinterpret_cast<const floatx4*>(base + (size_t)q * C3 + 8 * g + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] = a[e] * scale;
          x[4 + e] = b[e] * scale;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = 0.f;
      }
      split8(x, qh, ql);
    }
    floatx4 st[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) st[kt] = mfma3<PASSES>(kh[kt], kl[kt], qh, ql, floatx4{0.f, 0.f, 0.f, 0.f});
    // bias + mask (+ -inf on padded keys), then softmax over the query's 64 key slots
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const floatx4 b = *reinterpret_cast<const floatx4*>(tb + q * 64 + 16 * kt + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[kt][r] = st[kt][r] + b[r];
        m = fmaxf(m, st[kt][r]);
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[kt][r] = expf(st[kt][r] - m);
        sum += st[kt][r];
      }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    abf16x8 ph[2], pl[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = st[2 * s + (j >> 2)][j & 3] / sum;
      split8(x, ph[s], pl[s]);
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      floatx4 o = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) o = mfma3<PASSES>(vh[dt][s], vl[dt][s], ph[s], pl[s], o);
      if (q < kWinTok) {
        const size_t off = ((size_t)win_g * kWinTok + q) * C + h * kHeadDim + 16 * dt + 4 * g;
        if (out.f32) *reinterpret_cast<floatx4*>(out.f32 + off) = o;
        if (out.hi) {
          uint16_t hs[4], ls[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            hs[r] = f32_to_bf16_rne(o[r]);
            ls[r] = f32_to_bf16_rne(o[r] - __uint_as_float((uint32_t)hs[r] << 16));
          }
          *reinterpret_cast<uint2*>(out.hi + off) =
              make_uint2(hs[0] | ((uint32_t)hs[1] << 16), hs[2] | ((uint32_t)hs[3] << 16));
          if (out.lo)
            *reinterpret_cast<uint2*>(out.lo + off) =
                make_uint2(ls[0] | ((uint32_t)ls[1] << 16), ls[2] | ((uint32_t)ls[3] << 16));
        }
      }
    }
  }
}

__global__ void split_bf16_kernel(const float* __restrict__ x, RowOut out, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) store_val(out, i, x[i]);
}

inline unsigned blocks_for_rows(long rows) { return (unsigned)((rows + 3) / 4); }

}  // namespace

void launch_stem(const float* img, const float* w, const float* b, const float* ln_w, const float* ln_b, float* X,
                 int B, int H, int W, hipStream_t s) {
  const int Hs = H / 4, Ws = W / 4;
  stem_kernel<<<blocks_for_rows((long)B * Hs * Ws), 256, 0, s>>>(img, w, b, ln_w, ln_b, X, B, H, W, Hs, Ws);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_ln_partition(const float* X, const float* g, const float* b, float* XW, uint16_t* XWh, uint16_t* XWl,
                         int B, int C, const WinGeom& wg, hipStream_t s) {
  const long rows = (long)B * wg.nWin * kWinTok;
  const RowOut o{XW, XWh, XWl};
  switch ((C + 63) / 64) {
    case 2: ln_partition_kernel<2><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, B, C, wg); break;
    case 3: ln_partition_kernel<3><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, B, C, wg); break;
    case 6: ln_partition_kernel<6><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, B, C, wg); break;
    case 12: ln_partition_kernel<12><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, B, C, wg); break;
    default: throw std::runtime_error("ln_partition: unsupported C " + std::to_string(C));
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_layernorm(const float* X, const float* g, const float* b, float* Y, uint16_t* Yh, uint16_t* Yl,
                      int rows, int C, hipStream_t s) {
  const RowOut o{Y, Yh, Yl};
  switch ((C + 63) / 64) {
    case 2: layernorm_kernel<2><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, rows, C); break;
    case 3: layernorm_kernel<3><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, rows, C); break;
    case 4: layernorm_kernel<4><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, rows, C); break;
    case 6: layernorm_kernel<6><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, rows, C); break;
    case 12: layernorm_kernel<12><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, rows, C); break;
    default: throw std::runtime_error("layernorm: unsupported C " + std::to_string(C));
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_merge_ln(const float* X, const float* g, const float* b, float* Y, uint16_t* Yh, uint16_t* Yl, int B,
                     int H, int W, int C, hipStream_t s) {
  const RowOut o{Y, Yh, Yl};
  const long rows = (long)B * ((H + 1) / 2) * ((W + 1) / 2);
  switch ((4 * C + 63) / 64) {
    case 6: merge_ln_kernel<6><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, B, H, W, C); break;
    case 12: merge_ln_kernel<12><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, B, H, W, C); break;
    case 24: merge_ln_kernel<24><<<blocks_for_rows(rows), 256, 0, s>>>(X, g, b, o, B, H, W, C); break;
    default: throw std::runtime_error("merge_ln: unsupported C " + std::to_string(C));
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_window_attention(const float* QKV, const float* relbias, const float* relmask, float* O, uint16_t* Oh,
                             uint16_t* Ol, int B, int C, int heads, const WinGeom& wg, int passes, hipStream_t s) {
  if (passes == 0) {
    dim3 grid((unsigned)((long)B * wg.nWin), (unsigned)heads);
    window_attention_kernel<<<grid, 256, 0, s>>>(QKV, relbias, RowOut{O, Oh, Ol}, C, wg);
  } else {
    const long npairs = (long)B * wg.nWin * heads;
    const unsigned blocks = (unsigned)((npairs + 3) / 4);
    if (passes == 3)
      window_attention_mfma_kernel<3><<<blocks, 256, 0, s>>>(QKV, relmask, RowOut{O, Oh, Ol}, C, heads, npairs, wg);
    else if (passes == 1)
      window_attention_mfma_kernel<1><<<blocks, 256, 0, s>>>(QKV, relmask, RowOut{O, Oh, Ol}, C, heads, npairs, wg);
    else
      throw std::runtime_error("window_attention: passes must be 0, 1 or 3");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_split_bf16(const float* x, uint16_t* hi, uint16_t* lo, size_t n, hipStream_t s) {
  if (n == 0) return;
  const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 65536);
  split_bf16_kernel<<<blocks, 256, 0, s>>>(x, RowOut{nullptr, hi, lo}, n);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
