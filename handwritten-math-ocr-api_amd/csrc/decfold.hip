// Folded greedy decode step (kernels.h FoldGemmParams / FoldAttnParams): 5 dependent
// kernels per nn.TransformerDecoderLayer (torch/nn/modules/transformer.py:1143-1199)
// instead of 8.
//
// In a post-norm layer every projection reads a LayerNorm of a pre-norm sum y, which
// needs y's whole row.  For LN(y) = g (y - mu) rstd + b feeding W x + c:
//   W LN(y) + c = rstd (W' y - mu s) + c',   W' = W diag(g), s = W g, c' = W b + c,
// and W' y expands over y's own terms (y = residual + W_o a + b_o), so z = W' y is one
// more column block of the kernel that produces y, and the consumer only applies rstd,
// mu (y's slice statistics, merged as every other consumer merges them), s and c'.
// The CA q projection moves into the SA out-projection, FFN1 into the CA out-projection,
// the next layer's q|k|v projection into FFN2 (whose hidden is unfolded on load), and
// layer 0's q|k|v of a fed token into a [V, 3d] + [max_pos, 3d] table lookup.  The fold
// changes fp32 rounding only (weights folded with fp64 accumulation at load time).
//
// Loads are never predicated per element: out-of-range rows / keys read a clamped valid
// address and are masked after the load (hipcc turns `c ? *p : 0` into a branch and a
// full vmcnt(0) wait per element).
#include "kernels.h"
#include "lanes.h"
#include "select.h"

namespace mocr {

namespace {

constexpr int kD = 256;
constexpr int kSlices = kD / 16;
constexpr float kAttnScale = 0.17677669529663687f;  // 1/sqrt(32)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// 8 floats -> bf16 hi / lo planes (split2_bf16 per pair): the A fragment of a bf16x3 MFMA
__device__ __forceinline__ void split8(const floatx4& x0, const floatx4& x1, bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
  split2_bf16(x0[0], x0[1], h[0], l[0]);
  split2_bf16(x0[2], x0[3], h[1], l[1]);
  split2_bf16(x1[0], x1[1], h[2], l[2]);
  split2_bf16(x1[2], x1[3], h[3], l[3]);
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

__device__ __forceinline__ float ln_apply(float v, float mean, float rstd, float g, float b) {
  return fmaf((v - mean) * rstd, g, b);
}

// Row statistics from 16 (mean, M2) slice partials, merged by the fixed binary tree of
// decoder.hip (Chan et al.), so the values are bit-identical to every other consumer's.
__device__ __forceinline__ void merge_eq(float& m, float& q, float mb, float qb, float n) {
  const float delta = mb - m;
  q = q + qb + delta * delta * (n * 0.5f);
  m = m + delta * 0.5f;
}
template <int MASK>
__device__ __forceinline__ void merge_lanes(float& m, float& q, bool upper, float n) {
  const float mo = lane_partner<MASK>(m);  // lanes.h: DPP for MASK <= 8
  const float qo = lane_partner<MASK>(q);
  if (upper) {
    float mm = mo, qq = qo;
    merge_eq(mm, qq, m, q, n);
    m = mm;
    q = qq;
  } else {
    merge_eq(m, q, mo, qo, n);
  }
}
__device__ __forceinline__ float rstd_of(float m2) { return 1.0f / sqrtf(m2 * (1.0f / kD) + 1e-5f); }
// Layout 1 of decoder.hip: lane group g = 0..3 of a row holds slices 4g..4g+3 (loaded
// first, merged later, so several rows' partials can be in flight together).
struct Part4 {
  floatx4 p0, p1;
};
__device__ __forceinline__ Part4 load_part4(const float* __restrict__ part, int g) {
  return {*reinterpret_cast<const floatx4*>(part + 8 * g), *reinterpret_cast<const floatx4*>(part + 8 * g + 4)};
}
__device__ __forceinline__ void merge_part4(const Part4& pp, int g, float& mean, float& rstd) {
  const floatx4 p0 = pp.p0, p1 = pp.p1;
  float m = p0[0], q = p0[1], m2 = p1[0], q2 = p1[1];
  merge_eq(m, q, p0[2], p0[3], 16.f);
  merge_eq(m2, q2, p1[2], p1[3], 16.f);
  merge_eq(m, q, m2, q2, 32.f);
  merge_lanes<16>(m, q, (g & 1) != 0, 64.f);
  merge_lanes<32>(m, q, (g & 2) != 0, 128.f);
  mean = m;
  rstd = rstd_of(q);
}
__device__ __forceinline__ void row_stats_16lanes(const float* __restrict__ part, int c, float& mean, float& rstd) {
  float m = part[2 * c], q = part[2 * c + 1];
  merge_lanes<1>(m, q, (c & 1) != 0, 16.f);
  merge_lanes<2>(m, q, (c & 2) != 0, 32.f);
  merge_lanes<4>(m, q, (c & 4) != 0, 64.f);
  merge_lanes<8>(m, q, (c & 8) != 0, 128.f);
  mean = m;
  rstd = rstd_of(q);
}

// ------------------------------------------------------------------ fold row GEMM
// Workgroups x < 16 own a 16x16 tile of y (K = K1 over A1'), the others a 16x16 tile of
// z (K = K1 + d over [A1' | A2']).  4 waves split K and combine through LDS in a fixed
// order on v_mfma_f32_16x16x4_f32, as decoder.hip rowgemm_kernel; the y epilogue is its
// DEC_RESADD (y = A2' + (acc + by), then the (mean, M2) of the tile's 16 columns).  The
// 16-wide k chunks never straddle A1 / A2 (K1 % 16 == 0), so a chunk's source is
// wave-uniform.  S1 / S2: A1 / A2 carry statistics (unfold / LayerNorm on load).
// X3: bf16x3 on v_mfma_f32_16x16x32_bf16 (Wy / Wz as bf16 hi / lo planes, A split on
// load): a lane takes k = 32 s + 8 g .. +7 of its row / column per 32-deep step instead
// of k = 16 i + 4 g .. +3 per 16-deep chunk; the transforms, reductions and epilogue are
// the fp32 path's.
template <int NI, bool YT, bool S1, bool S2, int NW, bool X3>
__device__ __forceinline__ void fold_tile(const FoldGemmParams& p, int c0) {
  __shared__ float red[NW][16][17];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar branches on k ranges
  const int r0 = blockIdx.y * 16;
  const int ra = min(r0 + (lane & 15), p.B - 1);  // rows >= B compute discarded outputs
  const int cb = c0 + (lane & 15);
  const int g = lane >> 4;
  const int kbeg = wave * NI * 16;
  const int K1 = p.K1;
  const float* wrow = YT ? p.Wy + (size_t)cb * K1 : p.Wz + (size_t)cb * (K1 + kD);

  // The unfold / LayerNorm vectors depend on k only: the workgroup stages them in LDS
  // (one float4 of each per thread, issued first) instead of every lane loading its own
  // copies -- 16 lanes share each value, but a vector load returns 16 B per lane through
  // the CU's load-data path either way, and these were half of the kernel's loads.
  // (with S1; without it only the A2 quarter of a z tile needs LN vectors: per lane, below)
  constexpr int KUV = NI * 16 * NW;  // this tile's K
  constexpr bool UV = S1;
  __shared__ floatx4 uv_s[2][UV ? KUV / 4 : 1];
  floatx4 u4{}, v4{};
  const int kk4 = min(tid * 4, KUV - 4);
  if constexpr (UV) {
    static_assert(KUV / 4 <= 64 * NW, "one float4 of u and of v per thread");
    const bool in1 = kk4 < K1;
    const float* us = in1 ? (S1 ? p.a1_s + kk4 : p.a2_g) : (S2 ? p.a2_g + (kk4 - K1) : p.a1_s);
    const float* vs = in1 ? (S1 ? p.a1_c + kk4 : p.a2_b) : (S2 ? p.a2_b + (kk4 - K1) : p.a1_c);
    u4 = *reinterpret_cast<const floatx4*>(us);
    v4 = *reinterpret_cast<const floatx4*>(vs);
  }
  // every independent load first: A, W, the residual.  Slot i holds 4 consecutive k:
  // fp32, k = 16 i + 4 g (one 16x16x4 chunk); bf16x3, k = 32 (i / 2) + 8 g + 4 (i % 2)
  // (the two halves of a 32-deep step's 8 k)
  auto kof = [&](int i) { return X3 ? kbeg + 32 * (i >> 1) + 8 * g + 4 * (i & 1) : kbeg + i * 16 + 4 * g; };
  floatx4 a[NI], b[X3 ? 1 : NI], u[NI], v[NI];
  bf16x8 bh[X3 ? NI / 2 : 1], bl[X3 ? NI / 2 : 1];
  if constexpr (X3) {
    static_assert(NI % 2 == 0, "32-deep steps");
    const size_t wo = (size_t)cb * (YT ? K1 : K1 + kD);
    const uint16_t* whr = (YT ? p.Wy_hi : p.Wz_hi) + wo;
    const uint16_t* wlr = (YT ? p.Wy_lo : p.Wz_lo) + wo;
#pragma unroll
    for (int s2 = 0; s2 < NI / 2; ++s2) {
      const int k = kbeg + 32 * s2 + 8 * g;
      bh[s2] = *reinterpret_cast<const bf16x8*>(whr + k);
      bl[s2] = *reinterpret_cast<const bf16x8*>(wlr + k);
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int k = kof(i);
    const bool in1 = k < K1;  // uniform per slot: K1 % 32 == 0
    if constexpr (!X3) b[i] = *reinterpret_cast<const floatx4*>(wrow + k);
    a[i] = *reinterpret_cast<const floatx4*>(in1 ? p.A1 + (size_t)ra * K1 + k : p.A2 + (size_t)ra * kD + (k - K1));
    if constexpr (S2 && !S1 && !YT) {
      if ((X3 ? kbeg + 32 * (i >> 1) : kbeg + 16 * i) >= K1) {  // wave-uniform: LN2 of the A2 columns
        u[i] = *reinterpret_cast<const floatx4*>(p.a2_g + (k - K1));
        v[i] = *reinterpret_cast<const floatx4*>(p.a2_b + (k - K1));
      }
    }
  }
  if constexpr (UV) {
    if (tid * 4 < KUV) {
      uv_s[0][kk4 / 4] = u4;
      uv_s[1][kk4 / 4] = v4;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int k = kof(i);
      u[i] = uv_s[0][k / 4];
      v[i] = uv_s[1][k / 4];
    }
  }
  const int row = tid >> 4;
  const int col = tid & 15;
  const int grow = r0 + row;
  const int gcol = c0 + col;
  const int rrow = min(grow, p.B - 1);
  float rres = 0.f, rg = 0.f, rb = 0.f;
  if constexpr (YT) {
    rres = p.A2[(size_t)rrow * kD + gcol];
    if constexpr (S2) {
      rg = p.a2_g[gcol];
      rb = p.a2_b[gcol];
    }
  }
  const size_t srow = (size_t)ra * 2 * kSlices;
  Part4 pa1{}, pa2{};
  if constexpr (S1) pa1 = load_part4(p.a1_stats + srow, g);
  if constexpr (S2) pa2 = load_part4(p.a2_stats + srow, g);
  float m1 = 0.f, r1 = 0.f, m2 = 0.f, r2 = 0.f;
  if constexpr (S1) merge_part4(pa1, g, m1, r1);
  if constexpr (S2) merge_part4(pa2, g, m2, r2);
  if constexpr (S1 || S2) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int k = kof(i);
      if (k < K1) {
        if constexpr (S1)
#pragma unroll
          for (int s = 0; s < 4; ++s) a[i][s] = fmaxf(fmaf(r1, fmaf(-m1, u[i][s], a[i][s]), v[i][s]), 0.f);
      } else {
        if constexpr (S2)
#pragma unroll
          for (int s = 0; s < 4; ++s) a[i][s] = ln_apply(a[i][s], m2, r2, u[i][s], v[i][s]);
      }
    }
  }

  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if constexpr (X3) {
#pragma unroll
    for (int s2 = 0; s2 < NI / 2; ++s2) {
      bf16x8 ah, al;
      split8(a[2 * s2], a[2 * s2 + 1], ah, al);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[s2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[s2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[s2], acc, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[i][s], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][g * 4 + r][lane & 15] = acc[r];
  __syncthreads();
  if (tid >= 256) return;  // 16 x 16 outputs: the first 4 waves
  if constexpr (YT && S2) {  // all 16 lanes of a row take part in the merge
    float mean, rstd;
    row_stats_16lanes(p.a2_stats + (size_t)rrow * 2 * kSlices, col, mean, rstd);
    rres = ln_apply(rres, mean, rstd, rg, rb);
  }
  if (grow >= p.B || dec_skip(p.st, p.t)) return;  // uniform per 16-lane row group
  float val = red[0][row][col];
#pragma unroll
  for (int w = 1; w < NW; ++w) val += red[w][row][col];
  if constexpr (YT) {
    const float y = rres + (val + p.by[gcol]);
    p.y[(size_t)grow * kD + gcol] = y;
    const float m16 = row_sum<16>(y) * (1.0f / 16);  // the row's 16 lanes (DPP)
    const float q = row_sum<16>(sq_rn(y - m16));
    if (col == 0) {
      float* so = p.y_stats + ((size_t)grow * kSlices + c0 / 16) * 2;
      so[0] = m16;
      so[1] = q;
    }
  } else {
    p.z[(size_t)grow * p.NZ + gcol] = val + p.bz[gcol];
  }
}

// NW waves split K (4 or 8: 512-thread workgroups halve each wave's load chain).
template <int K1, bool S1, bool S2, int NW, bool X3>
__global__ void __launch_bounds__(64 * NW) foldgemm_kernel(FoldGemmParams p) {
  if (blockIdx.x < kD / 16)
    fold_tile<K1 / (16 * NW), true, S1, S2, NW, X3>(p, blockIdx.x * 16);
  else
    fold_tile<(K1 + kD) / (16 * NW), false, S1, S2, NW, X3>(p, (blockIdx.x - kD / 16) * 16);
}

#ifdef MOCR_FOLD_TS
// timing probe (tools/attn_ts.hip): thread 0's clocks per workgroup, as decwide.hip's
__device__ unsigned long long g_attn_ts[8192 * 8];
#define MOCR_ATS(i, v)                                                             \
  if (threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < 8192)             \
  g_attn_ts[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = (v)
#else
#define MOCR_ATS(i, v)
#endif

// ------------------------------------------------------------------ fold attention
// The newest position of row b against n keys for head h (one workgroup, 4 waves): the
// key loop of decoder.hip dec_attn_kernel (8 lanes per 32-float key row slice, every
// K/V load issued up front, per-wave softmax, wave partials merged after one barrier).
// Each lane unfolds its 4 columns of q -- and, self-attention, of the new k and v --
// from z; the lanes of key slot t take the new k/v from registers, and wave 0's first
// key group appends them to the cache.  ZS: z carries statistics (else z is final).
// SEL (layer 0 of steps t >= 1): the workgroup first runs the greedy selection of step
// t-1 for its row (select.h; the head-0 workgroup does the bookkeeping), then takes q|k|v
// of the selected token from the tables and writes its 32 columns of x = emb + pos --
// the work of a separate argmax kernel at the end of step t-1, without its launch.
// KVF: K/V (and the self-attention cache) in fp32 (0) or fp24 planes (1, common.h); 2:
// cross-attention K/V in int16 with per-column scales (the scales of K fold into q, those
// of V into the output); 3: the self-attention cache in int16 with one scale per (row,
// head, key) over its 32 values (the key's scale multiplies its score, the value's its
// softmax weight), the newest key / value quantised here by the same rule.
// NW waves (8 key rows each per pass; the selection runs on all 64 NW threads).
template <bool SELF, bool ZS, bool SEL, int NIT, int KVF, int NW, bool SLOT = false>
__global__ void __launch_bounds__(256) dec_foldattn_kernel(FoldAttnParams p) {
  MOCR_ATS(0, __builtin_amdgcn_s_memrealtime());
  MOCR_ATS(1, __builtin_amdgcn_s_memtime());
  constexpr int LPR = 8;  // lanes per key row
  constexpr int RPW = 8;  // key rows per wave instruction
  constexpr bool F24 = KVF == 1, I16 = KVF == 2, S16 = KVF == 3;
  static_assert(!(SELF && I16), "int16 K/V with per-column scales: cross-attention only");
  static_assert(!S16 || SELF, "int16 K/V with per-key scales: the self-attention cache");
  __shared__ floatx4 po[NW][LPR];
  __shared__ float pm[NW], ps[NW];

  const int b = blockIdx.x;
  const int h = blockIdx.y;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int rsub = lane / LPR;
  const int li = lane % LPR;
  const int cc = h * 32 + li * 4;  // this lane's 4 columns of the head
  const int t = p.t;
  const int n = p.n;
  const int n_cached = SELF ? t : n;
  const int m_first = wave * RPW + rsub;

  static_assert(!SLOT || (SELF && !SEL), "slot tables: the self-attention of beam hypotheses");
  // the K/V row: this decoder row, its image's memory row (cross-attention of beam
  // hypotheses: mem_div of them per image), or per key its slot row (SLOT, below)
  const int mb = SELF ? b : (p.mem_div > 1 ? b / p.mem_div : b);
  auto row_base = [&](int r) -> size_t {
    return KVF ? (size_t)r * p.f24_b + (size_t)h * p.f24_h + li * 4 : (size_t)r * p.kv_b_stride + cc;
  };
  const size_t kvb = row_base(mb);
  const size_t kvr = KVF ? 32 : (size_t)p.kv_row_stride;
  const size_t sbase = ((size_t)b * p.f24_b + (size_t)h * p.f24_h) / 32;  // S16: this (row, head)'s key scales
  int srow[SLOT ? NIT : 1];
  if constexpr (SLOT) {
    // key m < t of hypothesis b lives in the cache row of the ancestor that computed it; a
    // stale entry (after a batch stop) is clamped to a valid row
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int m = m_first + it * NW * RPW;
      const int sr = p.slot_rows[(size_t)b * p.slot_ld + (m < n_cached ? m : 0)];
      srow[it] = (unsigned)sr < (unsigned)p.B ? sr : 0;
    }
  }
  floatx4 kk[NIT], vv[NIT];
  float ksc[S16 ? NIT : 1], vsc[S16 ? NIT : 1];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int m = m_first + it * NW * RPW;
    const size_t o = (SLOT ? row_base(srow[it]) : kvb) + (size_t)(m < n_cached ? m : 0) * kvr;  // masked below
    if constexpr (F24) {
      kk[it] = ld_stream_fp24x4(p.K24, o);
      vv[it] = ld_stream_fp24x4(p.V24, o);
    } else if constexpr (I16) {
      kk[it] = ld_stream_i16x4(p.K16, o);
      vv[it] = ld_stream_i16x4(p.V16, o);
    } else if constexpr (S16) {
      kk[it] = ld_stream_i16x4(p.kc16, o);
      vv[it] = ld_stream_i16x4(p.vc16, o);
      const size_t so = (SLOT ? ((size_t)srow[it] * p.f24_b + (size_t)h * p.f24_h) / 32 : sbase) + (m < n_cached ? m : 0);
      ksc[it] = p.ksc[so];
      vsc[it] = p.vsc[so];
    } else {
      kk[it] = ld_stream4(p.K + o);
      vv[it] = ld_stream4(p.V + o);
    }
  }
  constexpr int NP = SELF ? 3 : 1;  // q (| k | v)
  floatx4 zv[NP], sv[NP], cv[NP];
  if constexpr (SEL) {
    static_assert(SELF && !ZS, "selection runs in layer 0's self-attention");
    const int tok = greedy_select<NW>(p.sel, b, h == 0);
    const int tk = max(tok, 0);  // -1: the batch stopped before step t-1 (nothing is written)
    const float* qt = p.qtab + (size_t)tk * 3 * kD + cc;
    const float* qp = p.qpos + (size_t)t * 3 * kD + cc;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const floatx4 a4 = *reinterpret_cast<const floatx4*>(qt + j * kD);
      const floatx4 b4 = *reinterpret_cast<const floatx4*>(qp + j * kD);
      zv[j] = a4 + b4;
    }
    if (tok >= 0 && wave == 0 && rsub == 0) {
      const floatx4 e4 = *reinterpret_cast<const floatx4*>(p.emb + (size_t)tk * kD + cc);
      const floatx4 p4 = *reinterpret_cast<const floatx4*>(p.pos + (size_t)t * kD + cc);
      *reinterpret_cast<floatx4*>(p.x + (size_t)b * kD + cc) = e4 + p4;
    }
  } else {
    const float* zr = p.z + (size_t)b * p.z_ld + cc;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      zv[j] = *reinterpret_cast<const floatx4*>(zr + j * kD);
      if constexpr (ZS) {
        sv[j] = *reinterpret_cast<const floatx4*>(p.s + j * kD + cc);
        cv[j] = *reinterpret_cast<const floatx4*>(p.c + j * kD + cc);
      }
    }
  }
  if constexpr (ZS) {
    float mean, rstd;
    row_stats_16lanes(p.z_stats + (size_t)b * 2 * kSlices, lane & 15, mean, rstd);
#pragma unroll
    for (int j = 0; j < NP; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) zv[j][e] = fmaf(rstd, fmaf(-mean, sv[j][e], zv[j][e]), cv[j][e]);
  }
#ifdef MOCR_FOLD_TS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  MOCR_ATS(2, __builtin_amdgcn_s_memtime());
  floatx4 q4 = zv[0];
  floatx4 vs4;
  if constexpr (I16) {
    q4 *= *reinterpret_cast<const floatx4*>(p.Ks + (size_t)mb * p.s_b + cc);
    vs4 = *reinterpret_cast<const floatx4*>(p.Vs + (size_t)mb * p.s_b + cc);
  }
  const floatx4 zero = {0.f, 0.f, 0.f, 0.f};
  if constexpr (SELF && F24) {  // the newest key / value as every later step reads them from the cache
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      zv[1][e] = fp24_round(zv[1][e]);
      zv[2][e] = fp24_round(zv[2][e]);
    }
  }
  float nks = 1.f, nvs = 1.f;  // S16: the newest key's / value's scale
  if constexpr (SELF && S16) {
    // int16 over the head's 32 values (the 8 lanes of a key row hold 4 each): scale max|x| /
    // 32767; a NaN anywhere makes the scale NaN (fmaxf drops it: tracked apart), so it
    // reaches the logits and the engine's non-finite check as on the fp32 / fp24 paths
    auto quant = [&](floatx4& v, float& sc) {
      float mx = 0.f, nan = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mx = fmaxf(mx, fabsf(v[e]));
        nan = v[e] != v[e] ? 1.f : nan;
      }
      mx = row_max8(mx);
      nan = row_max8(nan);
      const float inv = mx > 0.f ? 32767.f / mx : 0.f;
      sc = nan != 0.f ? __builtin_nanf("") : (mx > 0.f ? mx / 32767.f : 1.f);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fminf(fmaxf(rintf(v[e] * inv), -32767.f), 32767.f);
    };
    quant(zv[1], nks);
    quant(zv[2], nvs);
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int m = m_first + it * NW * RPW;
    if constexpr (SELF) {
      kk[it] = m == t ? zv[1] : kk[it];
      vv[it] = m == t ? zv[2] : (m < t ? vv[it] : zero);
      if constexpr (S16) {
        ksc[it] = m == t ? nks : ksc[it];
        // a masked key's value scale is 0 like its value (e = 0 times a stale NaN scale
        // would be NaN)
        vsc[it] = m == t ? nvs : (m < t ? vsc[it] : 0.f);
      }
    } else {
      vv[it] = m < n ? vv[it] : zero;
    }
  }
  if constexpr (SELF) {
    if (wave == 0 && rsub == 0 && !dec_skip(p.st, t)) {
      if constexpr (F24) {
        const size_t o = kvb + (size_t)t * 32;
        st_fp24x4(p.kc24, o, zv[1]);
        st_fp24x4(p.vc24, o, zv[2]);
      } else if constexpr (S16) {
        const size_t o = kvb + (size_t)t * 32;
        st_i16x4(p.kc16, o, zv[1]);
        st_i16x4(p.vc16, o, zv[2]);
        if (li == 0) {
          p.ksc[sbase + t] = nks;
          p.vsc[sbase + t] = nvs;
        }
      } else {
        const size_t o = kvb + (size_t)t * p.kv_row_stride;
        *reinterpret_cast<floatx4*>(p.kcache + o) = zv[1];
        *reinterpret_cast<floatx4*>(p.vcache + o) = zv[2];
      }
    }
  }

  float sc[NIT];
  float mx = -INFINITY;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float s = q4[0] * kk[it][0];
    s = fmaf(q4[1], kk[it][1], s);
    s = fmaf(q4[2], kk[it][2], s);
    s = fmaf(q4[3], kk[it][3], s);
    s = row_sum<8>(s);  // the 8 lanes of the key row (DPP, as the xor butterfly)
    if constexpr (S16) s *= ksc[it];
    s *= kAttnScale;
    sc[it] = (m_first + it * NW * RPW < n) ? s : -INFINITY;
    mx = fmaxf(mx, sc[it]);
  }
  mx = xmax8_16_32(mx);  // over the wave's 8 key-row groups
  float sum = 0.f;
  floatx4 o4 = {0.f, 0.f, 0.f, 0.f};
  if (mx != -INFINITY) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const float e = __expf(sc[it] - mx);  // v_exp_f32 (the libm expf's range reduction is ~10 VALU)
      sum += e;
      const float ev = S16 ? e * vsc[it] : e;
      o4[0] = fmaf(ev, vv[it][0], o4[0]);
      o4[1] = fmaf(ev, vv[it][1], o4[1]);
      o4[2] = fmaf(ev, vv[it][2], o4[2]);
      o4[3] = fmaf(ev, vv[it][3], o4[3]);
    }
  }
  sum = xsum8_16_32(sum);
#pragma unroll
  for (int e = 0; e < 4; ++e) o4[e] = xsum8_16_32(o4[e]);
  if constexpr (I16) o4 *= vs4;
  MOCR_ATS(3, __builtin_amdgcn_s_memtime());
  if (rsub == 0) {
    po[wave][li] = o4;
    if (li == 0) {
      pm[wave] = mx;
      ps[wave] = sum;
    }
  }
  __syncthreads();
  MOCR_ATS(4, __builtin_amdgcn_s_memtime());
  if (tid < 32 && !dec_skip(p.st, t)) {
    float m = pm[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) m = fmaxf(m, pm[w]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float f = pm[w] == -INFINITY ? 0.f : __expf(pm[w] - m);
      num = fmaf(po[w][tid / 4][tid % 4], f, num);
      den = fmaf(ps[w], f, den);
    }
    p.out[(size_t)b * kD + h * 32 + tid] = num * __builtin_amdgcn_rcpf(den);
  }
  MOCR_ATS(5, __builtin_amdgcn_s_memtime());
  MOCR_ATS(6, __builtin_amdgcn_s_memrealtime());
}

// ------------------------------------------------------------------ load-time folding
// out[i, j] = sum_k A[i, k] g[k] Bm[k sbk + j sbj] (+ add_row[i] + add_col[j]) in fp64,
// rounded once to fp32; Bm null: out = A diag(g).
__global__ void __launch_bounds__(256) fold_mm_kernel(const float* __restrict__ A, int lda,
                                                      const float* __restrict__ g, const float* __restrict__ Bm,
                                                      long sbk, long sbj, int K, const float* __restrict__ add_row,
                                                      const float* __restrict__ add_col, float* __restrict__ out,
                                                      int ldo, int cols) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y;
  if (j >= cols) return;
  const float* a = A + (size_t)i * lda;
  double acc = 0.0;
  if (Bm) {
    for (int k = 0; k < K; ++k)
      acc += (double)a[k] * (g ? (double)g[k] : 1.0) * (double)Bm[(long)k * sbk + (long)j * sbj];
  } else {
    acc = (double)a[j] * (g ? (double)g[j] : 1.0);
  }
  if (add_row) acc += (double)add_row[i];
  if (add_col) acc += (double)add_col[j];
  out[(size_t)i * ldo + j] = (float)acc;
}

}  // namespace

void launch_foldgemm(const FoldGemmParams& p, hipStream_t s) {
  if (p.NZ < 0 || p.NZ % 16 != 0 || (p.NZ && (!p.Wz || !p.bz || !p.z)))
    throw std::runtime_error("foldgemm: NZ must be a multiple of 16 with Wz, bz, z");
  const bool s1 = p.a1_stats != nullptr, s2 = p.a2_stats != nullptr;
  if ((s1 && (!p.a1_s || !p.a1_c)) || (s2 && (!p.a2_g || !p.a2_b)))
    throw std::runtime_error("foldgemm: statistics need their vectors");
  if (!p.A1 || !p.A2 || !p.Wy || !p.by || !p.y || !p.y_stats) throw std::runtime_error("foldgemm: null operand");
  if (p.B <= 0) return;
  const dim3 grid(kD / 16 + p.NZ / 16, (p.B + 15) / 16);
  // 4 waves split K (8-wave workgroups measured no faster)
  const bool x3 = p.Wy_hi != nullptr;
  if (x3 && (!p.Wy_lo || (p.NZ && (!p.Wz_hi || !p.Wz_lo))))
    throw std::runtime_error("foldgemm: bf16x3 needs hi and lo planes of Wy and Wz");
#define MOCR_FG(K1, S1, S2)                                      \
  if (x3)                                                        \
    foldgemm_kernel<K1, S1, S2, 4, true><<<grid, 256, 0, s>>>(p); \
  else                                                           \
    foldgemm_kernel<K1, S1, S2, 4, false><<<grid, 256, 0, s>>>(p);
  if (p.K1 == 256 && !s1 && !s2) {
    MOCR_FG(256, false, false)
  } else if (p.K1 == 256 && !s1 && s2) {
    MOCR_FG(256, false, true)
  } else if (p.K1 == 512 && s1 && s2) {
    MOCR_FG(512, true, true)
  } else {
    throw std::runtime_error("foldgemm: built for (K1 256, A2 plain or LayerNorm) and (K1 512, both)");
  }
#undef MOCR_FG
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_foldattn(const FoldAttnParams& p, bool self_attn, hipStream_t s) {
  if (p.n < 1 || p.n > 288) throw std::runtime_error("foldattn: 1..288 keys");
  const bool zs = p.z_stats != nullptr;
  if (zs && (!p.s || !p.c)) throw std::runtime_error("foldattn: statistics need s and c");
  if (self_attn && (!p.kcache || !p.vcache || p.n != p.t + 1 || p.z_ld < 3 * kD))
    throw std::runtime_error("foldattn: self-attention needs the cache, n = t + 1 and q|k|v");
  if (p.sel_on && (!self_attn || zs || !p.qtab || !p.qpos || !p.emb || !p.pos || !p.x || p.sel.t != p.t - 1 ||
                   (p.sel.part && p.sel.nparts > 512)))
    throw std::runtime_error("foldattn: the selection runs in layer 0's self-attention of step sel.t + 1");
  const bool f24 = p.K24 != nullptr, i16 = p.K16 != nullptr;
  if (f24 && (!p.V24 || (self_attn && (!p.kc24 || !p.vc24))))
    throw std::runtime_error("foldattn: fp24 K/V needs K and V (and the cache)");
  if (i16 && (self_attn || f24 || !p.V16 || !p.Ks || !p.Vs || p.s_b < kD))
    throw std::runtime_error("foldattn: int16 K/V is cross-attention only, with K, V and their scales");
  const bool s16 = p.kc16 != nullptr;
  if (s16 && (!self_attn || f24 || i16 || !p.vc16 || !p.ksc || !p.vsc || p.f24_h % 32 != 0))
    throw std::runtime_error("foldattn: the int16 cache is self-attention only, with K, V and their scales");
  if (p.B <= 0) return;
  // waves per workgroup: 2 unless the keys exceed 2 x 8 x 10 (tools/attn_ts: the 4-wave
  // kernel's per-wave fixed work -- statistics, unfold, the reductions -- made 8 waves per
  // SIMD VALU-bound: cross 9.9 -> 8.5 us, self at t = 16 6.9 -> 5.4, t = 120 10.8 -> 10.3)
  // (one wave up to 40 keys: self-attention at t = 16 5.42 -> 4.75 us; equal at t = 60,
  // slower from there and for the 144 memory keys, 8.5 -> 9.3 us)
  const int nw = p.waves ? p.waves : (p.n > 160 ? 4 : (p.n <= 40 ? 1 : 2));
  if (nw != 1 && nw != 2 && nw != 4) throw std::runtime_error("foldattn: 1, 2 or 4 waves");
  const int nit = (p.n + 8 * nw - 1) / (8 * nw);  // 8 nw key rows per workgroup pass
  const dim3 grid(p.B, kD / 32);
#define MOCR_FA2(N, F, W)                                                                  \
  if (self_attn && zs)                                                                     \
    dec_foldattn_kernel<true, true, false, N, F, W><<<grid, 64 * W, 0, s>>>(p);           \
  else if (self_attn && p.sel_on)                                                          \
    dec_foldattn_kernel<true, false, true, N, F, W><<<grid, 64 * W, 0, s>>>(p);           \
  else if (self_attn)                                                                      \
    dec_foldattn_kernel<true, false, false, N, F, W><<<grid, 64 * W, 0, s>>>(p);          \
  else if (zs)                                                                             \
    dec_foldattn_kernel<false, true, false, N, F, W><<<grid, 64 * W, 0, s>>>(p);          \
  else                                                                                     \
    dec_foldattn_kernel<false, false, false, N, F, W><<<grid, 64 * W, 0, s>>>(p);
#define MOCR_FA3(N, W)                                                                     \
  if (i16) {                                                                               \
    if (zs)                                                                                \
      dec_foldattn_kernel<false, true, false, N, 2, W><<<grid, 64 * W, 0, s>>>(p);        \
    else                                                                                   \
      dec_foldattn_kernel<false, false, false, N, 2, W><<<grid, 64 * W, 0, s>>>(p);       \
  } else if (s16) {                                                                        \
    if (zs)                                                                                \
      dec_foldattn_kernel<true, true, false, N, 3, W><<<grid, 64 * W, 0, s>>>(p);         \
    else if (p.sel_on)                                                                     \
      dec_foldattn_kernel<true, false, true, N, 3, W><<<grid, 64 * W, 0, s>>>(p);         \
    else                                                                                   \
      dec_foldattn_kernel<true, false, false, N, 3, W><<<grid, 64 * W, 0, s>>>(p);        \
  } else if (f24) {                                                                        \
    MOCR_FA2(N, 1, W)                                                                      \
  } else {                                                                                 \
    MOCR_FA2(N, 0, W)                                                                      \
  }
#define MOCR_FA(N, W) \
  case N:               \
    MOCR_FA3(N, W)      \
    break;
  if ((nw == 2 && nit > 10) || (nw == 1 && nit > 5))
    throw std::runtime_error("foldattn: at most 160 keys on 2 waves, 40 on 1");
  if (p.slot_rows) {
    // beam hypotheses' self-attention: the int16 cache (bf16x3 engines) or fp32 (fp32 engines)
    if (!self_attn || p.sel_on || f24 || p.slot_ld < p.n) throw std::runtime_error("foldattn: slot tables need "
                                                                                   "self-attention on the int16 or fp32 cache");
#define MOCR_FS(N, W)                                                                          \
  case N:                                                                                      \
    if (s16 && zs) dec_foldattn_kernel<true, true, false, N, 3, W, true><<<grid, 64 * W, 0, s>>>(p);       \
    else if (s16) dec_foldattn_kernel<true, false, false, N, 3, W, true><<<grid, 64 * W, 0, s>>>(p);       \
    else if (zs) dec_foldattn_kernel<true, true, false, N, 0, W, true><<<grid, 64 * W, 0, s>>>(p);         \
    else dec_foldattn_kernel<true, false, false, N, 0, W, true><<<grid, 64 * W, 0, s>>>(p);                \
    break;
    if (nw == 4) {
      switch (nit) {
        MOCR_FS(1, 4) MOCR_FS(2, 4) MOCR_FS(3, 4) MOCR_FS(4, 4) MOCR_FS(5, 4) MOCR_FS(6, 4) MOCR_FS(7, 4) MOCR_FS(8, 4)
        MOCR_FS(9, 4)
        default: throw std::runtime_error("foldattn: at most 288 keys");
      }
    } else if (nw == 2) {
      switch (nit) {
        MOCR_FS(1, 2) MOCR_FS(2, 2) MOCR_FS(3, 2) MOCR_FS(4, 2) MOCR_FS(5, 2) MOCR_FS(6, 2) MOCR_FS(7, 2) MOCR_FS(8, 2)
        MOCR_FS(9, 2) MOCR_FS(10, 2)
        default: break;
      }
    } else {
      switch (nit) {
        MOCR_FS(1, 1) MOCR_FS(2, 1) MOCR_FS(3, 1) MOCR_FS(4, 1) MOCR_FS(5, 1)
        default: break;
      }
    }
#undef MOCR_FS
    MOCR_HIP_CHECK(hipGetLastError());
    return;
  }
  if (nw == 4) {
    switch (nit) {
      MOCR_FA(1, 4) MOCR_FA(2, 4) MOCR_FA(3, 4) MOCR_FA(4, 4) MOCR_FA(5, 4) MOCR_FA(6, 4) MOCR_FA(7, 4) MOCR_FA(8, 4)
      MOCR_FA(9, 4)
      default: throw std::runtime_error("foldattn: at most 288 keys");
    }
  } else if (nw == 2) {
    switch (nit) {
      MOCR_FA(1, 2) MOCR_FA(2, 2) MOCR_FA(3, 2) MOCR_FA(4, 2) MOCR_FA(5, 2) MOCR_FA(6, 2) MOCR_FA(7, 2) MOCR_FA(8, 2)
      MOCR_FA(9, 2) MOCR_FA(10, 2)
      default: break;
    }
  } else {
    switch (nit) {
      MOCR_FA(1, 1) MOCR_FA(2, 1) MOCR_FA(3, 1) MOCR_FA(4, 1) MOCR_FA(5, 1)
      default: break;
    }
  }
#undef MOCR_FA
#undef MOCR_FA3
#undef MOCR_FA2
  MOCR_HIP_CHECK(hipGetLastError());
}

#ifdef MOCR_FOLD_TS
extern "C" int mocr_debug_attn_ts(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_attn_ts), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif

void launch_fold_mm(const float* A, int lda, const float* g, const float* Bm, long sbk, long sbj, int K,
                    const float* add_row, const float* add_col, float* out, int ldo, int rows, int cols,
                    hipStream_t s) {
  if (rows <= 0 || cols <= 0) return;
  const dim3 grid((cols + 255) / 256, rows);
  fold_mm_kernel<<<grid, 256, 0, s>>>(A, lda, g, Bm, sbk, sbj, K, add_row, add_col, out, ldo, cols);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
