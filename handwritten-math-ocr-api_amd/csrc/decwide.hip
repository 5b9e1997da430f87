// Wide-tile fold GEMM of the greedy decode step (kernels.h FoldGemmParams) for decode
// chains of 64-256+ rows: the same folded LayerNorm algebra as decfold.hip foldgemm_kernel
// (torch/nn/modules/transformer.py:1143-1199 post-norm layer, see decfold.hip's header),
// and the fc_out logits (src/model_swin.py:87) with the greedy selection's tile partials.
//
// decfold.hip computes 16x16 output tiles, so at R rows every tile re-reads its 16 A rows
// and 16 W columns over the whole K from L2: at R = 256 the FFN fold GEMM (N = 1024,
// K = 768) moves ~150 MB through L2 per launch for 0.2 GFLOP and takes 17 us
// (profiles/r03/chain1).  Here a workgroup owns a BM x BN tile (32 x 32 at R > 64), its 4
// waves split K four ways (each wave holds the whole tile's accumulators for its K range,
// so A and W are each loaded once per workgroup) and combine through LDS in a fixed
// order; loads run PD k-steps ahead of the MFMAs.  Blocks are numbered column tile
// fastest, so block b's column tile is b mod ncol and, with ncol a multiple of 8, each
// XCD (blocks b, b + 8, ...) streams 1/8 of W for every row tile.
//
// Columns [0, NY) are y tiles (K = K1 over A1'); columns [NY, NY + NZ) are z tiles over
// [A1' | A2'] (K = K1 + d), as foldgemm_kernel.  LOGITS (K1 = 0, NY = 0): the z tiles are
// fc_out over LN(A2), written to the logits slot of step t with the per-16-column
// (max, first argmax, sum exp) partials the selection reads (decoder.hip DEC_LOGITS).
#include "kernels.h"
#include "lanes.h"

namespace mocr {

#ifdef MOCR_FOLD_TS
// timing probe (tools/build_variant.sh DIR -DMOCR_FOLD_TS, tools/wide_bench.hip): per
// workgroup, thread 0's clocks at the tile's phase boundaries; slot 0 / 6 the 100-MHz
// real-time clock at entry / exit, 1..5 the shader clock (see wide_tile)
__device__ unsigned long long g_fold_ts[8192 * 8];
#define MOCR_TS(i, v) \
  if (threadIdx.x == 0 && blockIdx.x < 8192) g_fold_ts[blockIdx.x * 8 + (i)] = (v)
#else
#define MOCR_TS(i, v)
#endif

namespace {

constexpr int kD = 256;
constexpr int kSlices = kD / 16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split8(const floatx4& x0, const floatx4& x1, bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
  split2_bf16(x0[0], x0[1], h[0], l[0]);
  split2_bf16(x0[2], x0[3], h[1], l[1]);
  split2_bf16(x1[0], x1[1], h[2], l[2]);
  split2_bf16(x1[2], x1[3], h[3], l[3]);
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

// Row statistics from the 16 (mean, M2) slice partials, merged by decoder.hip's fixed
// binary tree (bit-identical to every other consumer of the same LayerNorm).
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
struct Part4 {
  floatx4 p0, p1;
};
// layout 1: the 4 lanes g = 0..3 of a row (lane, lane ^ 16, ^ 32, ^ 48) hold slices 4g..4g+3
__device__ __forceinline__ Part4 load_part4(const float* __restrict__ part, int g) {
  return {*reinterpret_cast<const floatx4*>(part + 8 * g), *reinterpret_cast<const floatx4*>(part + 8 * g + 4)};
}
__device__ __forceinline__ void merge_part4(const Part4& pp, int g, float& mean, float& rstd) {
  float m = pp.p0[0], q = pp.p0[1], m2 = pp.p1[0], q2 = pp.p1[1];
  merge_eq(m, q, pp.p0[2], pp.p0[3], 16.f);
  merge_eq(m2, q2, pp.p1[2], pp.p1[3], 16.f);
  merge_eq(m, q, m2, q2, 32.f);
  merge_lanes<16>(m, q, (g & 1) != 0, 64.f);
  merge_lanes<32>(m, q, (g & 2) != 0, 128.f);
  mean = m;
  rstd = rstd_of(q);
}
// the same tree with the 4 lanes of a row adjacent (lane ^ 1, lane ^ 2: coalesced layout)
__device__ __forceinline__ void merge_part4_quad(const Part4& pp, int g, float& mean, float& rstd) {
  float m = pp.p0[0], q = pp.p0[1], m2 = pp.p1[0], q2 = pp.p1[1];
  merge_eq(m, q, pp.p0[2], pp.p0[3], 16.f);
  merge_eq(m2, q2, pp.p1[2], pp.p1[3], 16.f);
  merge_eq(m, q, m2, q2, 32.f);
  merge_lanes<1>(m, q, (g & 1) != 0, 64.f);
  merge_lanes<2>(m, q, (g & 2) != 0, 128.f);
  mean = m;
  rstd = rstd_of(q);
}
// layout 2 from preloaded (mean, M2) of slice c
__device__ __forceinline__ void row_stats_16lanes_v(float m, float q, int c, float& mean, float& rstd) {
  merge_lanes<1>(m, q, (c & 1) != 0, 16.f);
  merge_lanes<2>(m, q, (c & 2) != 0, 32.f);
  merge_lanes<4>(m, q, (c & 4) != 0, 64.f);
  merge_lanes<8>(m, q, (c & 8) != 0, 128.f);
  mean = m;
  rstd = rstd_of(q);
}
// layout 2: the 16 lanes c = 0..15 of a row each hold slice c
__device__ __forceinline__ void row_stats_16lanes(const float* __restrict__ part, int c, float& mean, float& rstd) {
  float m = part[2 * c], q = part[2 * c + 1];
  merge_lanes<1>(m, q, (c & 1) != 0, 16.f);
  merge_lanes<2>(m, q, (c & 2) != 0, 32.f);
  merge_lanes<4>(m, q, (c & 4) != 0, 64.f);
  merge_lanes<8>(m, q, (c & 8) != 0, 128.f);
  mean = m;
  rstd = rstd_of(q);
}

// LDS of one tile: the k-vectors (u, v), each wave's A fragments of one k step (reused
// step after step: a wave's LDS accesses execute in order), the 4-wave reduction.
template <int BM, int BN, bool YT, int K1, bool X3, int NW>
struct TileLds {
  static constexpr int KT = YT ? K1 : K1 + kD;
  static constexpr int UV = 2 * KT * 4;
  static constexpr int AW = (BM / 16) * (X3 ? 2 : 1) * 1024;  // per wave: one step's fragments
  // the reduction's row pitch: 32 x 32 tiles on 8 waves read it 4 columns per lane (16-B
  // aligned rows), the others one column per lane
  static constexpr int RP = (BM == 32 && BN == 32 && NW == 8) ? BN + 4 : BN + 1;
  static constexpr int RED = NW * BM * RP * 4;
  static constexpr int BYTES = UV + NW * AW + RED;
};

// One BM x BN tile.  KT = the tile's K (K1 for y tiles, K1 + d for z tiles); each of the
// 4 waves takes KT / 4 consecutive k in steps of KS (32: bf16x3 16x16x32; 16: fp32 16x16x4
// in four MFMAs).
//  - Every load is issued up front, step by step (the step-s A pieces and W fragments
//    together), so each step waits only for its own data.
//  - A is loaded coalesced (lane = row (lane >> 2) x 16 bytes (lane & 3) of a 64-byte row
//    segment: every quad of lanes reads one segment), transformed once (FFN unfold + ReLU,
//    LayerNorm), split into bf16 hi / lo (X3) and written to the wave's LDS region in MFMA
//    fragment order, read back with one ds_read_b128 per fragment: a per-wave transpose,
//    no workgroup barrier in the k loop.
//  - W comes fragment-major (launch_frag_pack): one contiguous 1-KB load per 16-column x
//    k-step fragment and plane.
//  - Everything the epilogue reads (bias, LayerNorm vectors and statistics, residual) is
//    loaded before the first store: a load issued after a store waits for it (vmcnt).
// MFMA operands: row / column = lane & 15, k = 8 g .. 8 g + 7 of the step (X3) or
// 4 g .. 4 g + 3 (fp32), g = lane >> 4.
template <int BM, int BN, bool YT, int K1, bool S1, bool S2, bool X3, bool LOGITS, int NW, int PD>
__device__ __forceinline__ void wide_tile(const FoldGemmParams& p, int r0, int c0, char* smem) {
  using L = TileLds<BM, BN, YT, K1, X3, NW>;
  constexpr int MF = BM / 16, NF = BN / 16;
  constexpr int KT = L::KT;
  constexpr int KW = KT / NW;
  constexpr int KS = X3 ? 32 : 16;
  constexpr int NKS = KW / KS;
  constexpr int SPS = KS / 16;  // 64-byte row segments per k step
  static_assert(KW % KS == 0 && K1 % 32 == 0, "k steps never straddle A1 / A2");
  constexpr bool UV = S1 || (S2 && !YT);  // y tiles read A1 only; their LN2 residual uses 16-lane stats
  floatx4* uv_s = reinterpret_cast<floatx4*>(smem);                        // [2][KT / 4]
  char* a_s = smem + L::UV + (threadIdx.x >> 6) * L::AW;                   // this wave's fragments
  float* red = reinterpret_cast<float*>(smem + L::UV + NW * L::AW);       // [NW][BM][L::RP]
  MOCR_TS(0, __builtin_amdgcn_s_memrealtime());
  MOCR_TS(1, __builtin_amdgcn_s_memtime());
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 2;  // coalesced layout: row within a 16-row block
  const int c = lane & 3;   //                   16-byte piece of a 64-byte segment
  const int kbeg = wave * KW;
  const int B = p.B;
  const int ldw = YT ? K1 : K1 + kD;
  const int wt0 = (YT ? c0 : c0 - p.NY) / 16;  // first 16-column tile of W

  // ---- every load first: k-vectors, statistics, then A and W step by step, epilogue operands
  floatx4 u4{}, v4{};
  const int kk4 = min(tid * 4, KT - 4);
  if constexpr (UV) {
    static_assert(KT / 4 <= 64 * NW, "one float4 of u and of v per thread");
    const bool in1 = kk4 < K1;
    const float* us = in1 ? (S1 ? p.a1_s + kk4 : p.a2_g) : (S2 ? p.a2_g + (kk4 - K1) : p.a2_g);
    const float* vs = in1 ? (S1 ? p.a1_c + kk4 : p.a2_b) : (S2 ? p.a2_b + (kk4 - K1) : p.a2_b);
    u4 = *reinterpret_cast<const floatx4*>(us);
    v4 = *reinterpret_cast<const floatx4*>(vs);
  }
  int qrow[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) qrow[mf] = min(r0 + mf * 16 + q, B - 1);  // rows >= B: discarded outputs
  Part4 pa1[MF], pa2[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    if constexpr (S1) pa1[mf] = load_part4(p.a1_stats + (size_t)qrow[mf] * 2 * kSlices, c);
    if constexpr (S2 && !YT) pa2[mf] = load_part4(p.a2_stats + (size_t)qrow[mf] * 2 * kSlices, c);
  }
  // step s's A pieces and W fragments live in ring slot s % NR: the first NR steps are
  // loaded up front, step s + NR's right after step s's MFMAs (PD < NKS trades that step's
  // load latency for registers: the FFN kernel at 148 VGPRs holds one 8-wave workgroup per
  // CU, at PD = 2 two, so a chain of more than 256 rows is still one round)
  constexpr int NR = PD < NKS ? PD : NKS;
  floatx4 ra[NR][SPS][MF];
  floatx4 rw[NR][NF][X3 ? 2 : 1];
  auto load_step = [&](int s) {
    const int sl = s % NR;
#pragma unroll
    for (int h = 0; h < SPS; ++h) {
      const int sg = s * SPS + h;
      const int k = kbeg + sg * 16 + c * 4;
      const bool in1 = kbeg + sg * 16 < K1;  // wave-uniform
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
        ra[sl][h][mf] = *reinterpret_cast<const floatx4*>(in1 ? p.A1 + (size_t)qrow[mf] * K1 + k
                                                              : p.A2 + (size_t)qrow[mf] * kD + (k - K1));
    }
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) {
      const size_t fo = ((size_t)(wt0 + nf) * (ldw / KS) + kbeg / KS + s) * 64 + lane;
      if constexpr (X3) {
        rw[sl][nf][0] = reinterpret_cast<const floatx4*>(YT ? p.Fy_hi : p.Fz_hi)[fo];
        rw[sl][nf][1] = reinterpret_cast<const floatx4*>(YT ? p.Fy_lo : p.Fz_lo)[fo];
      } else {
        rw[sl][nf][0] = reinterpret_cast<const floatx4*>(YT ? p.Fy : p.Fz)[fo];
      }
    }
  };
#pragma unroll
  for (int s = 0; s < NR; ++s) load_step(s);
  // epilogue operands (the first 256 threads: row = tid >> 4 of each 16-row block, column
  // = tid & 15 of each 16-column block)
  const int erow = (tid & 255) >> 4;
  const int ecol = tid & 15;
  // 32 x 32 fold tiles (not the logits): the epilogue takes 4 consecutive columns of one row
  // per thread (row tid / 8, columns 4 (tid % 8) ..): float4 reduction reads and 16-B stores
  // instead of one column per thread and 4-B stores
  constexpr bool V4 = !LOGITS && BM == 32 && BN == 32 && NW == 8;
  constexpr int RP = L::RP;
  const int vrow = (tid & 255) >> 3;
  const int vj = tid & 7;
  const int vcol = vj * 4;
  floatx4 vres{}, vbias{}, vg{}, vb{}, vst{};
  if constexpr (V4) {
    const int col = (YT ? c0 : c0 - p.NY) + vcol;
    vbias = *reinterpret_cast<const floatx4*>((YT ? p.by : p.bz) + col);
    if constexpr (YT) {
      const int srow = min(r0 + vrow, B - 1);
      vres = *reinterpret_cast<const floatx4*>(p.A2 + (size_t)srow * kD + c0 + vcol);
      if constexpr (S2) {
        vg = *reinterpret_cast<const floatx4*>(p.a2_g + col);
        vb = *reinterpret_cast<const floatx4*>(p.a2_b + col);
        // slices 2 vj, 2 vj + 1 of the row's LayerNorm statistics (mean, M2)
        vst = reinterpret_cast<const floatx4*>(p.a2_stats + (size_t)srow * 2 * kSlices)[vj];
      }
    }
  }
  float rres[YT ? MF : 1][YT ? NF : 1], ebias[NF], eg[YT && S2 ? NF : 1], eb[YT && S2 ? NF : 1];
  float2 est[YT && S2 ? MF : 1];
#pragma unroll
  for (int nf = 0; nf < (V4 ? 0 : NF); ++nf) {
    const int col = (YT ? c0 : c0 - p.NY) + nf * 16 + ecol;
    ebias[nf] = (YT ? p.by : p.bz)[col];
    if constexpr (YT && S2) {
      eg[nf] = p.a2_g[col];
      eb[nf] = p.a2_b[col];
    }
  }
  if constexpr (YT && !V4) {
#pragma unroll
    for (int mf = 0; mf < MF; ++mf) {
      const int srow = min(r0 + mf * 16 + erow, B - 1);
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) rres[mf][nf] = p.A2[(size_t)srow * kD + c0 + nf * 16 + ecol];
      if constexpr (S2) est[mf] = reinterpret_cast<const float2*>(p.a2_stats + (size_t)srow * 2 * kSlices)[ecol];
    }
  }

  if constexpr (UV) {
    if (tid * 4 < KT) {
      uv_s[kk4 / 4] = u4;
      uv_s[KT / 4 + kk4 / 4] = v4;
    }
    __syncthreads();
  }
#ifdef MOCR_FOLD_TS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  MOCR_TS(2, __builtin_amdgcn_s_memtime());
  float m1[MF], rs1[MF], m2[MF], rs2[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    m1[mf] = rs1[mf] = m2[mf] = rs2[mf] = 0.f;
    if constexpr (S1) merge_part4_quad(pa1[mf], c, m1[mf], rs1[mf]);
    if constexpr (S2 && !YT) merge_part4_quad(pa2[mf], c, m2[mf], rs2[mf]);
  }

  // ---- k loop: transform + split step s's A pieces into the wave's LDS fragments, read
  // them back in MFMA order, MFMAs with the step's W fragments
  floatx4 acc[MF][NF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) acc[mf][nf] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
#pragma unroll
    for (int h = 0; h < SPS; ++h) {
      const int sg = s * SPS + h;
      const int kl = kbeg + sg * 16 + c * 4;  // the tile's k of the piece's first value
      const bool in1 = kbeg + sg * 16 < K1;
      floatx4 uu{}, vv{};
      if ((S1 && in1) || (S2 && !YT && !in1)) {
        uu = uv_s[kl / 4];
        vv = uv_s[KT / 4 + kl / 4];
      }
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        floatx4 x = ra[s % NR][h][mf];
        if ((S1 && in1) || (S2 && !YT && !in1)) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (in1) {
              if constexpr (S1) x[e] = fmaxf(fmaf(rs1[mf], fmaf(-m1[mf], uu[e], x[e]), vv[e]), 0.f);
            } else {
              if constexpr (S2 && !YT) x[e] = fmaf((x[e] - m2[mf]) * rs2[mf], uu[e], vv[e]);
            }
          }
        }
        if constexpr (X3) {
          // k within the step h 16 + 4 c = 8 g_t + 4 (c & 1)
          const int lt = q + 16 * (h * 2 + (c >> 1));
          uint32_t h0, l0, h1, l1;
          split2_bf16(x[0], x[1], h0, l0);
          split2_bf16(x[2], x[3], h1, l1);
          char* f = a_s + mf * 2048 + lt * 16 + (c & 1) * 8;
          *reinterpret_cast<uint2*>(f) = make_uint2(h0, h1);
          *reinterpret_cast<uint2*>(f + 1024) = make_uint2(l0, l1);
        } else {
          *reinterpret_cast<floatx4*>(a_s + mf * 1024 + (q + 16 * c) * 16) = x;  // k within the step 4 c
        }
      }
    }
    if constexpr (X3) {
      bf16x8 ah[MF], al[MF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const char* f = a_s + mf * 2048 + lane * 16;
        ah[mf] = *reinterpret_cast<const bf16x8*>(f);
        al[mf] = *reinterpret_cast<const bf16x8*>(f + 1024);
      }
      // the three passes over all MF x NF accumulators in turn (independent MFMAs between
      // two that update one accumulator; the per-element order hi*hi, hi*lo, lo*hi is kept)
#pragma unroll
      for (int pass = 0; pass < 3; ++pass)
#pragma unroll
        for (int mf = 0; mf < MF; ++mf)
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) {
            const bf16x8 a = pass == 2 ? al[mf] : ah[mf];
            const bf16x8 b = __builtin_bit_cast(bf16x8, rw[s % NR][nf][pass == 1 ? 1 : 0]);
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[mf][nf], 0, 0, 0);
          }
      if (s + NR < NKS) load_step(s + NR);
    } else {
      floatx4 a[MF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) a[mf] = *reinterpret_cast<const floatx4*>(a_s + mf * 1024 + lane * 16);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int mf = 0; mf < MF; ++mf)
#pragma unroll
          for (int nf = 0; nf < NF; ++nf)
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mf][e], rw[s % NR][nf][0][e], acc[mf][nf], 0, 0, 0);
      if (s + NR < NKS) load_step(s + NR);
    }
  }

  MOCR_TS(3, __builtin_amdgcn_s_memtime());
  // ---- combine the 4 waves' partial tiles in a fixed order
  const int g = lane >> 4;
  const int li = lane & 15;
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wave * BM + mf * 16 + g * 4 + r) * RP + nf * 16 + li] = acc[mf][nf][r];
  __syncthreads();
  MOCR_TS(4, __builtin_amdgcn_s_memtime());
  if (tid >= 256 || dec_skip(p.st, p.t)) return;
  if constexpr (V4) {
    const int orow = r0 + vrow;
    floatx4 val = *reinterpret_cast<const floatx4*>(red + vrow * RP + vcol);
#pragma unroll
    for (int w = 1; w < NW; ++w) val += *reinterpret_cast<const floatx4*>(red + (w * BM + vrow) * RP + vcol);
    if constexpr (YT) {
      floatx4 res = vres;
      if constexpr (S2) {
        // decoder.hip's fixed merge tree over the 16 slices: level 1 in the lane (slices 2 vj,
        // 2 vj + 1), then lanes vj ^ 1, ^ 2, ^ 4 -- the pairs row_stats_16lanes_v merges
        float m = vst[0], q = vst[1];
        merge_eq(m, q, vst[2], vst[3], 16.f);
        merge_lanes<1>(m, q, (vj & 1) != 0, 32.f);
        merge_lanes<2>(m, q, (vj & 2) != 0, 64.f);
        merge_lanes<4>(m, q, (vj & 4) != 0, 128.f);
        const float rstd = rstd_of(q);
#pragma unroll
        for (int e = 0; e < 4; ++e) res[e] = fmaf((res[e] - m) * rstd, vg[e], vb[e]);
      }
      floatx4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = res[e] + (val[e] + vbias[e]);
      // the 16-column slice's (mean, M2) over its 4 lanes (quad_perm xor 1, xor 2)
      float sm = (y[0] + y[1]) + (y[2] + y[3]);
      sm += dpp<0xB1>(sm);
      sm += dpp<0x4E>(sm);
      const float m16 = sm * (1.0f / 16);
      // the pairs row_sum<16> adds: (0 + 1) + (2 + 3) in the lane, then lanes ^ 1, ^ 2
      float qq = (sq_rn(y[0] - m16) + sq_rn(y[1] - m16)) + (sq_rn(y[2] - m16) + sq_rn(y[3] - m16));
      qq += dpp<0xB1>(qq);
      qq += dpp<0x4E>(qq);
      if (orow < B) {
        *reinterpret_cast<floatx4*>(p.y + (size_t)orow * kD + c0 + vcol) = y;
        if ((vj & 3) == 0) {
          float* so = p.y_stats + ((size_t)orow * kSlices + (c0 + vcol) / 16) * 2;
          so[0] = m16;
          so[1] = qq;
        }
      }
    } else {
      if (orow < B) *reinterpret_cast<floatx4*>(p.z + (size_t)orow * p.NZ + (c0 - p.NY) + vcol) = val + vbias;
    }
    MOCR_TS(5, __builtin_amdgcn_s_memtime());
    MOCR_TS(6, __builtin_amdgcn_s_memrealtime());
    return;
  }
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int orow = r0 + mf * 16 + erow;
    float mean = 0.f, rstd = 0.f;
    if constexpr (YT && S2) row_stats_16lanes_v(est[mf].x, est[mf].y, ecol, mean, rstd);
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) {
      const int lr = mf * 16 + erow, lc = nf * 16 + ecol;
      float val = red[lr * RP + lc];
#pragma unroll
      for (int w = 1; w < NW; ++w) val += red[(w * BM + lr) * RP + lc];
      const int ocol = c0 + nf * 16 + ecol;
      if constexpr (YT) {
        float res = rres[mf][nf];
        if constexpr (S2) res = fmaf((res - mean) * rstd, eg[nf], eb[nf]);
        const float y = res + (val + ebias[nf]);
        const float m16 = row_sum<16>(y) * (1.0f / 16);
        const float qq = row_sum<16>(sq_rn(y - m16));
        if (orow < B) {
          p.y[(size_t)orow * kD + ocol] = y;
          if (ecol == 0) {
            float* so = p.y_stats + ((size_t)orow * kSlices + ocol / 16) * 2;
            so[0] = m16;
            so[1] = qq;
          }
        }
      } else if constexpr (LOGITS) {
        const int zc = ocol - p.NY;
        const float v = val + ebias[nf];
        const bool cv = zc < p.n_valid;
        // z null: the greedy step without a logits history, whose selection reads only
        // the tile partials (select.h), stores no logits row
        if (p.z && orow < B && cv) p.z[(p.hist_stride ? (size_t)p.t * p.hist_stride : 0) + (size_t)orow * p.NZ + zc] = v;
        if (p.part) {
          // the 16-column tile's (max, first argmax, sum exp(l - max)) over the row's 16
          // lanes (DPP quad_perm xor 1, xor 2, row_half_mirror, row_mirror)
          float m = cv ? v : -INFINITY;
          int ix = zc;
          auto step = [&](float om, int oi) {
            if (om > m || (om == m && oi < ix)) {
              m = om;
              ix = oi;
            }
          };
          step(dpp<0xB1>(m), __builtin_amdgcn_mov_dpp(ix, 0xB1, 0xF, 0xF, false));
          step(dpp<0x4E>(m), __builtin_amdgcn_mov_dpp(ix, 0x4E, 0xF, 0xF, false));
          step(dpp<0x141>(m), __builtin_amdgcn_mov_dpp(ix, 0x141, 0xF, 0xF, false));
          step(dpp<0x140>(m), __builtin_amdgcn_mov_dpp(ix, 0x140, 0xF, 0xF, false));
          const float e = row_sum<16>(cv ? __expf(v - m) : 0.f);  // v_exp_f32
          if (ecol == 0 && orow < B)
            reinterpret_cast<floatx4*>(p.part)[(size_t)orow * (p.NZ / 16) + zc / 16] =
                floatx4{m, __int_as_float(ix), e, 0.f};
        }
      } else {
        const int zc = ocol - p.NY;
        if (orow < B) p.z[(size_t)orow * p.NZ + zc] = val + ebias[nf];
      }
    }
  }
  MOCR_TS(5, __builtin_amdgcn_s_memtime());
  MOCR_TS(6, __builtin_amdgcn_s_memrealtime());
}

template <int BM, int BN, int K1, bool S1, bool S2, bool X3, bool LOGITS, int NW, int PD>
__global__ void __launch_bounds__(64 * NW) foldwide_kernel(FoldGemmParams p) {
  constexpr int BYTES = LOGITS ? TileLds<BM, BN, false, 0, X3, NW>::BYTES
                               : (TileLds<BM, BN, true, K1, X3, NW>::BYTES > TileLds<BM, BN, false, K1, X3, NW>::BYTES
                                      ? TileLds<BM, BN, true, K1, X3, NW>::BYTES
                                      : TileLds<BM, BN, false, K1, X3, NW>::BYTES);
  __shared__ __attribute__((aligned(16))) char smem[BYTES];
  const int ncol = (p.NY + p.NZ) / BN;
  const int b = blockIdx.x;
  const int c0 = (b % ncol) * BN;
  const int r0 = (b / ncol) * BM;
  if constexpr (LOGITS) {
    wide_tile<BM, BN, false, 0, false, true, X3, true, NW, PD>(p, r0, c0, smem);
  } else {
    if (c0 < p.NY)
      wide_tile<BM, BN, true, K1, S1, S2, X3, false, NW, PD>(p, r0, c0, smem);
    else
      wide_tile<BM, BN, false, K1, S1, S2, X3, false, NW, PD>(p, r0, c0, smem);
  }
}

// Fragment-major copy of a row-major [N, K] fp32 weight (N % 16 == 0, K % 32 == 0):
// X3 planes hi / lo [N/16][K/32][64 lanes][8] (bf16 split as split2_bf16), or fp32
// [N/16][K/16][64 lanes][4]; lane L holds W[16 j + (L & 15)][k0 + (8 or 4) (L >> 4) + e].
// perm (planes only): lane L's 8 elements are k0 + 4 (L >> 4) + {0..3, 16..19}, the
// permuted k order of wattn.hip's proj GEMM (its B fragments are the attention's O^T
// accumulators of two 16-dim tiles).
__global__ void frag_pack_kernel(const float* __restrict__ W, int N, int K, uint16_t* __restrict__ hi,
                                 uint16_t* __restrict__ lo, float* __restrict__ f32, int perm) {
  const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // one lane-chunk
  const bool x3 = hi != nullptr;
  const int ks = x3 ? 32 : 16, per = x3 ? 8 : 4;
  const size_t nchunks = (size_t)N * K / per;
  if (idx >= nchunks) return;
  const int L = idx % 64;
  const size_t t = idx / 64;
  const int s = t % (K / ks);
  const int j = t / (K / ks);
  const float* src = W + (size_t)(16 * j + (L & 15)) * K + s * ks + (perm ? 4 : per) * (L >> 4);
  if (x3) {
    uint32_t h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k0 = perm && e >= 2 ? 12 : 0;  // elements 4..7 at +16 under perm
      split2_bf16(src[k0 + 2 * e], src[k0 + 2 * e + 1], h[e], l[e]);
    }
    reinterpret_cast<uint4*>(hi)[idx] = make_uint4(h[0], h[1], h[2], h[3]);
    reinterpret_cast<uint4*>(lo)[idx] = make_uint4(l[0], l[1], l[2], l[3]);
  } else {
    reinterpret_cast<floatx4*>(f32)[idx] = floatx4{src[0], src[1], src[2], src[3]};
  }
}

template <int BM, int BN, bool X3, bool LOGITS, int NW, int PD>
void launch_fw_pd(const FoldGemmParams& p, hipStream_t s) {
  const int ncol = (p.NY + p.NZ) / BN;
  const dim3 grid(ncol * ((p.B + BM - 1) / BM));
  if constexpr (LOGITS) {
    foldwide_kernel<BM, BN, 0, false, true, X3, true, NW, PD><<<grid, 64 * NW, 0, s>>>(p);
  } else {
    const bool s1 = p.a1_stats != nullptr, s2 = p.a2_stats != nullptr;
    if (p.K1 == 256 && !s1 && !s2) {
      foldwide_kernel<BM, BN, 256, false, false, X3, false, NW, PD><<<grid, 64 * NW, 0, s>>>(p);
    } else if (p.K1 == 256 && !s1 && s2) {
      foldwide_kernel<BM, BN, 256, false, true, X3, false, NW, PD><<<grid, 64 * NW, 0, s>>>(p);
    } else if (p.K1 == 512 && s1 && s2) {
      foldwide_kernel<BM, BN, 512, true, true, X3, false, NW, PD><<<grid, 64 * NW, 0, s>>>(p);
    } else {
      throw std::runtime_error("foldwide: built for (K1 256, A2 plain or LayerNorm), (K1 512, both), logits");
    }
  }
}

// the FFN kernel (K1 = 512, 32 x 32 tiles, 8 waves) with every k step's loads in flight
// holds one workgroup per CU; above 256 workgroups (chains of more than 256 rows) it keeps
// two k steps in flight instead, which fits two (profiles/r04/r04h)
template <int BM, int BN, bool X3, bool LOGITS, int NW>
void launch_fw_nw(const FoldGemmParams& p, hipStream_t s) {
  if constexpr (!LOGITS && NW == 8 && BM == 32 && BN == 32) {
    const int nblk = (p.NY + p.NZ) / BN * ((p.B + BM - 1) / BM);
    if (p.K1 == 512 && nblk > 256 && !p.no_prefetch_ring) {
      launch_fw_pd<BM, BN, X3, LOGITS, NW, 2>(p, s);
      return;
    }
  }
  launch_fw_pd<BM, BN, X3, LOGITS, NW, 8>(p, s);
}

// NW waves split K (p.waves: 4 or 8; 0 = kWideWaves).  The same NW at every row count, so
// a row's k order never depends on its chain's length.
// measured (tools/wide_bench, profiles/r03/wide_bench_v3.log): 8 waves for the fold GEMMs
// (FFN at 256 rows 9.1 -> 7.5 us), 4 for the logits (10.8 vs 11.8 us)
template <int BM, int BN, bool X3, bool LOGITS>
void launch_fw(const FoldGemmParams& p, hipStream_t s) {
  constexpr int kFoldWaves = 8, kLogitsWaves = 4;
  if ((p.waves ? p.waves : (LOGITS ? kLogitsWaves : kFoldWaves)) == 8)
    launch_fw_nw<BM, BN, X3, LOGITS, 8>(p, s);
  else
    launch_fw_nw<BM, BN, X3, LOGITS, 4>(p, s);
}

}  // namespace

// Wide fold GEMM (y tiles + z tiles) or, with p.K1 == 0 and the logits fields, fc_out.
void launch_foldwide(const FoldGemmParams& p, hipStream_t s) {
  const bool logits = p.K1 == 0;
  const bool x3 = logits ? p.Fz_hi != nullptr : p.Fy_hi != nullptr;
  if (logits) {
    if (p.NY != 0 || !p.a2_stats || !p.a2_g || !p.a2_b || !p.A2 || !p.bz || !(p.z || p.part) || p.NZ % 32 != 0)
      throw std::runtime_error("foldwide logits: A2 with LayerNorm, no y, z or partials, NZ % 32 == 0");
  } else {
    if (p.NY != kD || p.NZ % 32 != 0 || (p.NZ && (!p.bz || !p.z)))
      throw std::runtime_error("foldwide: NY == d and NZ a multiple of 32 with bz, z");
    // XCD placement (column tile = block % ncol, ncol % 8 == 0) holds for 16- and 32-wide tiles
    if (!p.A1 || !p.A2 || !p.by || !p.y || !p.y_stats) throw std::runtime_error("foldwide: null operand");
  }
  if ((p.a1_stats && (!p.a1_s || !p.a1_c)) || (p.a2_stats && (!p.a2_g || !p.a2_b)))
    throw std::runtime_error("foldwide: statistics need their vectors");
  const bool need_z = logits || p.NZ > 0;
  const bool have = x3 ? (!need_z || (p.Fz_hi && p.Fz_lo)) && (logits || (p.Fy_hi && p.Fy_lo))
                       : (!need_z || p.Fz) && (logits || p.Fy);
  if (!have) throw std::runtime_error("foldwide: fragment-major weights (launch_frag_pack) missing");
  if (p.B <= 0) return;
  // fold GEMMs: 16-row tiles up to 64 rows (more workgroups for a short chain), 32 above
  if (logits) {  // 16-row tiles; columns per tile p.tile_cols (A/B) or the default below
    // 64-column tiles above 64 rows (9.9 vs 10.9 us at 256 rows), 32 up to 64 (5.2 vs 5.9 us);
    // a row's k order does not depend on the tile width (profiles/r03/wide_bench_v4.log)
    const int bn = p.tile_cols ? p.tile_cols : (p.B > 64 ? 64 : 32);
    if (p.NZ % bn != 0) throw std::runtime_error("foldwide logits: NZ must be a multiple of the column tile");
    if (bn == 128) {
      if (x3) launch_fw<16, 128, true, true>(p, s); else launch_fw<16, 128, false, true>(p, s);
    } else if (bn == 64) {
      if (x3) launch_fw<16, 64, true, true>(p, s); else launch_fw<16, 64, false, true>(p, s);
    } else {
      if (x3) launch_fw<16, 32, true, true>(p, s); else launch_fw<16, 32, false, true>(p, s);
    }
  } else {
    // 16-column tiles when 32-column ones would leave CUs idle (e.g. N = 512 at 256 rows)
    const int bm = p.B <= 64 ? 16 : 32;
    const bool narrow_n = (p.NY + p.NZ) / 32 * ((p.B + bm - 1) / bm) < 256;
    if (bm == 16) {
      if (narrow_n) {
        if (x3) launch_fw<16, 16, true, false>(p, s); else launch_fw<16, 16, false, false>(p, s);
      } else {
        if (x3) launch_fw<16, 32, true, false>(p, s); else launch_fw<16, 32, false, false>(p, s);
      }
    } else {
      if (narrow_n) {
        if (x3) launch_fw<32, 16, true, false>(p, s); else launch_fw<32, 16, false, false>(p, s);
      } else {
        if (x3) launch_fw<32, 32, true, false>(p, s); else launch_fw<32, 32, false, false>(p, s);
      }
    }
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

#ifdef MOCR_FOLD_TS
extern "C" int mocr_debug_fold_ts(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fold_ts), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif

void launch_frag_pack(const float* W, int N, int K, uint16_t* hi, uint16_t* lo, float* f32, hipStream_t s,
                      bool perm) {
  if (N % 16 != 0 || K % 32 != 0 || (!hi != !lo) || (!hi && !f32)) throw std::runtime_error("frag_pack: N % 16, K % 32");
  if (perm && !hi) throw std::runtime_error("frag_pack: the permuted k order is built for bf16 planes");
  const size_t chunks = (size_t)N * K / (hi ? 8 : 4);
  frag_pack_kernel<<<(unsigned)((chunks + 255) / 256), 256, 0, s>>>(W, N, K, hi, lo, f32, perm ? 1 : 0);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
