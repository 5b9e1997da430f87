// Fused attention half of a Swin block on bf16 / bf16x3 MFMA (torchvision
// SwinTransformerBlock: x = x + proj(W-MSA(norm1(x)))), for one shifted window per
// workgroup and one head per wave.  Unfused, a stage-1 block moves ~2.3 GB through HBM
// for these four ops (the LN'd window partition as bf16 planes, QKV written and read
// back in fp32, the attention output planes, the residual); fused, X is read once and
// read-modify-written once per token.
//
//  A. norm1 of the window's 49 tokens (shift roll and zero padding applied on the
//     gather, as ln_partition_kernel) into LDS as bf16 hi / lo planes, 64 rows
//     (rows 49..63 and padded tokens are zero rows, F.pad after norm1);
//  B. wave h: q^T, k^T = W_{q,k}[head h] . LN^T and v = LN . W_v[head h]^T over the
//     C channels (W fragments straight from global, LN fragments from LDS).  The
//     accumulators ARE the attention operands (no data movement):
//       - K (A of S^T = K Q^T): lane (g, j) holds key j of a tile and dims
//         {4g..4g+3} of k^T tile 0, {16+4g..} of tile 1: a permuted k order, the
//         same for Q (B of S^T), so the contraction is unchanged;
//       - V^T (A of O^T = V^T P^T): lane (g, j) holds dim j and keys 4g+r of the
//         token tiles 2s, 2s+1 (swin.hip window_attention_mfma_kernel's key order);
//  C. S^T, bias + mask table, softmax, O^T as in window_attention_mfma_kernel;
//  D. O^T fragments (lane (g, j): token j, dims {4g+r, 16+4g+r} of head h) go to LDS
//     as the B fragments of proj's k-step h; wave w computes out^T rows 32w .. 32w+31
//     (A = W_proj rows, the same permuted k order), adds bias + residual and scatters
//     to the window-reversed, un-rolled pixel (EPI_WINRES's mapping).
//
// Stage 3 (C = 384, 12 heads: swin_attn_noproj_kernel) keeps A-C and drops D: the LN'd
// window alone fills 96 KB of LDS, so there is no room for proj's operands beside it.
// The waves loop over the heads, keep the LN rows in LDS for the whole kernel, and write
// O as bf16 hi / lo planes in window-token order -- the A operand of the proj GEMM
// (EPI_WINRES), exactly as window_attention_mfma_kernel writes it.  That removes the
// LN-partition kernel, the fp32 QKV round trip and the attention kernel's re-read
// (s3, PMC: 864 MB -> 195 MB of HBM traffic per block before proj).
#include "kernels.h"
#include "lanes.h"

namespace mocr {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void pack8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split2_bf16(v[2 * e], v[2 * e + 1], h[e], l[e]);
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

// c += a . b with a, b as bf16 hi (/ lo) planes: hi*hi (+ hi*lo + lo*hi for bf16x3)
template <bool X3>
__device__ __forceinline__ floatx4 mma(const bf16x8 (&a)[2], const bf16x8 (&b)[2], floatx4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
  if constexpr (X3) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
  }
  return c;
}

// WPB windows per workgroup, HEADS waves each: the waves of one head in the WPB windows
// load the same weight fragments at the same point of the same instruction stream (the
// block's barriers keep them in step), so the CU's L1 can serve the later ones.
template <int C, int PASSES, int OCC, int WPB>
__global__ void __launch_bounds__(2 * C * WPB) __attribute__((amdgpu_waves_per_eu(OCC))) swin_attn_kernel(SwinAttnParams p) {
  constexpr bool X3 = PASSES == 3;
  constexpr int PL = X3 ? 2 : 1;
  constexpr int HEADS = C / 32;  // = waves = k-steps of every GEMM here
  constexpr int NT = 64 * HEADS;
  constexpr int RC = C / 8;      // 16-B chunks per LN row
  // chunk c of row r at c ^ s(r): conflict-free ds_read_b128 fragment reads (mlp.hip W1 image)
  constexpr int SW = (RC % 16 == 0) ? 16 : ((RC % 8 == 0) ? 8 : 4);
  constexpr int SH = SW == 16 ? 0 : 1;
  constexpr int XB = 64 * C * 2;  // bytes per plane: the LN'd window, later proj's B fragments
  constexpr int LPR = C / 12;     // lanes per row in the LayerNorm (12 floats each)
  static_assert(RC % SW == 0 && 64 % LPR == 0, "layout");
  __shared__ __attribute__((aligned(16))) char lds_all[WPB * PL * XB];

  const int wsub = (int)threadIdx.x / NT;    // this wave's window within the workgroup
  const int tid = (int)threadIdx.x - wsub * NT;
  char* const lds = lds_all + wsub * PL * XB;
  const int lane = tid & 63;
  const int h = tid >> 6;
  const int j16 = lane & 15;
  const int g = lane >> 4;
  const WinGeom& wg = p.wg;
  // a window past the last (odd window count) recomputes the last one and stores nothing
  const long nwin_all = (long)p.B * wg.nWin;
  const long gw_raw = (long)blockIdx.x * WPB + wsub;
  const bool live = gw_raw < nwin_all;
  const long gw = live ? gw_raw : nwin_all - 1;
  const int b = (int)(gw / wg.nWin);
  const int win = (int)(gw - (long)b * wg.nWin);
  const int wy = win / wg.nWx;
  const int wx = win - wy * wg.nWx;
  // X row of window token tk, -1 for the padded tokens and slots 49..63
  auto pixel = [&](int tk) -> long {
    const int ty = tk / kWin;
    int y = wy * kWin + ty + wg.sh;
    int x = wx * kWin + (tk - ty * kWin) + wg.sw;
    if (y >= wg.pH) y -= wg.pH;
    if (x >= wg.pW) x -= wg.pW;
    return (tk < kWinTok && y < wg.H && x < wg.W) ? (long)(b * wg.H + y) * wg.W + x : -1L;
  };

  // ---- A: norm1 into LDS (ln_group_kernel's lanes per row and summation order; the xor
  // reductions as DPP moves, which add the same pairs; 1/C and rsqrt as multiplies)
  {
    constexpr int RPP = NT / LPR;              // rows per pass (24)
    constexpr int NP = (64 + RPP - 1) / RPP;   // passes (3)
    const int gi = lane % LPR;
    const int c0 = gi * 12;
    float v[NP][12];
    long px[NP];
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {  // every load first
      px[ps] = pixel(ps * RPP + tid / LPR);
      const float* src = p.X + (size_t)(px[ps] < 0 ? 0 : px[ps]) * C + c0;  // clamped, masked below
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const floatx4 t = *reinterpret_cast<const floatx4*>(src + 4 * e);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[ps][4 * e + k] = t[k];
      }
    }
    floatx4 gg[3], bb[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      gg[e] = *reinterpret_cast<const floatx4*>(p.ln_g + c0 + 4 * e);
      bb[e] = *reinterpret_cast<const floatx4*>(p.ln_b + c0 + 4 * e);
    }
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {
      const int r = ps * RPP + tid / LPR;
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) s += v[ps][e];
      s = row_sum<LPR>(s);
      const float mean = s * (1.0f / C);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) {
        const float d = v[ps][e] - mean;
        q += d * d;
      }
      q = row_sum<LPR>(q);
      const float rstd = rsqrtf(q * (1.0f / C) + 1e-5f);
      const bool zero = px[ps] < 0;
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        float y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = zero ? 0.f : (v[ps][4 * e + k] - mean) * rstd * gg[e][k] + bb[e][k];
        uint32_t h0, l0, h1, l1;
        split2_bf16(y[0], y[1], h0, l0);
        split2_bf16(y[2], y[3], h1, l1);
        const int c = c0 + 4 * e;
        const int off = r * (2 * C) + (((c >> 3) ^ ((r >> SH) & (SW - 1))) << 4) + ((c >> 2) & 1) * 8;
        if (ps * RPP + RPP <= 64 || r < 64) {
          *reinterpret_cast<uint2*>(lds + off) = make_uint2(h0, h1);
          if constexpr (X3) *reinterpret_cast<uint2*>(lds + XB + off) = make_uint2(l0, l1);
        }
      }
    }
  }
  __syncthreads();

  // ---- B: k^T, v, q^T of head h, one 8-tile GEMM at a time (each converted to its
  // attention fragments at once, so only one set of accumulators is live)
  // W_qkv fragment-major (launch_frag_pack): fragment (16-row tile, k-step) = 64 lanes x 16 B
  const bf16x8* wqh = static_cast<const bf16x8*>(p.wqkv_fm);
  const bf16x8* wql = static_cast<const bf16x8*>(p.wqkv_fm_lo);
  auto wfm = [&](int row0, int f, int ks, bf16x8(&w)[2]) {
    const int o = (((row0 >> 4) + f) * HEADS + ks) * 64 + lane;
    w[0] = wqh[o];
    if constexpr (X3) w[1] = wql[o];
  };
  const float* bq = p.bqkv;
  // LN fragment (tokens 16t + j16, channels 32ks + 8g ..): B of the k^T / q^T GEMMs, A of v's
  auto xfrag = [&](int ks, int t, bf16x8(&f)[2]) {
    const int r = 16 * t + j16;
    const int off = r * (2 * C) + (((4 * ks + g) ^ ((r >> SH) & (SW - 1))) << 4);
    f[0] = *reinterpret_cast<const bf16x8*>(lds + off);
    if constexpr (X3) f[1] = *reinterpret_cast<const bf16x8*>(lds + XB + off);
  };
  // acc[f][t] = W[row0 + 16f + j16, :] . LN^T (features x tokens)
  // the weight fragments of k-step ks + 1 are loaded while the MFMAs of ks run (a register
  // double buffer; the scheduling barrier keeps hipcc from sinking the loads to their use,
  // where each one waited out its whole L2 round trip)
  auto wload = [&](int row0, int ks, bf16x8(&w)[2][2]) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      wfm(row0, f, ks, w[f]);
    }
  };
  // PRE: the double buffer (the k^T GEMM; the q^T GEMM runs with k and v live and keeps
  // one buffer: two spilled)
  auto gemm_t = [&](int row0, floatx4(&acc)[2][4], auto pre) {
    constexpr bool PRE = decltype(pre)::value;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[f][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    bf16x8 w[PRE ? 2 : 1][2][2];
    wload(row0, 0, w[0]);
#pragma unroll
    for (int ks = 0; ks < HEADS; ++ks) {
      if (PRE && ks + 1 < HEADS) wload(row0, ks + 1, w[(ks + 1) & (PRE ? 1 : 0)]);
      else if (!PRE && ks > 0) wload(row0, ks, w[0]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bf16x8 xf[2];
        xfrag(ks, t, xf);
#pragma unroll
        for (int f = 0; f < 2; ++f)
          acc[f][t] = mma<X3>(w[ks & (PRE ? 1 : 0)][f], xf, acc[f][t]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  bf16x8 kf[4][2], vf[2][2][2], qf4[4][2];
  __builtin_amdgcn_s_setprio(1);
  {
    floatx4 acc[2][4];
    gemm_t(C + 32 * h, acc, std::true_type{});
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      float x[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        x[r] = acc[0][kt][r] + bq[C + 32 * h + 4 * g + r];
        x[4 + r] = acc[1][kt][r] + bq[C + 32 * h + 16 + 4 * g + r];
      }
      pack8(x, kf[kt][0], kf[kt][1]);
    }
  }
  // the three GEMMs one after the other: interleaved by the scheduler they spilled 72 B
  // per lane at C = 96 (s1.attn 935 -> 890 us per block pair, profiles/r02/ab_s12_sched_barrier.log)
  __builtin_amdgcn_sched_barrier(0);
  {
    // v [tokens x dims]: A = LN rows, B = W_v rows
    floatx4 acc[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t][0] = acc[t][1] = floatx4{0.f, 0.f, 0.f, 0.f};
    bf16x8 w[2][2][2];
    wload(2 * C + 32 * h, 0, w[0]);
#pragma unroll
    for (int ks = 0; ks < HEADS; ++ks) {
      if (ks + 1 < HEADS) wload(2 * C + 32 * h, ks + 1, w[(ks + 1) & 1]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bf16x8 xf[2];
        xfrag(ks, t, xf);
#pragma unroll
        for (int f = 0; f < 2; ++f)
          acc[t][f] = mma<X3>(xf, w[ks & 1][f], acc[t][f]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const float bv = bq[2 * C + 32 * h + 16 * dt + j16];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float x[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[r] = acc[2 * s][dt][r] + bv;
          x[4 + r] = acc[2 * s + 1][dt][r] + bv;
        }
        pack8(x, vf[dt][s][0], vf[dt][s][1]);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  {
    floatx4 acc[2][4];
    gemm_t(32 * h, acc, std::false_type{});
    const float scale = 0.17677669529663687f;  // 32 ** -0.5
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      float x[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        x[r] = (acc[0][qt][r] + bq[32 * h + 4 * g + r]) * scale;
        x[4 + r] = (acc[1][qt][r] + bq[32 * h + 16 + 4 * g + r]) * scale;
      }
      pack8(x, qf4[qt][0], qf4[qt][1]);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  __syncthreads();  // every wave is done with the LN rows: the region takes proj's operands

  // ---- C: attention per 16-query tile
  int type = 0;
  if (wg.sh + wg.sw > 0) type = 2 * (wy == wg.nWin / wg.nWx - 1) + (wx == wg.nWx - 1);
  const float* tb = p.table + ((size_t)type * HEADS + h) * 64 * 64;
  // bias + mask of the current query tile.  Key tile 3 holds keys 48 + 4 g + r: only key 48
  // (g = 0, r = 0) exists, keys 49..63 are -inf for every real query (build_relmask), so
  // r = 1..3 of that tile are skipped (exp = 0 exactly; max and sum unchanged) and only r = 0
  // of its bias is loaded.  The padded queries 49..63 change, but their rows are never stored.
  floatx4 bm[3];
  float bm3;
#pragma unroll
  for (int kt = 0; kt < 3; ++kt) bm[kt] = *reinterpret_cast<const floatx4*>(tb + j16 * 64 + 16 * kt + 4 * g);
  bm3 = tb[j16 * 64 + 48 + 4 * g];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    if (qt > 0) {
#pragma unroll
      for (int kt = 0; kt < 3; ++kt)
        bm[kt] = *reinterpret_cast<const floatx4*>(tb + (16 * qt + j16) * 64 + 16 * kt + 4 * g);
      bm3 = tb[(16 * qt + j16) * 64 + 48 + 4 * g];
    }
    floatx4 st[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) st[kt] = mma<X3>(kf[kt], qf4[qt], floatx4{0.f, 0.f, 0.f, 0.f});
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 3; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[kt][r] = st[kt][r] + bm[kt][r];
        m = fmaxf(m, st[kt][r]);
      }
    }
    st[3][0] = st[3][0] + bm3;
    m = fmaxf(m, st[3][0]);
    m = xmax16_32(m);
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 3; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[kt][r] = __expf(st[kt][r] - m);
        sum += st[kt][r];
      }
    st[3][0] = __expf(st[3][0] - m);
    sum += st[3][0];
    st[3][1] = st[3][2] = st[3][3] = 0.f;
    sum = xsum16_32(sum);
    bf16x8 pf[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = st[2 * s + (j >> 2)][j & 3];
      pack8(x, pf[s][0], pf[s][1]);
    }
    floatx4 o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      o[dt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) o[dt] = mma<X3>(vf[dt][s], pf[s], o[dt]);
    }
    // softmax normalisation after P.V (per query = per lane column); proj's B fragment
    // (token q, channels 32h + {4g+r, 16+4g+r}), lane-linear in LDS
    const float inv = __builtin_amdgcn_rcpf(sum);
    float x[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[r] = o[0][r] * inv;
      x[4 + r] = o[1][r] * inv;
    }
    bf16x8 ohl[2];
    pack8(x, ohl[0], ohl[1]);
    const int off = ((qt * HEADS + h) * 64 + lane) * 16;
    *reinterpret_cast<bf16x8*>(lds + off) = ohl[0];
    if constexpr (X3) *reinterpret_cast<bf16x8*>(lds + XB + off) = ohl[1];
  }
  __syncthreads();

  // ---- D: out^T rows 32h .. 32h+31 = W_proj . O^T, + bias + residual
  // W_proj fragment-major in the permuted k order (launch_frag_pack perm): lane (g, j) of
  // fragment (16-row tile, head hh) holds channels 32 hh + {4g..4g+3, 16+4g..16+4g+3}
  const bf16x8* wph = static_cast<const bf16x8*>(p.wproj_fm);
  const bf16x8* wpl = static_cast<const bf16x8*>(p.wproj_fm_lo);
  long pxo[4];
  floatx4 xres[2][4];  // the residual rows, loaded before the GEMM
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    pxo[t] = pixel(16 * t + j16);
#pragma unroll
    for (int f = 0; f < 2; ++f)
      xres[f][t] = *reinterpret_cast<const floatx4*>(p.X + (size_t)(pxo[t] < 0 ? 0 : pxo[t]) * C + 32 * h + 16 * f +
                                                     4 * g);
  }
  floatx4 ap[2][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) ap[0][t] = ap[1][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_s_setprio(1);
  // W_proj fragments one k-step ahead, as the qkv GEMMs.  At C = 192 (6 heads) a full
  // unroll hoisted every k-step's weight loads and spilled at 3 waves per SIMD: by 2
  auto pload = [&](int hh, bf16x8(&wa)[2][2]) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int o = ((2 * h + f) * HEADS + hh) * 64 + lane;
      wa[f][0] = wph[o];
      if constexpr (X3) wa[f][1] = wpl[o];
    }
  };
  bf16x8 wa[2][2][2];
  pload(0, wa[0]);
  constexpr int PU = C == 192 ? 2 : HEADS;
#pragma unroll PU
  for (int hh = 0; hh < HEADS; ++hh) {
    if (hh + 1 < HEADS) pload(hh + 1, wa[(hh + 1) & 1]);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bf16x8 of[2];
      const int off = ((t * HEADS + hh) * 64 + lane) * 16;
      of[0] = *reinterpret_cast<const bf16x8*>(lds + off);
      if constexpr (X3) of[1] = *reinterpret_cast<const bf16x8*>(lds + XB + off);
#pragma unroll
      for (int f = 0; f < 2; ++f)
        ap[f][t] = mma<X3>(wa[hh & 1][f], of, ap[f][t]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int ch = 32 * h + 16 * f + 4 * g;
    const floatx4 bp = *reinterpret_cast<const floatx4*>(p.bproj + ch);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (pxo[t] < 0 || !live) continue;
      floatx4 xv = xres[f][t];
#pragma unroll
      for (int r = 0; r < 4; ++r) xv[r] = xv[r] + (ap[f][t][r] + bp[r]);
      *reinterpret_cast<floatx4*>(p.X + (size_t)pxo[t] * C + ch) = xv;
    }
  }
}

// Stage 3: norm1 + qkv + W-MSA without proj (see the header): WAVES waves loop over the
// heads, O goes to the ATT planes.
// C of the no-proj kernels: attention of one head (K, V^T, Q^T fragments as B leaves
// them) per 16-query tile; O goes to the ATT planes [window token row, C] at channels
// ch0 + {4g.., 16+4g..} (tok0 = the window's first row)
// (16-B stores with lane pairs trading halves measured 1 % slower at C = 384: r05/r07t)
template <bool X3, int C>
__device__ __forceinline__ void attend_to_planes(const bf16x8 (&kf)[4][2], const bf16x8 (&vf)[2][2][2],
                                                 const bf16x8 (&qf4)[4][2], const float* tb, int j16, int g,
                                                 const long (&orow)[4], int ch0, uint16_t* att_hi,
                                                 uint16_t* att_lo) {
  floatx4 bm[4];  // bias + mask of the current query tile
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) bm[kt] = *reinterpret_cast<const floatx4*>(tb + j16 * 64 + 16 * kt + 4 * g);
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    if (qt > 0) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
        bm[kt] = *reinterpret_cast<const floatx4*>(tb + (16 * qt + j16) * 64 + 16 * kt + 4 * g);
    }
    floatx4 st[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) st[kt] = mma<X3>(kf[kt], qf4[qt], floatx4{0.f, 0.f, 0.f, 0.f});
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[kt][r] = st[kt][r] + bm[kt][r];
        m = fmaxf(m, st[kt][r]);
      }
    }
    m = xmax16_32(m);
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[kt][r] = __expf(st[kt][r] - m);
        sum += st[kt][r];
      }
    sum = xsum16_32(sum);
    bf16x8 pf[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = st[2 * s + (j >> 2)][j & 3];
      pack8(x, pf[s][0], pf[s][1]);
    }
    floatx4 o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      o[dt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) o[dt] = mma<X3>(vf[dt][s], pf[s], o[dt]);
    }
    // softmax normalisation after P.V (per query = per lane column)
    const float inv = __builtin_amdgcn_rcpf(sum);
    float x[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[r] = o[0][r] * inv;
      x[4 + r] = o[1][r] * inv;
    }
    // ATT planes [row, C]: query token 16qt + j16 -> row orow[qt] (-1: not written),
    // channels 32h + {4g.., 16+4g..}
    if (orow[qt] >= 0) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const size_t off = (size_t)orow[qt] * C + ch0 + 16 * dt + 4 * g;
        uint32_t h0, l0, h1, l1;
        split2_bf16(x[4 * dt], x[4 * dt + 1], h0, l0);
        split2_bf16(x[4 * dt + 2], x[4 * dt + 3], h1, l1);
        *reinterpret_cast<uint2*>(att_hi + off) = make_uint2(h0, h1);
        if constexpr (X3) *reinterpret_cast<uint2*>(att_lo + off) = make_uint2(l0, l1);
      }
    }
  }
}

template <int C, int PASSES, int OCC, int WAVES, int KU>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(OCC)))
swin_attn_noproj_kernel(SwinAttnParams p) {
  constexpr bool X3 = PASSES == 3;
  constexpr int PL = X3 ? 2 : 1;
  constexpr int HEADS = C / 32;  // = k-steps of every GEMM here
  constexpr int NT = 64 * WAVES;
  constexpr int RC = C / 8;      // 16-B chunks per LN row
  // chunk c of row r at c ^ s(r): conflict-free ds_read_b128 fragment reads (mlp.hip W1 image)
  constexpr int SW = (RC % 16 == 0) ? 16 : ((RC % 8 == 0) ? 8 : 4);
  constexpr int SH = SW == 16 ? 0 : 1;
  constexpr int XB = 64 * C * 2;  // bytes per plane: the LN'd window, later proj's B fragments
  constexpr int LPR = C / 12;     // lanes per row in the LayerNorm (12 floats each)
  static_assert(RC % SW == 0 && 64 % LPR == 0, "layout");
  __shared__ __attribute__((aligned(16))) char lds[PL * XB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int j16 = lane & 15;
  const int g = lane >> 4;
  const WinGeom& wg = p.wg;
  const int b = (int)(blockIdx.x / (unsigned)wg.nWin);
  const int win = (int)(blockIdx.x - (unsigned)b * wg.nWin);
  const int wy = win / wg.nWx;
  const int wx = win - wy * wg.nWx;
  // X row of window token tk, -1 for the padded tokens and slots 49..63
  auto pixel = [&](int tk) -> long {
    const int ty = tk / kWin;
    int y = wy * kWin + ty + wg.sh;
    int x = wx * kWin + (tk - ty * kWin) + wg.sw;
    if (y >= wg.pH) y -= wg.pH;
    if (x >= wg.pW) x -= wg.pW;
    return (tk < kWinTok && y < wg.H && x < wg.W) ? (long)(b * wg.H + y) * wg.W + x : -1L;
  };

  // ---- A: norm1 into LDS (ln_group_kernel's lanes per row and summation order; the xor
  // reductions as DPP moves, which add the same pairs; 1/C and rsqrt as multiplies)
  {
    constexpr int RPP = NT / LPR;              // rows per pass (24; 16 at C = 384)
    constexpr int NP = (64 + RPP - 1) / RPP;   // passes (3; 4)
    const int gi = lane % LPR;
    const int c0 = gi * 12;
    float v[NP][12];
    long px[NP];
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {  // every load first
      px[ps] = pixel(ps * RPP + tid / LPR);
      const float* src = p.X + (size_t)(px[ps] < 0 ? 0 : px[ps]) * C + c0;  // clamped, masked below
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const floatx4 t = *reinterpret_cast<const floatx4*>(src + 4 * e);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[ps][4 * e + k] = t[k];
      }
    }
    floatx4 gg[3], bb[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      gg[e] = *reinterpret_cast<const floatx4*>(p.ln_g + c0 + 4 * e);
      bb[e] = *reinterpret_cast<const floatx4*>(p.ln_b + c0 + 4 * e);
    }
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {
      const int r = ps * RPP + tid / LPR;
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) s += v[ps][e];
      s = row_sum<LPR>(s);
      const float mean = s * (1.0f / C);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) {
        const float d = v[ps][e] - mean;
        q += d * d;
      }
      q = row_sum<LPR>(q);
      const float rstd = rsqrtf(q * (1.0f / C) + 1e-5f);
      const bool zero = px[ps] < 0;
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        float y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = zero ? 0.f : (v[ps][4 * e + k] - mean) * rstd * gg[e][k] + bb[e][k];
        uint32_t h0, l0, h1, l1;
        split2_bf16(y[0], y[1], h0, l0);
        split2_bf16(y[2], y[3], h1, l1);
        const int c = c0 + 4 * e;
        const int off = r * (2 * C) + (((c >> 3) ^ ((r >> SH) & (SW - 1))) << 4) + ((c >> 2) & 1) * 8;
        if (ps * RPP + RPP <= 64 || r < 64) {
          *reinterpret_cast<uint2*>(lds + off) = make_uint2(h0, h1);
          if constexpr (X3) *reinterpret_cast<uint2*>(lds + XB + off) = make_uint2(l0, l1);
        }
      }
    }
  }
  __syncthreads();

  // ---- B-C per head: k^T, v, q^T of head h, one 8-tile GEMM at a time (each converted
  // to its attention fragments at once, so only one set of accumulators is live), then
  // attention per 16-query tile
  // W_qkv fragment-major (launch_frag_pack), as swin_attn_kernel
  const bf16x8* wqh = static_cast<const bf16x8*>(p.wqkv_fm);
  const bf16x8* wql = static_cast<const bf16x8*>(p.wqkv_fm_lo);
  auto wfm = [&](int row0, int f, int ks, bf16x8(&w)[2]) {
    const int o = (((row0 >> 4) + f) * HEADS + ks) * 64 + lane;
    w[0] = wqh[o];
    if constexpr (X3) w[1] = wql[o];
  };
  const float* bq = p.bqkv;
  // LN fragment (tokens 16t + j16, channels 32ks + 8g ..): B of the k^T / q^T GEMMs, A of v's
  auto xfrag = [&](int ks, int t, bf16x8(&f)[2]) {
    const int r = 16 * t + j16;
    const int off = r * (2 * C) + (((4 * ks + g) ^ ((r >> SH) & (SW - 1))) << 4);
    f[0] = *reinterpret_cast<const bf16x8*>(lds + off);
    if constexpr (X3) f[1] = *reinterpret_cast<const bf16x8*>(lds + XB + off);
  };
  // weight fragments of k-step ks + 1 loaded while the MFMAs of ks run (swin_attn_kernel)
  auto wload = [&](int row0, int ks, bf16x8(&w)[2][2]) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      wfm(row0, f, ks, w[f]);
    }
  };
  // acc[f][t] = W[row0 + 16f + j16, :] . LN^T (features x tokens)
  auto gemm_t = [&](int row0, floatx4(&acc)[2][4]) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[f][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    bf16x8 w[2][2][2];
    wload(row0, 0, w[0]);
#pragma unroll KU
    for (int ks = 0; ks < HEADS; ++ks) {
      if (ks + 1 < HEADS) wload(row0, ks + 1, w[(ks + 1) & 1]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bf16x8 xf[2];
        xfrag(ks, t, xf);
#pragma unroll
        for (int f = 0; f < 2; ++f)
          acc[f][t] = mma<X3>(w[ks & 1][f], xf, acc[f][t]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // destination row of each of this lane's 4 query tokens: the pixel row (window reverse,
  // un-roll and crop, padded tokens dropped: proj is then a plain residual-add GEMM over
  // the image's tokens), or the window-token row (the EPI_WINRES proj)
  long orow[4];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    const int q = 16 * qt + j16;
    orow[qt] = p.att_pixel_rows ? pixel(q) : (q < kWinTok ? ((long)b * wg.nWin + win) * kWinTok + q : -1L);
  }
#pragma unroll 1
  for (int h = wave; h < HEADS; h += WAVES) {
    bf16x8 kf[4][2], vf[2][2][2], qf4[4][2];
    __builtin_amdgcn_s_setprio(1);
    {
      floatx4 acc[2][4];
      gemm_t(C + 32 * h, acc);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        float x[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[r] = acc[0][kt][r] + bq[C + 32 * h + 4 * g + r];
          x[4 + r] = acc[1][kt][r] + bq[C + 32 * h + 16 + 4 * g + r];
        }
        pack8(x, kf[kt][0], kf[kt][1]);
      }
    }
    {
      // v [tokens x dims]: A = LN rows, B = W_v rows
      floatx4 acc[4][2];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t][0] = acc[t][1] = floatx4{0.f, 0.f, 0.f, 0.f};
      bf16x8 w[2][2][2];
      wload(2 * C + 32 * h, 0, w[0]);
#pragma unroll KU
      for (int ks = 0; ks < HEADS; ++ks) {
        if (ks + 1 < HEADS) wload(2 * C + 32 * h, ks + 1, w[(ks + 1) & 1]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          bf16x8 xf[2];
          xfrag(ks, t, xf);
#pragma unroll
          for (int f = 0; f < 2; ++f) acc[t][f] = mma<X3>(xf, w[ks & 1][f], acc[t][f]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const float bv = bq[2 * C + 32 * h + 16 * dt + j16];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float x[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            x[r] = acc[2 * s][dt][r] + bv;
            x[4 + r] = acc[2 * s + 1][dt][r] + bv;
          }
          pack8(x, vf[dt][s][0], vf[dt][s][1]);
        }
      }
    }
    {
      floatx4 acc[2][4];
      gemm_t(32 * h, acc);
      const float scale = 0.17677669529663687f;  // 32 ** -0.5
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        float x[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[r] = (acc[0][qt][r] + bq[32 * h + 4 * g + r]) * scale;
          x[4 + r] = (acc[1][qt][r] + bq[32 * h + 16 + 4 * g + r]) * scale;
        }
        pack8(x, qf4[qt][0], qf4[qt][1]);
      }
    }
    __builtin_amdgcn_s_setprio(0);

    // ---- C: attention per 16-query tile
    int type = 0;
    if (wg.sh + wg.sw > 0) type = 2 * (wy == wg.nWin / wg.nWx - 1) + (wx == wg.nWx - 1);
    attend_to_planes<X3, C>(kf, vf, qf4, p.table + ((size_t)type * HEADS + h) * 64 * 64, j16, g, orow, 32 * h,
                            p.att_hi, p.att_lo);
  }
}

// Stage 4 (C = 768, 24 heads): the LN'd window would take 192 KB of LDS, so the channels
// go through LDS in two halves of 384.  Each workgroup owns HPG heads of one window (one
// per wave) and keeps the head's k^T, v and q^T accumulators in registers across both
// halves: A0 the row statistics over all 768 channels, then per half A (normalise the
// half into LDS) and B (the half's 12 k-steps of the three GEMMs), then C as above.
template <int C, int PASSES, int OCC, int HPG, int KU>
__global__ void __launch_bounds__(64 * HPG) __attribute__((amdgpu_waves_per_eu(OCC)))
swin_attn_noproj_ks_kernel(SwinAttnParams p) {
  constexpr bool X3 = PASSES == 3;
  constexpr int PL = X3 ? 2 : 1;
  constexpr int HEADS = C / 32;
  constexpr int NG = HEADS / HPG;  // workgroups per window
  constexpr int NT = 64 * HPG;
  constexpr int KC = 384;          // channels per LDS half
  constexpr int NKC = C / KC;
  constexpr int KS = KC / 32;      // k-steps per half
  constexpr int RC = KC / 8;
  constexpr int SW = (RC % 16 == 0) ? 16 : ((RC % 8 == 0) ? 8 : 4);
  constexpr int SH = SW == 16 ? 0 : 1;
  constexpr int XB = 64 * KC * 2;
  constexpr int LPR = KC / 12;     // lanes per row of a half (12 floats each)
  static_assert(HEADS % HPG == 0 && C % KC == 0 && RC % SW == 0 && 64 % LPR == 0 && C == 64 * 12, "layout");
  __shared__ __attribute__((aligned(16))) char lds[PL * XB];
  __shared__ float2 stats[64];  // (mean, rstd) per window row

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int j16 = lane & 15;
  const int g = lane >> 4;
  const WinGeom& wg = p.wg;
  const unsigned wgi = blockIdx.x / (unsigned)NG;
  const int hg = (int)(blockIdx.x - wgi * NG);
  const int b = (int)(wgi / (unsigned)wg.nWin);
  const int win = (int)(wgi - (unsigned)b * wg.nWin);
  const int wy = win / wg.nWx;
  const int wx = win - wy * wg.nWx;
  auto pixel = [&](int tk) -> long {
    const int ty = tk / kWin;
    int y = wy * kWin + ty + wg.sh;
    int x = wx * kWin + (tk - ty * kWin) + wg.sw;
    if (y >= wg.pH) y -= wg.pH;
    if (x >= wg.pW) x -= wg.pW;
    return (tk < kWinTok && y < wg.H && x < wg.W) ? (long)(b * wg.H + y) * wg.W + x : -1L;
  };

  // ---- A0: mean and rstd of each row over the 768 channels (one wave per row, 12 each)
#pragma unroll 1
  for (int r = wave; r < 64; r += HPG) {
    const long px = pixel(r);
    const float* src = p.X + (size_t)(px < 0 ? 0 : px) * C + 12 * lane;
    float v[12];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const floatx4 t = *reinterpret_cast<const floatx4*>(src + 4 * e);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[4 * e + k] = t[k];
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 12; ++e) s += v[e];
    const float mean = row_sum<64>(s) * (1.0f / C);
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 12; ++e) {
      const float d = v[e] - mean;
      q += d * d;
    }
    const float rstd = rsqrtf(row_sum<64>(q) * (1.0f / C) + 1e-5f);
    if (lane == 0) stats[r] = make_float2(mean, rstd);
  }

  const int h = hg * HPG + wave;  // this wave's head
  // W_qkv fragment-major (launch_frag_pack), as swin_attn_kernel: fragment (16-row tile,
  // k-step of all C) = 64 lanes x 16 B
  const bf16x8* wqh = static_cast<const bf16x8*>(p.wqkv_fm);
  const bf16x8* wql = static_cast<const bf16x8*>(p.wqkv_fm_lo);
  auto wfm = [&](int row0, int f, int kstep, bf16x8(&w)[2]) {
    const int o = (((row0 >> 4) + f) * HEADS + kstep) * 64 + lane;
    w[0] = wqh[o];
    if constexpr (X3) w[1] = wql[o];
  };
  const float* bq = p.bqkv;
  auto xfrag = [&](int ks, int t, bf16x8(&f)[2]) {
    const int r = 16 * t + j16;
    const int off = r * (2 * KC) + (((4 * ks + g) ^ ((r >> SH) & (SW - 1))) << 4);
    f[0] = *reinterpret_cast<const bf16x8*>(lds + off);
    if constexpr (X3) f[1] = *reinterpret_cast<const bf16x8*>(lds + XB + off);
  };
  // acc[f][t] += W[row0 + 16f + j16, k0 ..] . LN_half^T
  auto gemm_t = [&](int row0, int k0, floatx4(&acc)[2][4]) {
#pragma unroll KU
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 w[2][2];
#pragma unroll
      for (int f = 0; f < 2; ++f) wfm(row0, f, k0 / 32 + ks, w[f]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bf16x8 xf[2];
        xfrag(ks, t, xf);
#pragma unroll
        for (int f = 0; f < 2; ++f) acc[f][t] = mma<X3>(w[f], xf, acc[f][t]);
      }
    }
  };
  floatx4 ak[2][4], aq[2][4], av[4][2];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int t = 0; t < 4; ++t) ak[f][t] = aq[f][t] = av[t][f] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int kc = 0; kc < NKC; ++kc) {
    __syncthreads();  // stats written (kc = 0) / the previous half's fragments read
    // ---- A: channels [KC kc, KC kc + KC) of the LN'd rows into LDS
    {
      constexpr int RPP = NT / LPR;
      constexpr int NP = (64 + RPP - 1) / RPP;
      const int gi = lane % LPR;
      const int c0 = gi * 12;
      const int cg = kc * KC + c0;
#pragma unroll 1
      for (int ps = 0; ps < NP; ++ps) {
        const int r = ps * RPP + tid / LPR;
        if (ps * RPP + RPP <= 64 || r < 64) {
          const long px = pixel(r);
          const float* src = p.X + (size_t)(px < 0 ? 0 : px) * C + cg;
          const float2 st = stats[r];
#pragma unroll
          for (int e = 0; e < 3; ++e) {
            const floatx4 t = *reinterpret_cast<const floatx4*>(src + 4 * e);
            const floatx4 gg = *reinterpret_cast<const floatx4*>(p.ln_g + cg + 4 * e);
            const floatx4 bb = *reinterpret_cast<const floatx4*>(p.ln_b + cg + 4 * e);
            float y[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = px < 0 ? 0.f : (t[k] - st.x) * st.y * gg[k] + bb[k];
            uint32_t h0, l0, h1, l1;
            split2_bf16(y[0], y[1], h0, l0);
            split2_bf16(y[2], y[3], h1, l1);
            const int c = c0 + 4 * e;
            const int off = r * (2 * KC) + (((c >> 3) ^ ((r >> SH) & (SW - 1))) << 4) + ((c >> 2) & 1) * 8;
            *reinterpret_cast<uint2*>(lds + off) = make_uint2(h0, h1);
            if constexpr (X3) *reinterpret_cast<uint2*>(lds + XB + off) = make_uint2(l0, l1);
          }
        }
      }
    }
    __syncthreads();
    // ---- B: this half's k-steps of k^T, v, q^T for head h
    __builtin_amdgcn_s_setprio(1);
    const int k0 = kc * KC;
    gemm_t(C + 32 * h, k0, ak);
#pragma unroll KU
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 w[2][2];
#pragma unroll
      for (int f = 0; f < 2; ++f) wfm(2 * C + 32 * h, f, k0 / 32 + ks, w[f]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bf16x8 xf[2];
        xfrag(ks, t, xf);
#pragma unroll
        for (int f = 0; f < 2; ++f) av[t][f] = mma<X3>(xf, w[f], av[t][f]);
      }
    }
    gemm_t(32 * h, k0, aq);
    __builtin_amdgcn_s_setprio(0);
  }

  // biases, scale, and the accumulators as attention operands (as swin_attn_noproj_kernel)
  bf16x8 kf[4][2], vf[2][2][2], qf4[4][2];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    float x[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[r] = ak[0][kt][r] + bq[C + 32 * h + 4 * g + r];
      x[4 + r] = ak[1][kt][r] + bq[C + 32 * h + 16 + 4 * g + r];
    }
    pack8(x, kf[kt][0], kf[kt][1]);
  }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const float bv = bq[2 * C + 32 * h + 16 * dt + j16];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        x[r] = av[2 * s][dt][r] + bv;
        x[4 + r] = av[2 * s + 1][dt][r] + bv;
      }
      pack8(x, vf[dt][s][0], vf[dt][s][1]);
    }
  }
  const float scale = 0.17677669529663687f;  // 32 ** -0.5
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    float x[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[r] = (aq[0][qt][r] + bq[32 * h + 4 * g + r]) * scale;
      x[4 + r] = (aq[1][qt][r] + bq[32 * h + 16 + 4 * g + r]) * scale;
    }
    pack8(x, qf4[qt][0], qf4[qt][1]);
  }

  // ---- C
  int type = 0;
  if (wg.sh + wg.sw > 0) type = 2 * (wy == wg.nWin / wg.nWx - 1) + (wx == wg.nWx - 1);
  // destination row of each of this lane's 4 query tokens: the pixel row (window reverse,
  // un-roll and crop, padded tokens dropped: proj is then a plain residual-add GEMM over
  // the image's tokens), or the window-token row (the EPI_WINRES proj)
  long orow[4];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    const int q = 16 * qt + j16;
    orow[qt] = p.att_pixel_rows ? pixel(q) : (q < kWinTok ? ((long)b * wg.nWin + win) * kWinTok + q : -1L);
  }
  attend_to_planes<X3, C>(kf, vf, qf4, p.table + ((size_t)type * HEADS + h) * 64 * 64, j16, g, orow, 32 * h,
                          p.att_hi, p.att_lo);
}

template <int C, int OCC, int WPB>
void launch_c(const SwinAttnParams& p, hipStream_t s) {
  const unsigned grid = (unsigned)(((long)p.B * p.wg.nWin + WPB - 1) / WPB);
  if (p.wqkv_lo)
    swin_attn_kernel<C, 3, OCC, WPB><<<grid, 2 * C * WPB, 0, s>>>(p);
  else
    swin_attn_kernel<C, 1, OCC, WPB><<<grid, 2 * C * WPB, 0, s>>>(p);
}
// windows per workgroup; at C = 192
// two windows need 3 waves per SIMD (12 waves per workgroup).  Measured per 512-image encode
// (two launches, profiles/r05/r06f/ops_*.log): C = 192 3.83-3.86 ms at two windows vs
// 4.77 at one (590 KB of W_qkv + W_proj per window, read once per window pair from L2 /
// L1); C = 96 6.86-6.90 ms at two vs 4.79 at one (147 KB per window; four 3-wave
// workgroups per CU overlap better than two 6-wave ones)
constexpr int kS1Wpb = 1, kS2Wpb = 2;

// waves per SIMD the register allocation targets: 3 at C = 96 (534 vs 651 us per s1
// block, 19 dwords spilled), 2 at C = 192 (509 vs 649 us: 94 spilled at 3).

}  // namespace

bool swin_attn_fused_supported(int C) { return C == 96 || C == 192; }
bool swin_attn_noproj_supported(int C) { return C == 384 || C == 768; }

void launch_swin_attn_fused(const SwinAttnParams& p, hipStream_t s) {
  if (p.B <= 0) return;
  if ((p.wqkv_lo == nullptr) != (p.wproj_lo == nullptr))
    throw std::runtime_error("swin_attn: lo planes for both or neither");
  if (!p.wqkv_fm || !p.wproj_fm || (p.wqkv_lo && (!p.wqkv_fm_lo || !p.wproj_fm_lo)))
    throw std::runtime_error("swin_attn: fragment-major weights (launch_frag_pack) missing");
  if (p.heads * 32 != p.C) throw std::runtime_error("swin_attn: head dim must be 32");
  switch (p.C) {
    case 96: launch_c<96, 3, kS1Wpb>(p, s); break;
    case 192: launch_c<192, kS2Wpb == 1 ? 2 : 3, kS2Wpb>(p, s); break;
    default: throw std::runtime_error("swin_attn: fused attention built for C = 96, 192");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_swin_attn_noproj(const SwinAttnParams& p, hipStream_t s) {
  if (p.B <= 0) return;
  if ((p.wqkv_lo == nullptr) != (p.att_lo == nullptr) || !p.att_hi)
    throw std::runtime_error("swin_attn_noproj: ATT planes must match the weight planes");
  if (p.heads * 32 != p.C) throw std::runtime_error("swin_attn: head dim must be 32");
  if (p.C != 384 && p.C != 768) throw std::runtime_error("swin_attn_noproj: built for C = 384, 768");
  if (!p.wqkv_fm || (p.wqkv_lo && !p.wqkv_fm_lo))
    throw std::runtime_error("swin_attn_noproj: fragment-major W_qkv (launch_frag_pack) missing");
  const unsigned grid = (unsigned)((long)p.B * p.wg.nWin);
  if (p.C == 768) {
    // two workgroups per window, 12 heads (waves) each
    if (p.wqkv_lo)
      swin_attn_noproj_ks_kernel<768, 3, 3, 12, 1><<<2 * grid, 768, 0, s>>>(p);
    else
      swin_attn_noproj_ks_kernel<768, 1, 3, 12, 1><<<2 * grid, 768, 0, s>>>(p);
    MOCR_HIP_CHECK(hipGetLastError());
    return;
  }
  // 12 waves (one head each, 3 per SIMD, 166 VGPRs) and k-steps unrolled by 2: 285 us per
  // s3 block at B=64, 384² vs 313 (8 waves over the 12 heads, 2 per SIMD), 302 (8 waves,
  // unroll 4), 318 (8 waves, no unroll)
  if (p.wqkv_lo)
    swin_attn_noproj_kernel<384, 3, 3, 12, 2><<<grid, 768, 0, s>>>(p);
  else
    swin_attn_noproj_kernel<384, 1, 3, 12, 2><<<grid, 768, 0, s>>>(p);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
