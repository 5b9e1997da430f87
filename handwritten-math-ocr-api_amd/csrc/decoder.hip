// Decoder step kernels: 8 post-norm nn.TransformerDecoderLayer (d=256, 8 heads, FFN 512,
// ReLU; torch/nn/modules/transformer.py:1143-1199) + fc_out + greedy argmax
// (src/model_swin.py:72-88, src/inference.py:18-25).
//
// The reference re-decodes the whole prefix every step (O(T^2)).  Here each step
// processes only the newest position: its K/V are appended to a per-layer cache and
// the cross-attention K/V of the encoder memory are precomputed once per image
// (gemm.hip).  With causal masking the newest position's output is the same
// function of the same inputs.
//
// Post-norm LayerNorms are never materialised: a sublayer writes its pre-norm sum
// y = x + f(x) plus, per row and 16-column slice, the slice's (mean, M2).  Every
// consumer of LN(y) (the next projection's A operand, the next residual) merges the
// 16 partials of a row in one fixed order (Chan et al.'s pairwise update) and
// normalises the values it reads, so all consumers see bit-identical LN(y) without a
// barrier or a re-read of the row.
//
// The step index t is a kernel argument (one captured hipGraph per chunk of 8 steps);
// no kernel reads device state before issuing its loads.  With the batch-global stop,
// the stop flag is read alongside the loads and checked before the first store.
#include "kernels.h"
#include "lanes.h"
#include "select.h"

namespace mocr {

namespace {

constexpr int kD = 256;  // d_model (engine config is checked to match)
constexpr float kAttnScale = 0.17677669529663687f;  // 1/sqrt(32)

__device__ __forceinline__ float ln_apply(float v, float mean, float rstd, float g, float b) {
  return fmaf((v - mean) * rstd, g, b);
}

// ------------------------------------------------------------------ row statistics
constexpr int kSlices = kD / 16;  // 16-column slices per row

// Pairwise merge of the (mean, M2) of two equal-size groups of n values each
// (Chan et al.): mean = ma + d/2, M2 = qa + qb + d^2 n/2.  The 16 slice partials of a
// row are merged as a fixed binary tree (n = 16, 32, 64, 128), lower group first, in
// every kernel, so all consumers of a LayerNorm compute bit-identical statistics.
__device__ __forceinline__ void merge_eq(float& m, float& q, float mb, float qb, float n) {
  const float delta = mb - m;
  q = q + qb + delta * delta * (n * 0.5f);
  m = m + delta * 0.5f;
}

// Cross-lane tree level: this lane's group and its partner's (lane ^ mask) are merged
// with the lower group first; both lanes get the same result.
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

// Layout 1 (A-operand prologue): the 4 lanes g = 0..3 of a row each load 4 slices
// (part[4g..4g+3]); levels 1-2 in-lane, levels 3-4 across lanes (lane ^ 16, ^ 32).
__device__ __forceinline__ void row_stats_4lanes(const float* __restrict__ part, int g, float& mean, float& rstd) {
  const floatx4 p0 = *reinterpret_cast<const floatx4*>(part + 8 * g);
  const floatx4 p1 = *reinterpret_cast<const floatx4*>(part + 8 * g + 4);
  float m = p0[0], q = p0[1], m2 = p1[0], q2 = p1[1];
  merge_eq(m, q, p0[2], p0[3], 16.f);
  merge_eq(m2, q2, p1[2], p1[3], 16.f);
  merge_eq(m, q, m2, q2, 32.f);
  merge_lanes<16>(m, q, (g & 1) != 0, 64.f);
  merge_lanes<32>(m, q, (g & 2) != 0, 128.f);
  mean = m;
  rstd = rstd_of(q);
}

// Layout 2 (epilogue): the 16 lanes c = 0..15 of a row each load slice c; levels 1-4
// across lanes (lane ^ 1, ^ 2, ^ 4, ^ 8).  Same tree as layout 1.
__device__ __forceinline__ void row_stats_16lanes(const float* __restrict__ part, int c, float& mean, float& rstd) {
  float m = part[2 * c], q = part[2 * c + 1];
  merge_lanes<1>(m, q, (c & 1) != 0, 16.f);
  merge_lanes<2>(m, q, (c & 2) != 0, 32.f);
  merge_lanes<4>(m, q, (c & 4) != 0, 64.f);
  merge_lanes<8>(m, q, (c & 8) != 0, 128.f);
  mean = m;
  rstd = rstd_of(q);
}

// ------------------------------------------------------------------ small-M GEMM
// out[B, N] = A[B, K] · W[N, K]^T + bias on v_mfma_f32_16x16x4_f32.  A workgroup
// owns a 16x16 output tile; its 4 waves split K and combine through LDS in a fixed
// order.  Each lane loads float4 runs of A and W straight into registers (no reuse
// inside the workgroup, so no LDS staging); lane group g = lane>>4 feeds
// k = 4g + s at MFMA step s.
template <int EPI, int KW, bool ALN, bool RLN>
__global__ void __launch_bounds__(256) rowgemm_kernel(RowGemmParams p) {
  const int t = p.t;
  constexpr int NI = KW / 16;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r0 = blockIdx.y * 16;
  const int c0 = blockIdx.x * 16;
  const int ra = r0 + (lane & 15);
  const int cb = c0 + (lane & 15);
  const int g = lane >> 4;
  const int kbeg = wave * KW;
  const bool row_ok = ra < p.B;
  const int rc = row_ok ? ra : p.B - 1;  // loads are never predicated (see dec_argmax_kernel)

  // issue every independent load first: the LayerNorm affine (one float4 of each per
  // thread, staged in LDS: 16 lanes share every value), A, W, residual
  __shared__ floatx4 gb_s[2][ALN ? kD / 4 : 1];
  floatx4 g4{}, b4{};
  if constexpr (ALN) {  // K == d == 256: 64 float4 of each
    const int k4 = (tid & 63) * 4;
    g4 = *reinterpret_cast<const floatx4*>(p.a_ln_g + k4);
    b4 = *reinterpret_cast<const floatx4*>(p.a_ln_b + k4);
  }
  floatx4 a[NI], b[NI];
  floatx4 gg[ALN ? NI : 1], bb[ALN ? NI : 1];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int k = kbeg + i * 16 + 4 * g;
    a[i] = *reinterpret_cast<const floatx4*>(p.A + (size_t)rc * p.K + k);
    if (!row_ok) a[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    b[i] = *reinterpret_cast<const floatx4*>(p.W + (size_t)cb * p.K + k);
  }
  if constexpr (ALN) {
    if (tid < 64) {
      gb_s[0][tid] = g4;
      gb_s[1][tid] = b4;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int k = kbeg + i * 16 + 4 * g;
      gg[i] = gb_s[0][k / 4];
      bb[i] = gb_s[1][k / 4];
    }
  }
  const int row = tid >> 4;
  const int col = tid & 15;
  const int grow = r0 + row;
  const int gcol = c0 + col;
  const bool out_ok = grow < p.B && gcol < p.n_valid;
  float rres = 0.f, rg = 0.f, rb = 0.f;
  if constexpr (EPI == DEC_RESADD) {  // N == n_valid == d: only the row can be out of range
    rres = p.resid[(size_t)min(grow, p.B - 1) * p.ldo + gcol];
    if constexpr (RLN) {
      rg = p.r_ln_g[gcol];
      rb = p.r_ln_b[gcol];
    }
  }
  if constexpr (ALN) {
    const size_t srow = (size_t)(row_ok ? ra : 0) * 2 * kSlices;
    float mean, rstd;
    row_stats_4lanes(p.a_stats + srow, g, mean, rstd);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) a[i][s] = row_ok ? ln_apply(a[i][s], mean, rstd, gg[i][s], bb[i][s]) : 0.f;
  }

  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[i][s], acc, 0, 0, 0);

  __shared__ float red[4][16][17];
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][g * 4 + r][lane & 15] = acc[r];
  __syncthreads();
  if constexpr (EPI == DEC_RESADD && RLN) {  // all 16 lanes of a row take part in the merge
    float mean, rstd;
    row_stats_16lanes(p.r_stats + (size_t)(grow < p.B ? grow : 0) * 2 * kSlices, col, mean, rstd);
    rres = ln_apply(rres, mean, rstd, rg, rb);
  }
  if constexpr (EPI == DEC_LOGITS) {
    if (grow >= p.B || dec_skip(p.st, t)) return;  // uniform per 16-lane row group
    const bool cv = gcol < p.n_valid;
    const float v = (((red[0][row][col] + red[1][row][col]) + red[2][row][col]) + red[3][row][col]) + p.bias[gcol];
    if (cv) p.out[(p.hist_stride ? (size_t)t * p.hist_stride : 0) + (size_t)grow * p.ldo + gcol] = v;
    if (p.part) {
      // the tile's (max, first argmax, sum exp(l - max)) over its 16 columns of the row
      // over the row's 16 lanes by DPP (quad_perm xor 1, xor 2, row_half_mirror,
      // row_mirror): the max with its first index is the same whichever lane pairs first
      float m = cv ? v : -INFINITY;
      int ix = gcol;
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
      const float e = row_sum<16>(cv ? expf(v - m) : 0.f);
      if (col == 0)
        reinterpret_cast<floatx4*>(p.part)[(size_t)grow * gridDim.x + blockIdx.x] = floatx4{m, __int_as_float(ix), e, 0.f};
    }
    return;
  }
  if (!out_ok || dec_skip(p.st, t)) return;  // uniform per 16-lane row group
  float v = ((red[0][row][col] + red[1][row][col]) + red[2][row][col]) + red[3][row][col];
  v += p.bias[gcol];
  if constexpr (EPI == DEC_STORE) {
    p.out[(size_t)grow * p.ldo + gcol] = v;
  } else if constexpr (EPI == DEC_RELU) {
    p.out[(size_t)grow * p.ldo + gcol] = fmaxf(v, 0.f);
  } else if constexpr (EPI == DEC_RESADD) {
    const float y = rres + v;
    p.out[(size_t)grow * p.ldo + gcol] = y;
    // (mean, M2) of this row's 16-column slice, reduced over the 16 lanes of the row (DPP)
    const float m16 = row_sum<16>(y) * (1.0f / 16);
    const float q = row_sum<16>(sq_rn(y - m16));
    if (col == 0) {
      float* so = p.out_stats + ((size_t)grow * kSlices + blockIdx.x) * 2;
      so[0] = m16;
      so[1] = q;
    }
  } else if constexpr (EPI == DEC_QKV) {
    if (gcol < p.d) {
      p.out[(size_t)grow * p.d + gcol] = v;
    } else if (gcol < 2 * p.d) {
      p.kcache[((size_t)grow * p.max_pos + t) * p.d + (gcol - p.d)] = v;
    } else {
      p.vcache[((size_t)grow * p.max_pos + t) * p.d + (gcol - 2 * p.d)] = v;
    }
  }
}

template <int EPI, bool ALN, bool RLN>
void launch_rowgemm_k(const RowGemmParams& p, dim3 grid, hipStream_t s) {
  if (p.K == 256) {
    rowgemm_kernel<EPI, 64, ALN, RLN><<<grid, 256, 0, s>>>(p);
  } else if (p.K == 512) {
    rowgemm_kernel<EPI, 128, ALN, RLN><<<grid, 256, 0, s>>>(p);
  } else {
    throw std::runtime_error("rowgemm: K must be 256 or 512");
  }
}

template <int EPI>
void launch_rowgemm_e(const RowGemmParams& p, dim3 grid, hipStream_t s) {
  const bool aln = p.a_ln_g != nullptr, rln = p.r_ln_g != nullptr;
  if (aln && rln) throw std::runtime_error("rowgemm: LayerNorm on both A and resid is not built");
  if (aln && (p.K != kD || !p.a_stats)) throw std::runtime_error("rowgemm: LayerNorm prologue needs K == d, stats");
  if (rln && !p.r_stats) throw std::runtime_error("rowgemm: residual LayerNorm needs stats");
  if (EPI == DEC_RESADD && (p.N != kD || !p.out_stats)) throw std::runtime_error("rowgemm: RESADD writes d + stats");
  if (aln) {
    launch_rowgemm_k<EPI, true, false>(p, grid, s);
  } else if (rln) {
    launch_rowgemm_k<EPI, false, true>(p, grid, s);
  } else {
    launch_rowgemm_k<EPI, false, false>(p, grid, s);
  }
}

// ------------------------------------------------------------------ embedding of step 0
// x[b] = embedding[feed[b][0]] + pos_encoder[0]   (src/model_swin.py:73-75).
__global__ void __launch_bounds__(256) dec_embed0_kernel(const int32_t* __restrict__ feed, int ld_ids,
                                                         const float* __restrict__ emb, const float* __restrict__ pos,
                                                         float* __restrict__ x, int d, const float* __restrict__ qtab,
                                                         const float* __restrict__ qpos, float* __restrict__ z) {
  const int b = blockIdx.x;
  const int tok = feed[(size_t)b * ld_ids];
  for (int c = threadIdx.x; c < d; c += blockDim.x) x[(size_t)b * d + c] = emb[(size_t)tok * d + c] + pos[c];
  if (qtab)
    for (int c = threadIdx.x; c < 3 * d; c += blockDim.x) z[(size_t)b * 3 * d + c] = qtab[(size_t)tok * 3 * d + c] + qpos[c];
}

// ------------------------------------------------------------------ attention
// Newest position of row b against n keys, HB heads per workgroup (4 waves).  A key
// row slice of HB*32 floats is read by 8*HB lanes (one float4 each); every K and V row
// load of a lane is issued up front.  Scores q·k·1/sqrt(32) are reduced over the 8
// lanes of a head.  Each wave runs a softmax over its own keys (local max, exp, sum,
// Σ e·v), and the 4 wave partials are merged after one barrier with the usual
// rescaling by exp(m_w - m); the result is Σ e v / Σ e, normalised at the end as in
// the CPU flash-attention SDPA kernel the reference's F.multi_head_attention_forward
// reaches.
// q row b at q + b*q_ld; K/V rows of row b start at row (kv_mod ? b % kv_mod : b) times
// kv_b_stride (kv_mod: the ResNet18-trans encoder, whose attention runs across the
// images of a position: rows b*M + w attend to rows b'*M + w).
template <int HB, int NIT>
__global__ void __launch_bounds__(256) dec_attn_kernel(const DecodeState* st, int t, const float* __restrict__ q,
                                                       const float* __restrict__ K, const float* __restrict__ V,
                                                       size_t kv_b_stride, int kv_row_stride, int n,
                                                       float* __restrict__ out, int d, int q_ld, int kv_mod) {
  constexpr int DIMS = 32 * HB;
  constexpr int LPR = DIMS / 4;  // lanes per key row
  constexpr int RPW = 64 / LPR;  // key rows per wave instruction
  __shared__ floatx4 po[4][LPR];
  __shared__ float pm[4][HB], ps[4][HB];

  const int b = blockIdx.x;
  const int hg = blockIdx.y;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int rsub = lane / LPR;
  const int li = lane % LPR;
  const int c4 = li * 4;
  const int hl = c4 / 32;

  const floatx4 q4 = *reinterpret_cast<const floatx4*>(q + (size_t)b * q_ld + hg * DIMS + c4);
  const size_t kvb = (size_t)(kv_mod ? b % kv_mod : b);
  const float* Kb = K + kvb * kv_b_stride + hg * DIMS + c4;
  const float* Vb = V + kvb * kv_b_stride + hg * DIMS + c4;
  const int m_first = wave * RPW + rsub;

  floatx4 kk[NIT], vv[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {  // unpredicated loads of a clamped key row, masked after
    const int m = m_first + it * 4 * RPW;
    const size_t ml = (size_t)(m < n ? m : 0);
    kk[it] = *reinterpret_cast<const floatx4*>(Kb + ml * kv_row_stride);
    vv[it] = *reinterpret_cast<const floatx4*>(Vb + ml * kv_row_stride);
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it)
    if (m_first + it * 4 * RPW >= n) {
      kk[it] = floatx4{0.f, 0.f, 0.f, 0.f};
      vv[it] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  float sc[NIT];
  float mx = -INFINITY;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float s = q4[0] * kk[it][0];
    s = fmaf(q4[1], kk[it][1], s);
    s = fmaf(q4[2], kk[it][2], s);
    s = fmaf(q4[3], kk[it][3], s);
    s = row_sum<8>(s);
    s *= kAttnScale;
    sc[it] = (m_first + it * 4 * RPW < n) ? s : -INFINITY;
    mx = fmaxf(mx, sc[it]);
  }
  static_assert(LPR == 8, "DPP reductions assume 8 lanes per key row");
  mx = xmax8_16_32(mx);
  float sum = 0.f;
  floatx4 o4 = {0.f, 0.f, 0.f, 0.f};
  if (mx != -INFINITY) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const float e = expf(sc[it] - mx);
      sum += e;
      o4[0] = fmaf(e, vv[it][0], o4[0]);
      o4[1] = fmaf(e, vv[it][1], o4[1]);
      o4[2] = fmaf(e, vv[it][2], o4[2]);
      o4[3] = fmaf(e, vv[it][3], o4[3]);
    }
  }
  sum = xsum8_16_32(sum);
#pragma unroll
  for (int e = 0; e < 4; ++e) o4[e] = xsum8_16_32(o4[e]);
  if (rsub == 0) {
    po[wave][li] = o4;
    if ((li & 7) == 0) {
      pm[wave][hl] = mx;
      ps[wave][hl] = sum;
    }
  }
  __syncthreads();
  if (tid < DIMS && !dec_skip(st, t)) {
    const int h = tid / 32;
    float m = pm[0][h];
#pragma unroll
    for (int w = 1; w < 4; ++w) m = fmaxf(m, pm[w][h]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = pm[w][h] == -INFINITY ? 0.f : expf(pm[w][h] - m);
      num = fmaf(po[w][tid / 4][tid % 4], f, num);
      den = fmaf(ps[w][h], f, den);
    }
    out[(size_t)b * d + hg * DIMS + tid] = num / den;
  }
}

// ------------------------------------------------------------------ projection + attention
// One workgroup per (row b, head h) does the head's q projection (self-attention: q, k
// and v) from the LayerNorm'd input row and then attends, so the projection needs no
// kernel of its own.  The cached K/V loads are issued first (they do not depend on this
// step); the input row is normalised once per workgroup into LDS (one element per
// thread, statistics merged by row_stats_16lanes: bit-identical to every other
// consumer of that LayerNorm); thread (o = tid/8, kc = tid%8) dots output o's weight
// row with k = 32kc..32kc+31, reduced over the 8 lanes in a fixed order.  The new
// position's k/v (self-attention) enter the score loop from LDS and are appended to the
// cache at t.  Attention: 8 lanes per key row, online softmax per wave, one barrier,
// wave partials merged as in dec_attn_kernel.
template <bool SELF, int NIT>
__global__ void __launch_bounds__(256, 3) dec_projattn_kernel(ProjAttnParams p) {
  constexpr int LPR = 8;  // lanes per key row (32 dims, float4 each)
  constexpr int RPW = 8;  // key rows per wave instruction
  constexpr int NP = SELF ? 3 : 1;
  constexpr int CH = NIT < 4 ? NIT : 4;  // key groups (of 32) held in registers at a time
  constexpr int NCH = (NIT + CH - 1) / CH;
  __shared__ float xs[kD];
  __shared__ float proj[NP][32];
  __shared__ floatx4 po[4][LPR];
  __shared__ float pm[4], ps[4];

  const int b = blockIdx.x;
  const int h = blockIdx.y;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int rsub = lane / LPR;
  const int li = lane % LPR;
  const int c4 = li * 4;
  const int t = p.t;
  const int n = p.n_cached + (SELF ? 1 : 0);
  const int m_first = wave * RPW + rsub;

  // key m of this row lives in K/V row slot_rows[b][m] (beam search: the hypothesis'
  // ancestor that computed position m), else row b / mem_div (beams share their image's
  // memory; 1 for greedy)
  const float* Kh = p.K + h * 32 + c4;
  const float* Vh = p.V + h * 32 + c4;
  const int32_t* slots = p.slot_rows ? p.slot_rows + (size_t)b * p.slot_ld : nullptr;
  const size_t fixed_row = (size_t)(b / p.mem_div);
  floatx4 kk[CH], vv[CH];
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int it = c * CH + j;
      const int m = m_first + it * 4 * RPW;
      if (it < NIT && m < p.n_cached) {
        // the slot tables of steps after a beam-search batch stop are not maintained (the
        // selection skips), but this step's loads are issued before the skip is read:
        // clamp the slot to a valid row so a stale entry cannot address past the cache
        const int sl = slots ? slots[m] : 0;
        const size_t r = slots ? (size_t)((unsigned)sl < (unsigned)p.B ? sl : 0) : fixed_row;
        kk[j] = *reinterpret_cast<const floatx4*>(Kh + r * p.kv_b_stride + (size_t)m * p.kv_row_stride);
        vv[j] = *reinterpret_cast<const floatx4*>(Vh + r * p.kv_b_stride + (size_t)m * p.kv_row_stride);
      } else {
        kk[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        vv[j] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  load_chunk(0);
  // weight rows of this head's projections (independent of the input row)
  const int o = tid >> 3;
  const int kc = tid & 7;
  floatx4 w[NP][8];
#pragma unroll
  for (int pj = 0; pj < NP; ++pj) {
    const float* wr = p.W + (size_t)(pj * kD + h * 32 + o) * kD + 32 * kc;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[pj][i] = *reinterpret_cast<const floatx4*>(wr + 4 * i);
  }
  float xv = p.A[(size_t)b * kD + tid];
  if (p.a_stats) {
    const float g = p.a_ln_g[tid], be = p.a_ln_b[tid];
    float mean, rstd;
    row_stats_16lanes(p.a_stats + (size_t)b * 2 * kSlices, lane & 15, mean, rstd);
    xv = ln_apply(xv, mean, rstd, g, be);
  }
  xs[tid] = xv;
  __syncthreads();
  float acc[NP];
#pragma unroll
  for (int pj = 0; pj < NP; ++pj) acc[pj] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const floatx4 x4 = *reinterpret_cast<const floatx4*>(&xs[32 * kc + 4 * i]);
#pragma unroll
    for (int pj = 0; pj < NP; ++pj)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[pj] = fmaf(x4[e], w[pj][i][e], acc[pj]);
  }
#pragma unroll
  for (int pj = 0; pj < NP; ++pj) {
    float a = acc[pj];
    a = row_sum<8>(a);
    if (kc == 0) proj[pj][o] = a + p.bias[pj * kD + h * 32 + o];
  }
  __syncthreads();
  const floatx4 q4 = *reinterpret_cast<const floatx4*>(&proj[0][c4]);
  floatx4 kn{}, vn{};
  if constexpr (SELF) {
    kn = *reinterpret_cast<const floatx4*>(&proj[1][c4]);
    vn = *reinterpret_cast<const floatx4*>(&proj[2][c4]);
    if (tid < 64 && !dec_skip(p.st, t)) {
      float* dst = (tid < 32 ? p.kcache : p.vcache) + ((size_t)b * p.max_pos + t) * kD + h * 32 + (tid & 31);
      *dst = proj[1 + (tid >> 5)][tid & 31];
    }
  }

  // online softmax over chunks of CH key groups with a wave-uniform running max (one
  // chunk: exactly the single-pass max / exp / sum)
  float mrun = -INFINITY, sum = 0.f;
  floatx4 o4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (c > 0) load_chunk(c);
    if constexpr (SELF) {
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (m_first + (c * CH + j) * 4 * RPW == t) {
          kk[j] = kn;
          vv[j] = vn;
        }
    }
    float sc[CH];
    float mc = -INFINITY;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      float sv = q4[0] * kk[j][0];
      sv = fmaf(q4[1], kk[j][1], sv);
      sv = fmaf(q4[2], kk[j][2], sv);
      sv = fmaf(q4[3], kk[j][3], sv);
      sv = row_sum<8>(sv);
      sv *= kAttnScale;
      const int it = c * CH + j;
      sc[j] = (it < NIT && m_first + it * 4 * RPW < n) ? sv : -INFINITY;
      mc = fmaxf(mc, sc[j]);
    }
    static_assert(LPR == 8, "DPP reductions assume 8 lanes per key row");
    mc = xmax8_16_32(mc);
    const float mnew = fmaxf(mrun, mc);
    if (mnew != -INFINITY) {
      const float scale = expf(mrun - mnew);
      sum *= scale;
      o4[0] *= scale;
      o4[1] *= scale;
      o4[2] *= scale;
      o4[3] *= scale;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const float e = expf(sc[j] - mnew);
        sum += e;
        o4[0] = fmaf(e, vv[j][0], o4[0]);
        o4[1] = fmaf(e, vv[j][1], o4[1]);
        o4[2] = fmaf(e, vv[j][2], o4[2]);
        o4[3] = fmaf(e, vv[j][3], o4[3]);
      }
      mrun = mnew;
    }
  }
  sum = xsum8_16_32(sum);
#pragma unroll
  for (int e = 0; e < 4; ++e) o4[e] = xsum8_16_32(o4[e]);
  if (rsub == 0) {
    po[wave][li] = o4;
    if (li == 0) {
      pm[wave] = mrun;
      ps[wave] = sum;
    }
  }
  __syncthreads();
  if (tid < 32 && !dec_skip(p.st, t)) {
    float m = pm[0];
#pragma unroll
    for (int wv = 1; wv < 4; ++wv) m = fmaxf(m, pm[wv]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv) {
      const float f = pm[wv] == -INFINITY ? 0.f : expf(pm[wv] - m);
      num = fmaf(po[wv][tid / 4][tid % 4], f, num);
      den = fmaf(ps[wv], f, den);
    }
    p.out[(size_t)b * kD + h * 32 + tid] = num / den;
  }
}

// ------------------------------------------------------------------ beam search
// Semantics: oracle/model_ref.py beam_search (the reference has none).
// Row r = b*K + k is hypothesis k of image b, kept in rank order.
__global__ void __launch_bounds__(256) beam_init_kernel(BeamParams p) {
  const int r = blockIdx.x;
  for (int c = threadIdx.x; c < p.d; c += blockDim.x)
    p.x[(size_t)r * p.d + c] = p.emb[(size_t)p.sos * p.d + c] + p.pos[c];
  if (p.qtab)  // folded step: layer 0's q|k|v of sos at position 0
    for (int c = threadIdx.x; c < 3 * p.d; c += blockDim.x)
      p.z[(size_t)r * 3 * p.d + c] = p.qtab[(size_t)p.sos * 3 * p.d + c] + p.qpos[c];
  if (threadIdx.x == 0) {
    p.score[r] = (r % p.K == 0) ? 0.f : -INFINITY;
    p.fin[r] = 0;
    p.seq_new[(size_t)r * p.ld] = p.sos;  // buffer of parity 0
  }
}

// (score, flat index) total order of the candidates: higher score, then lower index
__device__ __forceinline__ bool cand_before(float s1, int f1, float s2, int f2) {
  return s1 > s2 || (s1 == s2 && f1 < f2);
}

// sorted top-K lists with compile-time indices only (runtime-indexed arrays go to scratch)
template <int K>
__device__ __forceinline__ void topk_insert(float (&s)[K], int (&f)[K], float sv, int fv) {
  if (!cand_before(sv, fv, s[K - 1], f[K - 1])) return;
  s[K - 1] = sv;
  f[K - 1] = fv;
#pragma unroll
  for (int j = K - 1; j > 0; --j) {
    if (cand_before(s[j], f[j], s[j - 1], f[j - 1])) {
      const float ts = s[j];
      s[j] = s[j - 1];
      s[j - 1] = ts;
      const int tf = f[j];
      f[j] = f[j - 1];
      f[j - 1] = tf;
    }
  }
}

template <int K>
__device__ __forceinline__ void topk_merge(float (&s)[K], int (&f)[K], const float (&so)[K], const int (&fo)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) topk_insert<K>(s, f, so[k], fo[k]);
}

// One workgroup per image: log_softmax of the K beam rows (max, log Σ exp(l - max), as
// torch.log_softmax), the K best of the K*V candidates, then the new beam: scores,
// finished flags, token sequences and slot tables (double-buffered by step parity), and
// the embedding of each new hypothesis' last token at position t+1.
template <int K>
__global__ void __launch_bounds__(256) beam_select_kernel(BeamParams p) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int t = p.t;
  const int V = p.V;
  __shared__ float s_max[K], s_lse[K];
  __shared__ float ms[4][K];
  __shared__ int mf[4][K];
  __shared__ int s_par[K], s_tok[K];
  __shared__ float s_sc[K];
  __shared__ int s_fin[K];

  // 1. per-beam max and log Σ exp(l - max)
  for (int k = wave; k < K; k += 4) {
    const float* L = p.logits + (size_t)(b * K + k) * p.ldl;
    float m = -INFINITY, sm = 0.f;
    for (int v = lane; v < V; v += 64) {
      const float x = L[v];
      if (x > m) {
        sm = sm * expf(m - x) + 1.f;
        m = x;
      } else {
        sm += expf(x - m);
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float mo = __shfl_xor(m, off, 64);
      const float so = __shfl_xor(sm, off, 64);
      const float mm = fmaxf(m, mo);
      sm = (m == -INFINITY ? 0.f : sm * expf(m - mm)) + (mo == -INFINITY ? 0.f : so * expf(mo - mm));
      m = mm;
    }
    if (lane == 0) {
      s_max[k] = m;
      s_lse[k] = logf(sm);
    }
  }
  __syncthreads();
  // 2. candidates: live beam k offers score_k + logp_k[v]; a finished one, itself at k*V
  float ts[K];
  int tf[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    ts[k] = -INFINITY;
    tf[k] = 0x7fffffff;
  }
  for (int k = 0; k < K; ++k) {
    const int r = b * K + k;
    const float sc = p.score[r];
    const float* L = p.logits + (size_t)r * p.ldl;
    if (p.fin[r]) {
      if (tid == 0) topk_insert<K>(ts, tf, sc, k * V);
    } else {
      const float mk = s_max[k], lk = s_lse[k];
      for (int v = tid; v < V; v += 256) topk_insert<K>(ts, tf, sc + ((L[v] - mk) - lk), k * V + v);
    }
  }
  // 3. merge: 64 lanes by shuffles, then the 4 waves
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    float so[K];
    int fo[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      so[k] = __shfl_xor(ts[k], off, 64);
      fo[k] = __shfl_xor(tf[k], off, 64);
    }
    topk_merge<K>(ts, tf, so, fo);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      ms[wave][k] = ts[k];
      mf[wave][k] = tf[k];
    }
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) {
      float so[K];
      int fo[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        so[k] = ms[w][k];
        fo[k] = mf[w][k];
      }
      topk_merge<K>(ts, tf, so, fo);
    }
    int all_fin = 1;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (!(tf[k] >= 0 && tf[k] < K * V)) {  // no finite candidate (NaN logits): see dec_argmax_kernel
        atomicAdd(&p.st->bad_rows, 1);
        tf[k] = k * V;
      }
      const int parent = tf[k] / V;
      const int pr = b * K + parent;
      const int pfin = p.fin[pr];
      const int tok = pfin ? p.pad : tf[k] - parent * V;
      s_par[k] = pr;
      s_tok[k] = tok;
      s_sc[k] = ts[k];
      s_fin[k] = pfin || tok == p.eos;
      all_fin &= s_fin[k];
    }
    if (all_fin && p.stop_batch && !dec_skip(p.st, t)) {
      const int before = atomicAdd(&p.st->nfinished, 1);
      if (before == p.B - 1) p.st->done_step = t;
    }
  }
  __syncthreads();
  if (dec_skip(p.stop_batch ? p.st : nullptr, t)) return;
  // 4. the new beam (every read of the old beam of this image happened before the barrier)
  if (tid < K) {
    p.score[b * K + tid] = s_sc[tid];
    p.fin[b * K + tid] = s_fin[tid];
  }
  for (int i = tid; i < K * (t + 2); i += 256) {
    const int k = i / (t + 2), j = i - k * (t + 2);
    const size_t dst = (size_t)(b * K + k) * p.ld + j;
    p.seq_new[dst] = j <= t ? p.seq_old[(size_t)s_par[k] * p.ld + j] : s_tok[k];
    if (j < t) p.slot_new[dst] = p.slot_old[(size_t)s_par[k] * p.ld + j];
    else if (j == t) p.slot_new[dst] = s_par[k];
  }
  if (!p.last_step) {
    for (int i = tid; i < K * p.d; i += 256) {
      const int k = i / p.d, c = i - k * p.d;
      p.x[(size_t)(b * K + k) * p.d + c] = p.emb[(size_t)s_tok[k] * p.d + c] + p.pos[(size_t)(t + 1) * p.d + c];
    }
    if (p.qtab)
      for (int i = tid; i < K * 3 * p.d; i += 256) {
        const int k = i / (3 * p.d), c = i - k * 3 * p.d;
        p.z[(size_t)(b * K + k) * 3 * p.d + c] =
            p.qtab[(size_t)s_tok[k] * 3 * p.d + c] + p.qpos[(size_t)(t + 1) * 3 * p.d + c];
      }
  }
}

// ------------------------------------------------------------------ LayerNorm rows
// out[r] = LN(y[r]) from the producer's slice statistics (row_stats_16lanes, the same
// values every fused consumer computes): the ResNet18-trans encoder memory.
__global__ void __launch_bounds__(256) ln_rows_kernel(const float* __restrict__ y, const float* __restrict__ stats,
                                                      const float* __restrict__ g, const float* __restrict__ b,
                                                      float* __restrict__ out) {
  const int r = blockIdx.x;
  const int c = threadIdx.x;
  float mean, rstd;
  row_stats_16lanes(stats + (size_t)r * 2 * kSlices, c & 15, mean, rstd);
  out[(size_t)r * kD + c] = ln_apply(y[(size_t)r * kD + c], mean, rstd, g[c], b[c]);
}

// ------------------------------------------------------------------ greedy select
// select.h greedy_select for step t (one workgroup per row), then the embedding of the
// token fed to step t+1 (and, folded step, layer 0's q|k|v of it).  The folded step runs
// the selection of steps 0 .. n-2 inside the next step's layer-0 self-attention
// (decfold.hip), so this kernel only ends the last step there.
__global__ void __launch_bounds__(256) dec_argmax_kernel(SelectArgs a, int last_step, const float* __restrict__ emb,
                                                         const float* __restrict__ pos, float* __restrict__ x,
                                                         int d, const float* __restrict__ qtab,
                                                         const float* __restrict__ qpos, float* __restrict__ z) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int t = a.t;
  const int tok = greedy_select(a, b, true);
  if (tok < 0 || last_step) return;
  for (int c = tid; c < d; c += 256) x[(size_t)b * d + c] = emb[(size_t)tok * d + c] + pos[(size_t)(t + 1) * d + c];
  if (qtab)  // folded step: layer 0's q|k|v of the fed token at position t+1
    for (int c = tid; c < 3 * d; c += 256)
      z[(size_t)b * 3 * d + c] = qtab[(size_t)tok * 3 * d + c] + qpos[(size_t)(t + 1) * 3 * d + c];
}

}  // namespace

void launch_rowgemm(const RowGemmParams& p, hipStream_t s) {
  if (p.N % 16 != 0) throw std::runtime_error("rowgemm: N must be padded to 16");
  if (p.d != kD) throw std::runtime_error("rowgemm: d_model must be 256");
  dim3 grid(p.N / 16, (p.B + 15) / 16);
  switch (p.epi) {
    case DEC_STORE: launch_rowgemm_e<DEC_STORE>(p, grid, s); break;
    case DEC_RELU: launch_rowgemm_e<DEC_RELU>(p, grid, s); break;
    case DEC_RESADD: launch_rowgemm_e<DEC_RESADD>(p, grid, s); break;
    case DEC_QKV: launch_rowgemm_e<DEC_QKV>(p, grid, s); break;
    case DEC_LOGITS: launch_rowgemm_e<DEC_LOGITS>(p, grid, s); break;
    default: throw std::runtime_error("rowgemm: bad epilogue");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_embed0(const int32_t* feed, int ld_ids, const float* emb, const float* pos, float* x, int B, int d,
                       hipStream_t s, const float* qtab, const float* qpos, float* z) {
  dec_embed0_kernel<<<B, 256, 0, s>>>(feed, ld_ids, emb, pos, x, d, qtab, qpos, z);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_attn(const DecodeState* st, int t, const float* q, const float* K, const float* V,
                     size_t kv_b_stride, int kv_row_stride, int n_fixed, int n_max, float* out, int B, int d,
                     int heads, hipStream_t s, int q_ld, int kv_mod) {
  constexpr int HB = 1;
  if (d != kD || heads * 32 != d) throw std::runtime_error("dec_attn: d_model 256 with 8 heads of 32");
  if (n_max > 256 || n_fixed < 1) throw std::runtime_error("dec_attn: 1..256 keys");
  const int nit = (n_max + 31) / 32;  // 32 key rows per workgroup pass (4 waves x 8 rows)
  const dim3 grid(B, heads / HB);
#define MOCR_ATTN(N) \
  dec_attn_kernel<HB, N><<<grid, 256, 0, s>>>(st, t, q, K, V, kv_b_stride, kv_row_stride, n_fixed, out, d, \
                                               q_ld ? q_ld : d, kv_mod)
  switch (nit) {
    case 1: MOCR_ATTN(1); break;
    case 2: MOCR_ATTN(2); break;
    case 3: MOCR_ATTN(3); break;
    case 4: MOCR_ATTN(4); break;
    case 5: MOCR_ATTN(5); break;
    case 6: MOCR_ATTN(6); break;
    case 7: MOCR_ATTN(7); break;
    default: MOCR_ATTN(8); break;
  }
#undef MOCR_ATTN
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_argmax(const SelectArgs& a, int last_step, int B, const float* emb, const float* pos, float* x, int d,
                       hipStream_t s, const float* qtab, const float* qpos, float* z) {
  if (a.part && a.nparts > 512) throw std::runtime_error("argmax: at most 8192 logits with tile partials");
  dec_argmax_kernel<<<B, 256, 0, s>>>(a, last_step, emb, pos, x, d, qtab, qpos, z);
  MOCR_HIP_CHECK(hipGetLastError());
}


void launch_dec_projattn(const ProjAttnParams& p, bool self_attn, int n_max, hipStream_t s) {
  if (p.d != kD || p.heads * 32 != kD) throw std::runtime_error("projattn: d_model 256, 8 heads of 32");
  const int nit = (n_max + 31) / 32;
  const dim3 grid(p.B, p.heads);
#define MOCR_PA(N)                                                                        \
  case N:                                                                                 \
    if (self_attn)                                                                        \
      dec_projattn_kernel<true, N><<<grid, 256, 0, s>>>(p);                               \
    else                                                                                  \
      dec_projattn_kernel<false, N><<<grid, 256, 0, s>>>(p);                              \
    break;
  if (p.mem_div < 1) throw std::runtime_error("projattn: mem_div must be >= 1");
  switch (nit) {
    MOCR_PA(1) MOCR_PA(2) MOCR_PA(3) MOCR_PA(4) MOCR_PA(5) MOCR_PA(6) MOCR_PA(7) MOCR_PA(8) MOCR_PA(9)
    default: throw std::runtime_error("projattn: at most 288 keys");
  }
#undef MOCR_PA
  MOCR_HIP_CHECK(hipGetLastError());
}


void launch_beam_init(const BeamParams& p, hipStream_t s) {
  beam_init_kernel<<<p.B * p.K, 256, 0, s>>>(p);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_beam_select(const BeamParams& p, hipStream_t s) {
  switch (p.K) {
    case 1: beam_select_kernel<1><<<p.B, 256, 0, s>>>(p); break;
    case 2: beam_select_kernel<2><<<p.B, 256, 0, s>>>(p); break;
    case 3: beam_select_kernel<3><<<p.B, 256, 0, s>>>(p); break;
    case 4: beam_select_kernel<4><<<p.B, 256, 0, s>>>(p); break;
    case 5: beam_select_kernel<5><<<p.B, 256, 0, s>>>(p); break;
    case 6: beam_select_kernel<6><<<p.B, 256, 0, s>>>(p); break;
    case 7: beam_select_kernel<7><<<p.B, 256, 0, s>>>(p); break;
    case 8: beam_select_kernel<8><<<p.B, 256, 0, s>>>(p); break;
    default: throw std::runtime_error("beam: 1..8 hypotheses per image");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_ln_rows(const float* y, const float* stats, const float* g, const float* b, float* out, int rows,
                    hipStream_t s) {
  if (rows <= 0) return;
  ln_rows_kernel<<<rows, kD, 0, s>>>(y, stats, g, b, out);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
