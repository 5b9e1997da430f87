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
// y = x + f(x), and every consumer of LN(y) (the next projection's A operand, the
// next residual) normalises the rows it reads, from row statistics it computes itself
// with one fixed reduction order, so all consumers see bit-identical LN(y).
//
// The step index t is a kernel argument (one captured hipGraph per chunk of 8 steps);
// no kernel reads device state before issuing its loads.  With the batch-global stop,
// the stop flag is read alongside the loads and checked before the first store.
#include "kernels.h"

namespace mocr {

namespace {

constexpr int kD = 256;  // d_model (engine config is checked to match)
constexpr float kAttnScale = 0.17677669529663687f;  // 1/sqrt(32)

__device__ __forceinline__ float ln_apply(float v, float mean, float rstd, float g, float b) {
  return fmaf((v - mean) * rstd, g, b);
}

// ------------------------------------------------------------------ small-M GEMM
// out[B, N] = A[B, K] · W[N, K]^T + bias on v_mfma_f32_16x16x4_f32.  A workgroup
// owns a 16x16 output tile; its 4 waves split K and combine through LDS in a fixed
// order.  Each lane loads float4 runs of A and W straight into registers (no reuse
// inside the workgroup, so no LDS staging); lane group g = lane>>4 feeds
// k = 4g + s at MFMA step s.
//
// LN(A) / LN(resid) are fused: the 16 rows' statistics are reduced from fragments
// that are already in registers (A's own fragments, or the resid rows loaded in the
// same layout), two-pass mean / variance with a fixed order, so every consumer of a
// LayerNorm gets bit-identical values.
template <int NI>
__device__ __forceinline__ void frag_ln_stats(const floatx4 (&f)[NI], float (*red)[16], int lane, int wave,
                                              float& mean, float& rstd) {
  const int row = lane & 15;
  float ps = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int s = 0; s < 4; ++s) ps += f[i][s];
  ps += __shfl_xor(ps, 16, 64);
  ps += __shfl_xor(ps, 32, 64);
  if (lane < 16) red[wave][row] = ps;
  __syncthreads();
  mean = (((red[0][row] + red[1][row]) + red[2][row]) + red[3][row]) * (1.0f / kD);
  __syncthreads();
  float pq = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float t = f[i][s] - mean;
      pq += t * t;
    }
  pq += __shfl_xor(pq, 16, 64);
  pq += __shfl_xor(pq, 32, 64);
  if (lane < 16) red[wave][row] = pq;
  __syncthreads();
  const float var = (((red[0][row] + red[1][row]) + red[2][row]) + red[3][row]) * (1.0f / kD);
  rstd = 1.0f / sqrtf(var + 1e-5f);
}

template <int EPI, int KW, bool ALN, bool RLN>
__global__ void __launch_bounds__(256) rowgemm_kernel(RowGemmParams p) {
  const int t = p.t;
  constexpr int NI = KW / 16;
  constexpr int NR = kD / 4 / 16;  // resid fragments per lane (d split over 4 waves)
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

  floatx4 a[NI], b[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int k = kbeg + i * 16 + 4 * g;
    a[i] = row_ok ? *reinterpret_cast<const floatx4*>(p.A + (size_t)ra * p.K + k) : floatx4{0.f, 0.f, 0.f, 0.f};
    b[i] = *reinterpret_cast<const floatx4*>(p.W + (size_t)cb * p.K + k);
  }
  floatx4 rf[RLN ? NR : 1];
  if constexpr (RLN) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int k = wave * (kD / 4) + i * 16 + 4 * g;
      rf[i] = row_ok ? *reinterpret_cast<const floatx4*>(p.resid + (size_t)ra * p.ldo + k)
                     : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }

  __shared__ float red_s[4][16];
  __shared__ float rn[16][kD + 1];
  if constexpr (ALN) {
    float mean, rstd;
    frag_ln_stats<NI>(a, red_s, lane, wave, mean, rstd);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int k = kbeg + i * 16 + 4 * g;
      const floatx4 gg = *reinterpret_cast<const floatx4*>(p.a_ln_g + k);
      const floatx4 bb = *reinterpret_cast<const floatx4*>(p.a_ln_b + k);
#pragma unroll
      for (int s = 0; s < 4; ++s) a[i][s] = row_ok ? ln_apply(a[i][s], mean, rstd, gg[s], bb[s]) : 0.f;
    }
  }
  if constexpr (RLN) {
    float mean, rstd;
    frag_ln_stats<NR>(rf, red_s, lane, wave, mean, rstd);
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int k = wave * (kD / 4) + i * 16 + 4 * g;
#pragma unroll
      for (int s = 0; s < 4; ++s) rn[lane & 15][k + s] = ln_apply(rf[i][s], mean, rstd, p.r_ln_g[k + s], p.r_ln_b[k + s]);
    }
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
  const int row = tid >> 4;
  const int col = tid & 15;
  const int grow = r0 + row;
  const int gcol = c0 + col;
  if (grow >= p.B || gcol >= p.n_valid || dec_skip(p.st, t)) return;
  float v = ((red[0][row][col] + red[1][row][col]) + red[2][row][col]) + red[3][row][col];
  v += p.bias[gcol];
  if constexpr (EPI == DEC_STORE) {
    p.out[(size_t)grow * p.ldo + gcol] = v;
  } else if constexpr (EPI == DEC_RELU) {
    p.out[(size_t)grow * p.ldo + gcol] = fmaxf(v, 0.f);
  } else if constexpr (EPI == DEC_RESADD) {
    const float r = RLN ? rn[row][gcol] : p.resid[(size_t)grow * p.ldo + gcol];
    p.out[(size_t)grow * p.ldo + gcol] = r + v;
  } else if constexpr (EPI == DEC_QKV) {
    if (gcol < p.d) {
      p.out[(size_t)grow * p.d + gcol] = v;
    } else if (gcol < 2 * p.d) {
      p.kcache[((size_t)grow * p.max_pos + t) * p.d + (gcol - p.d)] = v;
    } else {
      p.vcache[((size_t)grow * p.max_pos + t) * p.d + (gcol - 2 * p.d)] = v;
    }
  } else {  // DEC_LOGITS
    float* slot = p.out + (p.hist_stride ? (size_t)t * p.hist_stride : 0);
    slot[(size_t)grow * p.ldo + gcol] = v;
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
  if (aln && p.K != kD) throw std::runtime_error("rowgemm: LayerNorm prologue needs K == d_model");
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
                                                         float* __restrict__ x, int d) {
  const int b = blockIdx.x;
  const int tok = feed[(size_t)b * ld_ids];
  for (int c = threadIdx.x; c < d; c += blockDim.x) x[(size_t)b * d + c] = emb[(size_t)tok * d + c] + pos[c];
}

// ------------------------------------------------------------------ attention
// Newest position of row b against n keys, HB heads per workgroup (4 waves).  A key
// row slice of HB*32 floats is read by 8*HB lanes (one float4 each), so one wave
// instruction covers 64/(8*HB) keys with full 128-B head rows; scores q·k·1/sqrt(32)
// are reduced over the 8 lanes of a head.  Softmax is exp(s - max) with the sum
// applied at the end (Σ e v / Σ e), as in the CPU flash-attention SDPA kernel the
// reference's F.multi_head_attention_forward reaches.
template <int HB, int NIT>
__global__ void __launch_bounds__(256) dec_attn_kernel(const DecodeState* st, int t, const float* __restrict__ q,
                                                       const float* __restrict__ K, const float* __restrict__ V,
                                                       size_t kv_b_stride, int kv_row_stride, int n_fixed,
                                                       float* __restrict__ out, int d) {
  constexpr int DIMS = 32 * HB;
  constexpr int LPR = DIMS / 4;  // lanes per key row
  constexpr int RPW = 64 / LPR;  // key rows per wave instruction
  constexpr int MAXN = NIT * 4 * RPW;  // key rows per lane: NIT (upper bound)
  __shared__ float S[HB][MAXN];
  __shared__ float ssum[HB];
  __shared__ floatx4 red[4][RPW][LPR];

  const int n = n_fixed ? n_fixed : t + 1;
  const int b = blockIdx.x;
  const int hg = blockIdx.y;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int rsub = lane / LPR;
  const int li = lane % LPR;
  const int c4 = li * 4;
  const int hl = c4 / 32;

  const floatx4 q4 = *reinterpret_cast<const floatx4*>(q + (size_t)b * d + hg * DIMS + c4);
  const float* Kb = K + (size_t)b * kv_b_stride + hg * DIMS + c4;
  const float* Vb = V + (size_t)b * kv_b_stride + hg * DIMS + c4;
  const int m_first = wave * RPW + rsub;
  const int niter = (n + 4 * RPW - 1) / (4 * RPW);

  // issue every K and V row load of this lane before using any of them
  floatx4 kk[NIT], vv[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int m = m_first + it * 4 * RPW;
    if (it < niter && m < n) {
      kk[it] = *reinterpret_cast<const floatx4*>(Kb + (size_t)m * kv_row_stride);
      vv[it] = *reinterpret_cast<const floatx4*>(Vb + (size_t)m * kv_row_stride);
    } else {
      kk[it] = floatx4{0.f, 0.f, 0.f, 0.f};
      vv[it] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int m = m_first + it * 4 * RPW;
    float s = q4[0] * kk[it][0];
    s = fmaf(q4[1], kk[it][1], s);
    s = fmaf(q4[2], kk[it][2], s);
    s = fmaf(q4[3], kk[it][3], s);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if ((li & 7) == 0 && it < niter && m < n) S[hl][m] = s * kAttnScale;
  }
  __syncthreads();

  for (int h = wave; h < HB; h += 4) {
    float mx = -INFINITY;
    for (int j = lane; j < n; j += 64) mx = fmaxf(mx, S[h][j]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int j = lane; j < n; j += 64) {
      const float e = expf(S[h][j] - mx);
      S[h][j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    if (lane == 0) ssum[h] = sum;
  }
  __syncthreads();

  floatx4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int m = m_first + it * 4 * RPW;
    if (it < niter && m < n) {
      const float pm = S[hl][m];
      o[0] = fmaf(pm, vv[it][0], o[0]);
      o[1] = fmaf(pm, vv[it][1], o[1]);
      o[2] = fmaf(pm, vv[it][2], o[2]);
      o[3] = fmaf(pm, vv[it][3], o[3]);
    }
  }
  red[wave][rsub][li] = o;
  __syncthreads();
  if (tid < DIMS && !dec_skip(st, t)) {
    const int l4 = tid / 4;
    const int e = tid % 4;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int r = 0; r < RPW; ++r) acc += red[w][r][l4][e];
    out[(size_t)b * d + hg * DIMS + tid] = acc / ssum[tid / 32];
  }
}

// ------------------------------------------------------------------ greedy select
// argmax over the vocabulary (first maximal index, as torch.argmax), log-prob of the
// chosen token log(softmax + 1e-10) (app/src/im2latex.py:33-39), EOS bookkeeping for
// the batch-global stop (src/inference.py:23-25), and the embedding of the token fed
// to step t+1.
__global__ void __launch_bounds__(256) dec_argmax_kernel(DecodeState* st, int t, int last_step,
                                                         const float* __restrict__ logits, size_t hist_stride, int ldl,
                                                         int V,
                                                         int32_t* __restrict__ ids, int32_t* __restrict__ feed,
                                                         const int32_t* __restrict__ forced, int ld_ids,
                                                         float* __restrict__ logp, int32_t* __restrict__ finished,
                                                         int eos, int stop_batch, const float* __restrict__ emb,
                                                         const float* __restrict__ pos, float* __restrict__ x,
                                                         int d) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const float* L = logits + (hist_stride ? (size_t)t * hist_stride : 0) + (size_t)b * ldl;
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int j = tid; j < V; j += 256) {
    const float v = L[j];
    if (v > best) {
      best = v;
      bidx = j;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ov > best || (ov == best && oi < bidx)) {
      best = ov;
      bidx = oi;
    }
  }
  __shared__ float sv[4];
  __shared__ int si_[4];
  __shared__ float ss[4];
  __shared__ int s_next;
  if (lane == 0) {
    sv[wave] = best;
    si_[wave] = bidx;
  }
  __syncthreads();
  best = sv[0];
  bidx = si_[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) {
    if (sv[w] > best || (sv[w] == best && si_[w] < bidx)) {
      best = sv[w];
      bidx = si_[w];
    }
  }
  float sum = 0.f;
  for (int j = tid; j < V; j += 256) sum += expf(L[j] - best);
  sum = wave_sum(sum);
  if (lane == 0) ss[wave] = sum;
  __syncthreads();
  if (dec_skip(stop_batch ? st : nullptr, t)) return;
  if (tid == 0) {
    sum = ((ss[0] + ss[1]) + ss[2]) + ss[3];
    const int next = forced ? forced[(size_t)b * ld_ids + t + 1] : bidx;
    ids[(size_t)b * ld_ids + t + 1] = bidx;
    feed[(size_t)b * ld_ids + t + 1] = next;
    logp[(size_t)b * (ld_ids - 1) + t] = logf(1.0f / sum + 1e-10f);
    s_next = next;
    if (bidx == eos && !finished[b]) {
      finished[b] = 1;
      atomicMax(&st->last_finish, t);
      __threadfence();
      const int before = atomicAdd(&st->nfinished, 1);
      if (before == st->batch - 1 && stop_batch) {
        __threadfence();
        st->done_step = atomicMax(&st->last_finish, t);
      }
    }
  }
  __syncthreads();
  if (!last_step) {
    const int tok = s_next;
    for (int c = tid; c < d; c += 256) x[(size_t)b * d + c] = emb[(size_t)tok * d + c] + pos[(size_t)(t + 1) * d + c];
  }
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
                       hipStream_t s) {
  dec_embed0_kernel<<<B, 256, 0, s>>>(feed, ld_ids, emb, pos, x, d);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_attn(const DecodeState* st, int t, const float* q, const float* K, const float* V,
                     size_t kv_b_stride, int kv_row_stride, int n_fixed, int n_max, float* out, int B, int d,
                     int heads, hipStream_t s) {
  constexpr int HB = 2;
  if (d != kD || heads * 32 != d) throw std::runtime_error("dec_attn: d_model 256 with 8 heads of 32");
  if (n_max > 256) throw std::runtime_error("dec_attn: at most 256 keys");
  const int nit = (n_max + 15) / 16;  // 16 key rows per workgroup pass (4 waves x 4 rows)
  const dim3 grid(B, heads / HB);
#define MOCR_ATTN(N) dec_attn_kernel<HB, N><<<grid, 256, 0, s>>>(st, t, q, K, V, kv_b_stride, kv_row_stride, n_fixed, out, d)
  if (nit <= 2) MOCR_ATTN(2);
  else if (nit <= 4) MOCR_ATTN(4);
  else if (nit <= 8) MOCR_ATTN(8);
  else if (nit <= 10) MOCR_ATTN(10);
  else if (nit <= 12) MOCR_ATTN(12);
  else MOCR_ATTN(16);
#undef MOCR_ATTN
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_argmax(DecodeState* st, int t, int last_step, const float* logits, size_t hist_stride, int ldl,
                       int V, int B, int32_t* ids, int32_t* feed, const int32_t* forced, int ld_ids, float* logp,
                       int32_t* finished, int eos, int stop_batch, const float* emb, const float* pos, float* x,
                       int d, hipStream_t s) {
  dec_argmax_kernel<<<B, 256, 0, s>>>(st, t, last_step, logits, hist_stride, ldl, V, ids, feed, forced, ld_ids, logp,
                                      finished, eos, stop_batch, emb, pos, x, d);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
