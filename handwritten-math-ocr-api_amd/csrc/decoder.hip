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
// Every kernel reads the step index from DecodeState in device memory, so one
// captured hipGraph of a step chunk is replayed for the whole decode; once the
// batch has stopped (all rows hit EOS, or max_steps) every kernel exits at entry.
#include "kernels.h"

namespace mocr {

namespace {

constexpr float kAttnScale = 0.17677669529663687f;  // 1/sqrt(32)

// ------------------------------------------------------------------ small-M GEMM
// out[B, N] = A[B, K] · W[N, K]^T + bias on v_mfma_f32_16x16x4_f32.  A workgroup
// owns a 16x16 output tile; its 4 waves split K and combine through LDS in a fixed
// order.  Each lane loads float4 runs of A and W straight into registers (no reuse
// inside the workgroup, so no LDS staging); lane group g = lane>>4 feeds
// k = 4g + s at MFMA step s.
template <int EPI, int KW>
__global__ void __launch_bounds__(256) rowgemm_kernel(RowGemmParams p) {
  if (p.st->done) return;
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

  floatx4 a[NI], b[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int k = kbeg + i * 16 + 4 * g;
    a[i] = ra < p.B ? *reinterpret_cast<const floatx4*>(p.A + (size_t)ra * p.K + k) : floatx4{0.f, 0.f, 0.f, 0.f};
    b[i] = *reinterpret_cast<const floatx4*>(p.W + (size_t)cb * p.K + k);
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
  if (grow >= p.B || gcol >= p.n_valid) return;
  float v = ((red[0][row][col] + red[1][row][col]) + red[2][row][col]) + red[3][row][col];
  v += p.bias[gcol];
  if constexpr (EPI == DEC_STORE) {
    p.out[(size_t)grow * p.ldo + gcol] = v;
  } else if constexpr (EPI == DEC_RELU) {
    p.out[(size_t)grow * p.ldo + gcol] = fmaxf(v, 0.f);
  } else if constexpr (EPI == DEC_RESADD) {
    p.out[(size_t)grow * p.ldo + gcol] = p.resid[(size_t)grow * p.ldo + gcol] + v;
  } else if constexpr (EPI == DEC_QKV) {
    const int t = p.st->t;
    if (gcol < p.d) {
      p.out[(size_t)grow * p.d + gcol] = v;
    } else if (gcol < 2 * p.d) {
      p.kcache[((size_t)grow * p.max_pos + t) * p.d + (gcol - p.d)] = v;
    } else {
      p.vcache[((size_t)grow * p.max_pos + t) * p.d + (gcol - 2 * p.d)] = v;
    }
  } else {  // DEC_LOGITS
    float* slot = p.out + (p.hist_stride ? (size_t)p.st->t * p.hist_stride : 0);
    slot[(size_t)grow * p.ldo + gcol] = v;
  }
}

template <int EPI>
void launch_rowgemm_k(const RowGemmParams& p, dim3 grid, hipStream_t s) {
  if (p.K == 256) {
    rowgemm_kernel<EPI, 64><<<grid, 256, 0, s>>>(p);
  } else if (p.K == 512) {
    rowgemm_kernel<EPI, 128><<<grid, 256, 0, s>>>(p);
  } else {
    throw std::runtime_error("rowgemm: K must be 256 or 512");
  }
}

// ------------------------------------------------------------------ embedding
// x[b] = embedding[feed[b][t]] + pos_encoder[t]   (src/model_swin.py:73-75).
// Single workgroup: it advances DecodeState.t before any other kernel of the step.
__global__ void __launch_bounds__(256) dec_embed_kernel(DecodeState* st, const int32_t* __restrict__ feed, int ld_ids,
                                                        const float* __restrict__ emb, const float* __restrict__ pos,
                                                        float* __restrict__ x, int B, int d) {
  __shared__ int s_t;
  if (threadIdx.x == 0) {
    int t = -1;
    if (!st->done) {
      t = st->t + 1;
      if (t >= st->max_steps) {
        st->done = 1;
        st->nsteps = st->max_steps;
        t = -1;
      } else {
        st->t = t;
      }
    }
    s_t = t;
  }
  __syncthreads();
  const int t = s_t;
  if (t < 0) return;
  for (int idx = threadIdx.x; idx < B * d; idx += blockDim.x) {
    const int b = idx / d;
    const int c = idx - b * d;
    const int tok = feed[(size_t)b * ld_ids + t];
    x[idx] = emb[(size_t)tok * d + c] + pos[(size_t)t * d + c];
  }
}

// ------------------------------------------------------------------ LayerNorm(d)
__global__ void __launch_bounds__(256) dec_layernorm_kernel(const DecodeState* st, const float* __restrict__ y,
                                                            const float* __restrict__ g,
                                                            const float* __restrict__ bta, float* __restrict__ x,
                                                            int B, int d) {
  if (st->done) return;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float* src = y + (size_t)row * d;
  float v[4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < d ? src[c] : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    if (c < d) {
      const float t = v[i] - mean;
      q += t * t;
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)d + 1e-5f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    if (c < d) x[(size_t)row * d + c] = (v[i] - mean) * rstd * g[c] + bta[c];
  }
}

// ------------------------------------------------------------------ attention
// One wave per (row b, head h).  Scores q·k * 1/sqrt(32) for n keys, softmax with a
// wave max/sum reduce, output Σ_j e_j v_j / Σ_j e_j (normalised at the end, like the
// CPU flash-attention SDPA kernel the reference's F.multi_head_attention_forward
// reaches).  Lane j scores keys j, j+64, ...; for P·V the two half-waves take even
// and odd keys with lane&31 as the head-dim index (coalesced 128-B rows).
__device__ __forceinline__ void attend(const float* __restrict__ qrow, const float* __restrict__ kbase,
                                       const float* __restrict__ vbase, size_t kv_stride, int n,
                                       float* __restrict__ out, float* p) {
  const int lane = threadIdx.x & 63;
  float qv[kHeadDim];
#pragma unroll
  for (int i = 0; i < kHeadDim / 4; ++i) {
    const floatx4 t = *reinterpret_cast<const floatx4*>(qrow + 4 * i);
    qv[4 * i] = t[0];
    qv[4 * i + 1] = t[1];
    qv[4 * i + 2] = t[2];
    qv[4 * i + 3] = t[3];
  }
  float m = -INFINITY;
  for (int j = lane; j < n; j += 64) {
    const float* kr = kbase + (size_t)j * kv_stride;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kHeadDim / 4; ++i) {
      const floatx4 kk = *reinterpret_cast<const floatx4*>(kr + 4 * i);
      s = fmaf(qv[4 * i], kk[0], s);
      s = fmaf(qv[4 * i + 1], kk[1], s);
      s = fmaf(qv[4 * i + 2], kk[2], s);
      s = fmaf(qv[4 * i + 3], kk[3], s);
    }
    s *= kAttnScale;
    p[j] = s;
    m = fmaxf(m, s);
  }
  m = wave_max(m);
  float sum = 0.f;
  for (int j = lane; j < n; j += 64) {
    const float e = expf(p[j] - m);
    p[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  const int dd = lane & 31;
  const int half = lane >> 5;
  float o = 0.f;
  for (int j = half; j < n; j += 2) o = fmaf(p[j], vbase[(size_t)j * kv_stride + dd], o);
  o += __shfl_xor(o, 32, 64);
  if (half == 0) out[dd] = o / sum;
}

__global__ void __launch_bounds__(64) dec_self_attn_kernel(const DecodeState* st, const float* __restrict__ q,
                                                           const float* __restrict__ kc,
                                                           const float* __restrict__ vc, float* __restrict__ out,
                                                           int d, int max_pos) {
  if (st->done) return;
  __shared__ float p[256];
  const int b = blockIdx.x;
  const int h = blockIdx.y;
  const int n = st->t + 1;
  const size_t base = (size_t)b * max_pos * d + h * kHeadDim;
  attend(q + (size_t)b * d + h * kHeadDim, kc + base, vc + base, d, n, out + (size_t)b * d + h * kHeadDim, p);
}

__global__ void __launch_bounds__(64) dec_cross_attn_kernel(const DecodeState* st, const float* __restrict__ q,
                                                            const float* __restrict__ memkv, int ld_kv, int koff,
                                                            int voff, float* __restrict__ out, int M, int d) {
  if (st->done) return;
  __shared__ float p[1024];
  const int b = blockIdx.x;
  const int h = blockIdx.y;
  const size_t base = (size_t)b * M * ld_kv + h * kHeadDim;
  attend(q + (size_t)b * d + h * kHeadDim, memkv + base + koff, memkv + base + voff, ld_kv, M,
         out + (size_t)b * d + h * kHeadDim, p);
}

// ------------------------------------------------------------------ greedy select
// argmax over the vocabulary (first maximal index, as torch.argmax), log-prob of the
// chosen token log(softmax + 1e-10) (app/src/im2latex.py:33-39), EOS bookkeeping for
// the batch-global stop (src/inference.py:23-25).
__global__ void __launch_bounds__(256) dec_argmax_kernel(DecodeState* st, const float* __restrict__ logits,
                                                         size_t hist_stride, int ldl, int V, int B,
                                                         int32_t* __restrict__ ids, int32_t* __restrict__ feed,
                                                         const int32_t* __restrict__ forced, int ld_ids,
                                                         float* __restrict__ logp, int32_t* __restrict__ finished,
                                                         int eos) {
  if (st->done) return;
  const int t = st->t;
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
  __shared__ int si[4];
  __shared__ float ss[4];
  if (lane == 0) {
    sv[wave] = best;
    si[wave] = bidx;
  }
  __syncthreads();
  best = sv[0];
  bidx = si[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) {
    if (sv[w] > best || (sv[w] == best && si[w] < bidx)) {
      best = sv[w];
      bidx = si[w];
    }
  }
  float sum = 0.f;
  for (int j = tid; j < V; j += 256) sum += expf(L[j] - best);
  sum = wave_sum(sum);
  if (lane == 0) ss[wave] = sum;
  __syncthreads();
  if (tid != 0) return;
  sum = ((ss[0] + ss[1]) + ss[2]) + ss[3];
  const int S1 = ld_ids;
  ids[(size_t)b * S1 + t + 1] = bidx;
  feed[(size_t)b * S1 + t + 1] = forced ? forced[(size_t)b * S1 + t + 1] : bidx;
  if (logp) logp[(size_t)b * (S1 - 1) + t] = logf(1.0f / sum + 1e-10f);
  if (bidx == eos && !finished[b]) {
    finished[b] = 1;
    const int before = atomicAdd(&st->nfinished, 1);
    if (before == B - 1 && st->stop_mode == 0) {
      st->nsteps = t + 1;
      __threadfence();
      st->done = 1;
    }
  }
}

}  // namespace

void launch_rowgemm(const RowGemmParams& p, hipStream_t s) {
  if (p.N % 16 != 0) throw std::runtime_error("rowgemm: N must be padded to 16");
  dim3 grid(p.N / 16, (p.B + 15) / 16);
  switch (p.epi) {
    case DEC_STORE: launch_rowgemm_k<DEC_STORE>(p, grid, s); break;
    case DEC_RELU: launch_rowgemm_k<DEC_RELU>(p, grid, s); break;
    case DEC_RESADD: launch_rowgemm_k<DEC_RESADD>(p, grid, s); break;
    case DEC_QKV: launch_rowgemm_k<DEC_QKV>(p, grid, s); break;
    case DEC_LOGITS: launch_rowgemm_k<DEC_LOGITS>(p, grid, s); break;
    default: throw std::runtime_error("rowgemm: bad epilogue");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_embed(DecodeState* st, const int32_t* feed, int ld_ids, const float* emb, const float* pos, float* x,
                      int B, int d, hipStream_t s) {
  dec_embed_kernel<<<1, 256, 0, s>>>(st, feed, ld_ids, emb, pos, x, B, d);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_layernorm(const DecodeState* st, const float* y, const float* g, const float* b, float* x, int B,
                          int d, hipStream_t s) {
  if (d > 256) throw std::runtime_error("dec_layernorm: d_model > 256");
  dec_layernorm_kernel<<<(B + 3) / 4, 256, 0, s>>>(st, y, g, b, x, B, d);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_self_attn(const DecodeState* st, const float* q, const float* kc, const float* vc, float* out, int B,
                          int d, int heads, int max_pos, hipStream_t s) {
  if (max_pos > 256) throw std::runtime_error("dec_self_attn: max_pos > 256");
  dec_self_attn_kernel<<<dim3(B, heads), 64, 0, s>>>(st, q, kc, vc, out, d, max_pos);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_cross_attn(const DecodeState* st, const float* q, const float* memkv, int ld_kv, int koff, int voff,
                           float* out, int B, int M, int d, int heads, hipStream_t s) {
  if (M > 1024) throw std::runtime_error("dec_cross_attn: more than 1024 memory tokens");
  dec_cross_attn_kernel<<<dim3(B, heads), 64, 0, s>>>(st, q, memkv, ld_kv, koff, voff, out, M, d);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_dec_argmax(DecodeState* st, const float* logits, size_t hist_stride, int ldl, int V, int B, int32_t* ids,
                       int32_t* feed, const int32_t* forced, int ld_ids, float* logp, int32_t* finished, int eos,
                       hipStream_t s) {
  dec_argmax_kernel<<<B, 256, 0, s>>>(st, logits, hist_stride, ldl, V, B, ids, feed, forced, ld_ids, logp, finished,
                                      eos);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
