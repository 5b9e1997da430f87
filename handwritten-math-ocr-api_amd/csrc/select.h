// Greedy token selection of one decoder row (device code shared by dec_argmax_kernel and
// the folded self-attention that runs it for the previous step, decfold.hip).
//
// argmax over the vocabulary (first maximal index, as torch.argmax), log-prob of the
// chosen token log(softmax + 1e-10) (app/src/im2latex.py:33-39), and the EOS bookkeeping
// of the batch-global stop (src/inference.py:23-25).
#pragma once

#include "kernels.h"

namespace mocr {

// running (max, first argmax, sum exp(l - max)) merge; ties go to the lower index
__device__ __forceinline__ void sel_merge(float& b1, int& i1, float& s1, float b2, int i2, float s2) {
  const float m = fmaxf(b1, b2);
  const float f1 = b1 == -INFINITY ? 0.f : __expf(b1 - m);
  const float f2 = b2 == -INFINITY ? 0.f : __expf(b2 - m);
  s1 = s1 * f1 + s2 * f2;
  if (b2 > b1 || (b2 == b1 && i2 < i1)) i1 = i2;
  b1 = m;
}

// Row b of step a.t, all 64 W threads of the workgroup.  Returns the token fed to step t+1
// (workgroup-uniform; the forced token when teacher forcing), or -1 when the batch stopped
// before step t.  `bookkeep`: this workgroup writes ids / feed / logp / the finished flags
// and the stop state (one workgroup per row may).
template <int W = 4>
__device__ __forceinline__ int greedy_select(const SelectArgs& a, int b, bool bookkeep) {
  constexpr int NT = 64 * W;
  constexpr int NP = (512 + NT - 1) / NT;  // partials per thread (nparts <= 512)
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int t = a.t;
  const int V = a.V;
  const float* L = a.logits + (a.hist_stride ? (size_t)t * a.hist_stride : 0) + (size_t)b * a.ldl;
  float best = -INFINITY, sum = 0.f;
  int bidx = 0x7fffffff;
  constexpr int CH = 20;  // loads in flight per thread: one round for V <= 5120
  if (a.part) {  // per-16-column-tile partials of the logits kernel (nparts <= 512)
    const floatx4* P = reinterpret_cast<const floatx4*>(a.part) + (size_t)b * a.nparts;
    floatx4 q[NP];
#pragma unroll
    for (int c = 0; c < NP; ++c) q[c] = P[min(tid + NT * c, a.nparts - 1)];
#pragma unroll
    for (int c = 0; c < NP; ++c)
      if (tid + NT * c < a.nparts) sel_merge(best, bidx, sum, q[c][0], __float_as_int(q[c][1]), q[c][2]);
  }
  for (int j0 = a.part ? V : tid; j0 < V; j0 += NT * CH) {
    float vals[CH];
    // unpredicated loads (a clamped column), masked after: a predicated load per element
    // becomes a branch + vmcnt(0) each
#pragma unroll
    for (int c = 0; c < CH; ++c) vals[c] = L[min(j0 + NT * c, V - 1)];
#pragma unroll
    for (int c = 0; c < CH; ++c) vals[c] = (j0 + NT * c < V) ? vals[c] : -INFINITY;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const float v = vals[c];
      if (v > best) {
        sum = sum * expf(best - v) + 1.0f;
        best = v;
        bidx = j0 + NT * c;
      } else if (v != -INFINITY) {
        sum += expf(v - best);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    const float os = __shfl_xor(sum, o, 64);
    sel_merge(best, bidx, sum, ob, oi, os);
  }
  __shared__ float sv[W], ss[W];
  __shared__ int si_[W];
  __shared__ int s_next;
  if ((tid & 63) == 0) {
    sv[wave] = best;
    si_[wave] = bidx;
    ss[wave] = sum;
  }
  __syncthreads();
  best = sv[0];
  bidx = si_[0];
  sum = ss[0];
#pragma unroll
  for (int w = 1; w < W; ++w) sel_merge(best, bidx, sum, sv[w], si_[w], ss[w]);
  DecodeState* st = a.st;
  if (dec_skip(a.stop_batch ? st : nullptr, t)) return -1;
  // A row without a finite maximum (NaN logits never win `v > best`) would leave bidx at
  // INT_MAX and gather the next embedding ~2^31 rows out of bounds: clamp it to a valid
  // id and count the row; the host turns the count into an error after the decode.
  if (!(bidx >= 0 && bidx < V && isfinite(best) && sum > 0.f)) {
    if (tid == 0 && bookkeep) atomicAdd(&st->bad_rows, 1);
    bidx = 0;
    sum = 1.f;
  }
  if (tid == 0) {
    int next = a.forced ? a.forced[(size_t)b * a.ld_ids + t + 1] : bidx;
    next = min(max(next, 0), V - 1);
    s_next = next;
    if (bookkeep) {
      a.ids[(size_t)b * a.ld_ids + t + 1] = bidx;
      a.feed[(size_t)b * a.ld_ids + t + 1] = next;
      a.logp[(size_t)b * (a.ld_ids - 1) + t] = logf(1.0f / sum + 1e-10f);
      if (bidx == a.eos && !a.finished[b]) {
        a.finished[b] = 1;
        atomicMax(&st->last_finish, t);
        __threadfence();
        const int before = atomicAdd(&st->nfinished, 1);
        if (before == st->batch - 1 && a.stop_batch) {
          __threadfence();
          st->done_step = atomicMax(&st->last_finish, t);
        }
      }
    }
  }
  __syncthreads();
  return s_next;
}

}  // namespace mocr
