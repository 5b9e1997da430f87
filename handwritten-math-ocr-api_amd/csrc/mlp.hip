// Fused norm2 + MLP + residual of a Swin block on bf16 / bf16x3 MFMA (torchvision
// SwinTransformerBlock: x = x + mlp(norm2(x)), mlp = Linear(C, 4C), GELU, Linear(4C, C)),
// for the memory-bound stages 1-2 (C = 96, 192): the 4C-wide hidden never leaves the
// chip.  Unfused, a stage-1 block moves 2.9 GB through HBM for these three ops (LN
// output, the hidden written and read as bf16 hi/lo planes, the residual); fused it
// reads and writes X once (0.45 GB).
//
// One workgroup (8 waves) per 128*TT rows; each wave owns 16*TT rows end to end, so
// only the weights are shared:
//  - LayerNorm of the wave's rows straight into the B fragments of GEMM 1 (lane (g, j)
//    holds row j, channels 32 ks + 8 g .. + 7: the 16x16x32 B layout), kept in registers;
//  - per chunk of NC hidden units: GEMM 1 computes hidden^T = W1 . LN(x)^T (A = W1 rows
//    from LDS), so lane (g, j) holds hidden units 4 g + r of row j; bias + GELU; those
//    accumulators ARE the B fragments of GEMM 2 under a permuted k order (k-step p takes
//    the hidden tiles 2p, 2p+1: lane group g supplies units {32p + 4g + r, 32p + 16 + 4g + r}),
//    and the A fragments (W2 rows) are read from LDS in the same order;
//  - GEMM 2 accumulates out^T = W2 . hidden^T over the chunks: lane (g, j) holds 4
//    consecutive channels of row j, so the residual update is one float4 read-modify-write.
// The W1 / W2 chunks are staged global -> LDS by global_load_lds (16 B per lane, lane
// -linear images with the 16-B chunks XOR-swizzled on the source address so the
// fragment reads are conflict-free), one buffer each, refilled while the other GEMM runs.
#include "kernels.h"

namespace mocr {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ float gelu_erf_fast(float x) {  // gemm.hip gelu_fast (A&S 7.1.26)
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  const float e = 1.0f - poly * t * __expf(-z * z);
  return x * 0.5f * (1.0f + copysignf(e, x));
}

// 8 floats -> bf16 hi / lo planes of one MFMA fragment
__device__ __forceinline__ void pack8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split2_bf16(v[2 * e], v[2 * e + 1], h[e], l[e]);
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

template <int C, int TT, int NC, int PASSES>
__global__ void __launch_bounds__(512) mlp_fused_kernel(MlpParams p) {
  constexpr bool X3 = PASSES == 3;
  constexpr int PL = X3 ? 2 : 1;
  constexpr int RC = C / 8;  // 16-B chunks per W1 row
  // W1 image: chunk c of row r at c ^ s(r), s spreading the 16 rows of a fragment read
  // over the 16 slots of a 256-B bank row (row pitch RC chunks)
  constexpr int SW1 = (RC % 16 == 0) ? 16 : ((RC % 8 == 0) ? 8 : 4);
  constexpr int SH1 = SW1 == 16 ? 0 : (SW1 == 8 ? 1 : 2);
  constexpr int RB = NC / 8;  // 16-B chunks per W2 row
  constexpr int SH2 = RB == 16 ? 0 : (RB == 8 ? 1 : 2);
  constexpr int W1B = NC * C * 2;  // bytes per plane
  constexpr int W2B = C * NC * 2;
  constexpr int KS1 = C / 32;
  constexpr int NH = NC / 16;
  constexpr int NCT = C / 16;
  constexpr int KP = NC / 32;
  constexpr int HID = 4 * C;
  constexpr int NCH = HID / NC;
  constexpr int ROWS = 8 * 16 * TT;
  constexpr int DMA1 = W1B / 1024;  // glds instructions per plane (1 KB each), dealt over the 8 waves
  constexpr int DMA2 = W2B / 1024;
  static_assert(DMA1 * 1024 == W1B && DMA2 * 1024 == W2B, "DMA split");
  static_assert(RC % SW1 == 0 && (RB == 16 || RB == 8 || RB == 4), "swizzle");
  constexpr int LDS_W = PL * (W1B + W2B);
  __shared__ __attribute__((aligned(16))) char lds[LDS_W + (HID + C) * 4];
  char* w1s = lds;
  char* w2s = lds + PL * W1B;
  float* b1s = reinterpret_cast<float*>(lds + LDS_W);
  float* b2s = b1s + HID;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int j16 = lane & 15;
  const int g = lane >> 4;
  const long row0 = (long)blockIdx.x * ROWS + wave * 16 * TT;
  const char* W1g[2] = {static_cast<const char*>(p.w1), static_cast<const char*>(p.w1lo)};
  const char* W2g[2] = {static_cast<const char*>(p.w2), static_cast<const char*>(p.w2lo)};

  auto issue_w1 = [&](int jc) {
#pragma unroll
    for (int q = 0; q < PL; ++q)
      for (int idx = wave; idx < DMA1; idx += 8) {
        const int s = idx * 64 + lane;  // 16-B slot of the image
        const int r = s / RC;
        const int c = (s - r * RC) ^ ((r >> SH1) & (SW1 - 1));
        const char* src = W1g[q] + ((size_t)(jc * NC + r) * C + c * 8) * 2;
        __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(w1s + q * W1B + idx * 1024), 16, 0, 0);
      }
  };
  auto issue_w2 = [&](int jc) {
#pragma unroll
    for (int q = 0; q < PL; ++q)
      for (int idx = wave; idx < DMA2; idx += 8) {
        const int s = idx * 64 + lane;
        const int r = s / RB;
        const int c = (s - r * RB) ^ ((r >> SH2) & (RB - 1));
        const char* src = W2g[q] + ((size_t)r * HID + jc * NC + c * 8) * 2;
        __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(w2s + q * W2B + idx * 1024), 16, 0, 0);
      }
  };

  issue_w1(0);
  issue_w2(0);
  for (int i = tid; i < HID; i += 512) b1s[i] = p.b1[i];
  for (int i = tid; i < C; i += 512) b2s[i] = p.b2[i];

  // LayerNorm(norm2) of this wave's rows into GEMM 1's B fragments
  bf16x8 xb[TT][KS1][PL];
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const long row = min(row0 + tt * 16 + j16, p.M - 1);
    const float* xr = p.X + (size_t)row * C + 8 * g;
    float v[KS1][8];
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(xr + 32 * ks);
      const floatx4 b = *reinterpret_cast<const floatx4*>(xr + 32 * ks + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[ks][e] = a[e];
        v[ks][4 + e] = b[e];
      }
    }
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[ks][e];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mean = s / (float)C;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[ks][e] - mean;
        q += d * d;
      }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rstd = 1.0f / sqrtf(q / (float)C + 1e-5f);
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      const int ch = 32 * ks + 8 * g;
      const floatx4 g0 = *reinterpret_cast<const floatx4*>(p.ln_g + ch);
      const floatx4 g1 = *reinterpret_cast<const floatx4*>(p.ln_g + ch + 4);
      const floatx4 c0 = *reinterpret_cast<const floatx4*>(p.ln_b + ch);
      const floatx4 c1 = *reinterpret_cast<const floatx4*>(p.ln_b + ch + 4);
      float y[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[e] = (v[ks][e] - mean) * rstd * g0[e] + c0[e];
        y[4 + e] = (v[ks][4 + e] - mean) * rstd * g1[e] + c1[e];
      }
      bf16x8 hi, lo;
      pack8(y, hi, lo);
      xb[tt][ks][0] = hi;
      if constexpr (X3) xb[tt][ks][PL - 1] = lo;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  floatx4 acc2[NCT][TT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) acc2[ct][tt] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int jc = 0; jc < NCH; ++jc) {
    const bool more = jc + 1 < NCH;
    // GEMM 1: hidden^T [NC x 16TT] = W1[chunk] . LN(x)^T
    floatx4 acc1[NH][TT];
#pragma unroll
    for (int ht = 0; ht < NH; ++ht)
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) acc1[ht][tt] = floatx4{0.f, 0.f, 0.f, 0.f};
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int ht = 0; ht < NH; ++ht) {
        const int r = ht * 16 + j16;
        const int pc = (4 * ks + g) ^ ((r >> SH1) & (SW1 - 1));
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(w1s + r * (C * 2) + pc * 16);
        bf16x8 al = ah;
        if constexpr (X3) al = *reinterpret_cast<const bf16x8*>(w1s + W1B + r * (C * 2) + pc * 16);
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
          acc1[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xb[tt][ks][0], acc1[ht][tt], 0, 0, 0);
          if constexpr (X3) {
            acc1[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xb[tt][ks][1], acc1[ht][tt], 0, 0, 0);
            acc1[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, xb[tt][ks][0], acc1[ht][tt], 0, 0, 0);
          }
        }
      }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of W2[chunk]
    __builtin_amdgcn_s_barrier();                      // w1s free; w2s[chunk] complete
    if (more) issue_w1(jc + 1);

    // bias + GELU; the accumulators of hidden tiles 2p, 2p+1 are GEMM 2's B fragment p
    bf16x8 hb[KP][TT][PL];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp)
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        const float* bb = b1s + jc * NC + 32 * kp + 4 * g;
        float h[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          h[r] = gelu_erf_fast(acc1[2 * kp][tt][r] + bb[r]);
          h[4 + r] = gelu_erf_fast(acc1[2 * kp + 1][tt][r] + bb[16 + r]);
        }
        bf16x8 hi, lo;
        pack8(h, hi, lo);
        hb[kp][tt][0] = hi;
        if constexpr (X3) hb[kp][tt][PL - 1] = lo;
      }

    // GEMM 2: out^T [C x 16TT] += W2[:, chunk] . hidden^T, k order as above
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kp = 0; kp < KP; ++kp)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const int r = ct * 16 + j16;
        const int t = (r >> SH2) & (RB - 1);
        const int s0 = 4 * kp + (g >> 1);
        const int o0 = r * (NC * 2) + ((s0 ^ t) * 16) + (g & 1) * 8;
        const int o1 = r * (NC * 2) + (((s0 + 2) ^ t) * 16) + (g & 1) * 8;
        const uint2 h0 = *reinterpret_cast<const uint2*>(w2s + o0);
        const uint2 h1 = *reinterpret_cast<const uint2*>(w2s + o1);
        const bf16x8 ah = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
        bf16x8 al = ah;
        if constexpr (X3) {
          const uint2 l0 = *reinterpret_cast<const uint2*>(w2s + W2B + o0);
          const uint2 l1 = *reinterpret_cast<const uint2*>(w2s + W2B + o1);
          al = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
        }
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
          acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, hb[kp][tt][0], acc2[ct][tt], 0, 0, 0);
          if constexpr (X3) {
            acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, hb[kp][tt][1], acc2[ct][tt], 0, 0, 0);
            acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, hb[kp][tt][0], acc2[ct][tt], 0, 0, 0);
          }
        }
      }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of W1[chunk + 1]
    __builtin_amdgcn_s_barrier();                      // w2s free; w1s[chunk + 1] complete
    if (more) issue_w2(jc + 1);
  }

  // x += out + b2 (4 consecutive channels of one row per lane and tile)
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const long row = row0 + tt * 16 + j16;
    if (row >= p.M) continue;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int ch = ct * 16 + 4 * g;
      float* xp = p.X + (size_t)row * C + ch;
      floatx4 x = *reinterpret_cast<const floatx4*>(xp);
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = x[r] + (acc2[ct][tt][r] + b2s[ch + r]);
      *reinterpret_cast<floatx4*>(xp) = x;
    }
  }
}

template <int C, int TT, int NC>
void launch_mlp_c(const MlpParams& p, hipStream_t s) {
  const unsigned grid = (unsigned)((p.M + 128 * TT - 1) / (128 * TT));
  if (p.w1lo && p.w2lo)
    mlp_fused_kernel<C, TT, NC, 3><<<grid, 512, 0, s>>>(p);
  else
    mlp_fused_kernel<C, TT, NC, 1><<<grid, 512, 0, s>>>(p);
}

}  // namespace

bool mlp_fused_supported(int C) { return C == 96 || C == 192; }

void launch_mlp_fused(const MlpParams& p, hipStream_t s) {
  if (p.M <= 0) return;
  if ((p.w1lo == nullptr) != (p.w2lo == nullptr)) throw std::runtime_error("mlp: lo planes for both or neither");
  switch (p.C) {
    case 96: launch_mlp_c<96, 2, 64>(p, s); break;
    case 192: launch_mlp_c<192, 1, 64>(p, s); break;
    default: throw std::runtime_error("mlp: fused MLP built for C = 96, 192");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
