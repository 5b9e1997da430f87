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
// The W1 / W2 chunks are staged global -> registers -> LDS (16 B per lane; the 16-B
// chunks of each row XOR-swizzled so the fragment reads are conflict-free),
// double-buffered: chunk j+1 is loaded while chunk j runs, one barrier per chunk.
#include "kernels.h"
#include "lanes.h"

namespace mocr {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// 2 x GELU(x) = x (1 + erf(x / sqrt 2)) (gemm.hip gelu_fast, A&S 7.1.26, without its factor
// 0.5): the fused MLP kernels' W2 chunk images hold W2 / 2 (mlp_pack_kernel, pack_img384's
// W2 image), so GEMM 2 multiplies the same bf16 products -- (2h) (W2 / 2) = h W2 exactly,
// splits included -- and the outputs are bitwise the unscaled ones whenever every W2 plane
// value is a normal bf16 whose half is normal too (exponent field > 1: half_bf16x2 is then an
// exact exponent decrement; below that, mostly lo-plane residuals of tiny weights, it halves
// through fp32 with truncation and FTZ), one multiply per hidden value fewer
__device__ __forceinline__ float gelu2_erf_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  const float e = 1.0f - poly * t * __expf(-z * z);
  return x * (1.0f + copysignf(e, x));
}

// 8 floats -> bf16 hi / lo planes of one MFMA fragment
__device__ __forceinline__ void pack8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split2_bf16(v[2 * e], v[2 * e + 1], h[e], l[e]);
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

// NST staging registers as a recursive struct (constant member offsets): an array indexed
// in an unrolled loop is left to AMDGPU promote-alloca, which put it in LDS / scratch.
template <int K, int N>
struct StgList {
  uint4 head;
  StgList<K + 1, N> tail;
  template <class F>
  __device__ __forceinline__ void load(F f) {
    head = f(K);
    tail.load(f);
  }
  template <class G>
  __device__ __forceinline__ void store(G g) const {
    g(K, head);
    tail.store(g);
  }
};
template <int N>
struct StgList<N, N> {
  template <class F>
  __device__ __forceinline__ void load(F) {}
  template <class G>
  __device__ __forceinline__ void store(G) const {}
};

// Piece rem (1 KB, 16 B per lane) of plane q of one W1 | W2 chunk's LDS image: pieces
// 0 .. DMA1 - 1 are the W1 image, the rest the W2 image.  The 16 bytes of lane `lane`
// (two 8-B loads, whichever image) and their offset in the image (the LDS byte order:
// [W1 planes | W2 planes]).  Both images' addresses are computed and selected.
template <int C, int NC, int DMA1, int RC, int SW1, int SH1, int RB, int SH2>
__device__ __forceinline__ uint4 mlp_piece_load(const MlpParams& p, int jc, int q, int rem, int lane) {
  const bool in1 = rem < DMA1;
  const int sl = (in1 ? rem : rem - DMA1) * 64 + lane;
  // W1 image: row r1 = hidden unit, slot = 8 channels, XOR-swizzled
  const int r1 = sl / RC;
  const int c1 = (sl - r1 * RC) ^ ((r1 >> SH1) & (SW1 - 1));
  // W2 image: row r2 = channel; logical slot s = 4 kp + g holds hidden units
  // {32 kp + 4 g .. +3} then {32 kp + 16 + 4 g .. +3} (GEMM 2's permuted k order)
  const int r2 = sl / RB;
  const int s2 = (sl - r2 * RB) ^ ((r2 >> SH2) & (RB - 1));
  const int h2 = 32 * (s2 >> 2) + 4 * (s2 & 3);
  const char* w1 = static_cast<const char*>(q ? p.w1lo : p.w1);
  const char* w2 = static_cast<const char*>(q ? p.w2lo : p.w2);
  const char* a1 = w1 + ((size_t)(jc * NC + r1) * C + c1 * 8) * 2;
  const char* a2 = w2 + ((size_t)r2 * 4 * C + jc * NC + h2) * 2;
  const uint2 lo = *reinterpret_cast<const uint2*>(in1 ? a1 : a2);
  const uint2 hi = *reinterpret_cast<const uint2*>(in1 ? a1 + 8 : a2 + 32);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
template <int PL, int DMA1, int W1B, int W2B>
__device__ __forceinline__ int mlp_piece_dst(int q, int rem, int lane) {
  const bool in1 = rem < DMA1;
  const int sl = (in1 ? rem : rem - DMA1) * 64 + lane;
  return in1 ? q * W1B + sl * 16 : PL * W1B + q * W2B + sl * 16;
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ int swz4(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }  // {0,2,3,1}

// GEMM 2's output channels are permuted (the W2 image's row i holds W2 row perm384(i), and
// b2 likewise), so that lane group g of output tiles 2 ks, 2 ks + 1 holds channels 32 ks +
// 8 g .. + 7: the B-fragment layout of the LayerNorm's input.  For GEMM 2 alone that only
// moves which lane computes a channel (bitwise the same outputs); with PROJ it lets the
// proj GEMM's accumulators be the LayerNorm's input in place.
__device__ __forceinline__ int perm384(int i) {
  return 32 * (i >> 5) + 8 * ((i >> 2) & 3) + 4 * ((i >> 4) & 1) + (i & 3);
}

__device__ __forceinline__ uint32_t lds_u32(const char* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((lds_ptr_t)(p));
}
// One 1-KB LDS-DMA piece: 16 B per lane from gbase + voff (uniform base, lane offset) to
// LDS lds + 16 * lane.  Issued by inline asm so that hipcc does not see an LDS write in
// flight: with __builtin_amdgcn_global_load_lds into a ring indexed at run time it puts a
// vmcnt(0) before every fragment read.  The kernel waits for its own DMA (counted vmcnt
// before each barrier); vector loads retire in order, so hipcc's own counts stay safe.
// M0 is a reserved register (no clobber list entry): the asm saves and restores it.
__device__ __forceinline__ void dma16(const char* gbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds)
      : "memory");
}

// Both bf16 halves of v times 0.5 (W2 / 2 for the fused MLPs, gelu2_erf_fast): the exponent
// minus one, exact for normal values; zeros, and the (never seen) smallest normals and
// subnormals, through fp32
__device__ __forceinline__ uint32_t half_bf16x2(uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint32_t h = (v >> (16 * i)) & 0xffffu;
    const uint32_t e = (h >> 7) & 0xffu;
    if (e > 1u && e < 255u)
      h -= 0x80u;
    else if (e <= 1u)
      h = __float_as_uint(__uint_as_float(h << 16) * 0.5f) >> 16;
    r |= h << (16 * i);
  }
  return r;
}
__device__ __forceinline__ uint4 half_bf16x8(uint4 v) {
  return make_uint4(half_bf16x2(v.x), half_bf16x2(v.y), half_bf16x2(v.z), half_bf16x2(v.w));
}


// The stage-1 kernel (C = 96, 4 waves) on three waves per SIMD: its W1 | W2 chunks go to
// LDS by LDS-DMA (dma16: no staging registers) and its residual rows are loaded in the
// epilogue, 158 VGPRs and no AGPRs instead of 152 + 68 (two waves per SIMD): s1.mlp 4.73 /
// 4.78 vs 5.36 / 5.40 ms per 512-image encode, bitwise the same memory (profiles/r05/r07e).
// The stage-2 kernel on 4-wave workgroups with one LDS buffer
// filled by LDS-DMA between two barriers: 148 VGPRs and 53 KB, three workgroups per CU
// (12 waves) instead of one 8-wave workgroup (229 VGPRs, 102 KB): s2.mlp 4.21 / 4.27 vs
// 4.53 / 4.61 ms per 512-image encode, bitwise the same memory (profiles/r05/r07h).  With
// register staging the same geometry measured slower (round 5, r06h: 4.9-5.0 vs 4.5 ms).
// Both run the DMA form (NWV = 4); NWV = 8 keeps round 4's register-staged chunks.
template <int C, int TT, int NC, int PASSES, int NWV = 8, int NBUF = 2>
__global__ void __launch_bounds__(64 * NWV)
__attribute__((amdgpu_waves_per_eu(NWV == 4 ? 3 : 1, 8)))
mlp_fused_kernel(MlpParams p) {
  constexpr bool PRERES = NWV != 4;
  constexpr bool X3 = PASSES == 3;
  constexpr int PL = X3 ? 2 : 1;
  constexpr int RC = C / 8;  // 16-B chunks per W1 row
  // W1 image: chunk c of row r at c ^ s(r), s spreading the 16 rows of a fragment read
  // over the 16 slots of a 256-B bank row (row pitch RC chunks)
  // (conflict-free for ds_read_b128's lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31},
  // ...: checked by enumerating the fragment reads, MI355X_MICROARCH.md §LDS)
  constexpr int SW1 = (RC % 16 == 0) ? 16 : ((RC % 8 == 0) ? 8 : 4);
  constexpr int SH1 = SW1 == 16 ? 0 : 1;
  constexpr int RB = NC / 8;  // 16-B slots per W2 row
  constexpr int SH2 = RB == 4 ? 1 : 0;
  constexpr int W1B = NC * C * 2;  // bytes per plane
  constexpr int W2B = C * NC * 2;
  constexpr int KS1 = C / 32;
  constexpr int NH = NC / 16;
  constexpr int NCT = C / 16;
  constexpr int KP = NC / 32;
  constexpr int HID = 4 * C;
  constexpr int NCH = HID / NC;
  constexpr int ROWS = NWV * 16 * TT;
  constexpr int DMA1 = W1B / 1024;  // 1-KB pieces per plane
  constexpr int DMA2 = W2B / 1024;
  static_assert(DMA1 * 1024 == W1B && DMA2 * 1024 == W2B, "DMA split");
  static_assert(RC % SW1 == 0 && (RB == 16 || RB == 8 || RB == 4), "swizzle");
  constexpr int BUF = PL * (W1B + W2B);  // one chunk of W1 and W2, double-buffered
  // NBUF = 2: chunk jc + 1 is stored into the other buffer while chunk jc is read; NBUF = 1
  // (half the LDS: two 4-wave workgroups per CU at C = 192): stored after a barrier
  constexpr int LDS_W = NBUF * BUF;
  __shared__ __attribute__((aligned(16))) char lds[LDS_W + (HID + C) * 4];
  static_assert(NWV == 8 || NWV == 4, "8 or 4 waves");
  float* b1s = reinterpret_cast<float*>(lds + LDS_W);
  float* b2s = b1s + HID;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int j16 = lane & 15;
  const int g = lane >> 4;
  const long row0 = (long)blockIdx.x * ROWS + wave * 16 * TT;

  // One chunk = PL x (DMA1 + DMA2) 1-KB pieces (W1 then W2 per plane), NWV waves x NST each.
  // Register-staged (global -> VGPR -> LDS): with LDS-DMA in flight hipcc drains it with
  // vmcnt(0) before the GEMM-2 fragment reads, which serialised the prefetch.  The packed
  // chunk image (launch_mlp_pack) holds the LDS bytes in order, so piece k of wave w is the
  // 1-KB block k NWV + w of the chunk, at the same offset in LDS.
  constexpr int NPIECE = PL * (DMA1 + DMA2);
  constexpr int NST = NPIECE / NWV;
  static_assert(NST * NWV == NPIECE, "pieces per wave");
  const char* wpk = static_cast<const char*>(p.wpack);
  auto pdst = [&](int k) { return (k * NWV + wave) * 1024 + lane * 16; };
  auto piece = [&](int jc, int k) { return *reinterpret_cast<const uint4*>(wpk + (size_t)jc * BUF + pdst(k)); };
  // !PRERES (the 3-wave stage-1 build): the chunks go global -> LDS by LDS-DMA (dma16, no
  // staging registers), issued at the start of the chunk before the one that reads them
  constexpr bool DMA = !PRERES;
  auto issue_chunk = [&](int jc, char* buf) {
    uint32_t lb = (uint32_t)(16 * lane);
    asm volatile("" : "+v"(lb));
#pragma unroll
    for (int k = 0; k < NST; ++k)
      dma16(wpk + (size_t)jc * BUF, (uint32_t)((k * NWV + wave) * 1024) + lb,
            __builtin_amdgcn_readfirstlane(lds_u32(buf) + (k * NWV + wave) * 1024));  // uniform
  };
  StgList<0, NST> stg;
  if constexpr (DMA)
    issue_chunk(0, lds);
  else
    stg.load([&](int k) { return piece(0, k); });
  for (int i = tid; i < HID; i += 64 * NWV) b1s[i] = p.b1[i];
  for (int i = tid; i < C; i += 64 * NWV) b2s[i] = p.b2[i];

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
    s = xsum16_32(s);  // permlane swaps (lanes.h), the butterfly's pairs
    const float mean = s / (float)C;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[ks][e] - mean;
        q += d * d;
      }
    q = xsum16_32(q);
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
  if constexpr (DMA)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else
    stg.store([&](int k, const uint4& v) { *reinterpret_cast<uint4*>(lds + pdst(k)) = v; });
  __syncthreads();

  floatx4 acc2[NCT][TT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) acc2[ct][tt] = floatx4{0.f, 0.f, 0.f, 0.f};

  // the residual rows of the epilogue, loaded at the start of the last chunk so that their
  // HBM round trip runs under its GEMMs (lane (g, j): 4 consecutive channels of row j)
  floatx4 xres[NCT][TT];
  for (int jc = 0; jc < NCH; ++jc) {
    const bool more = jc + 1 < NCH;
    if (PRERES && !more) {
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        const long row = min(row0 + tt * 16 + j16, p.M - 1);
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          xres[ct][tt] = *reinterpret_cast<const floatx4*>(p.X + (size_t)row * C + ct * 16 + 4 * g);
      }
    }
    if (more) {
      if constexpr (DMA && NBUF == 2)
        issue_chunk(jc + 1, lds + ((jc + 1) & 1) * BUF);
      else if constexpr (!DMA)
        stg.load([&](int k) { return piece(jc + 1, k); });
    }
    const char* w1s = lds + (NBUF == 2 ? (jc & 1) * BUF : 0);
    const char* w2s = w1s + PL * W1B;
    // GEMM 1: hidden^T [NC x 16TT] = W1[chunk] . LN(x)^T (b1 as the accumulator input, as in
    // mlp384_kernel, measured slower here: s2.mlp 4.55-4.59 vs 4.41-4.43 ms, profiles/r05/r07c)
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

    if constexpr (C == 192) {
      // bias + GELU of hidden tiles 2p, 2p+1 (GEMM 2's B fragment p) next to GEMM 2's k-step
      // p, without a priority bracket, so the scheduler overlaps the GELU of p + 1 with the
      // MFMAs of p: s2.mlp 793 -> 759 us per block pair; at C = 96 it measured 2.7 % slower
      // (profiles/r02/ab_mlp_interleave.log)
#pragma unroll
      for (int kp = 0; kp < KP; ++kp) {
        bf16x8 hb[TT][PL];
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
          const float* bb = b1s + jc * NC + 32 * kp + 4 * g;
          float h[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            h[r] = gelu2_erf_fast(acc1[2 * kp][tt][r] + bb[r]);
            h[4 + r] = gelu2_erf_fast(acc1[2 * kp + 1][tt][r] + bb[16 + r]);
          }
          bf16x8 hi, lo;
          pack8(h, hi, lo);
          hb[tt][0] = hi;
          if constexpr (X3) hb[tt][PL - 1] = lo;
        }
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          const int r = ct * 16 + j16;
          const int o = r * (NC * 2) + ((4 * kp + g) ^ ((r >> SH2) & (RB - 1))) * 16;
          const bf16x8 ah = *reinterpret_cast<const bf16x8*>(w2s + o);
          bf16x8 al = ah;
          if constexpr (X3) al = *reinterpret_cast<const bf16x8*>(w2s + W2B + o);
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) {
            acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, hb[tt][0], acc2[ct][tt], 0, 0, 0);
            if constexpr (X3) {
              acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, hb[tt][1], acc2[ct][tt], 0, 0, 0);
              acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, hb[tt][0], acc2[ct][tt], 0, 0, 0);
            }
          }
        }
      }
    } else {
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
            h[r] = gelu2_erf_fast(acc1[2 * kp][tt][r] + bb[r]);
            h[4 + r] = gelu2_erf_fast(acc1[2 * kp + 1][tt][r] + bb[16 + r]);
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
          const int o = r * (NC * 2) + ((4 * kp + g) ^ ((r >> SH2) & (RB - 1))) * 16;
          const bf16x8 ah = *reinterpret_cast<const bf16x8*>(w2s + o);
          bf16x8 al = ah;
          if constexpr (X3) al = *reinterpret_cast<const bf16x8*>(w2s + W2B + o);
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
    }
    // the other buffer was last read in chunk jc - 1, before the barrier that ended it
    if (DMA && NBUF == 1) {
      // one buffer: every wave is done with chunk jc before chunk jc + 1 lands in its place
      if (more) {
        __syncthreads();
        issue_chunk(jc + 1, lds);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk jc + 1 landed (this wave's pieces)
    } else if (more) {
      if constexpr (NBUF == 1) __syncthreads();  // every wave is done with the one buffer
      char* buf = lds + (NBUF == 2 ? ((jc + 1) & 1) * BUF : 0);
      stg.store([&](int k, const uint4& v) { *reinterpret_cast<uint4*>(buf + pdst(k)) = v; });
    }
    __syncthreads();  // chunk jc + 1 visible; buffer jc & 1 free
  }

  // x += out + b2 (4 consecutive channels of one row per lane and tile)
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const long row = row0 + tt * 16 + j16;
    if (row >= p.M) continue;
    if constexpr (!PRERES) {  // a row tile's loads all before its first store
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        xres[ct][tt] = *reinterpret_cast<const floatx4*>(p.X + (size_t)row * C + ct * 16 + 4 * g);
    }
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int ch = ct * 16 + 4 * g;
      float* xp = p.X + (size_t)row * C + ch;
      floatx4 x = xres[ct][tt];
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = x[r] + (acc2[ct][tt][r] + b2s[ch + r]);
      *reinterpret_cast<floatx4*>(xp) = x;
    }
  }
}

// ---------------------------------------------------------------- stage 3 (C = 384)
// The stage-1/2 kernel above keeps a whole W1 | W2 chunk double-buffered in LDS and
// stages it through registers.  At C = 384 a 32-unit chunk is 96 KB (hi + lo), and the
// LN'd rows (B fragments) plus the output accumulators of 128 rows take 384 registers
// per lane of a 4-wave workgroup, so this kernel runs one wave per SIMD (512 registers:
// 32 rows per wave) and fills its weight buffers by LDS-DMA (global_load_lds, no
// staging VGPRs).  One W1 buffer and one W2 buffer (48 KB each) are refilled in
// alternation: W2(jc) lands while GEMM 1 of chunk jc reads W1(jc), W1(jc + 1) lands
// while GEMM 2 reads W2(jc); two raw barriers per chunk behind vmcnt(0) (each wave waits
// for its own DMA, the barrier publishes it; __syncthreads would add a fence).
//
// GEMM 2's k order: the stage-1/2 kernel takes GEMM 2's B fragment p from hidden tiles
// 2p, 2p+1 (lane group g: units 32p + 4g + r and 32p + 16 + 4g + r), which needs a
// permuted W2 image that a 16-B DMA cannot build.  Here W1's rows are permuted instead:
// LDS row u of chunk jc holds hidden unit jc*32 + pi(u), pi(16t + 4g + r) = 8g + 4t + r,
// so lane group g's accumulators of the two hidden tiles are units 8g .. 8g + 7 in
// order -- the B fragment over W2's natural k order.
//
// LDS images (per plane; the lo plane follows at +24 KB), both of 64-B rows:
//  - W1: [12 k-steps][32 units] x 32 channels;
//  - W2: [384 channels] x the chunk's 32 units;
// the 16-B chunk c of row v stored at c ^ f((v >> 2) & 3), f = {0, 2, 3, 1} (the GEMM
// ring kernel's swizzle: the fragment reads' lane groups hit 16 distinct 16-B slots),
// applied on the DMA's per-lane source address (the LDS side of a DMA is lane-linear).
// Every DMA source is a uniform base + one lane base + uniform offsets, and every
// fragment read one lane base + an immediate.
// LDS chunk images of the C = 384 kernels, packed once at load: piece `rem` (1 KB) of plane
// q of chunk jc at (jc * PL + q) * 24 KB + rem * 1024 + 16 * lane holds the 16 B that lane
// `lane`'s DMA of that piece gathered from the row-major planes, so the kernels' DMA reads
// 1 KB of contiguous memory per piece instead of 16 rows x 64 B.
//  - W1 image (lngemm384's W, mlp384's W1; [N, 384], 32-unit chunks): piece rem = 2 ks + h,
//    row jc*32 + 4 h + 8 g + (lane / 4) % 4, bytes ks*64 + 16 ((lane & 3) ^ f(lane / 4));
//  - W2 image (mlp384's W2 [384, 1536]), mode 1: piece pp, row perm384(16 pp + lane / 4),
//    bytes jc*64 + 16 ((lane & 3) ^ f(lane / 4)), halved (gelu2_erf_fast);
//  - W_proj image (mlp384<PROJ>'s W_proj [384, 384]), mode 2: as W2's over 384 input
//    channels, not halved.
__global__ void pack_img384_kernel(const char* __restrict__ hi, const char* __restrict__ lo, int nch, int mode,
                                   char* __restrict__ out) {
  constexpr int C = 384, HID = 4 * C, PLB = 32 * C * 2;
  const int lane = threadIdx.x & 63;
  const int rem = (int)(blockIdx.x % 24) ;
  const int q = (int)(blockIdx.x / 24) % (lo ? 2 : 1);
  const int jc = (int)(blockIdx.x / 24) / (lo ? 2 : 1);
  if (jc >= nch || threadIdx.x >= 64) return;
  const int g = lane >> 4;
  const int chunk16 = ((lane & 3) ^ swz4(lane >> 2)) << 4;
  size_t src;
  if (mode == 0) {
    const int ks = rem >> 1, h = rem & 1;
    src = (size_t)(jc * 32 + 4 * h + 8 * g + ((lane >> 2) & 3)) * (C * 2) + ks * 64 + chunk16;
  } else {
    src = (size_t)perm384(rem * 16 + (lane >> 2)) * ((mode == 1 ? HID : C) * 2) + jc * 64 + chunk16;
  }
  const char* plane = q ? lo : hi;
  const uint4 v = *reinterpret_cast<const uint4*>(plane + src);
  // W2: W2 / 2 (gelu2_erf_fast)
  *reinterpret_cast<uint4*>(out + ((size_t)jc * (lo ? 2 : 1) + q) * PLB + rem * 1024 + 16 * lane) =
      mode == 1 ? half_bf16x8(v) : v;
}

void pack_img384(const void* hi, const void* lo, int nch, int mode, void* out, hipStream_t s) {
  pack_img384_kernel<<<nch * (lo ? 2 : 1) * 24, 64, 0, s>>>(static_cast<const char*>(hi), static_cast<const char*>(lo),
                                                            nch, mode, static_cast<char*>(out));
  MOCR_HIP_CHECK(hipGetLastError());
}


// NW waves of 128 / NW rows each (TT = 8 / NW row tiles): 4 (one wave per SIMD, 512
// registers); an 8-wave form (two per SIMD of 16 rows) measured no faster (profiles/r05/r07i).
//
// PROJ (the stage-3 block tail as one row-tile kernel): the block's
// attention output projection, residual add and norm2 run here too --
//   x_mid = X + (O W_proj^T + b_proj),  X = x_mid + mlp(norm2(x_mid))
// (torchvision SwinTransformerBlock: x = x + attn(norm1(x)); x = x + mlp(norm2(x))).  O
// (the attention kernel's bf16 hi / lo planes in X's row order) is loaded as the B
// fragments GEMM 1 later takes from the LayerNorm; W_proj streams through the same LDS ring
// as 12 chunk images of 32 input channels (W2's image geometry, rows permuted the same way)
// ahead of W1(0); the proj accumulators land in GEMM 2's accumulators, so x_mid is formed
// in the LayerNorm's lane layout and GEMM 2 then accumulates on top of it.  X is read once
// and written once; the separate proj GEMM's write and the MLP's two re-reads of X are gone.
template <int PASSES, bool PROJ, int NW = 4>
__global__ void __launch_bounds__(64 * NW) mlp384_kernel(MlpParams p) {
  constexpr int C = 384, HID = 4 * C, NC = 32, NCH = HID / NC, KS1 = C / 32, NCT = C / 16, TT = 8 / NW;
  constexpr int NPJ = C / NC;  // proj chunk images (32 input channels each)
  constexpr bool X3 = PASSES == 3;
  constexpr int PL = X3 ? 2 : 1;
  constexpr int PLB = NC * C * 2;              // bytes of one plane of a W1, W2 or W_proj chunk (24 KB)
  constexpr int NPW = PL * (PLB / 1024) / NW;  // 1-KB DMA pieces per wave per matrix and chunk
  static_assert(NPW * NW * 1024 == PL * PLB && NPW <= KS1 && 2 * NPW <= NCT, "DMA split");
  static_assert(NPJ % 3 == 0, "the proj chunks leave the ring's slot numbering of the MLP chunks unchanged");
  // a ring of three half-chunk slots (W1(0), W2(0), W1(1), ... in turn; PROJ: W_proj's 12
  // chunks first): two in flight while the MFMAs read the third
  constexpr int SLOT = PL * PLB;
  __shared__ __attribute__((aligned(16))) char ring[3 * SLOT];
  __shared__ __attribute__((aligned(16))) float b1s[HID];
  __shared__ __attribute__((aligned(16))) float b2s[C];                 // b2[perm384(i)]
  __shared__ __attribute__((aligned(16))) float bps[PROJ ? C : 1];      // b_proj[perm384(i)]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: piece offsets in SGPRs
  const int j16 = lane & 15;
  const int g = lane >> 4;
  const long row0 = (long)blockIdx.x * 128 + wave * 16 * TT;
  // the packed chunk images (pack_img384): W1's chunks, then W2's, then (PROJ) W_proj's
  const char* w1g = static_cast<const char*>(p.wpack);
  const char* w2g = w1g + (size_t)NCH * SLOT;
  const char* wpg = w2g + (size_t)NCH * SLOT;

  // W1 piece (plane q, k-step ks, half h): LDS rows u = 16 h + lane / 4 of block ks, slot
  // lane % 4; row u is hidden unit pi(u) = 8 g + 4 h + (lane / 4) % 4 of the chunk, and
  // slot s holds the channel chunk s ^ f(g) of k-step ks.
  // W2 / W_proj piece (plane q, pp): LDS rows r = 16 pp + lane / 4 (output channels
  // perm384(r)), slot s holds the chunk's k 8 (s ^ f(g)) .. + 7.
  // Every image has one piece geometry: piece i of this wave's share of chunk jc at
  // (jc * SLOT + q * PLB + rem * 1024) + 16 lane, only the image base differs.
  const uint32_t lb1 = (uint32_t)(16 * lane);
  // (the empty asm makes the lane base look new in every call: hipcc would otherwise hoist
  // the 24 per-piece 64-bit addresses out of the chunk loop and spill them)
  // pieces [i0, i0 + n) of this wave's share (the chunk loops issue one piece per MFMA step:
  // a burst of 12 DMA instructions stalls the wave's issue, and its MFMAs with it)
  auto issue = [&](const char* base, int jc, char* dst, int i0, int n) __attribute__((always_inline)) {
    uint32_t lb = lb1;
    asm volatile("" : "+v"(lb));
#pragma unroll
    for (int i = i0; i < i0 + n; ++i) {
      // piece i of this wave: plane q = i / (NPW / PL) (compile-time), piece 4 (i % ..) + wave
      const int q = i / (NPW / PL);
      const int rem = (i - q * (NPW / PL)) * NW + wave;
      const uint32_t off = (uint32_t)(jc * SLOT + q * PLB + rem * 1024) + lb;
      dma16(base, off, lds_u32(dst) + q * PLB + rem * 1024);
    }
  };

  // ring item hc (the MLP's half chunks; PROJ's 12 proj chunks are items -12 .. -1):
  // W1(hc / 2) if even, W2(hc / 2) if odd, in slot hc % 3
  auto slot = [&](int hc) { return ring + ((hc + 3 * NPJ) % 3) * SLOT; };
  // fragment reads: row v = 16 t + j16 of a 64-B-row image, chunk g at g ^ f(j16 / 4)
  const int fo = j16 * 64 + ((g ^ swz4(j16)) << 4);

  bf16x8 xb[TT][KS1][PL];  // GEMM 1's B fragments (PROJ: first O's, the proj GEMM's)
  floatx4 acc2[NCT][TT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) acc2[ct][tt] = floatx4{0.f, 0.f, 0.f, 0.f};

  if constexpr (PROJ) {
    // O rows as B fragments (lane (g, j): row j of tile tt, channels 32 kc + 8 g .. + 7),
    // loaded before the first DMA so that the ring's vmcnt waits cover them
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      const long row = min(row0 + tt * 16 + j16, p.M - 1);
#pragma unroll
      for (int kc = 0; kc < KS1; ++kc)
#pragma unroll
        for (int q = 0; q < PL; ++q)
          xb[tt][kc][q] = *reinterpret_cast<const bf16x8*>((q ? p.att_lo : p.att_hi) + (size_t)row * C + 32 * kc + 8 * g);
    }
    issue(wpg, 0, slot(-NPJ), 0, NPW);
    issue(wpg, 1, slot(-NPJ + 1), 0, NPW);
  } else {
    issue(w1g, 0, slot(0), 0, NPW);
    issue(w2g, 0, slot(1), 0, NPW);
  }
  for (int i = tid; i < HID; i += 64 * NW) b1s[i] = p.b1[i];
  for (int i = tid; i < C; i += 64 * NW) b2s[i] = p.b2[perm384(i)];
  if constexpr (PROJ)
    for (int i = tid; i < C; i += 64 * NW) bps[i] = p.bproj[perm384(i)];

  // GEMM 2's loop body over one W2-geometry chunk in slot `ws`: out^T [384 x 32] +=
  // W[:, chunk] . B^T, one channel tile per step, the fragments read two tiles ahead,
  // one DMA piece of the item two ahead issued every other step
  auto gemm2 = [&](const char* ws, auto bf, const char* nbase, int njc, char* ndst, bool nxt)
                   __attribute__((always_inline)) {
    bf16x8 fb[3][PL];
    auto rd2 = [&](int ct, bf16x8(&f)[PL]) {
      const int o = fo + ct * 1024;
      f[0] = *reinterpret_cast<const bf16x8*>(ws + o);
      if constexpr (X3) f[PL - 1] = *reinterpret_cast<const bf16x8*>(ws + PLB + o);
    };
    rd2(0, fb[0]);
    rd2(1, fb[1]);
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      if (ct + 2 < NCT) rd2(ct + 2, fb[(ct + 2) % 3]);
      if (nxt && (ct & 1) == 0 && ct / 2 < NPW) issue(nbase, njc, ndst, ct / 2, 1);
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        const bf16x8 ah = fb[ct % 3][0];
        acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bf(tt, 0), acc2[ct][tt], 0, 0, 0);
        if constexpr (X3) {
          const bf16x8 al = fb[ct % 3][PL - 1];
          acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bf(tt, 1), acc2[ct][tt], 0, 0, 0);
          acc2[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bf(tt, 0), acc2[ct][tt], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if constexpr (PROJ) {
    // proj^T [384 x 32] = W_proj[perm rows, chunk kc] . O^T, chunk by chunk; item kc + 2 is
    // W_proj(kc + 2), then W1(0) and W2(0)
#pragma unroll
    for (int kc = 0; kc < NPJ; ++kc) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
      __builtin_amdgcn_s_barrier();
      const int it2 = kc + 2;  // the item two ahead
      const char* nb = it2 < NPJ ? wpg : (it2 == NPJ ? w1g : w2g);
      gemm2(slot(kc - NPJ), [&](int tt, int q) __attribute__((always_inline)) { return xb[tt][kc][q]; }, nb,
            it2 < NPJ ? it2 : 0, slot(it2 - NPJ), true);
    }
    __builtin_amdgcn_sched_barrier(0);
    // x_mid = X + (proj + b_proj) in the LayerNorm's lane layout: output tile ct, lane group
    // g, element r is channel perm384(16 ct + 4 g + r) = 32 (ct / 2) + 8 g + 4 (ct % 2) + r,
    // so tiles 2 ks, 2 ks + 1 are the channels GEMM 1's B fragment ks takes
    // (one row tile at a time, its 24 loads in flight together: the scheduling barriers
    // keep hipcc from hoisting the other tile's loads into this one's registers)
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      const long row = min(row0 + tt * 16 + j16, p.M - 1);
      const float* xr = p.X + (size_t)row * C + 8 * g;
      floatx4 x4[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) x4[ct] = *reinterpret_cast<const floatx4*>(xr + 32 * (ct >> 1) + 4 * (ct & 1));
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const floatx4 b4 = *reinterpret_cast<const floatx4*>(bps + 16 * ct + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc2[ct][tt][r] = x4[ct][r] + (acc2[ct][tt][r] + b4[r]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // LayerNorm(norm2) of this wave's TT x 16 rows into GEMM 1's B fragments (lane (g, j):
  // row j of tile tt, channels 32 ks + 8 g .. + 7); PROJ: from x_mid in acc2, which then
  // stays there as GEMM 2's accumulator input (the residual)
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    float v[KS1][8];
    if constexpr (PROJ) {
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[ks][e] = acc2[2 * ks + (e >> 2)][tt][e & 3];
    } else {
      const long row = min(row0 + tt * 16 + j16, p.M - 1);
      const float* xr = p.X + (size_t)row * C + 8 * g;
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
    }
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[ks][e];
    s = xsum16_32(s);
    const float mean = s / (float)C;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[ks][e] - mean;
        q += d * d;
      }
    q = xsum16_32(q);
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
    if constexpr (PROJ) __builtin_amdgcn_sched_barrier(0);  // (registers: one tile's LN at a time)
  }

  for (int jc = 0; jc < NCH; ++jc) {
    // W1(jc) landed (this wave's pieces; W2(jc)'s may stay in flight), then visible to all;
    // every wave is past GEMM 2 of chunk jc - 1, so its slot takes W1(jc + 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
    __builtin_amdgcn_s_barrier();
    const bool nxt = jc + 1 < NCH;
    char* s_w1n = slot(2 * jc + 2);
    char* s_w2n = slot(2 * jc + 3);
    const char* w1s = slot(2 * jc);
    const char* w2s = slot(2 * jc + 1);
    // GEMM 1: hidden^T [32 x 32] = W1[chunk, permuted rows] . LN(x)^T.  The fragments of
    // k-step ks + 1 are read while the MFMAs of ks run; the scheduling barriers keep hipcc
    // from hoisting every fragment read of the chunk to the top
    // b1 as the accumulator input: tile ht, lane group g holds units 8 g + 4 ht .. + 3
    floatx4 acc1[2][TT];
#pragma unroll
    for (int ht = 0; ht < 2; ++ht) {
      const floatx4 b4 = *reinterpret_cast<const floatx4*>(b1s + jc * NC + 8 * g + 4 * ht);
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) acc1[ht][tt] = b4;
    }
    bf16x8 fa[2][2][PL];
    auto rd1 = [&](int ks, bf16x8(&f)[2][PL]) {
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        const int o = fo + ks * 2048 + ht * 1024;
        f[ht][0] = *reinterpret_cast<const bf16x8*>(w1s + o);
        if constexpr (X3) f[ht][PL - 1] = *reinterpret_cast<const bf16x8*>(w1s + PLB + o);
      }
    };
    rd1(0, fa[0]);
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      if (ks + 1 < KS1) rd1(ks + 1, fa[(ks + 1) & 1]);
      if (nxt && ks < NPW) issue(w1g, jc + 1, s_w1n, ks, 1);
#pragma unroll
      for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
          const bf16x8 ah = fa[ks & 1][ht][0];
          acc1[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xb[tt][ks][0], acc1[ht][tt], 0, 0, 0);
          if constexpr (X3) {
            const bf16x8 al = fa[ks & 1][ht][PL - 1];
            acc1[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xb[tt][ks][1], acc1[ht][tt], 0, 0, 0);
            acc1[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, xb[tt][ks][0], acc1[ht][tt], 0, 0, 0);
          }
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    // W2(jc) landed and visible (W1(jc + 1)'s pieces may stay in flight); every wave is past
    // GEMM 1, so its slot takes W2(jc + 1)
    if (jc + 1 < NCH)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // bias + GELU: lane group g holds hidden units jc*32 + 8 g .. + 7 of row j (tile ht,
    // element r: unit 8 g + 4 ht + r), GEMM 2's B fragment
    bf16x8 hb[TT][PL];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      float h[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h[r] = gelu2_erf_fast(acc1[0][tt][r]);
        h[4 + r] = gelu2_erf_fast(acc1[1][tt][r]);
      }
      bf16x8 hi, lo;
      pack8(h, hi, lo);
      hb[tt][0] = hi;
      if constexpr (X3) hb[tt][PL - 1] = lo;
    }
    // GEMM 2: out^T [384 x 32] += W2[perm rows, chunk] . hidden^T
    gemm2(w2s, [&](int tt, int q) __attribute__((always_inline)) { return hb[tt][q]; }, w2g, jc + 1, s_w2n, nxt);
  }

  // out = x + mlp + b2 at channels perm384(16 ct + 4 g ..): 4 consecutive channels of one
  // row per lane and tile.  PROJ: acc2 already holds x_mid + mlp.  Otherwise a row tile's 24
  // loads are all issued before its first store (hipcc keeps a load behind an earlier store
  // to the same buffer: one HBM round trip per tile otherwise)
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const long row = row0 + tt * 16 + j16;
    if (row >= p.M) continue;
    float* xr = p.X + (size_t)row * C + 8 * g;
    floatx4 x[NCT];
    if constexpr (!PROJ) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) x[ct] = *reinterpret_cast<const floatx4*>(xr + 32 * (ct >> 1) + 4 * (ct & 1));
    }
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const floatx4 b4 = *reinterpret_cast<const floatx4*>(b2s + 16 * ct + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        x[ct][r] = PROJ ? acc2[ct][tt][r] + b4[r] : x[ct][r] + (acc2[ct][tt][r] + b4[r]);
      *reinterpret_cast<floatx4*>(xr + 32 * (ct >> 1) + 4 * (ct & 1)) = x[ct];
    }
  }
}


// ---------------------------------------------------------------- LayerNorm + Linear, C = 384
// out = LN(X) W^T + b for stage 3's norm1 + qkv over the image tokens at >= 128 images
// (torchvision SwinTransformerBlock norm1 -> ShiftedWindowAttention's qkv Linear; the
// attention itself is window_attention_mfma_kernel over `out`).  mlp384_kernel's design
// without GEMM 2: a wave's 16 TT LN'd rows stay in registers as B fragments, W streams
// through the same 3-slot LDS-DMA ring a 32-unit chunk at a time (W(jc + 2) issued one
// piece per k-step while the MFMAs read W(jc)), and every chunk's 32 output columns are
// stored as soon as they are done, so the output leaves in a steady stream instead of one
// burst per tile (the GEMM's epilogue), and the LN output never goes through HBM.
// Chunk rows are permuted as mlp384's W1 (row u = unit pi(u)), so lane group g holds
// units 8 g .. 8 g + 7 of the chunk: two 16-B stores per row tile.
template <int PASSES, int TT>
__global__ void __launch_bounds__(256) lngemm384_kernel(LnGemm384Params p) {
  constexpr int C = 384, NC = 32, KS1 = C / 32;
  constexpr bool X3 = PASSES == 3;
  constexpr int PL = X3 ? 2 : 1;
  constexpr int PLB = NC * C * 2;             // one plane of a chunk (24 KB)
  constexpr int NPW = PL * (PLB / 1024) / 4;  // 1-KB DMA pieces per wave and chunk
  constexpr int NST = 2 * TT;                 // output stores per wave and chunk
  static_assert(NPW * 4 * 1024 == PL * PLB && NPW <= KS1 && NPW + NST < 64, "DMA split");
  constexpr int SLOT = PL * PLB;
  __shared__ __attribute__((aligned(16))) char ring[3 * SLOT];
  __shared__ __attribute__((aligned(16))) float bs[kLnGemm384MaxN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j16 = lane & 15;
  const int g = lane >> 4;
  const int N = p.N;
  const int nch = N / NC;
  const long row0 = (long)blockIdx.x * 64 * TT + wave * 16 * TT;
  const char* wpk = static_cast<const char*>(p.wpk);  // the packed chunk images (pack_img384)

  // piece i of this wave (plane q = i / (NPW / PL)): LDS rows u = 16 h + lane / 4 of k-step
  // ks's block, unit pi(u) = 8 g + 4 h + (lane / 4) % 4, slot s holds channel chunk s ^ f(g)
  const uint32_t lb1 = (uint32_t)(16 * lane);
  auto issue = [&](int jc, char* ws, int i0, int n) {
    uint32_t lb = lb1;
    asm volatile("" : "+v"(lb));
#pragma unroll
    for (int i = i0; i < i0 + n; ++i) {
      const int q = i / (NPW / PL);
      const int rem = (i - q * (NPW / PL)) * 4 + wave;
      const uint32_t off = (uint32_t)(jc * SLOT + q * PLB + rem * 1024) + lb;
      dma16(wpk, off, lds_u32(ws) + q * PLB + rem * 1024);
    }
  };
  auto slot = [&](int jc) { return ring + (jc % 3) * SLOT; };
  issue(0, slot(0), 0, NPW);
  if (nch > 1) issue(1, slot(1), 0, NPW);
  for (int i = tid; i < N; i += 256) bs[i] = p.b ? p.b[i] : 0.f;

  // LayerNorm of this wave's TT x 16 rows into the B fragments (lane (g, j): row j of tile
  // tt, channels 32 ks + 8 g .. + 7); rows >= M repeat row M - 1 (their stores rewrite its
  // values, so every lane stores and the vmcnt counts below hold)
  bf16x8 xb[TT][KS1][PL];
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const long row = min(row0 + tt * 16 + j16, p.M - 1);
    // the row's 384 channels: X's row, or PatchMerging's gather [x(0,0), x(1,0), x(0,1),
    // x(1,1)] of 96 channels each (swin.hip MODE_MERGE; pixels past the map are zeros)
    const float* src[4];
    bool valid[4];
    if (p.merge_H) {
      const int Ho = (p.merge_H + 1) / 2, Wo = (p.merge_W + 1) / 2;
      const int bi = (int)(row / ((long)Ho * Wo));
      const int rem = (int)(row - (long)bi * Ho * Wo);
      const int oy = rem / Wo, ox = rem - oy * Wo;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int y = 2 * oy + (q & 1), x = 2 * ox + (q >> 1);
        valid[q] = y < p.merge_H && x < p.merge_W;
        src[q] = p.X + ((size_t)(bi * p.merge_H + min(y, p.merge_H - 1)) * p.merge_W + min(x, p.merge_W - 1)) * 96;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        valid[q] = true;
        src[q] = p.X + (size_t)row * C + 96 * q;
      }
    }
    float v[KS1][8];
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      const int ch = 32 * ks + 8 * g;
      const int q = ch / 96;  // lane-dependent piece
      const float* xr = (q == 0 ? src[0] : q == 1 ? src[1] : q == 2 ? src[2] : src[3]) + (ch - 96 * q);
      const bool ok = q == 0 ? valid[0] : q == 1 ? valid[1] : q == 2 ? valid[2] : valid[3];
      const floatx4 a = *reinterpret_cast<const floatx4*>(xr);
      const floatx4 b = *reinterpret_cast<const floatx4*>(xr + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[ks][e] = ok ? a[e] : 0.f;
        v[ks][4 + e] = ok ? b[e] : 0.f;
      }
    }
    float sm = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) sm += v[ks][e];
    sm = xsum16_32(sm);
    const float mean = sm / (float)C;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[ks][e] - mean;
        q += d * d;
      }
    q = xsum16_32(q);
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
    __builtin_amdgcn_sched_barrier(0);  // one row tile's 96 values live at a time
  }
  const int fo = j16 * 64 + ((g ^ swz4(j16)) << 4);
  size_t orow[TT];
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) orow[tt] = (size_t)min(row0 + tt * 16 + j16, p.M - 1) * N;

  // W(0) landed (W(1) may stay in flight), then visible to all
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
  __builtin_amdgcn_s_barrier();
  for (int jc = 0; jc < nch; ++jc) {
    const bool nxt = jc + 2 < nch;
    char* s_n = slot(jc + 2);
    const char* ws = slot(jc);
    floatx4 acc[2][TT];
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) acc[ht][tt] = floatx4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa[2][2][PL];
    auto rd = [&](int ks, bf16x8(&f)[2][PL]) {
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        const int o = fo + ks * 2048 + ht * 1024;
        f[ht][0] = *reinterpret_cast<const bf16x8*>(ws + o);
        if constexpr (X3) f[ht][PL - 1] = *reinterpret_cast<const bf16x8*>(ws + PLB + o);
      }
    };
    rd(0, fa[0]);
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      if (ks + 1 < KS1) rd(ks + 1, fa[(ks + 1) & 1]);
      if (nxt && ks < NPW) issue(jc + 2, s_n, ks, 1);
#pragma unroll
      for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
          const bf16x8 ah = fa[ks & 1][ht][0];
          acc[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xb[tt][ks][0], acc[ht][tt], 0, 0, 0);
          if constexpr (X3) {
            const bf16x8 al = fa[ks & 1][ht][PL - 1];
            acc[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xb[tt][ks][1], acc[ht][tt], 0, 0, 0);
            acc[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, xb[tt][ks][0], acc[ht][tt], 0, 0, 0);
          }
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    // + bias; lane group g: units jc*32 + 8 g + 4 ht + r of row j (tile tt)
    const int col = jc * NC + 8 * g;
    const floatx4 bb0 = *reinterpret_cast<const floatx4*>(bs + col);
    const floatx4 bb1 = *reinterpret_cast<const floatx4*>(bs + col + 4);
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      float* o = p.out + orow[tt] + col;
      // plain stores: the two 16-B halves of a lane's 32 B leave in two instructions, and
      // L2 merges them into whole lines (non-temporal stores wrote each 64-B segment twice:
      // WRITE_SIZE 1365 vs 680 MB per launch at B = 256)
      *reinterpret_cast<floatx4*>(o) = acc[0][tt] + bb0;
      *reinterpret_cast<floatx4*>(o + 4) = acc[1][tt] + bb1;
    }
    // W(jc + 1) landed: in issue order W(jc + 2) and stores(jc) may be outstanding behind
    // it (and stores(jc - 1) is waited for: a per-chunk count that differs in chunk 0 makes
    // hipcc peel it, 134 VGPRs spilled and 553 vs 499 us per launch at B = 256); then
    // visible to all, and every wave is past chunk jc, whose slot takes W(jc + 3)
    if (nxt)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW + NST) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    __builtin_amdgcn_s_barrier();
  }
}

// mlp_fused_kernel<C, TT, NC, PASSES, NWV>'s chunk images: chunk jc at jc * BUF in the LDS
// byte order, piece rem of plane q holding what mlp_piece_load gathers for it (one 64-lane
// block per piece; the kernel copies 1-KB blocks whatever its wave count).
template <int C, int NC, int PASSES>
struct MlpImage {
  static constexpr int PL = PASSES == 3 ? 2 : 1, RC = C / 8;
  static constexpr int SW1 = (RC % 16 == 0) ? 16 : ((RC % 8 == 0) ? 8 : 4), SH1 = SW1 == 16 ? 0 : 1;
  static constexpr int RB = NC / 8, SH2 = RB == 4 ? 1 : 0;
  static constexpr int W1B = NC * C * 2, W2B = C * NC * 2, DMA1 = W1B / 1024, DMA2 = W2B / 1024;
  static constexpr int NPIECE = PL * (DMA1 + DMA2), BUF = PL * (W1B + W2B), NCH = 4 * C / NC;
};
template <int C, int NC, int PASSES>
__global__ void __launch_bounds__(64) mlp_pack_kernel(MlpParams p, char* __restrict__ out) {
  using I = MlpImage<C, NC, PASSES>;
  const int lane = threadIdx.x;
  const int P = blockIdx.x % I::NPIECE;
  const int jc = blockIdx.x / I::NPIECE;
  const int q = P / (I::DMA1 + I::DMA2);
  const int rem = P - q * (I::DMA1 + I::DMA2);
  const uint4 v = mlp_piece_load<C, NC, I::DMA1, I::RC, I::SW1, I::SH1, I::RB, I::SH2>(p, jc, q, rem, lane);
  // pieces >= DMA1 are W2's: W2 / 2 (gelu2_erf_fast)
  *reinterpret_cast<uint4*>(out + (size_t)jc * I::BUF + mlp_piece_dst<I::PL, I::DMA1, I::W1B, I::W2B>(q, rem, lane)) =
      rem < I::DMA1 ? v : half_bf16x8(v);
}
template <int C, int NC>
void launch_pack_c(const MlpParams& p, void* out, hipStream_t s) {
  if (p.w1lo) {
    using I = MlpImage<C, NC, 3>;
    mlp_pack_kernel<C, NC, 3><<<I::NCH * I::NPIECE, 64, 0, s>>>(p, static_cast<char*>(out));
  } else {
    using I = MlpImage<C, NC, 1>;
    mlp_pack_kernel<C, NC, 1><<<I::NCH * I::NPIECE, 64, 0, s>>>(p, static_cast<char*>(out));
  }
}

template <int C, int TT, int NC, int NWV = 8, int NBUF = 2>
void launch_mlp_c(const MlpParams& p, hipStream_t s) {
  const unsigned grid = (unsigned)((p.M + 16 * NWV * TT - 1) / (16 * NWV * TT));
  if (p.w1lo && p.w2lo)
    mlp_fused_kernel<C, TT, NC, 3, NWV, NBUF><<<grid, 64 * NWV, 0, s>>>(p);
  else
    mlp_fused_kernel<C, TT, NC, 1, NWV, NBUF><<<grid, 64 * NWV, 0, s>>>(p);
}
// stage-1 MLP geometry: 4 waves (128 rows) per workgroup with 32-unit chunks (49 KB of LDS,
// 152 VGPRs: three workgroups per CU, whose LayerNorm prologues and residual epilogues
// overlap the others' chunk loops) instead of 8 waves with 64-unit chunks (100 KB, 256
// VGPRs, one per CU): 5.30-5.39 vs 5.72-5.75 ms per 512-image encode (profiles/r05/r06f).
// stage 2: 4-wave workgroups of 64 rows, one LDS buffer filled by LDS-DMA
constexpr int kS1MlpNWV = 4, kS2MlpNWV = 4;
constexpr int kS1MlpNC = kS1MlpNWV == 4 ? 32 : 64;

}  // namespace

bool mlp_fused_supported(int C) { return C == 96 || C == 192 || C == 384; }

void launch_lngemm384(const LnGemm384Params& p, hipStream_t s) {
  if (p.M <= 0) return;
  if (p.N <= 0 || p.N % 32 != 0 || p.N > kLnGemm384MaxN || !p.X || !p.w || !p.wpk || !p.out || !p.ln_g || !p.ln_b)
    throw std::runtime_error("lngemm384: N must be a multiple of 32 up to kLnGemm384MaxN, with every operand");
  if (p.merge_H && (p.merge_H < 1 || p.merge_W < 1 ||
                    p.M % ((long)((p.merge_H + 1) / 2) * ((p.merge_W + 1) / 2)) != 0))
    throw std::runtime_error("lngemm384: PatchMerging rows must be B x ceil(H/2) x ceil(W/2)");
  // 128 rows per workgroup (2 row tiles per wave, the LN rows in 192 of the 256 arch VGPRs;
  // the prologue spills, the chunk loop does not): 1152 workgroups at B = 256
  constexpr int TT = 2;
  const unsigned grid = (unsigned)((p.M + 64 * TT - 1) / (64 * TT));
  if (p.wlo)
    lngemm384_kernel<3, TT><<<grid, 256, 0, s>>>(p);
  else
    lngemm384_kernel<1, TT><<<grid, 256, 0, s>>>(p);
  MOCR_HIP_CHECK(hipGetLastError());
}

// hidden chunk NC per C as launch_mlp_fused runs the kernel; C = 384: W1's then W2's images
size_t mlp_pack_bytes(int C, bool x3) {
  if (C != 96 && C != 192 && C != 384) return 0;
  // PL x (W1 + W2) bf16, and at C = 384 the W_proj images of the PROJ kernel
  return (size_t)(x3 ? 2 : 1) * (4 * C * C * 2 + (C == 384 ? C * C : 0)) * 2;
}

void launch_lngemm384_pack(const void* w, const void* wlo, int N, void* out, hipStream_t s) {
  if (!w || !out || N <= 0 || N % 32 != 0 || N > kLnGemm384MaxN) throw std::runtime_error("lngemm384_pack: N % 32");
  pack_img384(w, wlo, N / 32, 0, out, s);
}

void launch_mlp_pack(const MlpParams& p, void* out, hipStream_t s) {
  if ((p.w1lo == nullptr) != (p.w2lo == nullptr) || !p.w1 || !p.w2 || !out)
    throw std::runtime_error("mlp_pack: planes");
  switch (p.C) {
    case 96: launch_pack_c<96, kS1MlpNC>(p, out, s); break;
    case 192: launch_pack_c<192, 32>(p, out, s); break;
    case 384: {
      const size_t img = (size_t)4 * 384 * 384 * 2 * (p.w1lo ? 2 : 1);  // W1's 48 chunk images
      pack_img384(p.w1, p.w1lo, 48, 0, out, s);
      pack_img384(p.w2, p.w2lo, 48, 1, static_cast<char*>(out) + img, s);
      // mlp384<PROJ>'s W_proj: 12 chunk images after W2's (mlp_pack_bytes counts them)
      if (p.wproj) pack_img384(p.wproj, p.wproj_lo, 12, 2, static_cast<char*>(out) + 2 * img, s);
      break;
    }
    default: throw std::runtime_error("mlp_pack: built for C = 96, 192, 384");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_mlp_fused(const MlpParams& p, hipStream_t s) {
  if (p.M <= 0) return;
  if ((p.w1lo == nullptr) != (p.w2lo == nullptr)) throw std::runtime_error("mlp: lo planes for both or neither");
  if (!p.wpack) throw std::runtime_error("mlp: packed chunk images (launch_mlp_pack) missing");
  switch (p.C) {
    // rows per wave 16 TT and hidden chunk NC measured best (TT = 1 at C = 96: 514 vs 420 us
    // per s1 block; TT = 2 at C = 192 spills)
    case 96: launch_mlp_c<96, 2, kS1MlpNC, kS1MlpNWV>(p, s); break;  // NC: launch_mlp_pack's chunks
    case 192: launch_mlp_c<192, 1, 32, kS2MlpNWV, kS2MlpNWV == 4 ? 1 : 2>(p, s); break;
    case 384: {
      const unsigned grid = (unsigned)((p.M + 127) / 128);
      const bool proj = p.att_hi != nullptr;
      if (proj && (!p.bproj || (p.att_lo == nullptr) != (p.w1lo == nullptr)))
        throw std::runtime_error("mlp384 proj: attention planes like the weights' and b_proj");
      if (p.w1lo) {
        if (proj) mlp384_kernel<3, true><<<grid, 256, 0, s>>>(p);
        else mlp384_kernel<3, false><<<grid, 256, 0, s>>>(p);
      } else {
        if (proj) mlp384_kernel<1, true><<<grid, 256, 0, s>>>(p);
        else mlp384_kernel<1, false><<<grid, 256, 0, s>>>(p);
      }
      break;
    }
    default: throw std::runtime_error("mlp: fused MLP built for C = 96, 192, 384");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
