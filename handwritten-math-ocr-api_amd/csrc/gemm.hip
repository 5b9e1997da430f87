// Encoder GEMMs on the gfx950 matrix cores.
//
// C[M,N] (op)= A[M,K] · W[N,K]^T + bias with fused epilogues (GELU, residual add,
// window-reverse + un-roll + crop + residual add).  These are every Linear of the
// Swin-T encoder (qkv, proj, mlp.0, mlp.3, reduction; torchvision
// shifted_window_attention / SwinTransformerBlock / PatchMerging) plus the memory
// projection (src/model_swin.py:37,45) and the per-layer cross-attention K/V
// projection of the decoder (torch/nn/functional.py _in_projection_packed), which
// the engine runs once per image instead of once per step.
//
// fp32 path: v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, 64 FLOP/clk/SIMD).
// Tile BM x BN x 32, 4 waves, each wave owns TM x TN blocks of 32x32.  A and W
// tiles are staged global -> registers -> LDS (rows padded to 36 floats so the
// 16-row ds_read_b128 groups hit 16 distinct slots); the next K-tile's global
// loads are issued before the current tile's MFMAs.  Within a 16-deep k chunk,
// lane half h feeds k = 8h + s at MFMA step s, so each lane reads 8 contiguous
// floats (two ds_read_b128) per operand instead of 8 scattered ones.
#include <cstdlib>

#include "kernels.h"

namespace mocr {

namespace {

constexpr int BK = 32;
constexpr int LDS_STRIDE = BK + 4;

// XCD-aware tile order (1-D grid): workgroups b and b+8 are dispatched to the same XCD,
// so logical tile L = (b % 8) * ceil(n/8) + b / 8 (bijective form for n % 8 != 0) gives
// each XCD a contiguous range of row-panel-major tiles, and the N-tiles that share an A
// row panel share that XCD's L2.  Placement only affects speed, never results.
__device__ __forceinline__ void tile_of(int gx, int& tx, int& ty) {
  const int n = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q = n >> 3, r = n & 7;
  const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  ty = L / gx;
  tx = L - ty * gx;
}

template <int EPI>
__device__ __forceinline__ void epi_store(const GemmParams& p, int row, int col, float v) {
  if (p.bias) v += p.bias[col];
  if constexpr (EPI == EPI_STORE) {
    if (p.col_split) {
      const int blk = col / p.col_split;
      p.C[blk * p.split_stride + (size_t)row * p.col_split + (col - blk * p.col_split)] = v;
    } else {
      p.C[(size_t)row * p.ldc + col] = v;
    }
  } else if constexpr (EPI == EPI_GELU) {
    p.C[(size_t)row * p.ldc + col] = gelu_erf(v);
  } else if constexpr (EPI == EPI_RESADD) {
    float* c = p.C + (size_t)row * p.ldc + col;
    *c = *c + v;
  } else {  // EPI_WINRES
    const WinGeom& g = p.win;
    const int per_img = g.nWin * kWinTok;
    const int b = row / per_img;
    const int rem = row - b * per_img;
    const int win = rem / kWinTok;
    const int tk = rem - win * kWinTok;
    const int wy = win / g.nWx;
    const int wx = win - wy * g.nWx;
    int y = wy * kWin + tk / kWin + g.sh;
    int x = wx * kWin + tk % kWin + g.sw;
    if (y >= g.pH) y -= g.pH;
    if (x >= g.pW) x -= g.pW;
    if (y < g.H && x < g.W) {
      float* c = p.C + ((size_t)(b * g.H + y) * g.W + x) * p.ldc + col;
      *c = *c + v;
    }
  }
}

template <int TM, int TN, int WGM, int WGN, int EPI>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_f32_kernel(GemmParams p) {
  constexpr int BM = 32 * TM * WGM;
  constexpr int BN = 32 * TN * WGN;
  constexpr int NT = 64 * WGM * WGN;
  constexpr int A_F4 = BM * BK / 4 / NT;
  constexpr int W_F4 = BN * BK / 4 / NT;
  static_assert(A_F4 * NT * 4 == BM * BK, "A tile split");
  static_assert(W_F4 * NT * 4 == BN * BK, "W tile split");

  __shared__ float lds[(BM + BN) * LDS_STRIDE];
  float* As = lds;
  float* Ws = lds + BM * LDS_STRIDE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN;
  const int wn = wave % WGN;
  int tx, ty;
  tile_of(p.N / BN, tx, ty);
  const int row0 = ty * BM;
  const int col0 = tx * BN;
  const float* A = static_cast<const float*>(p.A);
  const float* W = static_cast<const float*>(p.W);

  floatx4 ra[A_F4];
  floatx4 rw[W_F4];

  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int idx = tid + i * NT;
      const int r = idx >> 3;
      const int c = (idx & 7) * 4;
      const int gr = row0 + r;
      ra[i] = gr < p.M ? *reinterpret_cast<const floatx4*>(A + (size_t)gr * p.lda + k0 + c)
                       : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < W_F4; ++i) {
      const int idx = tid + i * NT;
      const int r = idx >> 3;
      const int c = (idx & 7) * 4;
      rw[i] = *reinterpret_cast<const floatx4*>(W + (size_t)(col0 + r) * p.ldw + k0 + c);
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int idx = tid + i * NT;
      *reinterpret_cast<floatx4*>(&As[(idx >> 3) * LDS_STRIDE + (idx & 7) * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < W_F4; ++i) {
      const int idx = tid + i * NT;
      *reinterpret_cast<floatx4*>(&Ws[(idx >> 3) * LDS_STRIDE + (idx & 7) * 4]) = rw[i];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gload(0);
  sstore();
  __syncthreads();

  const int half = lane >> 5;
  const int l32 = lane & 31;
  for (int k0 = 0; k0 < p.K; k0 += BK) {
    const bool more = k0 + BK < p.K;
    if (more) gload(k0 + BK);
#pragma unroll
    for (int kc = 0; kc < BK; kc += 16) {
      floatx4 a0[TM], a1[TM], b0[TN], b1[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* src = &As[(wm * 32 * TM + i * 32 + l32) * LDS_STRIDE + kc + 8 * half];
        a0[i] = *reinterpret_cast<const floatx4*>(src);
        a1[i] = *reinterpret_cast<const floatx4*>(src + 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* src = &Ws[(wn * 32 * TN + j * 32 + l32) * LDS_STRIDE + kc + 8 * half];
        b0[j] = *reinterpret_cast<const floatx4*>(src);
        b1[j] = *reinterpret_cast<const floatx4*>(src + 4);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[i][s], b0[j][s], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[i][s], b1[j][s], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (more) {
      sstore();
      __syncthreads();
    }
  }

#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + wm * 32 * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        const int col = col0 + wn * 32 * TN + j * 32 + l32;
        if (row < p.M) epi_store<EPI>(p, row, col, acc[i][j][r]);
      }
}

template <int TM, int TN, int WGM, int WGN>
void launch_tile(const GemmParams& p, hipStream_t s) {
  constexpr int BM = 32 * TM * WGM;
  constexpr int BN = 32 * TN * WGN;
  dim3 grid((p.N / BN) * ((p.M + BM - 1) / BM));
  dim3 block(64 * WGM * WGN);
  switch (p.epi) {
    case EPI_STORE: gemm_f32_kernel<TM, TN, WGM, WGN, EPI_STORE><<<grid, block, 0, s>>>(p); break;
    case EPI_GELU: gemm_f32_kernel<TM, TN, WGM, WGN, EPI_GELU><<<grid, block, 0, s>>>(p); break;
    case EPI_RESADD: gemm_f32_kernel<TM, TN, WGM, WGN, EPI_RESADD><<<grid, block, 0, s>>>(p); break;
    case EPI_WINRES: gemm_f32_kernel<TM, TN, WGM, WGN, EPI_WINRES><<<grid, block, 0, s>>>(p); break;
    default: throw std::runtime_error("gemm: bad epilogue");
  }
}

}  // namespace

void launch_gemm_f32(const GemmParams& p, hipStream_t s) {
  if (p.K % BK != 0) throw std::runtime_error("gemm_f32: K must be a multiple of 32");
  if (p.M <= 0) return;
  if (p.N % 128 == 0) {
    launch_tile<2, 2, 2, 2>(p, s);   // 128 x 128, 4 waves of 64 x 64
  } else if (p.N % 96 == 0) {
    launch_tile<1, 3, 4, 1>(p, s);   // 128 x 96, 4 waves of 32 x 96
  } else {
    throw std::runtime_error("gemm_f32: N must be a multiple of 96 or 128");
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

// ================================================================ bf16 MFMA path
// v_mfma_f32_16x16x32_bf16 with fp32 accumulate.  PASSES = 1: plain bf16 operands.
// PASSES = 3 ("bf16x3"): every fp32 operand x is carried as hi = bf16(x) and
// lo = bf16(x - hi) and the product is hi·hi + hi·lo + lo·hi (the dropped lo·lo term
// is ~2^-16 relative), i.e. near-fp32 accuracy on the bf16 matrix pipes.
// Tile BM x BN x 32, 4 waves (2 x 2), wave tile (16 TM) x (16 TN); A/W planes are
// staged global -> registers -> LDS with 80-B rows (16 rows of a ds_read_b128 group
// land on 16 distinct 16-B slots).  MFMA operand maps: lane l holds
// A[row l&15][k = 8(l>>4) + j], B[k][col l&15]; C/D: col = l&15, row = 4(l>>4) + r.
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

constexpr int BK16 = 32;

// GELU for the bf16 / bf16x3 epilogues: erf by Abramowitz & Stegun 7.1.26 (one
// reciprocal, one exp, 6 FMAs, no branches; |erf error| <= 1.5e-7, two orders below the
// bf16x3 products' ~1e-5).  The fp32 path keeps the library erff (gelu_erf).  The
// reciprocal is the 1-ulp v_rcp_f32: __frcp_rn expands to the ~10-instruction IEEE
// division sequence, which made this epilogue cost a fifth of s3.fc1's time.
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  const float e = 1.0f - poly * t * __expf(-z * z);  // erf(|x| / sqrt 2)
  return x * 0.5f * (1.0f + copysignf(e, x));
}

// Row-vector epilogue: 8 consecutive columns of one output row (col % 8 == 0), the same
// arithmetic as epi_store element by element, but 16/32-B loads and stores.
template <int EPI>
__device__ __forceinline__ void epi_vec8(const GemmParams& p, int row, int col, float (&v)[8]) {
  if constexpr (EPI == EPI_KV16) {  // int16 K/V: v already biased and quantised (stagq kernel)
    const int blk = col / p.col_split;
    const int c = col - blk * p.col_split;
    const int b = row / p.kv_M;
    const size_t o = blk * p.split_stride + ((size_t)(b * 2 + (c >> 8)) * 8 + ((c >> 5) & 7)) * p.kv_M * 32 +
                     (size_t)(row - b * p.kv_M) * 32 + (c & 31);
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = ((uint32_t)(int)v[2 * e] & 0xffffu) | ((uint32_t)(int)v[2 * e + 1] << 16);
    *reinterpret_cast<uint4*>(p.kv16 + o) = make_uint4(w[0], w[1], w[2], w[3]);
    return;
  }
  if (p.bias) {
    const floatx4 b0 = *reinterpret_cast<const floatx4*>(p.bias + col);
    const floatx4 b1 = *reinterpret_cast<const floatx4*>(p.bias + col + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] += b0[e];
      v[4 + e] += b1[e];
    }
  }
  if constexpr (EPI == EPI_RESRELU) {
    const size_t off = (size_t)row * p.ldc + col;
    float* c = p.C + off;
    const floatx4 r0 = *reinterpret_cast<const floatx4*>(c);
    const floatx4 r1 = *reinterpret_cast<const floatx4*>(c + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = fmaxf(r0[e] + v[e], 0.f);
      v[4 + e] = fmaxf(r1[e] + v[4 + e], 0.f);
    }
    *reinterpret_cast<floatx4*>(c) = floatx4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<floatx4*>(c + 4) = floatx4{v[4], v[5], v[6], v[7]};
    if (p.C16) {
      uint32_t hi[4], lo[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) split2_bf16(v[2 * e], v[2 * e + 1], hi[e], lo[e]);
      *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.C16) + off) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
      if (p.C16lo)
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.C16lo) + off) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    }
  } else if constexpr (EPI == EPI_RESADD || EPI == EPI_WINRES) {
    float* c;
    if constexpr (EPI == EPI_RESADD) {
      c = p.C + (size_t)row * p.ldc + col;
    } else {
      const WinGeom& g = p.win;
      const int per_img = g.nWin * kWinTok;
      const int b = row / per_img;
      const int rem = row - b * per_img;
      const int win = rem / kWinTok;
      const int tk = rem - win * kWinTok;
      const int wy = win / g.nWx;
      const int wx = win - wy * g.nWx;
      int y = wy * kWin + tk / kWin + g.sh;
      int x = wx * kWin + tk % kWin + g.sw;
      if (y >= g.pH) y -= g.pH;
      if (x >= g.pW) x -= g.pW;
      if (y >= g.H || x >= g.W) return;  // padding token: cropped
      c = p.C + ((size_t)(b * g.H + y) * g.W + x) * p.ldc + col;
    }
    floatx4 r0 = *reinterpret_cast<const floatx4*>(c);
    floatx4 r1 = *reinterpret_cast<const floatx4*>(c + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r0[e] = r0[e] + v[e];
      r1[e] = r1[e] + v[4 + e];
    }
    *reinterpret_cast<floatx4*>(c) = r0;
    *reinterpret_cast<floatx4*>(c + 4) = r1;
  } else {
    if constexpr (EPI == EPI_GELU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gelu_fast(v[e]);
    }
    if constexpr (EPI == EPI_RELU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    const size_t off = (size_t)row * p.ldc + col;
    if (EPI == EPI_STORE && p.kv24) {  // packed fp24 K/V, 8 columns of one head
      const int blk = col / p.col_split;
      const int c = col - blk * p.col_split;
      const int b = row / p.kv_M;
      const size_t o = blk * p.split_stride + ((size_t)(b * 2 + (c >> 8)) * 8 + ((c >> 5) & 7)) * p.kv_M * 32 +
                       (size_t)(row - b * p.kv_M) * 32 + (c & 31);
      st_fp24x4(p.kv24, o, floatx4{v[0], v[1], v[2], v[3]});
      st_fp24x4(p.kv24, o + 4, floatx4{v[4], v[5], v[6], v[7]});
    }
    if (p.C) {
      float* c = p.C + off;
      if (EPI == EPI_STORE && p.col_split) {
        const int blk = col / p.col_split;
        c = p.C + blk * p.split_stride + (size_t)row * p.col_split + (col - blk * p.col_split);
      }
      *reinterpret_cast<floatx4*>(c) = floatx4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<floatx4*>(c + 4) = floatx4{v[4], v[5], v[6], v[7]};
    }
    if (p.C16) {
      uint32_t hi[4], lo[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) split2_bf16(v[2 * e], v[2 * e + 1], hi[e], lo[e]);
      *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.C16) + off) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
      if (p.C16lo)
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.C16lo) + off) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    }
  }
}

// ---------------------------------------------------------------- LDS-DMA ring version
// The operand tiles go global -> LDS by global_load_lds (16 B per lane, no VGPR
// staging) into a 3-stage ring, so two k-tiles are in flight while the MFMAs consume a
// third.  One raw s_barrier per k-tile, with a counted vmcnt: the DMA of the newest
// tiles stays in flight across it (hipcc's __syncthreads would drain it).  Rows are
// 64 B (32 bf16); the 16-B chunk c of row r is stored at chunk c ^ f((r >> 2) & 3) with
// f = {0, 2, 3, 1}, applied on the DMA's per-lane source address (the LDS side of a
// DMA is lane-linear), which makes every ds_read_b128 lane group of the MFMA
// fragment reads hit 16 distinct 16-B slots.
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ int swz(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }  // {0,2,3,1}

template <int TM, int TN, int WGM, int WGN, int EPI, int PASSES, int NSTAGE, bool CONV = false>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_bf16_ring_kernel(GemmParams p) {
  constexpr int BM = 16 * TM * WGM;
  constexpr int BN = 16 * TN * WGN;
  constexpr int NW = WGM * WGN;
  // PASSES 13: bf16x3 as one bf16 GEMM over concatenated operands, K' = 3K:
  // A' = [A_hi | A_hi | A_lo], W' = [W_hi | W_lo | W_hi] (one LDS plane, one MFMA per step).
  // Measured slower than the two-plane form on every encoder shape except K = 96 (it
  // moves 1.5x the operand bytes through the CU's L2 path), so no launcher selects it.
  constexpr bool KC = PASSES == 13;
  constexpr int PL = PASSES == 3 ? 2 : 1;
  constexpr int ROWB = BK16 * 2;                 // 64 B per tile row
  constexpr int A_BYTES = BM * ROWB, W_BYTES = BN * ROWB;
  constexpr int STAGE = PL * (A_BYTES + W_BYTES);
  static_assert(NSTAGE >= 2 && NSTAGE <= 4, "ring depth");
  // 1-KB DMA pieces (16 rows) per wave per plane; when the pieces do not split evenly
  // (BN = 96: 6 over 4 waves) the spare slots re-load the last piece, identical bytes to
  // the same LDS place, so every wave issues the same count and one vmcnt fits all
  constexpr int A_DMA = (BM / 16 + NW - 1) / NW;
  constexpr int W_DMA = (BN / 16 + NW - 1) / NW;
  constexpr int DMA_PER_TILE = PL * (A_DMA + W_DMA);  // per wave

  // epilogue: each wave transposes its accumulators through a private LDS slab, 32 rows
  // of its 16*TN columns at a time (row stride padded by 4 floats)
  constexpr int EW = 16 * TN, ES = EW + 4, ER = 32;
  constexpr int EPI_BYTES = NW * ER * ES * 4;
  static_assert(TM % 2 == 0 && (ER * EW / 8) % 64 == 0, "epilogue split");
  __shared__ __attribute__((aligned(16))) char lds[NSTAGE * STAGE > EPI_BYTES ? NSTAGE * STAGE : EPI_BYTES];
  const char* Ag[2] = {static_cast<const char*>(p.A), static_cast<const char*>(p.A_lo)};
  const char* Wg[2] = {static_cast<const char*>(p.W), static_cast<const char*>(p.W_lo)};

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN;
  const int wn = wave % WGN;
  int tx, ty;
  tile_of(p.N / BN, tx, ty);
  const int row0 = ty * BM;
  const int col0 = tx * BN;
  const int nk = (KC ? 3 : 1) * p.K / BK16;

  // per-lane DMA source: piece row = 16*piece + lane/4, chunk lane%4 (swizzled)
  const int prow = lane >> 2;
  const int pch = lane & 3;
  // implicit-GEMM conv: this lane's output pixel per A piece -> input origin (iy0, ix0)
  int cv_b[A_DMA], cv_iy[A_DMA], cv_ix[A_DMA];
  if constexpr (CONV) {
    const ConvGeom& g = p.conv;
#pragma unroll
    for (int i = 0; i < A_DMA; ++i) {
      const int pc = min(wave * A_DMA + i, BM / 16 - 1);
      const int gr = row0 + pc * 16 + prow;
      const int hw = g.Hout * g.Wout;
      const int b = gr / hw;
      const int rem = gr - b * hw;
      const int oy = rem / g.Wout;
      cv_b[i] = gr < p.M ? b : -1;
      cv_iy[i] = oy * g.stride - g.pad;
      cv_ix[i] = (rem - oy * g.Wout) * g.stride - g.pad;
    }
  }
  auto issue = [&](int kt) {
    char* st = lds + (kt % NSTAGE) * STAGE;
    int kel = kt * BK16;  // k within the (segment's) operand
    int seg = 0;
    if constexpr (KC) {
      seg = kel / p.K;
      kel -= seg * p.K;
    }
    const int kb = kel * 2;
    const char* Aseg = KC ? Ag[seg == 2 ? 1 : 0] : nullptr;
    const char* Wseg = KC ? Wg[seg == 1 ? 1 : 0] : nullptr;
    int ky = 0, kx = 0, c0 = 0;
    if constexpr (CONV) {
      const int k0 = kel;
      const int tap = k0 / p.conv.Cin;
      c0 = k0 - tap * p.conv.Cin;
      ky = tap / p.conv.ks;
      kx = tap - ky * p.conv.ks;
    }
#pragma unroll
    for (int q = 0; q < PL; ++q) {
#pragma unroll
      for (int i = 0; i < A_DMA; ++i) {
        const int pc = min(wave * A_DMA + i, BM / 16 - 1);
        const int r = pc * 16 + prow;
        const char* src;
        if constexpr (CONV) {
          const ConvGeom& g = p.conv;
          const int iy = cv_iy[i] + ky, ix = cv_ix[i] + kx;
          const bool ok = cv_b[i] >= 0 && iy >= 0 && iy < g.Hin && ix >= 0 && ix < g.Win;
          src = ok ? (KC ? Aseg : Ag[q]) + ((((size_t)cv_b[i] * g.Hin + iy) * g.Win + ix) * g.Cin + c0) * 2 +
                         16 * (pch ^ swz(r))
                   : static_cast<const char*>(p.zero) + 16 * pch;
        } else {
          const int gr = min(row0 + r, p.M - 1);
          src = (KC ? Aseg : Ag[q]) + (size_t)gr * p.lda * 2 + kb + 16 * (pch ^ swz(r));
        }
        __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(st + q * A_BYTES + pc * 1024), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < W_DMA; ++i) {
        const int pc = min(wave * W_DMA + i, BN / 16 - 1);
        const int r = pc * 16 + prow;
        const char* src = (KC ? Wseg : Wg[q]) + (size_t)(col0 + r) * p.ldw * 2 + kb + 16 * (pch ^ swz(r));
        __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(st + PL * A_BYTES + q * W_BYTES + pc * 1024), 16, 0, 0);
      }
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int k = 0; k < NSTAGE - 1 && k < nk; ++k) issue(k);
  const int l16 = lane & 15;
  const int kq = lane >> 4;  // 16-B chunk of the fragment (k = 8*kq .. 8*kq+7)
  for (int kt = 0; kt < nk; ++kt) {
    // retire tile kt's DMA (tile kt+1's may stay in flight), then make it visible to all waves
    // tiles kt+1 .. kt+NSTAGE-2 may stay in flight
    const int ahead = min(NSTAGE - 2, nk - 1 - kt);
    if (NSTAGE >= 4 && ahead >= 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DMA_PER_TILE) : "memory");
    } else if (NSTAGE >= 3 && ahead >= 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_TILE) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    // into the stage every wave finished reading before the barrier
    if (kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1);
    const char* st = lds + (kt % NSTAGE) * STAGE;
    bf16x8 a[PL][TM], b[PL][TN];
#pragma unroll
    for (int q = 0; q < PL; ++q) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * 16 * TM + i * 16 + l16;
        a[q][i] = *reinterpret_cast<const bf16x8*>(st + q * A_BYTES + r * ROWB + 16 * (kq ^ swz(r)));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * 16 * TN + j * 16 + l16;
        b[q][j] = *reinterpret_cast<const bf16x8*>(st + PL * A_BYTES + q * W_BYTES + r * ROWB + 16 * (kq ^ swz(r)));
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
        if constexpr (PASSES == 3) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
        }
      }
  }

  __builtin_amdgcn_s_barrier();  // every wave is done reading the ring; no DMA in flight
  float* ep = reinterpret_cast<float*>(lds) + wave * ER * ES;
#pragma unroll
  for (int h = 0; h < TM / 2; ++h) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ep[(i2 * 16 + 4 * kq + r) * ES + j * 16 + l16] = acc[2 * h + i2][j][r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < ER * EW / 8 / 64; ++it) {
      const int idx = it * 64 + lane;
      const int rr = idx / (EW / 8);
      const int cc = idx - rr * (EW / 8);
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(ep + rr * ES + cc * 8);
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(ep + rr * ES + cc * 8 + 4);
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const int row = row0 + wm * 16 * TM + h * 32 + rr;
      if (row < p.M) epi_vec8<EPI>(p, row, col0 + wn * EW + cc * 8, v);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <int TM, int TN, int WGM, int WGN, int PASSES, int RING>
void launch_tile16(const GemmParams& p, hipStream_t s) {
  constexpr int BM = 16 * TM * WGM;
  constexpr int BN = 16 * TN * WGN;
  dim3 grid((p.N / BN) * ((p.M + BM - 1) / BM));
  dim3 block(64 * WGM * WGN);
#define MOCR_G16(E) gemm_bf16_ring_kernel<TM, TN, WGM, WGN, E, PASSES, RING><<<grid, block, 0, s>>>(p);
  switch (p.epi) {
    case EPI_STORE: MOCR_G16(EPI_STORE); break;
    case EPI_GELU: MOCR_G16(EPI_GELU); break;
    case EPI_RESADD: MOCR_G16(EPI_RESADD); break;
    case EPI_WINRES: MOCR_G16(EPI_WINRES); break;
    default: throw std::runtime_error("gemm_bf16: bad epilogue");
  }
#undef MOCR_G16
}

// Implicit-GEMM convolutions (ResNet18 3x3 / 1x1): the ring kernel with the conv A
// loader; Cout = 64 uses a 128 x 64 tile.
template <int TM, int TN, int PASSES>
void launch_conv_tile(const GemmParams& p, hipStream_t s) {
  constexpr int BM = 16 * TM * 2, BN = 16 * TN * 2;
  const dim3 grid((p.N / BN) * ((p.M + BM - 1) / BM));
  switch (p.epi) {
    case EPI_STORE: gemm_bf16_ring_kernel<TM, TN, 2, 2, EPI_STORE, PASSES, 2, true><<<grid, 256, 0, s>>>(p); break;
    case EPI_RELU: gemm_bf16_ring_kernel<TM, TN, 2, 2, EPI_RELU, PASSES, 2, true><<<grid, 256, 0, s>>>(p); break;
    case EPI_RESRELU:
      gemm_bf16_ring_kernel<TM, TN, 2, 2, EPI_RESRELU, PASSES, 2, true><<<grid, 256, 0, s>>>(p);
      break;
    default: throw std::runtime_error("conv: epilogue must be STORE, RELU or RESRELU");
  }
}

template <int PASSES>
void launch_conv_passes(const GemmParams& p, hipStream_t s) {
  if (p.N % 128 == 0)
    launch_conv_tile<4, 4, PASSES>(p, s);
  else if (p.N % 64 == 0)
    launch_conv_tile<4, 2, PASSES>(p, s);
  else
    throw std::runtime_error("conv: Cout must be a multiple of 64");
}

// ---------------------------------------------------------------- 256 x 256 staggered kernel
// 8 waves (wr = wave / 4: rows 128*wr.., wc = wave % 4: cols 64*wc..), each owning a
// 128 x 64 output = 4 quadrants of 64 x 32 (4 x 2 MFMA tiles).  A K-tile is 64 k (bf16)
// or 32 k in hi|lo planes (bf16x3): either way 128-B LDS rows, 32 KB of A + 32 KB of W,
// two buffers (128 KB).  Each K-tile runs 4 phases (one per quadrant), each phase a LOAD
// section (the quadrant's fragments by ds_read_b128, the next K-tile's DMA in phases
// 0-1, lgkmcnt(0)) and a COMPUTE section (the quadrant's MFMAs), separated by raw
// s_barriers.  Wave group 1 (wr = 1) starts one barrier late, so on every SIMD (one wave
// of each group) one wave's MFMAs run while the other loads.  Each group drains its
// DMA (vmcnt(0)) right before the barrier after which the other group first reads the
// buffer; every LOAD ends with lgkmcnt(0), so a buffer is refilled only after every
// wave's reads of it completed (the barrier that ends K-tile t-1's last LOAD).
// LDS row r holds global 16-B chunk c at chunk c ^ ((r >> 1) & 7): the 16 lanes of a
// ds_read_b128 group (16 consecutive rows, one chunk) hit 16 distinct slots.
__device__ __forceinline__ int swz8(int r) { return (r >> 1) & 7; }

template <int EPI, int PASSES>
__global__ void __launch_bounds__(512) gemm_bf16_stag_kernel(GemmParams p) {
  constexpr int BM = 256, BN = 256;
  constexpr bool X3 = PASSES == 3;
  constexpr int KT = X3 ? 32 : 64;        // k per K-tile
  constexpr int ROWB = 128;               // LDS row bytes
  constexpr int OPB = 256 * ROWB;         // one operand per buffer: 32 KB
  constexpr int BUF = 2 * OPB;            // A + W: 64 KB
  constexpr int EW = 64, ES = EW + 4, ER = 32;
  static_assert(8 * ER * ES * 4 <= 2 * BUF, "epilogue slab");
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2;
  const int wc = wave & 3;
  int tx, ty;
  tile_of(p.N / BN, tx, ty);
  const int row0 = ty * BM;
  const int col0 = tx * BN;
  const int nk = p.K / KT;
  const char* A0 = static_cast<const char*>(p.A);
  const char* A1 = static_cast<const char*>(X3 ? p.A_lo : p.A);
  const char* W0 = static_cast<const char*>(p.W);
  const char* W1 = static_cast<const char*>(X3 ? p.W_lo : p.W);

  // DMA: one glds instruction = 8 rows x 128 B; half-tile h (0,1: A rows 128h..; 2,3: W
  // rows 128(h-2)..) = 16 instructions, 2 per wave.  Lane: row +lane/8, chunk lane%8.
  const int drow = lane >> 3;
  const int dch = lane & 7;
  auto issue_half = [&](int kt, int h) {
    char* buf = lds + (kt & 1) * BUF + (h >> 1) * OPB;
    const int k0 = kt * KT;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (h & 1) * 128 + (wave * 2 + i) * 8 + drow;  // row within the operand tile
      const int sc = dch ^ swz8(r);                              // global chunk this lane fetches
      const char* src;
      if (h < 2) {
        const size_t gr = (size_t)min(row0 + r, p.M - 1);
        if constexpr (X3) src = (sc < 4 ? A0 : A1) + (gr * p.lda + k0 + 8 * (sc & 3)) * 2;
        else src = A0 + (gr * p.lda + k0 + 8 * sc) * 2;
      } else {
        const size_t gr = (size_t)(col0 + r);
        if constexpr (X3) src = (sc < 4 ? W0 : W1) + (gr * p.ldw + k0 + 8 * (sc & 3)) * 2;
        else src = W0 + (gr * p.ldw + k0 + 8 * sc) * 2;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(buf + ((h & 1) * 128 + (wave * 2 + i) * 8) * ROWB), 16, 0,
                                       0);
    }
  };

  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int l16 = lane & 15;
  const int kq = lane >> 4;
  // fragments of the current quadrant: A 4 row-tiles x 2 (k-steps or planes), W 2 x 2
  bf16x8 fa[4][2], fb[2][2];
  auto load_a = [&](const char* buf, int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wr * 128 + qm * 64 + i * 16 + l16;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        fa[i][s2] = *reinterpret_cast<const bf16x8*>(buf + r * ROWB + 16 * ((4 * s2 + kq) ^ swz8(r)));
    }
  };
  auto load_b = [&](const char* buf, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = wc * 64 + qn * 32 + j * 16 + l16;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        fb[j][s2] = *reinterpret_cast<const bf16x8*>(buf + OPB + r * ROWB + 16 * ((4 * s2 + kq) ^ swz8(r)));
    }
  };
  auto compute = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        floatx4& c = acc[qm * 4 + i][qn * 2 + j];
        if constexpr (X3) {  // planes: s2 = 0 hi, 1 lo
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
        } else {  // k-steps
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
        }
      }
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: K-tile 0 into buffer 0, visible to all; group 1 then falls one barrier behind
#pragma unroll
  for (int h = 0; h < 4; ++h) issue_half(0, h);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();

  // quadrant order (0,0) (0,1) (1,1) (1,0): A changes once, W every other phase
  for (int kt = 0; kt < nk; ++kt) {
    const char* buf = lds + (kt & 1) * BUF;
    const bool more = kt + 1 < nk;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int qm = (ph == 1 || ph == 2) ? (ph == 2 ? 1 : 0) : (ph == 3 ? 1 : 0);
      const int qn = (ph == 1 || ph == 2) ? 1 : 0;
      // LOAD
      if (ph == 0) {
        load_b(buf, 0);
        load_a(buf, 0);
      } else if (ph == 1) {
        load_b(buf, 1);
      } else if (ph == 2) {
        load_a(buf, 1);
      } else {
        load_b(buf, 0);
      }
      if (more && ph < 2) {
        issue_half(kt + 1, 2 * ph);
        issue_half(kt + 1, 2 * ph + 1);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (ph == 3 && wr == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // COMPUTE
      compute(qm, qn);
      if (ph == 3 && wr == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // pair group 1's extra barrier
  __builtin_amdgcn_s_barrier();

  // epilogue: per-wave LDS transpose, 32 rows x 64 columns per round
  float* ep = reinterpret_cast<float*>(lds) + wave * ER * ES;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ep[(i2 * 16 + 4 * kq + r) * ES + j * 16 + l16] = acc[2 * h + i2][j][r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < ER * EW / 8 / 64; ++it) {
      const int idx = it * 64 + lane;
      const int rr = idx / (EW / 8);
      const int cc = idx - rr * (EW / 8);
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(ep + rr * ES + cc * 8);
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(ep + rr * ES + cc * 8 + 4);
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const int row = row0 + wr * 128 + h * 32 + rr;
      if (row < p.M) epi_vec8<EPI>(p, row, col0 + wc * EW + cc * 8, v);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------- staggered kernel, whole rounds
// gemm_bf16_stag_kernel's schedule (two wave groups one barrier apart, LOAD / COMPUTE
// sections, counted DMA drains) for bf16x3 on BM x BN = 32 WTM x 64 WTN tiles: waves as
// 2 (rows) x 4 (cols), each owning WTM x WTN MFMA tiles of 16 x 16, computed in phases of
// PM x PN tiles visited in serpentine order, so a phase reloads only the A or only the W
// fragments.  The shapes are picked so the tile count fills whole rounds of the 256 CUs on
// the stage-3 GEMMs (M = 576 B, a multiple of 288): 288 x 256 on s3.fc1 is 768 tiles =
// 3 rounds (256 x 256: 864 tiles, a 4th round 38 % full), 288 x 192 on s3.fc2 / s3.proj
// 256 tiles = 1 round (128 x 128: 864 tiles).  Per output element the MFMA sequence is the
// other kernels' (hi·hi, hi·lo, lo·hi per 32-deep k-tile, k ascending), so the results
// are bitwise equal to theirs.
template <int EPI, int WTM, int WTN, int PM, int PN>
__global__ void __launch_bounds__(512) gemm_x3_stagq_kernel(GemmParams p) {
  constexpr int BM = 32 * WTM, BN = 64 * WTN;
  constexpr int KT = 32, ROWB = 128;  // one LDS row: 32 k of the hi plane | 32 k of the lo plane
  constexpr int A_B = BM * ROWB;
  constexpr int BUF = (BM + BN) * ROWB;
  constexpr int NPM = WTM / PM, NPN = WTN / PN, NPH = NPM * NPN;
  static_assert(NPM * PM == WTM && NPN * PN == WTN && NPH >= 2, "phase split");
  static_assert(BM % 16 == 0, "the W rows keep the A rows' swizzle phase");
  constexpr int PIECES = (BM + BN) / 8;   // one glds = 8 rows x 128 B
  constexpr int PPW = (PIECES + 7) / 8;   // per wave; spare slots repeat the last piece
  constexpr int PPH0 = (PPW + 1) / 2;     // issued in phase 0, the rest in phase 1
  constexpr int CR = WTM % 3 == 0 ? 3 : 2;  // epilogue: CR row tiles per slab round
  static_assert(WTM % CR == 0, "epilogue rounds");
  constexpr int EW = 16 * WTN, ES = EW + 4, ER = 16 * CR;
  constexpr int EV = ER * EW / 8;  // 8-float vectors per slab round per wave
  static_assert(8 * ER * ES * 4 <= 2 * BUF, "epilogue slab");
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2;
  const int wc = wave & 3;
  int tx, ty;
  tile_of(p.N / BN, tx, ty);
  const int row0 = ty * BM;
  const int col0 = tx * BN;
  const int nk = p.K / KT;
  const char* A0 = static_cast<const char*>(p.A);
  const char* A1 = static_cast<const char*>(p.A_lo);
  const char* W0 = static_cast<const char*>(p.W);
  const char* W1 = static_cast<const char*>(p.W_lo);

  // DMA piece pc = rows 8 pc .. 8 pc + 7 of the [A | W] image; lane: row + lane / 8,
  // LDS chunk lane % 8, which holds global chunk (lane % 8) ^ swz8(row)
  const int drow = lane >> 3;
  const int dch = lane & 7;
  const int lda = p.lda, ldw = p.ldw, M = p.M;
  // lo-plane offsets as integers: a select between two captured pointers put them in scratch
  const ptrdiff_t dA = A1 - A0, dW = W1 - W0;
  auto issue1 = [&](int kt, int i) {  // this wave's piece i of K-tile kt
    char* buf = lds + (kt & 1) * BUF;
    const int k0 = kt * KT;
    {
      const int pc = min(wave * PPW + i, PIECES - 1);
      const int r = pc * 8 + drow;
      const int sc = dch ^ swz8(r);
      const char* src;
      if (pc < BM / 8) {
        const size_t gr = (size_t)min(row0 + r, M - 1);
        src = A0 + (sc < 4 ? 0 : dA) + (gr * lda + k0 + 8 * (sc & 3)) * 2;
      } else {
        const size_t gr = (size_t)(col0 + r - BM);
        src = W0 + (sc < 4 ? 0 : dW) + (gr * ldw + k0 + 8 * (sc & 3)) * 2;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(buf + pc * 8 * ROWB), 16, 0, 0);
    }
  };

  floatx4 acc[WTM][WTN];
#pragma unroll
  for (int i = 0; i < WTM; ++i)
#pragma unroll
    for (int j = 0; j < WTN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int l16 = lane & 15;
  const int kq = lane >> 4;
  bf16x8 fa[PM][2], fb[PN][2];  // [tile][plane: 0 hi, 1 lo]
  auto load_a = [&](const char* buf, int qm) {
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      const int r = wr * (BM / 2) + (qm * PM + i) * 16 + l16;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        fa[i][s2] = *reinterpret_cast<const bf16x8*>(buf + r * ROWB + 16 * ((4 * s2 + kq) ^ swz8(r)));
    }
  };
  auto load_b = [&](const char* buf, int qn) {
#pragma unroll
    for (int j = 0; j < PN; ++j) {
      const int r = wc * EW + (qn * PN + j) * 16 + l16;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        fb[j][s2] = *reinterpret_cast<const bf16x8*>(buf + A_B + r * ROWB + 16 * ((4 * s2 + kq) ^ swz8(r)));
    }
  };

  // prologue: K-tile 0 into buffer 0, visible to all; group 1 then falls one barrier behind
#pragma unroll
  for (int i = 0; i < PPW; ++i) issue1(0, i);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < nk; ++kt) {
    const char* buf = lds + (kt & 1) * BUF;
    const bool more = kt + 1 < nk;
#pragma unroll
    for (int ph = 0; ph < NPH; ++ph) {
      const int qm = ph / NPN;
      const int qn = (qm & 1) ? NPN - 1 - ph % NPN : ph % NPN;  // serpentine
      // LOAD
      if (ph == 0) {
        load_b(buf, qn);
        load_a(buf, qm);
      } else if (ph % NPN == 0) {
        load_a(buf, qm);
      } else {
        load_b(buf, qn);
      }
      if (more) {
        if (ph == 0)
#pragma unroll
          for (int i = 0; i < PPH0; ++i) issue1(kt + 1, i);
        if (ph == 1)
#pragma unroll
          for (int i = PPH0; i < PPW; ++i) issue1(kt + 1, i);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (ph == NPH - 1 && wr == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // COMPUTE
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < PM; ++i)
#pragma unroll
        for (int j = 0; j < PN; ++j) {
          floatx4& c = acc[qm * PM + i][qn * PN + j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
        }
      __builtin_amdgcn_s_setprio(0);
      if (ph == NPH - 1 && wr == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // pair group 1's extra barrier
  __builtin_amdgcn_s_barrier();

  if constexpr (EPI == EPI_KV16) {
    static_assert(BM == 288, "each wave's 144 rows are one image");
    {
      // int16 K/V: this wave's 144 rows are one image; per column, the bias is added, the
      // max |value| over the image's rows taken (lanes l16 + 16 kq) and the values quantised
      const int img_row = row0 + wr * (BM / 2);
#pragma unroll
      for (int j = 0; j < WTN; ++j) {
        const int col = col0 + wc * EW + j * 16 + l16;
        const float bj = p.bias ? p.bias[col] : 0.f;
        float m = 0.f, nan = 0.f;
#pragma unroll
        for (int i = 0; i < WTM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc[i][j][r] += bj;
            m = fmaxf(m, fabsf(acc[i][j][r]));  // fmaxf drops NaN operands: tracked apart
            nan = acc[i][j][r] != acc[i][j][r] ? 1.f : nan;
          }
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        nan = fmaxf(nan, __shfl_xor(nan, 16, 64));
        nan = fmaxf(nan, __shfl_xor(nan, 32, 64));
        const float inv = m > 0.f ? 32767.f / m : 0.f;
        if (kq == 0 && img_row < M) {
          const int blk = col / p.col_split;
          // a NaN anywhere in the column makes its scale NaN, so it reaches the logits and the
          // engine's non-finite check as on the fp32 / fp24 paths (inf gives an inf scale)
          p.kv16_scale[blk * p.kv16_sstride + (size_t)(img_row / p.kv_M) * p.col_split + (col - blk * p.col_split)] =
              nan != 0.f ? __builtin_nanf("") : (m > 0.f ? m / 32767.f : 1.f);
        }
#pragma unroll
        for (int i = 0; i < WTM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = fminf(fmaxf(rintf(acc[i][j][r] * inv), -32767.f), 32767.f);
      }
    }
  }

  // epilogue: per-wave LDS transpose, ER rows x EW columns per round
  float* ep = reinterpret_cast<float*>(lds) + wave * ER * ES;
#pragma unroll
  for (int h = 0; h < WTM / CR; ++h) {
#pragma unroll
    for (int i2 = 0; i2 < CR; ++i2)
#pragma unroll
      for (int j = 0; j < WTN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ep[(i2 * 16 + 4 * kq + r) * ES + j * 16 + l16] = acc[h * CR + i2][j][r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < (EV + 63) / 64; ++it) {
      const int idx = it * 64 + lane;
      if (EV % 64 == 0 || idx < EV) {
        const int rr = idx / (EW / 8);
        const int cc = idx - rr * (EW / 8);
        const floatx4 v0 = *reinterpret_cast<const floatx4*>(ep + rr * ES + cc * 8);
        const floatx4 v1 = *reinterpret_cast<const floatx4*>(ep + rr * ES + cc * 8 + 4);
        float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        const int row = row0 + wr * (BM / 2) + h * ER + rr;
        if (row < M) epi_vec8<EPI>(p, row, col0 + wc * EW + cc * 8, v);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <int WTM, int WTN, int PM, int PN>
void launch_stagq(const GemmParams& p, hipStream_t s) {
  constexpr int BM = 32 * WTM, BN = 64 * WTN;
  const dim3 grid((unsigned)((p.N / BN) * ((p.M + BM - 1) / BM)));
  switch (p.epi) {
    case EPI_STORE: gemm_x3_stagq_kernel<EPI_STORE, WTM, WTN, PM, PN><<<grid, 512, 0, s>>>(p); break;
    case EPI_GELU: gemm_x3_stagq_kernel<EPI_GELU, WTM, WTN, PM, PN><<<grid, 512, 0, s>>>(p); break;
    case EPI_RESADD: gemm_x3_stagq_kernel<EPI_RESADD, WTM, WTN, PM, PN><<<grid, 512, 0, s>>>(p); break;
    case EPI_WINRES: gemm_x3_stagq_kernel<EPI_WINRES, WTM, WTN, PM, PN><<<grid, 512, 0, s>>>(p); break;
    case EPI_KV16:
      if constexpr (WTM == 9 && WTN == 4) {
        gemm_x3_stagq_kernel<EPI_KV16, WTM, WTN, PM, PN><<<grid, 512, 0, s>>>(p);
        break;
      }
      [[fallthrough]];
    default: throw std::runtime_error("gemm_bf16: bad epilogue");
  }
}

// Staggered 256 x 256 kernel: measured (B=64, 384²) faster than the ring kernels on bf16x3
// GEMMs with K <= N and at least 384 tiles (s3.fc1 225 -> 217 us, s4.fc1 163 -> 154),
// slower with K > N or fewer tiles and in plain bf16.
constexpr long kBigMinTiles = 384;
template <int PASSES>
bool try_stag(const GemmParams& p, hipStream_t s) {
  if (PASSES != 3 || p.K > p.N || p.N % 256 != 0 || p.K % 32 != 0) return false;
  const long tiles = (long)((p.M + 255) / 256) * (p.N / 256);
  if (tiles < kBigMinTiles) return false;
  const dim3 grid((unsigned)tiles);
  switch (p.epi) {
    case EPI_STORE: gemm_bf16_stag_kernel<EPI_STORE, PASSES><<<grid, 512, 0, s>>>(p); break;
    case EPI_GELU: gemm_bf16_stag_kernel<EPI_GELU, PASSES><<<grid, 512, 0, s>>>(p); break;
    case EPI_RESADD: gemm_bf16_stag_kernel<EPI_RESADD, PASSES><<<grid, 512, 0, s>>>(p); break;
    case EPI_WINRES: gemm_bf16_stag_kernel<EPI_WINRES, PASSES><<<grid, 512, 0, s>>>(p); break;
    default: throw std::runtime_error("gemm_bf16: bad epilogue");
  }
  return true;
}

// 256-row tiles: 8 waves as 2 (M) x 4 (N), each 128 x 16*TN, 2-stage ring (bf16x3: 2 x
// 64 KB of LDS, 1 block per CU).  Half the operand re-reads per MFMA of the 128-row
// tiles, but one k-tile in flight at one block per CU: measured (B=64, 384²) faster on
// bf16x3 GEMMs with K <= N (s1.fc1 435 -> 393 us, s2.qkv 212 -> 174, s2.fc1 276 -> 237,
// s4.qkv 149 -> 136) and slower with K > N (s2.fc2 232 -> 257, s3.fc2 180 -> 191) and in
// plain bf16.  Used for bf16x3 with K <= N and >= kBigMinTiles tiles.
template <int TN, int PASSES>
void launch_big_tile(const GemmParams& p, hipStream_t s) {
  constexpr int BM = 256, BN = 64 * TN;
  const dim3 grid((p.N / BN) * ((p.M + BM - 1) / BM));
  switch (p.epi) {
    case EPI_STORE: gemm_bf16_ring_kernel<8, TN, 2, 4, EPI_STORE, PASSES, 2><<<grid, 512, 0, s>>>(p); break;
    case EPI_GELU: gemm_bf16_ring_kernel<8, TN, 2, 4, EPI_GELU, PASSES, 2><<<grid, 512, 0, s>>>(p); break;
    case EPI_RESADD: gemm_bf16_ring_kernel<8, TN, 2, 4, EPI_RESADD, PASSES, 2><<<grid, 512, 0, s>>>(p); break;
    case EPI_WINRES: gemm_bf16_ring_kernel<8, TN, 2, 4, EPI_WINRES, PASSES, 2><<<grid, 512, 0, s>>>(p); break;
    default: throw std::runtime_error("gemm_bf16: bad epilogue");
  }
}

template <int PASSES>
bool try_big_tile(const GemmParams& p, hipStream_t s) {
  constexpr long min_tiles = kBigMinTiles;
  if (PASSES != 3 || p.K > p.N) return false;
  const long mt = (p.M + 255) / 256;
  if (p.N % 256 == 0 && mt * (p.N / 256) >= min_tiles) {
    launch_big_tile<4, PASSES>(p, s);
  } else if (p.N % 192 == 0 && mt * (p.N / 192) >= min_tiles) {
    launch_big_tile<3, PASSES>(p, s);
  } else if (p.N % 128 == 0 && mt * (p.N / 128) >= min_tiles) {
    launch_big_tile<2, PASSES>(p, s);
  } else {
    return false;
  }
  return true;
}

// force_kernel values (tools/gemm_bench A/B; 0 = the dispatch's choice)
enum : int { kKernelAuto = -1, kKernelStag = 1, kKernelBig = 2, kKernelTile = 3, kKernelQ288x256 = 10, kKernelQ288x192 = 11,
             kKernelQ288x128 = 12 };

template <int PASSES>
void launch_forced(const GemmParams& p, hipStream_t s) {
  const bool x3 = PASSES == 3;
  switch (p.force_kernel) {
    case kKernelAuto:  // the dispatch before the 288-row tiles
      if (try_stag<PASSES>(p, s) || try_big_tile<PASSES>(p, s)) return;
      if (p.N % 128 == 0) return launch_tile16<4, 4, 2, 2, PASSES, 2>(p, s);
      if (p.N % 96 == 0) return launch_tile16<4, 3, 2, 2, PASSES, 2>(p, s);
      break;
    case kKernelStag:
      if (try_stag<PASSES>(p, s)) return;
      break;
    case kKernelBig:
      if (try_big_tile<PASSES>(p, s)) return;
      break;
    case kKernelTile:
      if (p.N % 128 == 0) return launch_tile16<4, 4, 2, 2, PASSES, 2>(p, s);
      if (p.N % 96 == 0) return launch_tile16<4, 3, 2, 2, PASSES, 2>(p, s);
      break;
    case kKernelQ288x256:
      if (x3 && p.N % 256 == 0) return launch_stagq<9, 4, 3, 2>(p, s);
      break;
    case kKernelQ288x192:
      if (x3 && p.N % 192 == 0) return launch_stagq<9, 3, 3, 3>(p, s);
      break;
    case kKernelQ288x128:
      if (x3 && p.N % 128 == 0) return launch_stagq<9, 2, 3, 2>(p, s);
      break;
  }
  throw std::runtime_error("gemm_bf16: forced kernel does not fit the shape");
}

// 288-row staggered tiles where they fill whole rounds of the 256 CUs (bf16x3; measured
// on the stage-3 shapes, tools/gemm_bench: s3.fc2 175 -> 143 us, s3.proj 52 -> 46,
// s3.fc1 194 -> 183; equal on s4.fc1; slower than the 256 x 256 / ring kernels on the
// stage-4 shapes that leave a partial round, which keep those)
template <int PASSES>
bool try_stagq(const GemmParams& p, hipStream_t s) {
  if (PASSES != 3) return false;
  const long mt = (p.M + 287) / 288;
  auto whole = [](long tiles) { return tiles >= 256 && tiles % 256 == 0; };
  if (p.K <= p.N && p.N % 256 == 0 && whole(mt * (p.N / 256))) {
    launch_stagq<9, 4, 3, 2>(p, s);
    return true;
  }
  if (p.N % 192 == 0 && whole(mt * (p.N / 192))) {
    launch_stagq<9, 3, 3, 3>(p, s);
    return true;
  }
  return false;
}

template <int PASSES>
void launch_bf16_passes(const GemmParams& p, hipStream_t s) {
  if (p.epi == EPI_KV16) {  // the quantising epilogue lives in the 288 x 256 staggered kernel only
    if (PASSES != 3 || !p.kv16 || p.C || p.C16 || p.kv24 || p.kv_M != 144 || p.col_split != 512 ||
        p.N % 512 != 0 || !p.kv16_scale || p.kv16_sstride < (size_t)(p.M / 144) * 512 || p.M % 144 != 0)
      throw std::runtime_error("gemm_bf16: int16 K/V needs bf16x3, EPI_STORE, no other output, 144-row images, "
                               "512-column blocks");
    return launch_stagq<9, 4, 3, 2>(p, s);
  }
  if (p.force_kernel) return launch_forced<PASSES>(p, s);
  if (try_stagq<PASSES>(p, s)) return;
  if (try_stag<PASSES>(p, s)) return;
  if (try_big_tile<PASSES>(p, s)) return;
  if (p.N % 128 == 0) {  // 128 x 128, waves of 64 x 64
    launch_tile16<4, 4, 2, 2, PASSES, 2>(p, s);
  } else if (p.N % 96 == 0) {  // 128 x 96, waves of 64 x 48
    launch_tile16<4, 3, 2, 2, PASSES, 2>(p, s);
  } else {
    throw std::runtime_error("gemm_bf16: N must be a multiple of 96 or 128");
  }
}

}  // namespace

void launch_gemm_bf16(const GemmParams& p, hipStream_t s) {
  if (p.K % BK16 != 0) throw std::runtime_error("gemm_bf16: K must be a multiple of 32");
  if (p.M <= 0) return;
  if (p.conv.on) {
    const ConvGeom& g = p.conv;
    if (g.Cin % BK16 != 0 || p.K != g.ks * g.ks * g.Cin || p.M % (g.Hout * g.Wout) != 0 || !p.zero)
      throw std::runtime_error("conv: geometry does not match the GEMM");
    if (p.A_lo && p.W_lo)
      launch_conv_passes<3>(p, s);
    else
      launch_conv_passes<1>(p, s);
  } else if (p.A_lo && p.W_lo) {
    launch_bf16_passes<3>(p, s);
  } else {
    launch_bf16_passes<1>(p, s);
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
