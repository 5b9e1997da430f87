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
constexpr int LDS16 = BK16 + 8;  // 40 bf16 = 80 B per row

__device__ __forceinline__ uint16_t bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

template <int EPI>
__device__ __forceinline__ void epi_store16(const GemmParams& p, int row, int col, float v) {
  if constexpr (EPI == EPI_RESADD || EPI == EPI_WINRES) {
    epi_store<EPI>(p, row, col, v);  // fp32 residual stream
  } else {
    if (p.bias) v += p.bias[col];
    if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
    const size_t off = (size_t)row * p.ldc + col;
    if (p.C) {
      if (EPI == EPI_STORE && p.col_split) {
        const int blk = col / p.col_split;
        p.C[blk * p.split_stride + (size_t)row * p.col_split + (col - blk * p.col_split)] = v;
      } else {
        p.C[off] = v;
      }
    }
    if (p.C16) {
      const uint16_t hi = bf16_rne(v);
      static_cast<uint16_t*>(p.C16)[off] = hi;
      if (p.C16lo) static_cast<uint16_t*>(p.C16lo)[off] = bf16_rne(v - bf16_to_f32(hi));
    }
  }
}

template <int TM, int TN, int WGM, int WGN, int EPI, int PASSES>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_bf16_kernel(GemmParams p) {
  constexpr int BM = 16 * TM * WGM;
  constexpr int BN = 16 * TN * WGN;
  constexpr int NT = 64 * WGM * WGN;
  constexpr int PL = PASSES == 3 ? 2 : 1;  // planes per operand
  constexpr int A_CHUNKS = BM * (BK16 / 8);  // 16-B chunks per plane
  constexpr int W_CHUNKS = BN * (BK16 / 8);
  constexpr int A_CH = (A_CHUNKS + NT - 1) / NT;  // per thread
  constexpr int W_CH = (W_CHUNKS + NT - 1) / NT;

  __shared__ uint16_t lds[PL * (BM + BN) * LDS16];
  uint16_t* As[PL];
  uint16_t* Ws[PL];
#pragma unroll
  for (int q = 0; q < PL; ++q) {
    As[q] = lds + q * BM * LDS16;
    Ws[q] = lds + PL * BM * LDS16 + q * BN * LDS16;
  }
  const uint16_t* Ag[2] = {static_cast<const uint16_t*>(p.A), static_cast<const uint16_t*>(p.A_lo)};
  const uint16_t* Wg[2] = {static_cast<const uint16_t*>(p.W), static_cast<const uint16_t*>(p.W_lo)};

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN;
  const int wn = wave % WGN;
  int tx, ty;
  tile_of(p.N / BN, tx, ty);
  const int row0 = ty * BM;
  const int col0 = tx * BN;

  u16x8 ra[PL][A_CH];
  u16x8 rw[PL][W_CH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < PL; ++q) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int idx = tid + i * NT;
        const int r = idx >> 2;
        const int c = (idx & 3) * 8;
        const int gr = row0 + r;
        ra[q][i] = (idx < A_CHUNKS && gr < p.M)
                       ? *reinterpret_cast<const u16x8*>(Ag[q] + (size_t)gr * p.lda + k0 + c) : u16x8{};
      }
#pragma unroll
      for (int i = 0; i < W_CH; ++i) {
        const int idx = tid + i * NT;
        const int r = idx >> 2;
        const int c = (idx & 3) * 8;
        rw[q][i] = idx < W_CHUNKS ? *reinterpret_cast<const u16x8*>(Wg[q] + (size_t)(col0 + r) * p.ldw + k0 + c)
                                  : u16x8{};
      }
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int q = 0; q < PL; ++q) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int idx = tid + i * NT;
        if (idx < A_CHUNKS) *reinterpret_cast<u16x8*>(&As[q][(idx >> 2) * LDS16 + (idx & 3) * 8]) = ra[q][i];
      }
#pragma unroll
      for (int i = 0; i < W_CH; ++i) {
        const int idx = tid + i * NT;
        if (idx < W_CHUNKS) *reinterpret_cast<u16x8*>(&Ws[q][(idx >> 2) * LDS16 + (idx & 3) * 8]) = rw[q][i];
      }
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  sstore();
  __syncthreads();
  const int l16 = lane & 15;
  const int kq = 8 * (lane >> 4);
  for (int k0 = 0; k0 < p.K; k0 += BK16) {
    const bool more = k0 + BK16 < p.K;
    if (more) gload(k0 + BK16);
    bf16x8 a[PL][TM], b[PL][TN];
#pragma unroll
    for (int q = 0; q < PL; ++q) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[q][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(
                                                 &As[q][(wm * 16 * TM + i * 16 + l16) * LDS16 + kq]));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[q][j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(
                                                 &Ws[q][(wn * 16 * TN + j * 16 + l16) * LDS16 + kq]));
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
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * 16 * TM + i * 16 + 4 * (lane >> 4) + r;
        const int col = col0 + wn * 16 * TN + j * 16 + l16;
        if (row < p.M) epi_store16<EPI>(p, row, col, acc[i][j][r]);
      }
}

template <int TM, int TN, int WGM, int WGN, int PASSES>
void launch_tile16(const GemmParams& p, hipStream_t s) {
  constexpr int BM = 16 * TM * WGM;
  constexpr int BN = 16 * TN * WGN;
  dim3 grid((p.N / BN) * ((p.M + BM - 1) / BM));
  dim3 block(64 * WGM * WGN);
  switch (p.epi) {
    case EPI_STORE: gemm_bf16_kernel<TM, TN, WGM, WGN, EPI_STORE, PASSES><<<grid, block, 0, s>>>(p); break;
    case EPI_GELU: gemm_bf16_kernel<TM, TN, WGM, WGN, EPI_GELU, PASSES><<<grid, block, 0, s>>>(p); break;
    case EPI_RESADD: gemm_bf16_kernel<TM, TN, WGM, WGN, EPI_RESADD, PASSES><<<grid, block, 0, s>>>(p); break;
    case EPI_WINRES: gemm_bf16_kernel<TM, TN, WGM, WGN, EPI_WINRES, PASSES><<<grid, block, 0, s>>>(p); break;
    default: throw std::runtime_error("gemm_bf16: bad epilogue");
  }
}

template <int PASSES>
void launch_bf16_passes(const GemmParams& p, hipStream_t s) {
  if (p.N % 128 == 0) {
    launch_tile16<4, 4, 2, 2, PASSES>(p, s);  // 128 x 128, waves of 64 x 64
  } else if (p.N % 96 == 0) {
    launch_tile16<4, 3, 2, 2, PASSES>(p, s);  // 128 x 96, waves of 64 x 48
  } else {
    throw std::runtime_error("gemm_bf16: N must be a multiple of 96 or 128");
  }
}

}  // namespace

void launch_gemm_bf16(const GemmParams& p, hipStream_t s) {
  if (p.K % BK16 != 0) throw std::runtime_error("gemm_bf16: K must be a multiple of 32");
  if (p.M <= 0) return;
  if (p.A_lo && p.W_lo) {
    launch_bf16_passes<3>(p, s);
  } else {
    launch_bf16_passes<1>(p, s);
  }
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
