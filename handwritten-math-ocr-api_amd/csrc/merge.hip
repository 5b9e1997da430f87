// Stage 1's PatchMerging as one streaming kernel (torchvision PatchMerging: the 2 x 2
// gather x0 = x[0::2, 0::2], x1 = x[1::2, 0::2], x2 = x[0::2, 1::2], x3 = x[1::2, 1::2]
// concatenated to 4C = 384 channels, LayerNorm(384), Linear(384, 192, bias=False)), on
// bf16 / bf16x3 MFMA.  VERDICT r05 "What's weak" 5: merge 1 ran on lngemm384_kernel, a
// GEMM-shaped kernel at 0.25 of its HBM roofline (one 128-row workgroup per CU whose
// load, LayerNorm and GEMM phases ran one after the other, W streamed through LDS again
// for every 128 rows).  The op is a stream: 2.26 GB in, 1.13 GB out per 640 images.
//
// Persistent workgroups (one per CU) loop over tiles of 16 output rows, i.e. 32 pixels
// of two consecutive image rows, which are two contiguous 12 KB runs of X:
//  - the tile's 24 KB reach LDS by LDS-DMA (global_load_lds, 16 B per lane) already in
//    gathered order [row][384], four tiles ahead (no staging registers);
//  - LayerNorm: 16 lanes per row, 24 channels each, the sums over the row's 16 lanes on
//    DPP; the normalised rows are split into bf16 hi / lo and written to LDS as the MFMA B
//    fragments (k-step, plane, lane);
//  - W (192 x 384, fragment-major hi / lo planes, launch_frag_pack) stays in registers for
//    the whole kernel: wave w owns output channels 48 w .. 48 w + 47 (3 tiles of 16), 72
//    A fragments; out^T [48 x 16] = W_w . LN^T, three MFMAs per product in bf16x3;
//  - each lane stores 4 consecutive channels of one row per output tile (16-B stores).
// A software pipeline with one raw barrier per tile: tile i's MFMAs beside tile i+1's
// LayerNorm (double-buffered fragments); the DMA waits count this wave's own vector-memory
// operations (see the loop).
#include "kernels.h"
#include "lanes.h"

namespace mocr {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kMC = 96;           // stage-1 channels
constexpr int kMK = 4 * kMC;      // LayerNorm / GEMM k
constexpr int kMN = 2 * kMC;      // output channels
constexpr int kMRows = 16;        // output rows per tile
constexpr int kRawBytes = kMRows * kMK * 4;  // 24 KB: one tile, gathered, fp32
constexpr int kRing = 4;          // tiles in flight (LDS: 4 x 24 KB raw + 2 x 24 KB fragments)
constexpr int kDmaPerWave = kRawBytes / 1024 / 4;  // 1-KB pieces per wave and tile (6)
constexpr int kStoresPerTile = 3; // 16-B stores per lane and tile (3 output tiles per wave)
static_assert(kDmaPerWave * 4 * 1024 == kRawBytes, "four waves split the tile's pieces");

typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((lds_ptr_t)(p));
}
// one 1-KB LDS-DMA piece: 16 B per lane from gbase + voff to LDS lds + 16 lane (mlp.hip dma16:
// inline asm so that hipcc does not see an LDS write in flight; M0 saved and restored)
__device__ __forceinline__ void dma16(const char* gbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds)
      : "memory");
}
// 8 floats -> bf16 hi / lo (split2_bf16 per pair)
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split2_bf16(v[2 * e], v[2 * e + 1], h[e], l[e]);
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

template <int PASSES>
__global__ void __launch_bounds__(256) merge1_kernel(Merge1Params p) {
  constexpr bool X3 = PASSES == 3;
  __shared__ __attribute__((aligned(16))) char raw[kRing][kRawBytes];
  __shared__ __attribute__((aligned(16))) char frag[2][12 * 2 * 1024];  // [tile % 2][k-step][plane][lane] x 16 B
  __shared__ __attribute__((aligned(16))) float gam[kMK], bet[kMK];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H2 = p.H / 2, W2 = p.W / 2, JT = W2 / kMRows;
  const int ntiles = p.B * H2 * JT;  // < 2^31 (launch_merge1)
  const int G = gridDim.x;
  const int my = (ntiles - (int)blockIdx.x + G - 1) / G;  // this workgroup's tiles: blockIdx.x + i G
  if (my <= 0) return;

  // The raw tile [16 rows][96 16-B chunks]: chunk c of a row (gathered channels 4c .. 4c+3)
  // sits at position 16 (c % 6) + c / 6 of the row, so the LayerNorm's 16 lanes of a row
  // (lane l16 owns chunks 6 l16 .. 6 l16 + 5) read 16 consecutive chunks per instruction.
  // LDS unit u = 64 piece + lane of the DMA (lane-linear) is row u / 96, position u % 96; its
  // source offset within the tile is the same for every tile, computed here once:
  // gathered chunk c is part c / 24 (x0 .. x3 of torchvision's cat) of pixel
  // (2 oi + part % 2, 2 (16 jt + row) + part / 2), channels 4 (c % 24) ..
  uint32_t doff[kDmaPerWave];
#pragma unroll
  for (int k = 0; k < kDmaPerWave; ++k) {
    const int u = (wave * kDmaPerWave + k) * 64 + lane;
    const int t = u / 96, pos = u - (u / 96) * 96;
    const int c = 6 * (pos & 15) + (pos >> 4);
    const int part = c / 24, ch = 4 * (c - part * 24);
    doff[k] = (uint32_t)((((part & 1) * p.W + 2 * t + (part >> 1)) * kMC + ch) * 4);
  }
  // Tile T = (image b, output row oi, 16-pixel column block jt); local tile i is blockIdx.x +
  // i G.  Two cursors walk this workgroup's tiles, one for the DMA (kRing tiles ahead) and
  // one for the stores, advanced by G's own decomposition with carries (scalar adds instead
  // of three integer divisions per tile and cursor)
  const int HJ = H2 * JT;
  const int gb = G / HJ, grem = G - (G / HJ) * HJ, goi = grem / JT, gjt = grem - (grem / JT) * JT;
  struct Cur {
    int b, oi, jt;
  };
  const int r0 = (int)blockIdx.x - ((int)blockIdx.x / HJ) * HJ;
  const Cur first = {(int)blockIdx.x / HJ, r0 / JT, r0 - (r0 / JT) * JT};
  auto step = [&](Cur& c) __attribute__((always_inline)) {
    c.jt += gjt;
    c.oi += goi;
    c.b += gb;
    if (c.jt >= JT) {
      c.jt -= JT;
      ++c.oi;
    }
    if (c.oi >= H2) {
      c.oi -= H2;
      ++c.b;
    }
  };
  auto in_base = [&](const Cur& c) __attribute__((always_inline)) {
    return reinterpret_cast<const char*>(p.X + (((size_t)c.b * p.H + 2 * c.oi) * p.W + 2 * kMRows * c.jt) * kMC);
  };
  const char* const base0 = in_base(first);
  Cur dcur = first;
  // the DMA of local tile i, issued in order (a tile past the end re-reads the first: the
  // ring's wait counts stay those of the steady state, and the LayerNorm of "tile my" reads
  // valid data; neither result is used); the tile's base (uniform) goes into the DMA's
  // scalar address
  auto issue = [&](int i) __attribute__((always_inline)) {
    const char* base = i < my ? in_base(dcur) : base0;
    step(dcur);
    char* dst = raw[i % kRing];
#pragma unroll
    for (int k = 0; k < kDmaPerWave; ++k)
      dma16(base, doff[k], lds_u32(dst + (wave * kDmaPerWave + k) * 1024));
  };
#pragma unroll
  for (int i = 0; i < kRing; ++i) issue(i);
  for (int i = tid; i < kMK; i += 256) {
    gam[i] = p.ln_g[i];
    bet[i] = p.ln_b[i];
  }
  // this wave's W fragments: output tiles 3 wave + t, k-steps ks, planes hi / lo
  bf16x8 wf[3][12][PASSES == 3 ? 2 : 1];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int ks = 0; ks < 12; ++ks) {
      const size_t o = ((size_t)(3 * wave + t) * 12 + ks) * 64 + lane;
      wf[t][ks][0] = reinterpret_cast<const bf16x8*>(p.w_hi)[o];
      if constexpr (X3) wf[t][ks][1] = reinterpret_cast<const bf16x8*>(p.w_lo)[o];
    }

  const int row = tid >> 4;  // LayerNorm: tile row, and this lane's 24 channels
  const int l16 = tid & 15;
  const int j16 = lane & 15, g = lane >> 4;
  // LayerNorm of tile i's row `row`, channels 24 l16 .. + 23, into B-fragment buffer i % 2
  auto layernorm = [&](int i) __attribute__((always_inline)) {
    const float* xr = reinterpret_cast<const float*>(raw[i % kRing]) + row * kMK + 4 * l16;
    float v[24];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(xr + 64 * e);  // chunk 6 l16 + e
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * e + r] = a[r];
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 24; ++e) s += v[e];
    const float mean = row_sum<16>(s) * (1.0f / kMK);
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 24; ++e) {
      const float d = v[e] - mean;
      q += d * d;
    }
    const float rstd = 1.0f / sqrtf(row_sum<16>(q) * (1.0f / kMK) + 1e-5f);
#pragma unroll
    for (int h = 0; h < 3; ++h) {  // k8 group 3 l16 + h: k-step k8 / 4, lane group k8 % 4
      const int k8 = 3 * l16 + h;
      float y[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 8 * k8 + e;
        y[e] = (v[8 * h + e] - mean) * rstd * gam[k] + bet[k];
      }
      bf16x8 hi, lo;
      split8(y, hi, lo);
      // fragment lane (lane group k8 % 4, row) at slot row ^ (k8 % 16) of its lane group: the
      // 16 lanes of a row write 16 distinct slots (k8 = 3 l16 + h is distinct mod 16)
      const int fl = (k8 & 3) * 16 + (row ^ (k8 & 15));
      char* fp = frag[i & 1] + ((k8 >> 2) * 2 * 64 + fl) * 16;
      *reinterpret_cast<bf16x8*>(fp) = hi;
      if constexpr (X3) *reinterpret_cast<bf16x8*>(fp + 1024) = lo;
    }
  };

  // software pipeline, one barrier per tile: iteration i runs tile i's MFMAs (fragment
  // buffer i % 2) beside tile i+1's LayerNorm (raw slot (i+1) % kRing -> buffer (i+1) % 2), so
  // the LayerNorm's VALU work fills the MFMAs' issue gaps
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kRing - 1) * kDmaPerWave) : "memory");  // tile 0 landed (this wave's pieces)
  __builtin_amdgcn_s_barrier();
  layernorm(0);
  Cur scur = first;  // the store cursor: tile i
  for (int i = 0; i < my; ++i) {
    // tile i+1's DMA landed: after it this wave issued the DMAs of tiles i+2 .. i+kRing-1
    // (iterations i+2-kRing .. i-1, or the prologue) and the stores of iterations
    // i+1-kRing .. i-1
    static_assert(kRing == 4, "the wait counts below are those of a 4-slot ring");
    if (i == 0)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * kDmaPerWave) : "memory");
    else if (i == 1)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * kDmaPerWave + kStoresPerTile) : "memory");
    else if (i == 2)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * kDmaPerWave + 2 * kStoresPerTile) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * kDmaPerWave + 3 * kStoresPerTile) : "memory");
    // every wave: tile i's fragments written, tile i+1's pieces landed, tile i-1's MFMAs (the
    // other fragment buffer) and tile i's LayerNorm (its raw slot) done
    __builtin_amdgcn_s_barrier();
    issue(i + kRing);  // into tile i's raw slot
    // ---- out^T [48 x 16] = W_w . LN^T over 12 k-steps (three passes per product in bf16x3)
    floatx4 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    const char* fb = frag[i & 1];
#pragma unroll
    for (int ks = 0; ks < 12; ++ks) {
      const char* fp = fb + (ks * 2 * 64 + 16 * g + (j16 ^ ((4 * ks + g) & 15))) * 16;
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(fp);
      bf16x8 bl;
      if constexpr (X3) bl = *reinterpret_cast<const bf16x8*>(fp + 1024);
#pragma unroll
      for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][ks][0], bh, acc[t], 0, 0, 0);
      if constexpr (X3) {
#pragma unroll
        for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][ks][0], bl, acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][ks][1], bh, acc[t], 0, 0, 0);
      }
    }
    layernorm(i + 1);  // independent of the MFMAs above: the scheduler interleaves them
    // lane (g, j16): output row j16, channels 16 (3 wave + t) + 4 g .. + 3
    {
      float* o = p.out + (((size_t)scur.b * H2 + scur.oi) * W2 + scur.jt * kMRows + j16) * kMN + 48 * wave + 4 * g;
      step(scur);
#pragma unroll
      for (int t = 0; t < 3; ++t) *reinterpret_cast<floatx4*>(o + 16 * t) = acc[t];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing DMAs land before the workgroup ends
}

}  // namespace

bool merge1_supported(int H, int W) { return H % 2 == 0 && W % 2 == 0 && (W / 2) % kMRows == 0; }

void launch_merge1(const Merge1Params& p, hipStream_t s) {
  if (p.B <= 0) return;
  if (!merge1_supported(p.H, p.W) || !p.X || !p.out || !p.ln_g || !p.ln_b || !p.w_hi)
    throw std::runtime_error("merge1: even H and W with W / 2 a multiple of 16, and every operand");
  if ((size_t)p.H * p.W * kMC * 4 >= (1ull << 32)) throw std::runtime_error("merge1: an image's map must fit 32-bit offsets");
  const long ntiles = (long)p.B * (p.H / 2) * (p.W / 2 / kMRows);
  if (ntiles >= (1l << 31)) throw std::runtime_error("merge1: tile count must fit int");
  int dev = 0, cus = 256;
  MOCR_HIP_CHECK(hipGetDevice(&dev));
  MOCR_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const unsigned grid = (unsigned)std::min<long>(ntiles, cus);  // one persistent workgroup per CU
  if (p.w_lo)
    merge1_kernel<3><<<grid, 256, 0, s>>>(p);
  else
    merge1_kernel<1><<<grid, 256, 0, s>>>(p);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
