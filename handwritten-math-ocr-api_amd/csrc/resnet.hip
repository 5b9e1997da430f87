// ResNet18 + Transformer-encoder variant (src/model_res18trans.py:13-64, BASELINE
// config 5): the kernels that are not GEMMs.  The 3x3 / 1x1 convolutions are implicit
// GEMMs on the bf16 LDS-DMA ring (gemm.hip, ConvGeom); the encoder transformer runs on
// the decoder's row kernels (decoder.hip).  BatchNorm (eval) is folded into the conv
// weights and a per-channel bias when the weights are loaded (engine.hip).
#include "kernels.h"

namespace mocr {

namespace {

__device__ __forceinline__ uint16_t bf16_bits(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// conv1 7x7 / stride 2 / pad 3 (1 -> 64 channels, BN folded) + ReLU + maxpool 3x3 /
// stride 2 / pad 1, fused (torchvision resnet18 conv1, bn1, relu, maxpool).  One
// workgroup per (image, 8x8 tile of pooled outputs): the 17x17 conv outputs the tile's
// windows cover are computed into LDS, 32 channels per pass, from a 39x39 input patch.
// Pool windows skip conv positions outside the map; after ReLU every value is >= 0
// and every window holds at least one valid position, so a 0 stands in for them.
constexpr int kPT = 8;                 // pooled tile edge
constexpr int kCT = 2 * kPT + 1;       // conv outputs per edge (17)
constexpr int kIT = 2 * kCT + 5;       // input patch edge (39)

__global__ void __launch_bounds__(256) res_stem_kernel(const float* __restrict__ img, const float* __restrict__ w,
                                                       const float* __restrict__ bias, float* __restrict__ X,
                                                       uint16_t* __restrict__ Xh, uint16_t* __restrict__ Xl, int H,
                                                       int W, int Hc, int Wc, int Hp, int Wp) {
  __shared__ float patch[kIT * kIT];
  __shared__ float wt[64 * 49];
  __shared__ float cv[kCT * kCT * 32];
  const int tid = threadIdx.x;
  const int tilesx = (Wp + kPT - 1) / kPT;
  const int b = blockIdx.y;
  const int py0 = (blockIdx.x / tilesx) * kPT, px0 = (blockIdx.x % tilesx) * kPT;
  const int cy0 = 2 * py0 - 1, cx0 = 2 * px0 - 1;  // first conv position of the tile's windows
  const int iy0 = 2 * cy0 - 3, ix0 = 2 * cx0 - 3;  // first input pixel
  const float* im = img + (size_t)b * H * W;
  for (int i = tid; i < kIT * kIT; i += 256) {
    const int y = iy0 + i / kIT, x = ix0 + i % kIT;
    patch[i] = (y >= 0 && y < H && x >= 0 && x < W) ? im[(size_t)y * W + x] : 0.f;
  }
  for (int i = tid; i < 64 * 49; i += 256) wt[i] = w[i];
  __syncthreads();
  for (int pass = 0; pass < 2; ++pass) {
    for (int pos = tid; pos < kCT * kCT; pos += 256) {
      const int ly = pos / kCT, lx = pos % kCT;
      const int cy = cy0 + ly, cx = cx0 + lx;
      float acc[32];
      const float* bp = bias + 32 * pass;
#pragma unroll
      for (int c = 0; c < 32; ++c) acc[c] = 0.f;
      for (int ky = 0; ky < 7; ++ky)
#pragma unroll
        for (int kx = 0; kx < 7; ++kx) {
          const float x = patch[(2 * ly + ky) * kIT + 2 * lx + kx];
          const float* wr = wt + (32 * pass) * 49 + ky * 7 + kx;
#pragma unroll
          for (int c = 0; c < 32; ++c) acc[c] = fmaf(x, wr[c * 49], acc[c]);
        }
      const bool valid = cy >= 0 && cy < Hc && cx >= 0 && cx < Wc;
#pragma unroll
      for (int c = 0; c < 32; ++c) cv[pos * 32 + c] = valid ? fmaxf(acc[c] + bp[c], 0.f) : 0.f;
    }
    __syncthreads();
    for (int i = tid; i < kPT * kPT * 32; i += 256) {
      const int c = i & 31, q = i >> 5;
      const int ty = q / kPT, tx = q % kPT;
      const int py = py0 + ty, px = px0 + tx;
      if (py < Hp && px < Wp) {
        float m = 0.f;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) m = fmaxf(m, cv[((2 * ty + dy) * kCT + 2 * tx + dx) * 32 + c]);
        const size_t off = (((size_t)b * Hp + py) * Wp + px) * 64 + 32 * pass + c;
        if (X) X[off] = m;
        if (Xh) {
          const uint16_t h = bf16_bits(m);
          Xh[off] = h;
          if (Xl) Xl[off] = bf16_bits(m - __uint_as_float((uint32_t)h << 16));
        }
      }
    }
    __syncthreads();
  }
}

// AdaptiveAvgPool2d((1, None)) of NHWC [B, h, w, C] -> rows (b, x) of [B*w, C]: the
// mean over the h rows, summed in row order and divided by h.
__global__ void res_avgpool_kernel(const float* __restrict__ X, float* __restrict__ P, int B, int h, int w, int C) {
  const size_t n = (size_t)B * w * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const size_t r = i / C;
    const int x = (int)(r % w);
    const int b = (int)(r / w);
    float s = 0.f;
    for (int y = 0; y < h; ++y) s += X[(((size_t)b * h + y) * w + x) * C + c];
    P[i] = s / (float)h;
  }
}

// rows r of the replicated per-forward positional table: out[r] = pos[r % M]
__global__ void res_posrep_kernel(const float* __restrict__ pos, float* __restrict__ out, int rows, int M, int d) {
  const size_t n = (size_t)rows * d;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / d;
    out[i] = pos[(r % M) * d + i % d];
  }
}

}  // namespace

void launch_res_stem(const float* img, const float* w, const float* bias, float* X, uint16_t* Xh, uint16_t* Xl, int B,
                     int H, int W, hipStream_t s) {
  const int Hc = (H + 6 - 7) / 2 + 1, Wc = (W + 6 - 7) / 2 + 1;
  const int Hp = (Hc + 2 - 3) / 2 + 1, Wp = (Wc + 2 - 3) / 2 + 1;
  const dim3 grid(((Hp + kPT - 1) / kPT) * ((Wp + kPT - 1) / kPT), B);
  res_stem_kernel<<<grid, 256, 0, s>>>(img, w, bias, X, Xh, Xl, H, W, Hc, Wc, Hp, Wp);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_res_avgpool(const float* X, float* P, int B, int h, int w, int C, hipStream_t s) {
  const size_t n = (size_t)B * w * C;
  res_avgpool_kernel<<<(unsigned)std::min<size_t>((n + 255) / 256, 65536), 256, 0, s>>>(X, P, B, h, w, C);
  MOCR_HIP_CHECK(hipGetLastError());
}

void launch_res_posrep(const float* pos, float* out, int rows, int M, int d, hipStream_t s) {
  const size_t n = (size_t)rows * d;
  res_posrep_kernel<<<(unsigned)std::min<size_t>((n + 255) / 256, 65536), 256, 0, s>>>(pos, out, rows, M, d);
  MOCR_HIP_CHECK(hipGetLastError());
}

}  // namespace mocr
