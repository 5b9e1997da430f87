// FETCH_SIZE / WRITE_SIZE calibration for the decode step's access patterns (VERDICT r05
// "Counter caveat": tools/pmc_traffic.py doubles FETCH_SIZE for every kernel, which the
// guide validates only for 16-B-per-lane coalesced streaming reads).
//
// Each kernel touches a known number of bytes exactly once, from a region no earlier
// kernel touched (a 512 MB flush write runs between kernels, so neither L2 nor the
// Infinity Cache holds the region).  Run under
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d D -o run -- tools/fetch_calib
//   rocprofv3 --pmc WRITE_SIZE --output-format csv -d D -o run -- tools/fetch_calib
// and divide each dispatch's counter (KiB) by the bytes printed here.
//
// Patterns (the fold GEMMs of decwide.hip, the attention kernels of decfold.hip):
//   r16     16 B per lane, 1 KB contiguous per wave instruction (the guide's calibrated case;
//           also the fragment-major weight loads)
//   rquad1k the fold GEMM's A rows: lane -> row (lane >> 2), 16 B (lane & 3) of a 64-B
//           segment; 16 rows x 64 B per instruction, row pitch 1 KB (K = 256 fp32), the
//           two halves of a 128-B line read by consecutive instructions
//   rquad2k the same with a 2 KB row pitch (K = 512)
//   r8      8 B per lane, 512 B contiguous per instruction (int16 K/V rows)
//   r4      4 B per lane, 256 B contiguous per instruction (scalar epilogue operands)
//   w16     16 B per lane stores, 1 KB per instruction
//   w16row  the V4 epilogue: 8 lanes x 16 B = one 128-B row piece, rows 1 KB apart
//   w4      4 B per lane stores
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
      return 1;                                                           \
    }                                                                     \
  } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));

// one wave instruction = 1 KB; grid-stride over n16 float4s
__global__ void k_r16(const floatx4* __restrict__ in, float* __restrict__ sink, size_t n16) {
  floatx4 s{};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) s += in[i];
  if (s[0] + s[1] + s[2] + s[3] == 1.2345f) sink[threadIdx.x] = s[0];
}

// each wave owns 16-row blocks; per instruction 16 rows x 64 B; walks the row's segments
__global__ void k_rquad(const float* __restrict__ in, float* __restrict__ sink, int rows, int pitch_floats) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int q = lane >> 2, c = lane & 3;
  floatx4 s{};
  for (int rb = wave; rb * 16 < rows; rb += nwaves) {
    const float* row = in + (size_t)(rb * 16 + q) * pitch_floats + c * 4;
#pragma unroll 4
    for (int seg = 0; seg < pitch_floats / 16; ++seg) s += *reinterpret_cast<const floatx4*>(row + seg * 16);
  }
  if (s[0] + s[1] + s[2] + s[3] == 1.2345f) sink[threadIdx.x] = s[0];
}

__global__ void k_r8(const uint2* __restrict__ in, float* __restrict__ sink, size_t n8) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 v = in[i];
    s += v.x ^ v.y;
  }
  if (s == 12345u) sink[threadIdx.x] = (float)s;
}

__global__ void k_r4(const float* __restrict__ in, float* __restrict__ sink, size_t n4) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) s += in[i];
  if (s == 1.2345f) sink[threadIdx.x] = s;
}

__global__ void k_w16(floatx4* __restrict__ out, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    out[i] = floatx4{1.f, 2.f, 3.f, (float)i};
}

// V4 epilogue stores: 8 lanes x 16 B = 128 B of one row (32 columns of a 256-wide fp32
// row), 8 rows per instruction; column tiles walk the row
__global__ void k_w16row(float* __restrict__ out, int rows) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int r = lane >> 3, j = lane & 7;
  for (int rb = wave; rb * 8 < rows; rb += nwaves)
    for (int ct = 0; ct < 8; ++ct)
      *reinterpret_cast<floatx4*>(out + (size_t)(rb * 8 + r) * 256 + ct * 32 + j * 4) = floatx4{1.f, 2.f, 3.f, (float)rb};
}

__global__ void k_w4(float* __restrict__ out, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) out[i] = (float)i;
}

__global__ void k_flush(floatx4* __restrict__ out, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    out[i] = floatx4{0.f, 0.f, 0.f, (float)i};
}

int main() {
  const size_t region = 64ull << 20;  // bytes each kernel touches
  const int nreg = 8;
  const size_t flush_bytes = 512ull << 20;
  char* buf;
  float* sink;
  floatx4* fl;
  CK(hipMalloc(&buf, region * nreg));
  CK(hipMalloc(&fl, flush_bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 0, region * nreg));
  CK(hipDeviceSynchronize());
  const int grid = 2048, block = 256;
  auto flush = [&]() { k_flush<<<grid, block>>>(fl, flush_bytes / 16); };
  char* r[nreg];
  for (int i = 0; i < nreg; ++i) r[i] = buf + i * region;
  printf("bytes per kernel: %zu (%.1f KiB)\n", region, region / 1024.0);
  printf("dispatch order (after each a flush): r16 rquad1k rquad2k r8 r4 w16 w16row w4\n");
  flush();
  k_r16<<<grid, block>>>(reinterpret_cast<const floatx4*>(r[0]), sink, region / 16);
  flush();
  k_rquad<<<grid, block>>>(reinterpret_cast<const float*>(r[1]), sink, (int)(region / 1024), 256);
  flush();
  k_rquad<<<grid, block>>>(reinterpret_cast<const float*>(r[2]), sink, (int)(region / 2048), 512);
  flush();
  k_r8<<<grid, block>>>(reinterpret_cast<const uint2*>(r[3]), sink, region / 8);
  flush();
  k_r4<<<grid, block>>>(reinterpret_cast<const float*>(r[4]), sink, region / 4);
  flush();
  k_w16<<<grid, block>>>(reinterpret_cast<floatx4*>(r[5]), region / 16);
  flush();
  k_w16row<<<grid, block>>>(reinterpret_cast<float*>(r[6]), (int)(region / 1024));
  flush();
  k_w4<<<grid, block>>>(reinterpret_cast<float*>(r[7]), region / 4);
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
