// Checks the cross-lane helpers of wattn.hip (DPP row sums, permlane16/32 swaps) against
// __shfl_xor on one wave.  hipcc --offload-arch=gfx950 -O3 tools/lane_ops_test.hip -o tools/lane_ops_test
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__global__ void k(float* out) {
  const int l = threadIdx.x;
  const float x = (float)((l * 37) % 64) + 0.25f * l;
  float s8 = x, r8 = x;
  s8 += dpp<0xB1>(s8); s8 += dpp<0x4E>(s8); s8 += dpp<0x141>(s8);
  for (int m = 1; m < 8; m <<= 1) r8 += __shfl_xor(r8, m, 64);
  float s16 = x, r16 = x;
  s16 += dpp<0xB1>(s16); s16 += dpp<0x4E>(s16); s16 += dpp<0x141>(s16); s16 += dpp<0x140>(s16);
  for (int m = 1; m < 16; m <<= 1) r16 += __shfl_xor(r16, m, 64);
  auto a = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, x), false, false);
  const float p16a = __builtin_bit_cast(float, a[0]), p16b = __builtin_bit_cast(float, a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, x), false, false);
  const float p32a = __builtin_bit_cast(float, b[0]), p32b = __builtin_bit_cast(float, b[1]);
  float a16 = x, b16 = x, a32 = x, b32 = x;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a16), "+v"(b16));
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a32), "+v"(b32));
  float* o = out + l * 14;
  o[10] = a16; o[11] = b16; o[12] = a32; o[13] = b32;
  o[0] = x; o[1] = s8; o[2] = r8; o[3] = s16; o[4] = r16;
  o[5] = p16a; o[6] = p16b; o[7] = p32a; o[8] = p32b; o[9] = __shfl_xor(x, 16, 64);
}
int main() {
  float* d; hipMalloc(&d, 896 * 4);
  k<<<1, 64>>>(d);
  float h[896]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  int bad8 = 0, bad16 = 0;
  for (int l = 0; l < 64; ++l) {
    bad8 += h[l * 14 + 1] != h[l * 14 + 2];
    bad16 += h[l * 14 + 3] != h[l * 14 + 4];
  }
  printf("row_sum8 mismatches %d, row_sum16 mismatches %d\n", bad8, bad16);
  for (int l = 0; l < 64; l += 5)
    printf("lane %2d x %7.2f | p16 %7.2f %7.2f | p32 %7.2f %7.2f | x^16 %7.2f x^32 %7.2f\n", l, h[l * 14], h[l * 14 + 5],
           h[l * 14 + 6], h[l * 14 + 7], h[l * 14 + 8], h[(l ^ 16) * 14], h[(l ^ 32) * 14]);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const float* o = h + l * 14;
    const float x = o[0], x16 = h[(l ^ 16) * 14], x32 = h[(l ^ 32) * 14];
    bad += !((o[10] == x && o[11] == x16) || (o[10] == x16 && o[11] == x));
    bad += !((o[12] == x && o[13] == x32) || (o[12] == x32 && o[13] == x));
  }
  printf("asm swap pair mismatches %d\n", bad);
  return bad != 0;
}
