// Host-side launchers of the gfx950 kernels (one translation unit per kernel family).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace mocr {

// ------------------------------------------------------------------ encoder GEMM
// C[M,N] (op)= A[M,K] · W[N,K]^T + bias   — row-major, K contiguous (torch Linear layout).
enum Epi : int {
  EPI_STORE = 0,   // C = acc + bias
  EPI_GELU = 1,    // C = gelu(acc + bias)
  EPI_RESADD = 2,  // C += acc + bias                 (x = x + mlp(...), torchvision block)
  EPI_WINRES = 3,  // X[b, y, x] += acc + bias, row m in shifted-window order (window reverse,
                   // roll(+s), crop)  (torchvision shifted_window_attention tail)
};

struct WinGeom {
  int H, W;      // unpadded stage map
  int pH, pW;    // padded to multiples of 7
  int sh, sw;    // effective shift (0 when the window covers the padded axis)
  int nWx;       // windows per padded row
  int nWin;      // windows per image
};

struct GemmParams {
  const void* A;     // [M, lda] fp32 (precision 0) or bf16 (precision 1)
  const void* W;     // [N, ldw] fp32 or bf16
  const float* bias; // [N] or nullptr
  float* C;          // [M, ldc] (EPI_WINRES: X [B,H,W,ldc])
  void* C16;         // optional bf16 copy of the output (EPI_STORE/EPI_GELU), may be null
  int M, N, K;
  int lda, ldw, ldc;
  int epi;
  WinGeom win;
};

void launch_gemm_f32(const GemmParams& p, hipStream_t s);
void launch_gemm_bf16(const GemmParams& p, hipStream_t s);

// ------------------------------------------------------------------ Swin pieces
// Stem: Conv2d(1,96,4,4,bias) + Permute + LayerNorm(96) -> X [B, H/4, W/4, 96].
void launch_stem(const float* img, const float* w, const float* b, const float* ln_w, const float* ln_b,
                 float* X, int B, int H, int W, hipStream_t s);

// LayerNorm(norm1) + zero-pad + roll(-s) + window partition -> XW [B*nWin*49, C] (fp32 and/or bf16).
void launch_ln_partition(const float* X, const float* g, const float* b, float* XW, uint16_t* XW16, int B, int C,
                         const WinGeom& wg, hipStream_t s);

// Plain row LayerNorm over C: Y[r] = LN(X[r]) (fp32 and/or bf16 outputs).
void launch_layernorm(const float* X, const float* g, const float* b, float* Y, uint16_t* Y16, int rows, int C,
                      hipStream_t s);

// Window MSA: QKV [B*nWin*49, 3C] -> O [B*nWin*49, C] (fp32 and/or bf16 outputs).
void launch_window_attention(const float* QKV, const float* relbias /*[heads,49,49]*/, float* O, uint16_t* O16,
                             int B, int C, int heads, const WinGeom& wg, hipStream_t s);

// PatchMerging gather (x0,x1,x2,x3 with zero pad) + LayerNorm(4C) -> Y [B*Ho*Wo, 4C].
void launch_merge_ln(const float* X, const float* g, const float* b, float* Y, uint16_t* Y16, int B, int H, int W,
                     int C, hipStream_t s);

void launch_f32_to_bf16(const float* x, uint16_t* y, size_t n, hipStream_t s);

// ------------------------------------------------------------------ decoder
enum DecEpi : int {
  DEC_STORE = 0,   // out = acc + bias
  DEC_RELU = 1,    // out = relu(acc + bias)
  DEC_RESADD = 2,  // out = resid + (acc + bias)   (pre-LayerNorm sum of a post-norm sublayer)
  DEC_QKV = 3,     // cols [0,d) -> q ; [d,2d) -> K cache[t] ; [2d,3d) -> V cache[t]
  DEC_LOGITS = 4,  // out = acc + bias -> logits slot of step t
};

struct RowGemmParams {
  const float* A;      // [B, K]
  const float* W;      // [N, K]
  const float* bias;   // [N]
  float* out;          // [B, ldo]
  const float* resid;  // DEC_RESADD
  float* kcache;       // DEC_QKV: [B, max_pos, d] for this layer
  float* vcache;
  int B, N, K, ldo;
  int d, max_pos;
  int n_valid;         // columns < n_valid are real (fc_out padding)
  size_t hist_stride;  // DEC_LOGITS: floats between step slots (0: single slot)
  int epi;
  const DecodeState* st;
};
void launch_rowgemm(const RowGemmParams& p, hipStream_t s);

// Embedding of step t (single block; advances the step counter).
void launch_dec_embed(DecodeState* st, const int32_t* feed, int ld_ids, const float* emb, const float* pos,
                      float* x, int B, int d, hipStream_t s);

// Decoder LayerNorm over d (one wave per row).
void launch_dec_layernorm(const DecodeState* st, const float* y, const float* g, const float* b, float* x, int B,
                          int d, hipStream_t s);

// Self-attention over the KV cache (keys 0..t) and cross-attention over memory K/V.
void launch_dec_self_attn(const DecodeState* st, const float* q, const float* kc, const float* vc, float* out,
                          int B, int d, int heads, int max_pos, hipStream_t s);
void launch_dec_cross_attn(const DecodeState* st, const float* q, const float* memkv, int ld_kv, int koff,
                           int voff, float* out, int B, int M, int d, int heads, hipStream_t s);

// Argmax + log-prob + finish flags + next fed token.
void launch_dec_argmax(DecodeState* st, const float* logits, size_t hist_stride, int ldl, int V, int B,
                       int32_t* ids, int32_t* feed, const int32_t* forced, int ld_ids, float* logp,
                       int32_t* finished, int eos, hipStream_t s);

}  // namespace mocr
