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
  EPI_RELU = 4,    // C = relu(acc + bias)            (conv + folded BN + ReLU, ResNet BasicBlock)
  EPI_RESRELU = 5, // C = relu(C + (acc + bias))      (BasicBlock: out += identity; relu)
  EPI_KV16 = 6,    // acc + bias quantised to the int16 cross-attention K/V (GemmParams kv16)
};

// Implicit-GEMM convolution (gemm_bf16 only): A row m = output pixel (b, oy, ox) of an
// NHWC [B, Hin, Win, Cin] input, k = (ky, kx, cin) with cin fastest (Cin % 32 == 0), so
// a 32-deep k-tile is 64 contiguous bytes of one input pixel; taps outside the map read
// `zero`.  W is [Cout][ks][ks][Cin].
struct ConvGeom {
  int on;
  int Hin, Win, Cin, Hout, Wout, ks, stride, pad;
};

struct WinGeom {
  int H, W;      // unpadded stage map
  int pH, pW;    // padded to multiples of 7
  int sh, sw;    // effective shift (0 when the window covers the padded axis)
  int nWx;       // windows per padded row
  int nWin;      // windows per image
};

struct GemmParams {
  const void* A;     // [M, lda] fp32 (gemm_f32) or bf16 hi plane (gemm_bf16)
  const void* W;     // [N, ldw] fp32 or bf16 hi plane
  const void* A_lo;  // bf16x3: lo planes (x - bf16(x)); nullptr for plain bf16
  const void* W_lo;
  const float* bias; // [N] or nullptr
  float* C;          // [M, ldc] (EPI_WINRES: X [B,H,W,ldc]); may be null for EPI_STORE/GELU with C16
  void* C16;         // optional bf16 hi plane of the output (EPI_STORE/EPI_GELU, gemm_bf16 only)
  void* C16lo;       // optional bf16 lo plane of the output
  int M, N, K;
  int lda, ldw, ldc;
  int epi;
  WinGeom win;
  int col_split;       // EPI_STORE: column block width of a split layout (0 = plain [M, ldc])
  size_t split_stride; // floats between column blocks: C[col/cs][row][col%cs]
  ConvGeom conv;       // conv.on: A is the implicit im2col of an NHWC map (bf16 planes)
  const void* zero;    // >= 64 zero bytes (conv padding taps)
  int force_kernel;    // 0: the dispatch's choice; tools/gemm_bench A/B: launch_gemm_bf16 kKernel*
  // EPI_STORE with col_split (gemm_bf16 only): also write the output as the greedy step's
  // packed fp24 cross-attention K/V (common.h), head-major [col block][row / kv_M][k | v]
  // [8 heads][kv_M][32] elements per block (col_split = 512); C may then be null
  uint8_t* kv24;
  int kv_M;
  // ... or as int16 with one scale per (image, column) over its kv_M rows (FoldAttnParams
  // K16): kv16 in the same head-major order, kv16_scale[col block][row / kv_M][512] at
  // kv16_sstride floats per block.  EPI_KV16 on the 288 x 256 staggered kernel only,
  // kv_M = 144 (each wave's 144 rows are one image); C must be null
  int16_t* kv16;
  float* kv16_scale;
  size_t kv16_sstride;
};

void launch_gemm_f32(const GemmParams& p, hipStream_t s);
void launch_gemm_bf16(const GemmParams& p, hipStream_t s);

// ------------------------------------------------------------------ ResNet18 pieces
// conv1 7x7/2 (BN folded, w [64][49]) + ReLU + maxpool 3x3/2 -> X [B, H/4, W/4, 64].
void launch_res_stem(const float* img, const float* w, const float* bias, float* X, uint16_t* Xh, uint16_t* Xl, int B,
                     int H, int W, hipStream_t s);
// AdaptiveAvgPool2d((1, None)): NHWC [B, h, w, C] -> [B*w, C].
void launch_res_avgpool(const float* X, float* P, int B, int h, int w, int C, hipStream_t s);
// out[r] = pos[r % M] for r < rows (the per-forward positional table, per image).
void launch_res_posrep(const float* pos, float* out, int rows, int M, int d, hipStream_t s);

// ------------------------------------------------------------------ Swin pieces
// Stem: Conv2d(1,96,4,4,bias) + Permute + LayerNorm(96) -> X [B, H/4, W/4, 96].
void launch_stem(const float* img, const float* w, const float* b, const float* ln_w, const float* ln_b,
                 float* X, int B, int H, int W, hipStream_t s);

// Outputs of the producers below: fp32 (Y) and/or bf16 hi plane (Yh) and/or lo plane
// (Yl = bf16(y - hi)); each pointer may be null.

// LayerNorm(norm1) + zero-pad + roll(-s) + window partition -> XW [B*nWin*49, C].
void launch_ln_partition(const float* X, const float* g, const float* b, float* XW, uint16_t* XWh, uint16_t* XWl,
                         int B, int C, const WinGeom& wg, hipStream_t s);

// Plain row LayerNorm over C: Y[r] = LN(X[r]).
void launch_layernorm(const float* X, const float* g, const float* b, float* Y, uint16_t* Yh, uint16_t* Yl,
                      int rows, int C, hipStream_t s);

// Window MSA: QKV [B*nWin*49, 3C] fp32 -> O [B*nWin*49, C].  passes 0: fp32 MFMA with
// relbias [heads,49,49] and the region mask computed in-kernel; 1 / 3: bf16 / bf16x3
// MFMA with relmask [types][heads][64][64] (bias + shift mask + -inf key padding; 4
// window types for shifted blocks, 1 otherwise).
// bqkv != nullptr (MFMA kernels only): QKV / O rows are the image's tokens in X's order and
// the padded tokens' k / v are synthesised from the qkv bias (see swin.hip)
void launch_window_attention(const float* QKV, const float* relbias, const float* relmask, float* O, uint16_t* Oh,
                             uint16_t* Ol, int B, int C, int heads, const WinGeom& wg, int passes, hipStream_t s,
                             const float* bqkv = nullptr);

// PatchMerging gather (x0,x1,x2,x3 with zero pad) + LayerNorm(4C) -> Y [B*Ho*Wo, 4C].
void launch_merge_ln(const float* X, const float* g, const float* b, float* Y, uint16_t* Yh, uint16_t* Yl, int B,
                     int H, int W, int C, hipStream_t s);

// Fused norm2 + MLP + residual of a Swin block (mlp.hip): X[r] += W2 gelu(W1 LN(X[r]) + b1)
// + b2 on bf16 (w*lo null) or bf16x3 MFMA, the 4C-wide hidden kept on chip.  C = 96, 192.
struct MlpParams {
  float* X;                 // [M, C] fp32 residual stream, updated in place
  long M;
  int C;
  const float *ln_g, *ln_b; // norm2
  const void *w1, *w1lo;    // [4C, C] bf16 hi / lo planes
  const float* b1;          // [4C]
  const void *w2, *w2lo;    // [C, 4C]
  const float* b2;          // [C]
  const void* wpack;        // W1 | W2 as the kernel's LDS chunk images (launch_mlp_pack)
  // C = 384 only: the block's attention output projection fused in front (mlp384_kernel
  // PROJ): X = x_mid + mlp(norm2(x_mid)), x_mid = X + O W_proj^T + b_proj.  att_hi / att_lo:
  // O as bf16 planes [M, C] in X's row order; wproj / wproj_lo: W_proj's planes, packed
  // by launch_mlp_pack after W2 (null: no proj, or no proj images packed)
  const uint16_t *att_hi, *att_lo;
  const void *wproj, *wproj_lo;
  const float* bproj;
};
bool mlp_fused_supported(int C);
void launch_mlp_fused(const MlpParams& p, hipStream_t s);
// The fused MLP kernels' weight chunks in their LDS image order (swizzled, permuted k or
// unit order), packed once at load from w1 / w2 (/ lo) so that each 1-KB piece -- a staged
// load at C = 96, 192, an LDS-DMA at C = 384 -- reads 1 KB of contiguous memory:
// mlp_pack_bytes(C, x3) bytes at `out`.
size_t mlp_pack_bytes(int C, bool x3);
void launch_mlp_pack(const MlpParams& p, void* out, hipStream_t s);

// out = LayerNorm(X) W^T + b at C = 384 (mlp.hip lngemm384_kernel): stage 3's norm1 + qkv
// over the image tokens at >= 128 images, and merge 1 (PatchMerging of the 96-channel
// stage-1 map: gather, norm, reduction), the LN'd rows kept in registers, W streamed
// through LDS, each 32-column chunk stored when done.  bf16 (wlo null) or bf16x3.
constexpr int kLnGemm384MaxN = 1152;
struct LnGemm384Params {
  const float* X;            // [M, 384]
  long M;
  const float *ln_g, *ln_b;  // [384]
  const void *w, *wlo;       // [N, 384] bf16 hi / lo planes
  const float* b;            // [N] or null (no bias)
  float* out;                // [M, N]
  const void* wpk;           // W as the kernel's LDS chunk images (launch_lngemm384_pack)
  int N;
  int merge_H, merge_W;      // > 0: X is a [B, H, W, 96] map and row r is PatchMerging's
                             // 2 x 2 gather of output pixel r (M = B ceil(H/2) ceil(W/2))
};
void launch_lngemm384(const LnGemm384Params& p, hipStream_t s);
// W [N, 384] (bf16 hi (/ lo) planes) as lngemm384_kernel's LDS chunk images: N * 384 * 2 *
// (lo ? 2 : 1) bytes at `out`
void launch_lngemm384_pack(const void* w, const void* wlo, int N, void* out, hipStream_t s);

// Stage 1's PatchMerging (merge.hip): 2 x 2 gather of X [B, H, W, 96] + LayerNorm(384) +
// Linear(384, 192) -> out [B * H/2 * W/2, 192], bf16 (w_lo null) or bf16x3, W in the
// fragment-major planes of launch_frag_pack(W, 192, 384).  H, W even and W / 2 % 16 == 0
// (merge1_supported); other maps take lngemm384.
struct Merge1Params {
  const float* X;
  int B, H, W;
  const float *ln_g, *ln_b;         // [384]
  const uint16_t *w_hi, *w_lo;      // [12][12][64 lanes][8] bf16
  float* out;
};
bool merge1_supported(int H, int W);
void launch_merge1(const Merge1Params& p, hipStream_t s);

// Fused norm1 + window qkv + W-MSA + proj + residual of one Swin block (wattn.hip),
// bf16 / bf16x3 (lo planes present) for C = 96, 192 (head dim 32).
struct SwinAttnParams {
  float* X;                   // [B, H, W, C] fp32 residual stream, updated in place
  const float *ln_g, *ln_b;   // norm1
  const void *wqkv, *wqkv_lo; // [3C, C] bf16 hi / lo planes
  const float* bqkv;          // [3C]
  const void *wproj, *wproj_lo;  // [C, C]
  const float* bproj;         // [C]
  // the fused stage-1/2 kernel (launch_swin_attn_fused) and the stage-3 no-proj kernel
  // (launch_swin_attn_noproj at C = 384, W_qkv only): the same weights fragment-major
  // (launch_frag_pack: one contiguous 1-KB load per 16-row x 32-k fragment and plane),
  // proj in its permuted k order
  const void *wqkv_fm, *wqkv_fm_lo, *wproj_fm, *wproj_fm_lo;
  const float* table;         // [4 window types][heads][64 q][64 key] bias + mask (build_relmask)
  uint16_t *att_hi, *att_lo;  // noproj: O planes [B * nWin * 49, C] (window-token rows), or
                              // att_pixel_rows: [B * H * W, C] in X's row order, padding dropped
  int att_pixel_rows;
  int B, C, heads;
  WinGeom wg;
};
bool swin_attn_fused_supported(int C);
void launch_swin_attn_fused(const SwinAttnParams& p, hipStream_t s);
// norm1 + qkv + W-MSA only (no proj), O written for the proj GEMM (EPI_WINRES)
bool swin_attn_noproj_supported(int C);
void launch_swin_attn_noproj(const SwinAttnParams& p, hipStream_t s);

// x -> bf16 hi (and lo) planes.
void launch_split_bf16(const float* x, uint16_t* hi, uint16_t* lo, size_t n, hipStream_t s);
// Cross-attention K/V [rows = B * M][2 * 256] fp32 -> packed fp24 (common.h fp24_*),
// head-major [B][k | v][8 heads][M][32] elements (FoldAttnParams f24_*)
void launch_split_kv_fp24(const float* kv, uint8_t* kv24, int B, int M, hipStream_t s);
// Cross-attention K/V of L layers [L][layer_stride elements] fp32 -> int16 in the same
// head-major order, with scale[l][b][512] = max over the M keys of |column| / 32767
// (common.h ld_stream_i16x4; FoldAttnParams K16)
void launch_quant_kv_i16(const float* kv, int16_t* q, float* scale, int B, int M, int L, size_t layer_stride,
                         size_t scale_stride, hipStream_t s);

// ------------------------------------------------------------------ decoder
// Every decode kernel takes its step index t as an argument (one captured graph per
// chunk of steps) and `st` (nullable) for the batch-global stop.
enum DecEpi : int {
  DEC_STORE = 0,   // out = acc + bias
  DEC_RELU = 1,    // out = relu(acc + bias)
  DEC_RESADD = 2,  // out = resid + (acc + bias)   (pre-LayerNorm sum of a post-norm sublayer)
  DEC_QKV = 3,     // cols [0,d) -> q ; [d,2d) -> K cache[t] ; [2d,3d) -> V cache[t]
  DEC_LOGITS = 4,  // out = acc + bias -> logits slot of step t
};

struct RowGemmParams {
  const float* A;      // [B, K]  (pre-LayerNorm sums when a_ln_g is set)
  const float* W;      // [N, K]
  const float* bias;   // [N]
  float* out;          // [B, ldo]
  const float* resid;  // DEC_RESADD: [B, ldo] (pre-LayerNorm sums when r_ln_g is set)
  const float* a_ln_g; const float* a_ln_b;  // A := LayerNorm(A) * g + b, fused prologue
  const float* a_stats;                      // ... with A's row statistics partials [B][16][2]
  const float* r_ln_g; const float* r_ln_b;  // resid := LayerNorm(resid) * g + b
  const float* r_stats;                      // ... with resid's row statistics partials
  float* out_stats;    // DEC_RESADD: write (mean, M2) of each 16-column slice of every output row
  float* kcache;       // DEC_QKV: [B, max_pos, d] for this layer
  float* vcache;
  int B, N, K, ldo;
  int d, max_pos;
  int n_valid;         // columns < n_valid are real (fc_out padding)
  size_t hist_stride;  // DEC_LOGITS: floats between step slots (0: single slot)
  float* part;         // DEC_LOGITS (nullable): per row and 16-column tile {max, argmax bits, sum exp(l - max), 0}
  int epi;
  int t;               // decode step
  const DecodeState* st;
};
void launch_rowgemm(const RowGemmParams& p, hipStream_t s);

// ------------------------------------------------------------------ folded greedy step
// The post-norm LayerNorm in front of each projection is folded into the producer of its
// input (engine.hip fold_decoder, decfold.hip): for LN(y) = g (y - mu) rstd + b feeding
// W x + c, W LN(y) + c = rstd (W' y - mu s) + c' with W' = W diag(g), s = W g,
// c' = W b + c, and W' y is expanded over y's own terms (residual + projection), so it
// is one more column block of y's producer.  The consumer applies rstd and mu (y's slice
// statistics), s and c' when it loads z = W' y.
//
// Fold row GEMM over A = [A1 (K1 columns) | A2 (d columns)]:
//   A1' = A1, or relu(rstd (A1 - mu s) + c) with the statistics a1_stats (the FFN hidden)
//   A2' = A2 (embedding), or LN(A2) with a2_stats, a2_g, a2_b (the sublayer input)
//   y[:, 0:d)  = A2' + (Wy A1' + by), and y's slice statistics      (pre-norm sum)
//   z[:, 0:NZ) = Wz [A1' | A2'] + bz                                 (next projection, folded)
struct FoldGemmParams {
  const float* A1;
  int K1;
  const float *a1_stats, *a1_s, *a1_c;
  const float* A2;
  const float *a2_stats, *a2_g, *a2_b;
  const float *Wy, *by;
  float *y, *y_stats;
  const float *Wz, *bz;
  float* z;
  int NZ;
  int B, t;
  const DecodeState* st;
  // launch_foldwide only: y columns (d, or 0 for the logits), and the logits form (K1 = 0:
  // z = fc_out LN(A2) + b into slot t * hist_stride, n_valid real columns, per-16-column
  // partials `part` [B][NZ / 16] for the greedy selection)
  int NY;
  int n_valid;
  size_t hist_stride;
  float* part;
  // launch_foldwide: Wy / Wz fragment-major (launch_frag_pack): bf16x3 hi / lo planes, or fp32
  const uint16_t *Fy_hi, *Fy_lo, *Fz_hi, *Fz_lo;
  const float *Fy, *Fz;
  int waves;      // launch_foldwide: waves splitting K (0: the default; tools/wide_bench A/B 4 vs 8)
  int tile_cols;  // launch_foldwide logits: columns per tile, 32 / 64 / 128 (0: the default; A/B)
  int no_prefetch_ring;  // launch_foldwide: every k step's loads up front at any grid (A/B)
  // bf16x3 (optional): bf16 hi / lo planes of Wy and Wz; A is split on load and each
  // product is hi·hi + hi·lo + lo·hi on v_mfma_f32_16x16x32_bf16 (fp32 MFMA otherwise)
  const uint16_t *Wy_hi, *Wy_lo, *Wz_hi, *Wz_lo;
};
void launch_foldgemm(const FoldGemmParams& p, hipStream_t s);
// The same fold GEMM on BM x BN tiles with the K range split over 4 waves (decwide.hip),
// for decode chains of 64-256+ rows; with K1 = 0 the fc_out logits (+ partials).
void launch_foldwide(const FoldGemmParams& p, hipStream_t s);
// Fragment-major copy of a row-major [N, K] fp32 weight for launch_foldwide: bf16x3 hi / lo
// planes (hi, lo non-null) or fp32 (f32).  N % 16 == 0, K % 32 == 0.
void launch_frag_pack(const float* W, int N, int K, uint16_t* hi, uint16_t* lo, float* f32, hipStream_t s,
                      bool perm = false);

// Attention of the newest position with folded inputs, one workgroup per (row, head):
// q = rstd (z_q - mu s) + c from z [B, z_ld] and z_stats (plain z when z_stats is null).
// Self-attention: z holds q|k|v (s, c: [3d]); the new k/v are appended to the cache at t
// and the keys are cache rows 0..t.  Cross-attention: K/V = the memory K/V, n = M.
// Greedy selection of step t (select.h): logits (or the logits kernel's per-16-column
// (max, first argmax, sum exp) partials, nparts per row) -> ids / feed / logp, finished
// flags and the batch-global stop state.
struct SelectArgs {
  DecodeState* st;
  int t;
  const float* logits;
  size_t hist_stride;  // logits of step t at logits + t * hist_stride (0: one slot)
  int ldl, V;
  int32_t *ids, *feed;
  const int32_t* forced;  // teacher forcing (parity tests), or null
  int ld_ids;
  float* logp;
  int32_t* finished;
  int eos, stop_batch;
  const float* part;
  int nparts;
};

struct FoldAttnParams {
  const DecodeState* st;
  int t;
  const float* z;
  int z_ld;
  const float *z_stats, *s, *c;
  const float* K;
  const float* V;
  float *kcache, *vcache;  // self only: this layer's cache (same strides as K/V)
  // packed fp24 K/V (common.h): replace K / V / kcache / vcache when K24 is set.  Head-
  // major: key m of head h of row b at element b * f24_b + h * f24_h + 32 m (a head's
  // keys are adjacent: each lane's 4 columns are one 12-byte load, 8 key rows of a wave
  // instruction 768 contiguous bytes)
  const uint8_t *K24, *V24;
  uint8_t *kc24, *vc24;
  size_t f24_b, f24_h;
  // cross-attention only: int16 K/V in the same head-major order (f24_b, f24_h), scaled
  // per (row, column): K = K16 * Ks[b * s_b + column], V = V16 * Vs[...]
  const int16_t *K16, *V16;
  const float *Ks, *Vs;
  int s_b;
  // self-attention only: the cache in int16 (kc16 / vc16, the fp24 layout's element order)
  // with one scale per (row, head, key) over its 32 values: key m of head h of row b is
  // kc16[b f24_b + h f24_h + 32 m ..] * ksc[(b f24_b + h f24_h) / 32 + m]
  int16_t *kc16, *vc16;
  float *ksc, *vsc;
  size_t kv_b_stride;
  int kv_row_stride;
  int n;                   // keys (self: t + 1)
  int waves;               // waves per workgroup, 2 or 4 (0: the launcher's choice; tools/attn_ts A/B)
  float* out;              // [B, d]
  int B;
  // layer 0 of step t >= 1: the greedy selection of step t-1 runs here (sel.t = t - 1),
  // q|k|v of the selected token come from the tables, x = emb + pos is written
  int sel_on;
  SelectArgs sel;
  const float *qtab, *qpos, *emb, *pos;
  float* x;
  // beam search (rows = hypotheses): self-attention key m < t of row b lives in cache row
  // slot_rows[b * slot_ld + m] (the hypothesis' ancestor that computed it); the
  // cross-attention reads memory row b / mem_div (0: 1)
  const int32_t* slot_rows;
  int slot_ld;
  int mem_div;
};
void launch_dec_foldattn(const FoldAttnParams& p, bool self_attn, hipStream_t s);

// out[i, j] = sum_k A[i, k] g[k] Bm[k*sbk + j*sbj] + add_row[i] + add_col[j], accumulated in
// fp64 and rounded once (g null: 1; Bm null: out = A diag(g), K unused).  Load-time
// weight folding only.
void launch_fold_mm(const float* A, int lda, const float* g, const float* Bm, long sbk, long sbj, int K,
                    const float* add_row, const float* add_col, float* out, int ldo, int rows, int cols,
                    hipStream_t s);

// x[b] = embedding[feed[b][0]] + pos[0] and DecodeState init (outside the graph).  With
// qtab: z[b] = qtab[feed[b][0]] + qpos[0], the first layer's folded q|k|v ([V, 3d] and
// [max_pos, 3d] tables).
void launch_dec_embed0(const int32_t* feed, int ld_ids, const float* emb, const float* pos, float* x, int B, int d,
                       hipStream_t s, const float* qtab = nullptr, const float* qpos = nullptr, float* z = nullptr);

// Attention of the newest position over n keys (self: n = t+1 from the KV cache;
// cross: n = M memory tokens).  K/V rows for image b start at K + b*kv_b_stride.
// Fused head projection + attention of the newest position (decoder.hip
// dec_projattn_kernel), one workgroup per (row, head).  Self-attention: W/bias are the
// in_proj [3d][d] rows (q, k, v); K/V = the layer's cache (kv_b_stride = max_pos*d,
// row stride d), n_cached = t; the new k/v are appended at t.  Cross-attention: W/bias
// the q rows of the in_proj, K/V = the precomputed memory K/V, n_cached = M.
struct ProjAttnParams {
  const DecodeState* st;
  int t;
  const float* A;        // [B, d] layer input (pre-norm sum)
  const float* a_stats;  // its LayerNorm slice stats [B][16][2], or null (embedding input)
  const float* a_ln_g;
  const float* a_ln_b;
  const float* W;
  const float* bias;
  const float* K;
  const float* V;
  size_t kv_b_stride;
  int kv_row_stride;
  int n_cached;
  float* kcache;  // self-attention only
  float* vcache;
  float* out;     // [B, d]
  int B, d, heads, max_pos;
  const int32_t* slot_rows;  // beam self-attention: [B][slot_ld] K/V row of key m, or null
  int slot_ld;
  int mem_div;               // K/V row = b / mem_div when slot_rows is null (>= 1)
};
void launch_dec_projattn(const ProjAttnParams& p, bool self_attn, int n_max, hipStream_t s);

// Beam search state and step kernels (decoder.hip; semantics oracle/model_ref.py
// beam_search).  Rows r = b*K + k.
struct BeamParams {
  DecodeState* st;
  int t, last_step, stop_batch;
  int B, K, V, ldl, d, ld;  // ld = max_pos + 1 (sequence / slot table row stride)
  int sos, eos, pad;
  const float* logits;      // [B*K, ldl]
  float* score;             // [B*K]
  int32_t* fin;             // [B*K]
  const int32_t* seq_old;   // [B*K, ld] token sequences, step parity t & 1
  int32_t* seq_new;         // parity (t + 1) & 1
  const int32_t* slot_old;  // [B*K, ld] K/V cache row of each position
  int32_t* slot_new;
  const float* emb;
  const float* pos;
  float* x;                 // [B*K, d] next step's input
  // folded step (qtab set): layer 0's q|k|v of each new hypothesis' token at position t+1,
  // z[r] = qtab[tok] + qpos[t + 1] ([B*K, 3d], decfold.hip's table lookup)
  const float *qtab, *qpos;
  float* z;
};
void launch_beam_init(const BeamParams& p, hipStream_t s);
void launch_beam_select(const BeamParams& p, hipStream_t s);

// out[r] = LayerNorm(y[r]) from slice statistics [rows][16][2] (d = 256).
void launch_ln_rows(const float* y, const float* stats, const float* g, const float* b, float* out, int rows,
                    hipStream_t s);

void launch_dec_attn(const DecodeState* st, int t, const float* q, const float* K, const float* V,
                     size_t kv_b_stride, int kv_row_stride, int n_fixed, int n_max, float* out, int B, int d,
                     int heads, hipStream_t s, int q_ld = 0, int kv_mod = 0);

// Argmax + log-prob + finish flags + next fed token + next step's embedding.  With `part`
// (the logits kernel's tile partials [B][ldl/16] float4) the logits are not re-read.
void launch_dec_argmax(const SelectArgs& a, int last_step, int B, const float* emb, const float* pos, float* x, int d,
                       hipStream_t s, const float* qtab = nullptr, const float* qpos = nullptr, float* z = nullptr);

}  // namespace mocr
