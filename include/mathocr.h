/*
 * mathocr.h — C-ABI of libmathocr.so, the MI355X (gfx950) engine for the
 * Swin-T encoder + 8-layer Transformer decoder greedy-decode hot path of
 * PTD504/handwritten-math-ocr-api.
 *
 * The reference has no FFI for this path: its boundary is two Python calls that
 * FastAPI consumes.  These entry points replace them:
 *
 *   app/src/im2latex.py:7    load_model(path, vocab, device)            -> mocr_create + mocr_load_weights
 *   app/src/im2latex.py:15   predict(model, image[1,1,H,W], ...)        -> mocr_set_images + mocr_encode
 *                                                                          + mocr_decode(stop_mode=MOCR_STOP_BATCH, logp_out)
 *   src/inference.py:7       predict(images[B,1,H,W], model, ...)       -> mocr_set_images + mocr_encode
 *                                                                          + mocr_decode(stop_mode=MOCR_STOP_BATCH)
 *   src/model_swin.py:39-46  EncoderSwin.forward                        -> mocr_encode (+ mocr_get_memory)
 *   src/model_swin.py:72-88  DecoderTransformer.forward (per step)      -> one step of mocr_decode
 *
 * The Python host layer (handwritten-math-ocr-api_amd/engine.py) binds these with
 * ctypes and mirrors the reference's call signatures; see INTEGRATION.md.
 *
 * Conventions
 *  - Every function returns 0 on success and a negative code on failure; the
 *    message is in mocr_last_error(engine) (or mocr_last_error(NULL) for errors
 *    raised before an engine exists).
 *  - Host buffers are owned by the caller and are complete when the call returns
 *    (all calls are synchronous).  Device buffers are owned by the engine, except
 *    the *_device variants, which read/write caller-owned device memory on the
 *    engine's device.
 *  - One engine per device; calls on one engine must be serialised by the caller.
 *    Calls release no locks of their own, so different engines may run in
 *    different host threads concurrently.
 */
#ifndef MATHOCR_H_
#define MATHOCR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MOCR_ABI_VERSION 6

/* Arithmetic of the engine. */
enum {
  MOCR_PRECISION_FP32 = 0,   /* fp32 everywhere; encoder GEMMs on fp32-input MFMA                     */
  MOCR_PRECISION_BF16 = 1,   /* encoder GEMMs on bf16 MFMA (bf16 operands, fp32 accumulate); ~6e-3    */
                             /* relative memory error, NOT token-exact                                */
  MOCR_PRECISION_BF16X3 = 2  /* encoder GEMMs on bf16 MFMA with split operands x = hi + lo,            */
                             /* hi*hi + hi*lo + lo*hi (~1e-5 relative); decoder fp32                  */
};

/* Model family (the Swin path, and the f3 ResNet18 + Transformer-encoder
 * variant of src/model_res18trans.py, BASELINE config 5). */
enum {
  MOCR_ARCH_SWIN = 0,       /* src/model_swin.py: Swin-T encoder, memory = (H/32 x W/32) tokens        */
  MOCR_ARCH_RES18TRANS = 1  /* src/model_res18trans.py: ResNet18 (eval BN) + 8 post-norm encoder layers */
                            /* whose attention runs across the batch (:61-62), memory = W/32 tokens;   */
                            /* its per-forward random positional table is an input                     */
                            /* (mocr_set_encoder_pos); convs run bf16x3 (bf16 with MOCR_PRECISION_BF16)  */
};

/* Kernel-path variants (mocr_config.variant).  0 is the production path; the others keep
 * the unfused kernel sequences the fused kernels replaced selectable, so the parity tests
 * can check fused against unfused on the same engine build (they are bit-for-bit different
 * roundings of the same math, each held to the oracle's tolerance). */
enum {
  MOCR_VARIANT_DEFAULT = 0,
  MOCR_VARIANT_UNFUSED_ATTN = 1, /* Swin stages 1-2: LN-partition, qkv GEMM, window attention, proj */
                                 /* GEMM as separate kernels instead of wattn.hip's fused kernel     */
  MOCR_VARIANT_UNFUSED_MLP = 2,  /* Swin stages 1-2 (and 3 at >= 128 images): LN, fc1, fc2 instead  */
                                 /* of mlp.hip's fused kernels                                       */
  MOCR_VARIANT_DEC_UNFOLDED = 4, /* greedy decoder on the 8-kernel step (LayerNorms applied by their */
                                 /* consumers) instead of the folded 5-kernel step (decfold.hip)     */
  MOCR_VARIANT_S4_FUSED_ATTN = 8, /* Swin stage 4 (C = 768): norm1 + qkv + W-MSA in one kernel (two  */
                                  /* 384-channel LDS halves) -- measured slower than the unfused     */
                                  /* sequence at 384x384, so off in production                       */
  MOCR_VARIANT_WINDOW_ROWS = 16,  /* unfused Swin attention (stage 4, or with UNFUSED_ATTN) over the */
                                  /* partitioned window rows, padded tokens included, instead of the */
                                  /* image's tokens in pixel order                                   */
  MOCR_VARIANT_DEC_NARROW = 32,   /* folded greedy step on decfold.hip's 16x16-tile fold GEMMs and    */
                                  /* decoder.hip's logits kernel instead of decwide.hip's wide tiles */
  MOCR_VARIANT_LOGITS_F32 = 64,   /* bf16x3 engines: the greedy step's fc_out on fp32-input MFMA     */
                                  /* instead of bf16x3 (fc_out hi / lo planes)                        */
  MOCR_VARIANT_S3_LARGE_BATCH = 128, /* Swin stage 3 takes its >= 128-image kernels at any batch     */
                                     /* (unfused attention over the image tokens, mlp.hip's fused    */
                                     /* C = 384 MLP), so small-batch parity tests cover that path    */
  MOCR_VARIANT_KV_F32 = 256,         /* bf16x3 engines: the greedy step streams fp32 K/V instead of  */
                                     /* fp24 (packed 16 + 8 bits, relative rounding <= 2^-16) and    */
                                     /* int16 cross-attention K/V                                    */
  MOCR_VARIANT_CROSS_KV_F24 = 512,   /* bf16x3 engines: cross-attention K/V in fp24 instead of int16 */
                                     /* with one scale per (row, column) over the memory's keys      */
  MOCR_VARIANT_UNFUSED_LN_GEMM = 1024, /* norm + Linear pairs at 384 channels (stage 3's norm1 + qkv */
                                     /* at >= 128 images, merge 1) as two kernels instead of         */
                                     /* mlp.hip's lngemm384_kernel                                   */
  MOCR_VARIANT_SELF_KV_F24 = 2048,   /* bf16x3 engines: the self-attention cache in fp24 instead of  */
                                     /* int16 with one scale per (row, head, key) over its 32 values */
  MOCR_VARIANT_BEAM_UNFOLDED = 4096, /* beam search on round 2's projection+attention step (fp32    */
                                     /* K/V, row GEMMs) instead of the folded wide-tile step         */
  MOCR_VARIANT_UNFUSED_S3_TAIL = 8192 /* Swin stage 3 at >= 128 images: the attention output         */
                                     /* projection as its own residual-add GEMM in front of the      */
                                     /* fused MLP, instead of inside it (mlp.hip mlp384_kernel PROJ) */
};

/* Greedy stopping rule (src/inference.py:23-25). */
enum {
  MOCR_STOP_BATCH = 0, /* stop once every row has produced EOS (the reference); rows keep generating */
  MOCR_STOP_NONE = 1   /* run exactly max_steps steps (bench: fixed work)                            */
};

typedef struct mocr_config {
  int32_t img_h, img_w;  /* input image size, e.g. 384x384 (bench) or 96x320 (src/config.py:17-18) */
  int32_t vocab;         /* V = 5075 for the published checkpoint                                  */
  int32_t d_model;       /* 256  (src/config.py:19)                                                */
  int32_t n_heads;       /* 8    (src/config.py:20)                                                */
  int32_t d_ff;          /* 512  (src/config.py:21)                                                */
  int32_t n_layers;      /* 8    (src/config.py:32)                                                */
  int32_t max_pos;       /* 150  rows of the learned positional table (src/model_swin.py:54)       */
  int32_t sos_id, eos_id, pad_id; /* 1, 2, 0 (src/utils.py:111)                                    */
  int32_t max_batch;     /* device buffers are sized for this many images                          */
  int32_t precision;     /* MOCR_PRECISION_*                                                       */
  int32_t max_beam;      /* 0: greedy only; K <= 8: decoder buffers for max_batch*K hypotheses      */
  int32_t arch;          /* MOCR_ARCH_*                                                            */
  int32_t variant;       /* MOCR_VARIANT_* flags; 0 in production                                  */
} mocr_config;

typedef struct mocr_engine mocr_engine;

int mocr_abi_version(void);

/* sha256 (16 hex digits) of the sources the library was built from (the .hip and .h files of
 * csrc sorted by name, then this header): the Python binding refuses a library whose sources
 * changed. */
const char* mocr_source_hash(void);

/* "production", or what made a non-production build: "defs:" and the compile-time
 * definitions of a Makefile MOCR_DEFS build (e.g. the phase-clock -DMOCR_FOLD_TS), "ab:" and
 * the tools/ script of an A/B build.  The Python binding refuses a non-production library
 * unless it is loaded as an A/B build (the bench's --lib, which reports the tag). */
const char* mocr_build_tag(void);

/* HIP devices visible to the process (serving /health "device_available"); negative on a
 * HIP error, message in mocr_last_error(NULL). */
int mocr_device_count(void);

/* Number of float32 values mocr_load_weights expects for this config.  The blob
 * is the concatenation, in order, of the tensors listed by
 * handwritten-math-ocr-api_amd/synth.py:param_specs (reference state_dict names,
 * encoder.features.* alias; relative_position_index buffers, decoder.tgt_mask
 * and the unused swin.norm/head are not part of it). */
size_t mocr_weight_count(const mocr_config* cfg);

/* Encoder memory tokens per image: ceil-merged (H/4, W/4) map after 3 merges. */
int mocr_memory_tokens(const mocr_config* cfg);

int mocr_create(const mocr_config* cfg, int hip_device, mocr_engine** out);
int mocr_destroy(mocr_engine* eng);
const char* mocr_last_error(const mocr_engine* eng);

/* Upload fp32 weights (host).  Derived tensors (expanded relative-position
 * biases, bf16 copies, padded fc_out) are built on the device. */
int mocr_load_weights(mocr_engine* eng, const float* blob, size_t n_floats);

/* Images [B,1,H,W] fp32 NCHW in [-1,1] (app/src/preprocess.py:6-17) -> engine buffer. */
int mocr_set_images(mocr_engine* eng, const float* img_host, int batch);
int mocr_set_images_device(mocr_engine* eng, const float* img_dev, int batch);

/* MOCR_ARCH_RES18TRANS: the positional table [M, d_model] the encoder adds after the
 * projection.  The reference draws it fresh in every forward (nn.Embedding(M, d) inside
 * EncoderCNN.forward, src/model_res18trans.py:57-59); the caller supplies the draw. */
int mocr_set_encoder_pos(mocr_engine* eng, const float* table, int tokens);

/* Encoder on the resident images: memory [B, M, d_model] and every layer's
 * cross-attention K/V (computed once, not per step as in the reference). */
int mocr_encode(mocr_engine* eng, int batch);

/* Copy the encoder memory [B, M, d_model] fp32 to the host (parity tests). */
int mocr_get_memory(mocr_engine* eng, float* host_out);

/* Greedy decode of the encoded batch (src/inference.py:13-27).
 *   forced_ids  nullable [B, max_steps+1]: teacher forcing — step t feeds
 *               forced_ids[b][t] instead of the previous argmax (parity tests);
 *   ids_out     [B, max_steps+1] int32, column 0 = sos; columns past *n_steps_out are pad;
 *   n_steps_out number of steps run (< max_steps only with MOCR_STOP_BATCH);
 *   logp_out    nullable [B, max_steps]: log(softmax(logits)[argmax] + 1e-10) per step
 *               (app/src/im2latex.py:33-39);
 *   logits_out  nullable [B, max_steps, vocab] fp32 last-position logits (parity only). */
int mocr_decode(mocr_engine* eng, int max_steps, int stop_mode, const int32_t* forced_ids,
                int32_t* ids_out, int32_t* n_steps_out, float* logp_out, float* logits_out);

/* Beam search of the encoded batch.  The reference's beam_size
 * argument (src/inference.py:7, src/config.py:50) is accepted but unused, so the
 * semantics are this engine's, restated on the CPU by oracle/model_ref.py
 * beam_search: K hypotheses per image in rank order, score = sum of log_softmax of
 * the chosen tokens (no length penalty), finished hypotheses retained at unchanged
 * score, ties broken by the lower (beam * V + token) index.
 *   beam         1 <= K <= cfg.max_beam;
 *   ids_out      nullable [B, max_steps+1]: the best hypothesis, column 0 = sos, pad after;
 *   scores_out   nullable [B, K] hypothesis scores, rank order;
 *   beam_ids_out nullable [B, K, max_steps+1] every hypothesis;
 *   n_steps_out  steps run (< max_steps only with MOCR_STOP_BATCH: every hypothesis of
 *                every image finished). */
int mocr_decode_beam(mocr_engine* eng, int beam, int max_steps, int stop_mode, int32_t* ids_out, float* scores_out,
                     int32_t* beam_ids_out, int32_t* n_steps_out);

/* Same, ids written to caller device memory [B, max_steps+1] (e.g. a torch tensor
 * that is then all-gathered over RCCL). */
int mocr_decode_device(mocr_engine* eng, int max_steps, int stop_mode, int32_t* ids_dev,
                       int32_t* n_steps_out);

/* Parity debugging: run the encoder only up to torchvision features[k] (0 = stem,
 * 1,3,5,7 = stages, 2,4,6 = PatchMerging) and copy that NHWC map (n floats) out. */
int mocr_debug_encode_until(mocr_engine* eng, int batch, int k, float* host_out, size_t n);

/* Per-kernel-class timing measured with HIP events on the engine stream while
 * enabled (bench.py roofline).  Each record: {name, launches, total_ms, flops, bytes}. */
typedef struct mocr_kernel_stat {
  char name[48];
  int64_t launches;
  double total_ms;
  double flops;  /* algorithmic FLOP summed over launches */
  double bytes;  /* algorithmic HBM bytes summed over launches */
} mocr_kernel_stat;

int mocr_set_timing(mocr_engine* eng, int enabled); /* also resets the counters */

/* Restrict the engine's HIP stream to a set of CUs (hipExtStreamCreateWithCUMask: bit i
 * of mask[i / 32] enables CU i); n_words = 0 restores an unmasked stream.  HIP makes a
 * stream with a CU mask or a priority, not both: a mask on a stream with a non-zero
 * priority (and a non-zero priority on a masked stream) fails. */
int mocr_set_cu_mask(mocr_engine* eng, const uint32_t* mask, int n_words);

/* Recreate the engine's stream at a HIP stream priority: > 0 the device's highest, < 0
 * its lowest, 0 normal (pipeline experiments: a decode chain above a concurrent encoder). */
int mocr_set_stream_priority(mocr_engine* eng, int priority);
int mocr_get_timing(mocr_engine* eng, mocr_kernel_stat* out, int max_records);

/* ---- Image-parallel group (BASELINE config 3) ----------------
 * One process per GPU.  Each rank encodes and decodes its own contiguous shard of the
 * global batch on its own engine (no collective on the data path); the decoded token
 * streams are then all-gathered over RCCL (xGMI) into every rank's device memory.  The
 * reference has no multi-GPU inference (src/test_model.py:38-40 wraps the model in a
 * non-working nn.DataParallel); this replaces the survey's sketch
 * mocr_group_create(n_dev, devs) / mocr_group_predict with one process per device.
 *
 * RCCL is loaded at run time (librccl.so.1).  Rank 0 makes the 128-byte unique id with
 * mocr_group_unique_id and hands it to the other ranks over the caller's own channel
 * (bench.py: the torch.distributed store); every rank then calls mocr_group_create
 * collectively.  Errors: negative return, message in mocr_group_last_error(). */
#define MOCR_GROUP_ID_BYTES 128
typedef struct mocr_group mocr_group;

int mocr_group_unique_id(uint8_t* id_out /* [MOCR_GROUP_ID_BYTES] */);
int mocr_group_create(const uint8_t* id /* [MOCR_GROUP_ID_BYTES] */, int world, int rank, int hip_device,
                      mocr_group** out);
int mocr_group_destroy(mocr_group* g);
const char* mocr_group_last_error(void);

/* Ranks in the group as RCCL's communicator counts them (ncclCommCount): bench.py records
 * it beside n_gpus ("rccl_ranks"), so the record shows RCCL saw every rank. */
int mocr_group_size(const mocr_group* g, int* ranks_out);

/* Collective: every rank passes its shard's ids [rows, width] int32 (device memory, e.g.
 * the ids mocr_decode_device wrote); ids_all_dev [world*rows, width] receives all shards
 * in rank order.  The group's HIP stream first waits for everything queued so far on
 * producer_stream (the hipStream_t that wrote ids_dev or last used ids_all_dev, e.g.
 * torch's current stream; NULL = the null stream), then all-gathers every rank's
 * (rows, width) and fails on every rank, before the data gather, unless all are equal.
 * Returns when the result is complete. */
int mocr_group_gather_ids(mocr_group* g, const int32_t* ids_dev, int rows, int width, int32_t* ids_all_dev,
                          void* producer_stream);

#ifdef __cplusplus
}
#endif

#endif /* MATHOCR_H_ */
