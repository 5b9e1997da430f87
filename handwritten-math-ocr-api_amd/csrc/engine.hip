// libmathocr.so: engine state, weight layout, encoder schedule, hipGraph-captured
// decode loop, and the C-ABI of include/mathocr.h.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/mathocr.h"
#include <cstdlib>

#include "kernels.h"

using namespace mocr;

namespace {

thread_local std::string g_last_error;

constexpr int kStages = 4;
constexpr int kDepth[kStages] = {2, 2, 6, 2};
constexpr int kHeads[kStages] = {3, 6, 12, 24};
constexpr int kEmbed = 96;
constexpr int kEncDim = 768;
constexpr int kDecodeChunk = 8;  // steps per captured graph
constexpr int kSyncStopRows = 16;  // batch-stop check after every chunk up to this many rows (decode())

struct StageGeom {
  int H, W, C, heads;
  WinGeom win[2];  // block parity 0: no shift, 1: shift 3 (disabled per axis when 7 >= padded size)
};

struct SwinBlockW {
  size_t n1w, n1b, qkvw, qkvb, projw, projb, table, n2w, n2b, fc1w, fc1b, fc2w, fc2b;
};
struct MergeW {
  size_t nw, nb, redw;
};
struct DecLayerW {
  size_t sa_inw, sa_inb, sa_ow, sa_ob, ca_inw, ca_inb, ca_ow, ca_ob, l1w, l1b, l2w, l2b, n1w, n1b, n2w, n2b, n3w,
      n3b;
};

// ResNet18-trans pieces (synth.py:param_specs_res18 order).
struct ConvW {
  size_t w, bn_w, bn_b, bn_m, bn_v;
  int cin, cout, ks, stride;
};
struct ResBlockW {
  ConvW c1, c2, ds;
  bool has_ds;
};
struct EncLayerW {
  size_t inw, inb, ow, ob, l1w, l1b, l2w, l2b, n1w, n1b, n2w, n2b;
};
constexpr int kResCh[4] = {64, 128, 256, 512};

// ResNet18 map sizes: conv1 /2 then maxpool /2 (H/4 for H % 4 == 0), then 3 stride-2 stages.
inline int res_out(int n, int k, int s, int p) { return (n + 2 * p - k) / s + 1; }
inline int res_h1(int h) { return res_out(res_out(h, 7, 2, 3), 3, 2, 1); }
inline int res_h4(int h) {
  h = res_h1(h);
  for (int i = 0; i < 3; ++i) h = res_out(h, 3, 2, 1);
  return h;
}

// Blob layout: the order of synth.py:param_specs (Swin) / param_specs_res18.
struct Layout {
  int arch = MOCR_ARCH_SWIN;
  size_t stem_w, stem_b, stem_lnw, stem_lnb;
  std::vector<SwinBlockW> blocks;  // 12
  MergeW merge[3];
  ConvW r_conv1{};
  std::vector<ResBlockW> rblocks;  // 8
  std::vector<EncLayerW> elayers;  // 8
  size_t projw, projb, emb, pos;
  std::vector<DecLayerW> layers;
  size_t fcw, fcb;
  size_t total;

  explicit Layout(const mocr_config& c) {
    size_t off = 0;
    auto take = [&](size_t n) {
      size_t o = off;
      off += n;
      return o;
    };
    const size_t d = c.d_model, ff = c.d_ff;
    arch = c.arch;
    if (arch == MOCR_ARCH_RES18TRANS) {
      auto conv = [&](int cin, int cout, int ks, int stride) {
        ConvW w;
        w.w = take((size_t)cout * cin * ks * ks);
        w.bn_w = take(cout);
        w.bn_b = take(cout);
        w.bn_m = take(cout);
        w.bn_v = take(cout);
        w.cin = cin;
        w.cout = cout;
        w.ks = ks;
        w.stride = stride;
        return w;
      };
      r_conv1 = conv(1, 64, 7, 2);
      int cin = 64;
      for (int li = 0; li < 4; ++li) {
        const int ch = kResCh[li];
        for (int blk = 0; blk < 2; ++blk) {
          const int stride = (li > 0 && blk == 0) ? 2 : 1;
          ResBlockW b{};
          b.c1 = conv(blk == 0 ? cin : ch, ch, 3, stride);
          b.c2 = conv(ch, ch, 3, 1);
          b.has_ds = blk == 0 && (stride != 1 || cin != ch);
          if (b.has_ds) b.ds = conv(cin, ch, 1, stride);
          rblocks.push_back(b);
        }
        cin = ch;
      }
      projw = take(d * 512);
      projb = take(d);
      for (int l = 0; l < 8; ++l) {
        EncLayerW e;
        e.inw = take(3 * d * d);
        e.inb = take(3 * d);
        e.ow = take(d * d);
        e.ob = take(d);
        e.l1w = take(ff * d);
        e.l1b = take(ff);
        e.l2w = take(d * ff);
        e.l2b = take(d);
        e.n1w = take(d);
        e.n1b = take(d);
        e.n2w = take(d);
        e.n2b = take(d);
        elayers.push_back(e);
      }
      decoder_part(c, take);
      total = off;
      return;
    }
    stem_w = take(kEmbed * 16);
    stem_b = take(kEmbed);
    stem_lnw = take(kEmbed);
    stem_lnb = take(kEmbed);
    size_t dim = kEmbed;
    for (int s = 0; s < kStages; ++s) {
      for (int j = 0; j < kDepth[s]; ++j) {
        SwinBlockW b;
        b.n1w = take(dim);
        b.n1b = take(dim);
        b.qkvw = take(3 * dim * dim);
        b.qkvb = take(3 * dim);
        b.projw = take(dim * dim);
        b.projb = take(dim);
        b.table = take(169 * (size_t)kHeads[s]);
        b.n2w = take(dim);
        b.n2b = take(dim);
        b.fc1w = take(4 * dim * dim);
        b.fc1b = take(4 * dim);
        b.fc2w = take(4 * dim * dim);
        b.fc2b = take(dim);
        blocks.push_back(b);
      }
      if (s < kStages - 1) {
        merge[s].nw = take(4 * dim);
        merge[s].nb = take(4 * dim);
        merge[s].redw = take(8 * dim * dim);
        dim *= 2;
      }
    }
    projw = take(d * kEncDim);
    projb = take(d);
    decoder_part(c, take);
    total = off;
  }

  template <typename Take>
  void decoder_part(const mocr_config& c, Take& take) {
    const size_t d = c.d_model, ff = c.d_ff, V = c.vocab;
    emb = take(V * d);
    pos = take((size_t)c.max_pos * d);
    for (int l = 0; l < c.n_layers; ++l) {
      DecLayerW w;
      w.sa_inw = take(3 * d * d);
      w.sa_inb = take(3 * d);
      w.sa_ow = take(d * d);
      w.sa_ob = take(d);
      w.ca_inw = take(3 * d * d);
      w.ca_inb = take(3 * d);
      w.ca_ow = take(d * d);
      w.ca_ob = take(d);
      w.l1w = take(ff * d);
      w.l1b = take(ff);
      w.l2w = take(d * ff);
      w.l2b = take(d);
      w.n1w = take(d);
      w.n1b = take(d);
      w.n2w = take(d);
      w.n2b = take(d);
      w.n3w = take(d);
      w.n3b = take(d);
      layers.push_back(w);
    }
    fcw = take(V * d);
    fcb = take(V);
  }
};

void check_config(const mocr_config& c) {
  auto req = [](bool ok, const char* what) {
    if (!ok) throw std::runtime_error(std::string("invalid config: ") + what);
  };
  req(c.img_h >= 4 && c.img_w >= 4, "image smaller than one patch");
  req(c.vocab > 0, "vocab");
  req(c.d_model == 256 && c.n_heads == 8, "decoder kernels are built for d_model=256, 8 heads");
  req(c.d_ff == 512, "decoder kernels are built for d_ff=512");
  req(c.n_layers >= 1 && c.n_layers <= 64, "n_layers");
  req(c.max_pos >= 2 && c.max_pos <= 288, "max_pos in [2,288]");
  req(c.max_beam >= 0 && c.max_beam <= 8, "max_beam in [0,8]");
  req(c.arch == MOCR_ARCH_SWIN || c.arch == MOCR_ARCH_RES18TRANS, "arch");
  if (c.arch == MOCR_ARCH_RES18TRANS) {
    req(c.img_h >= 32 && c.img_w >= 32, "ResNet18 needs images of at least 32x32");
    req(c.max_batch <= 256, "ResNet18-trans: the encoder attends across at most 256 images");
  }
  req(c.max_batch >= 1 && c.max_batch <= 4096, "max_batch");
  req(c.precision == MOCR_PRECISION_FP32 || c.precision == MOCR_PRECISION_BF16 ||
          c.precision == MOCR_PRECISION_BF16X3,
      "precision");
  req((c.variant & ~(MOCR_VARIANT_UNFUSED_ATTN | MOCR_VARIANT_UNFUSED_MLP | MOCR_VARIANT_DEC_UNFOLDED |
                      MOCR_VARIANT_S4_FUSED_ATTN | MOCR_VARIANT_WINDOW_ROWS | MOCR_VARIANT_DEC_NARROW |
                      MOCR_VARIANT_LOGITS_F32 | MOCR_VARIANT_S3_LARGE_BATCH | MOCR_VARIANT_KV_F32 |
                      MOCR_VARIANT_CROSS_KV_F24 | MOCR_VARIANT_UNFUSED_LN_GEMM | MOCR_VARIANT_SELF_KV_F24 |
                      MOCR_VARIANT_BEAM_UNFOLDED | MOCR_VARIANT_UNFUSED_S3_TAIL)) == 0,
      "variant: unknown MOCR_VARIANT_* flag");
  req(c.sos_id >= 0 && c.sos_id < c.vocab && c.eos_id >= 0 && c.eos_id < c.vocab, "special ids");
}

StageGeom make_win(int H, int W, int C, int heads) {
  StageGeom g{};
  g.H = H;
  g.W = W;
  g.C = C;
  g.heads = heads;
  for (int par = 0; par < 2; ++par) {
    WinGeom& w = g.win[par];
    w.H = H;
    w.W = W;
    w.pH = (H + kWin - 1) / kWin * kWin;
    w.pW = (W + kWin - 1) / kWin * kWin;
    const int shift = par ? kWin / 2 : 0;
    w.sh = (kWin >= w.pH) ? 0 : shift;
    w.sw = (kWin >= w.pW) ? 0 : shift;
    w.nWx = w.pW / kWin;
    w.nWin = (w.pH / kWin) * w.nWx;
  }
  return g;
}


template <typename T>
T* dalloc(size_t n) {
  void* p = nullptr;
  if (n == 0) n = 1;
  MOCR_HIP_CHECK(hipMalloc(&p, n * sizeof(T)));
  return static_cast<T*>(p);
}

struct TimingRec {
  std::string name;
  hipEvent_t e0, e1;
  double flops, bytes;
};

}  // namespace

struct mocr_engine {
  mocr_config cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  // the engine stream's CU mask (mocr_set_cu_mask) and priority (mocr_set_stream_priority):
  // HIP creates a stream with one or the other, so the two settings exclude each other
  bool stream_cu_masked = false;
  int stream_priority = 0;
  std::string err;
  std::unique_ptr<Layout> lay;

  // geometry
  int H1 = 0, W1 = 0, Hm = 0, Wm = 0, M = 0, Vpad = 0;
  StageGeom stage[kStages];

  // weights
  float* dw = nullptr;
  std::vector<float*> relbias;  // per Swin block [heads,49,49] (fp32 attention)
  std::vector<float*> relmask;  // per Swin block [types][heads][64][64] (bf16 attention)
  float* fcw_pad = nullptr;
  float* fcb_pad = nullptr;
  float* kvw_all = nullptr;  // [L*2d, d] cross-attention k/v in_proj rows of every layer
  float* kvb_all = nullptr;
  bool weights_loaded = false;

  // encoder activations
  float *img = nullptr, *X = nullptr, *X2 = nullptr, *XW = nullptr, *QKV = nullptr, *ATT = nullptr, *HID = nullptr;
  float *MEM = nullptr, *MEMKV = nullptr;
  size_t szX = 0, szXW = 0, szQKV = 0, szHID = 0;
  // bf16 modes: hi/lo planes of the GEMM A operands and of every weight
  uint16_t *XWh = nullptr, *XWl = nullptr, *ATTh = nullptr, *ATTl = nullptr, *HIDh = nullptr, *HIDl = nullptr;
  uint16_t *MEMh = nullptr, *MEMl = nullptr, *dwh = nullptr, *dwl = nullptr, *kvwh = nullptr, *kvwl = nullptr;
  int cur_batch = 0;
  bool encoded = false;
  int partial_stage = -1;

  // decoder state
  float *dx = nullptr, *dq = nullptr, *datt = nullptr, *dh = nullptr, *dlogits = nullptr;
  float *dy_sa = nullptr, *dy_ca = nullptr, *dy_ff = nullptr;
  float *ds_sa = nullptr, *ds_ca = nullptr, *ds_ff = nullptr;  // row-stat partials [B][16][2]
  float* dlogits_hist = nullptr;
  float *kcache = nullptr, *vcache = nullptr;
  // packed fp24 (common.h) cross-attention K/V and self-attention cache that the folded
  // greedy step streams in bf16x3 engines (kv24()); 3 bytes per element
  uint8_t *MEMKV24 = nullptr, *kc24 = nullptr, *vc24 = nullptr;
  // the self-attention cache in int16 with per-(row, head, key) scales (self16())
  int16_t *kc16 = nullptr, *vc16 = nullptr;
  float *ksc16 = nullptr, *vsc16 = nullptr;
  // int16 cross-attention K/V (kvx16(), replaces the fp24 planes of MEMKV24) and its
  // per-(layer, row, column) scales [L][max_batch][2d]
  int16_t* MEMKV16 = nullptr;
  float* MEMKVS = nullptr;
  int32_t *ids = nullptr, *feed = nullptr, *forced = nullptr, *finished = nullptr;
  float* logp = nullptr;
  DecodeState* st = nullptr;
  DecodeState* st_host = nullptr;          // pinned, 2 slots: the state after alternate chunks
  hipEvent_t chunk_ev[2] = {nullptr, nullptr};
  int ld_ids = 0;
  const SelectArgs* sel_prev = nullptr;  // record_step -> record_layers_fold (layer 0 of step t >= 1)
  int max_rows = 0;  // decoder rows the buffers hold: max_batch * max(1, max_beam)
  // beam search: scores, finished flags, token sequences and K/V slot tables [2 parities]
  float* bscore = nullptr;
  int32_t* bfin = nullptr;
  int32_t* bseq[2] = {nullptr, nullptr};
  int32_t* bslot[2] = {nullptr, nullptr};
  std::map<std::tuple<int, int, int>, hipGraphExec_t> graphs;
  // folded greedy step (kernels.h FoldGemmParams): per-layer folded weights in one buffer,
  // layer 0's q|k|v tables, and the folded q|k|v of the next layer [rows, 3d]
  struct FoldW {
    float *wzq, *bzq, *sq, *cq;          // z_q = W_q' y_sa:  [d, 2d] over [attn | x]
    float *wzh, *bzh, *sh, *ch;          // z_h = W_1' y_ca:  [ff, 2d] over [attn | LN1(y_sa)]
    float *wzqkv, *bzqkv, *sqkv, *cqkv;  // z_qkv(l+1) = W_in' y_ff: [3d, ff + d] over [hidden | LN2(y_ca)]
  };
  std::vector<FoldW> foldw;
  float* fold_buf = nullptr;
  size_t fold_floats = 0;
  uint16_t *fold_h = nullptr, *fold_l = nullptr;  // bf16x3: hi / lo planes of fold_buf
  float *qtab = nullptr, *qpos = nullptr, *dzqkv = nullptr;
  float* dpart = nullptr;  // greedy: logits tile partials [rows][Vpad/16] float4 for the argmax
  // decwide.hip: fragment-major copies (launch_frag_pack) of every layer's fold GEMM weights
  // (y_sa, z_q, y_ca, z_h, y_ff, z_qkv) and of fc_out; bf16x3 hi / lo planes or fp32
  struct FragW {
    uint16_t *hi = nullptr, *lo = nullptr;
    float* f = nullptr;
  };
  std::vector<std::array<FragW, 6>> fragw;
  FragW frag_logits;
  // wattn.hip swin_attn_kernel: fragment-major W_qkv and (permuted k order) W_proj of the
  // stage-1/2 blocks, bf16 hi / lo planes
  std::vector<std::array<FragW, 2>> swinfrag;
  std::vector<void*> mlppack;  // mlp.hip: the fused MLP kernels' W1 | W2 chunk images per block
  std::vector<void*> lngpack;  // mlp.hip: lngemm384's W_qkv chunk images per stage-3 block
  void* mergepack = nullptr;   // and of merge 1's reduction
  FragW mergefrag;             // merge 1's reduction, fragment-major (merge.hip)
  std::vector<void*> frag_allocs;

  // timing
  bool timing = false;
  std::vector<TimingRec> pending;
  std::map<std::string, mocr_kernel_stat> stats;
  std::vector<hipEvent_t> event_pool;

  ~mocr_engine() {
    free_res18();
    (void)hipSetDevice(device);
    for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);
    for (auto e : event_pool) (void)hipEventDestroy(e);
    for (auto e : chunk_ev)
      if (e) (void)hipEventDestroy(e);
    if (st_host) (void)hipHostFree(st_host);
    for (auto& r : pending) {
      (void)hipEventDestroy(r.e0);
      (void)hipEventDestroy(r.e1);
    }
    void* bufs[] = {dw,      fcw_pad, fcb_pad, kvw_all, kvb_all, img,  X,        X2,       XW,     QKV,
                    ATT,     HID,     MEM,     MEMKV,   dx,      dq,   datt,     dy_sa,    dy_ca,  dy_ff, dh, dlogits,
                    ds_sa,   ds_ca,   ds_ff,
                    dlogits_hist, kcache, vcache, ids, feed, forced, finished, logp, st, XWh, XWl, ATTh, ATTl,
                    HIDh, HIDl, MEMh, MEMl, dwh, dwl, kvwh, kvwl, bscore, bfin, bseq[0], bseq[1],
                    bslot[0], bslot[1], fold_buf, qtab, qpos, dzqkv, dpart, MEMKV24, kc24, vc24, MEMKV16, MEMKVS,
                    kc16, vc16, ksc16, vsc16};
    for (void* p : bufs)
      if (p) (void)hipFree(p);
    for (void* p : frag_allocs)
      if (p) (void)hipFree(p);
    for (float* p : relbias)
      if (p) (void)hipFree(p);
    for (float* p : relmask)
      if (p) (void)hipFree(p);
    if (stream) (void)hipStreamDestroy(stream);
  }

  const float* W(size_t off) const { return dw + off; }

  // ---------------------------------------------------------------- ResNet18-trans state
  struct DevConv {
    uint16_t* wh = nullptr;  // [cout][ks][ks][cin] BN-folded, bf16 hi / lo planes
    uint16_t* wl = nullptr;
    float* bias = nullptr;   // BN shift
    int cin = 0, cout = 0, ks = 0, stride = 1;
  };
  struct DevBlock {
    DevConv c1, c2, ds;
    bool has_ds = false;
  };
  std::vector<DevBlock> rdev;
  float* rstem_w = nullptr;  // [64][49] BN-folded conv1
  float* rstem_b = nullptr;
  float* RX[2] = {nullptr, nullptr};           // fp32 block input / identity maps (NHWC)
  uint16_t *RXh = nullptr, *RXl = nullptr;     // planes of the block input
  uint16_t *RTh = nullptr, *RTl = nullptr;     // planes of a block's conv1 output
  void* rzero = nullptr;                       // zero taps of the implicit-GEMM convs
  float *RP = nullptr, *RPOS = nullptr, *RPOSB = nullptr;  // pooled rows, pos table, replicated table
  float *EX0 = nullptr, *EQKV = nullptr, *EATT = nullptr, *EY1 = nullptr, *EY2 = nullptr, *EH = nullptr;
  float *ES0 = nullptr, *ES1 = nullptr, *ES2 = nullptr;  // LayerNorm slice stats [rows][16][2]
  bool pos_set = false;
  int rH1 = 0, rW1 = 0, rH4 = 0;

  bool res_x3() const { return cfg.precision != MOCR_PRECISION_BF16; }  // conv passes: 3 unless plain bf16

  void init_res18() {
    const size_t B = cfg.max_batch, d = cfg.d_model, L = cfg.n_layers;
    rH1 = res_h1(cfg.img_h);
    rW1 = res_h1(cfg.img_w);
    rH4 = res_h4(cfg.img_h);
    M = res_h4(cfg.img_w);
    Hm = 1;
    Wm = M;
    const size_t rows = B * M;
    // the largest NHWC map is layer1's (channels double as the map quarters)
    const size_t szmap = B * (size_t)rH1 * rW1 * 64;
    dw = dalloc<float>(lay->total);
    fcw_pad = dalloc<float>((size_t)Vpad * d);
    fcb_pad = dalloc<float>(Vpad);
    kvw_all = dalloc<float>(L * 2 * d * d);
    kvb_all = dalloc<float>(L * 2 * d);
    img = dalloc<float>(B * cfg.img_h * cfg.img_w);
    MEM = dalloc<float>(rows * d);
    MEMKV = dalloc<float>(rows * L * 2 * d);
    RX[0] = dalloc<float>(szmap);
    RX[1] = dalloc<float>(szmap);
    RXh = dalloc<uint16_t>(szmap);
    RTh = dalloc<uint16_t>(szmap);
    if (res_x3()) {
      RXl = dalloc<uint16_t>(szmap);
      RTl = dalloc<uint16_t>(szmap);
    }
    rzero = dalloc<char>(256);
    // on the engine's stream: a kernel on the null stream claims one of the process's
    // hardware queues (GPU_MAX_HW_QUEUES, 4), and engines created after it then share
    // queues (profiles/r04/r04i: config 4's four replicas on three queues)
    MOCR_HIP_CHECK(hipMemsetAsync(rzero, 0, 256, stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    RP = dalloc<float>(rows * 512);
    RPOS = dalloc<float>((size_t)M * d);
    RPOSB = dalloc<float>(rows * d);
    EX0 = dalloc<float>(rows * d);
    EQKV = dalloc<float>(rows * 3 * d);
    EATT = dalloc<float>(rows * d);
    EY1 = dalloc<float>(rows * d);
    EY2 = dalloc<float>(rows * d);
    EH = dalloc<float>(rows * cfg.d_ff);
    ES0 = dalloc<float>(rows * 32);
    ES1 = dalloc<float>(rows * 32);
    ES2 = dalloc<float>(rows * 32);
    rstem_w = dalloc<float>(64 * 49);
    rstem_b = dalloc<float>(64);
    for (const ResBlockW& b : lay->rblocks) {
      DevBlock db;
      auto mk = [&](const ConvW& c) {
        DevConv dc;
        const size_t n = (size_t)c.cout * c.ks * c.ks * c.cin;
        dc.wh = dalloc<uint16_t>(n);
        if (res_x3()) dc.wl = dalloc<uint16_t>(n);
        dc.bias = dalloc<float>(c.cout);
        dc.cin = c.cin;
        dc.cout = c.cout;
        dc.ks = c.ks;
        dc.stride = c.stride;
        return dc;
      };
      db.c1 = mk(b.c1);
      db.c2 = mk(b.c2);
      db.has_ds = b.has_ds;
      if (b.has_ds) db.ds = mk(b.ds);
      rdev.push_back(db);
    }
  }

  void free_res18() {
    for (DevBlock& b : rdev)
      for (DevConv* c : {&b.c1, &b.c2, &b.ds})
        for (void* q : {(void*)c->wh, (void*)c->wl, (void*)c->bias})
          if (q) (void)hipFree(q);
    void* bufs[] = {RX[0], RX[1], RXh, RXl, RTh, RTl, rzero, RP, RPOS, RPOSB, EX0, EQKV, EATT, EY1, EY2, EH, ES0, ES1,
                    ES2, rstem_w, rstem_b};
    for (void* q : bufs)
      if (q) (void)hipFree(q);
  }

  // Eval BatchNorm folded into the conv (torch: y = (conv(x) - mean) / sqrt(var + eps) * g + b):
  // w' = w * g / sqrt(var + eps) reordered to [cout][ky][kx][cin], bias = b - mean * g / sqrt(var + eps).
  static void fold_bn(const float* blob, const ConvW& c, std::vector<float>& w, std::vector<float>& bias) {
    const int K = c.ks * c.ks;
    w.assign((size_t)c.cout * K * c.cin, 0.f);
    bias.assign(c.cout, 0.f);
    for (int o = 0; o < c.cout; ++o) {
      const float sc = blob[c.bn_w + o] / std::sqrt(blob[c.bn_v + o] + 1e-5f);
      bias[o] = blob[c.bn_b + o] - blob[c.bn_m + o] * sc;
      for (int i = 0; i < c.cin; ++i)
        for (int k = 0; k < K; ++k) w[((size_t)o * K + k) * c.cin + i] = blob[c.w + ((size_t)o * c.cin + i) * K + k] * sc;
    }
  }

  void load_res18(const float* blob) {
    std::vector<float> w, bias;
    fold_bn(blob, lay->r_conv1, w, bias);
    MOCR_HIP_CHECK(hipMemcpy(rstem_w, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    MOCR_HIP_CHECK(hipMemcpy(rstem_b, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
    float* tmp = dalloc<float>((size_t)512 * 512 * 9);
    for (size_t i = 0; i < rdev.size(); ++i) {
      const ResBlockW& b = lay->rblocks[i];
      auto up = [&](const ConvW& c, DevConv& dc) {
        fold_bn(blob, c, w, bias);
        MOCR_HIP_CHECK(hipMemcpy(tmp, w.data(), w.size() * 4, hipMemcpyHostToDevice));
        MOCR_HIP_CHECK(hipDeviceSynchronize());  // before the non-blocking stream reads tmp
        launch_split_bf16(tmp, dc.wh, dc.wl, w.size(), stream);
        MOCR_HIP_CHECK(hipStreamSynchronize(stream));
        MOCR_HIP_CHECK(hipMemcpy(dc.bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
      };
      up(b.c1, rdev[i].c1);
      up(b.c2, rdev[i].c2);
      if (b.has_ds) up(b.ds, rdev[i].ds);
    }
    (void)hipFree(tmp);
  }

  void set_encoder_pos(const float* table, int tokens) {
    if (cfg.arch != MOCR_ARCH_RES18TRANS) throw std::runtime_error("mocr_set_encoder_pos: only for MOCR_ARCH_RES18TRANS");
    if (tokens != M) throw std::runtime_error("positional table has " + std::to_string(tokens) + " rows, the encoder "
                                              "makes " + std::to_string(M) + " tokens");
    MOCR_HIP_CHECK(hipSetDevice(device));
    MOCR_HIP_CHECK(hipMemcpy(RPOS, table, (size_t)M * cfg.d_model * 4, hipMemcpyHostToDevice));
    MOCR_HIP_CHECK(hipDeviceSynchronize());  // visible to the engine's non-blocking stream
    pos_set = true;
    encoded = false;
  }

  // One implicit-GEMM conv: NHWC [B, h, w, cin] planes -> [B, ho, wo, cout].
  void conv(const char* name, const DevConv& c, const uint16_t* Ah, const uint16_t* Al, int B, int h, int w,
            float* C, uint16_t* Ch, uint16_t* Cl, int epi) {
    const int pad = c.ks / 2;
    const int ho = res_out(h, c.ks, c.stride, pad), wo = res_out(w, c.ks, c.stride, pad);
    GemmParams p{};
    p.A = Ah;
    p.A_lo = res_x3() ? Al : nullptr;
    p.W = c.wh;
    p.W_lo = res_x3() ? c.wl : nullptr;
    p.bias = c.bias;
    p.C = C;
    p.C16 = Ch;
    p.C16lo = res_x3() ? Cl : nullptr;
    p.M = B * ho * wo;
    p.N = c.cout;
    p.K = c.ks * c.ks * c.cin;
    p.lda = p.K;
    p.ldw = p.K;
    p.ldc = c.cout;
    p.epi = epi;
    p.conv = ConvGeom{1, h, w, c.cin, ho, wo, c.ks, c.stride, pad};
    p.zero = rzero;
    const double flops = 2.0 * p.M * p.N * p.K;
    const double bytes = (res_x3() ? 4.0 : 2.0) * ((double)B * h * w * c.cin + (double)p.N * p.K) +
                         4.0 * (double)p.M * p.N * (epi == EPI_RESRELU ? 3 : 1);
    timed(name, flops, bytes, [&] { launch_gemm_bf16(p, stream); });
  }

  void encode_res18(int B) {
    if (!pos_set) throw std::runtime_error("MOCR_ARCH_RES18TRANS: mocr_set_encoder_pos before mocr_encode");
    const int d = cfg.d_model, rows = B * M;
    static const char* c1n[] = {"l1.conv1", "l1.conv1", "l2.conv1", "l2.conv1", "l3.conv1", "l3.conv1", "l4.conv1",
                                "l4.conv1"};
    static const char* c2n[] = {"l1.conv2", "l1.conv2", "l2.conv2", "l2.conv2", "l3.conv2", "l3.conv2", "l4.conv2",
                                "l4.conv2"};
    static const char* dsn[] = {"", "", "l2.down", "", "l3.down", "", "l4.down", ""};
    timed("r.stem", 2.0 * B * (res_out(cfg.img_h, 7, 2, 3) * (double)res_out(cfg.img_w, 7, 2, 3)) * 64 * 49,
          4.0 * B * ((double)cfg.img_h * cfg.img_w + (double)rH1 * rW1 * 64 * (res_x3() ? 2 : 1.5)),
          [&] { launch_res_stem(img, rstem_w, rstem_b, RX[0], RXh, RXl, B, cfg.img_h, cfg.img_w, stream); });
    int h = rH1, w = rW1;
    float* x = RX[0];
    float* spare = RX[1];
    for (size_t i = 0; i < rdev.size(); ++i) {
      const DevBlock& b = rdev[i];
      conv(c1n[i], b.c1, RXh, RXl, B, h, w, nullptr, RTh, RTl, EPI_RELU);
      const int ho = res_out(h, 3, b.c1.stride, 1), wo = res_out(w, 3, b.c1.stride, 1);
      float* ident = x;
      if (b.has_ds) {
        conv(dsn[i], b.ds, RXh, RXl, B, h, w, spare, nullptr, nullptr, EPI_STORE);
        ident = spare;
      }
      conv(c2n[i], b.c2, RTh, RTl, B, ho, wo, ident, RXh, RXl, EPI_RESRELU);
      if (b.has_ds) std::swap(x, spare);
      h = ho;
      w = wo;
    }
    // AdaptiveAvgPool2d((1, None)) -> [B*M, 512]; projection + positional table
    timed("r.avgpool", 0, 4.0 * B * (double)h * w * 512, [&] { launch_res_avgpool(x, RP, B, h, w, 512, stream); });
    launch_res_posrep(RPOS, RPOSB, rows, M, d, stream);
    auto rg = [&]() {
      RowGemmParams p{};
      p.B = rows;
      p.d = d;
      p.max_pos = cfg.max_pos;
      return p;
    };
    RowGemmParams p = rg();
    p.A = RP; p.W = W(lay->projw); p.bias = W(lay->projb); p.resid = RPOSB; p.out = EX0; p.out_stats = ES0;
    p.N = d; p.K = 512; p.ldo = d; p.n_valid = d; p.epi = DEC_RESADD;
    timed("r.proj", 2.0 * rows * d * 512, 4.0 * (rows * 512.0 + d * 512.0 + 2.0 * rows * d),
          [&] { launch_rowgemm(p, stream); });
    // 8 post-norm TransformerEncoderLayers (batch_first on [M, B, d]: attention across images)
    const float *xin = EX0, *xs = nullptr, *xg = nullptr, *xb = nullptr;
    for (size_t l = 0; l < lay->elayers.size(); ++l) {
      const EncLayerW& e = lay->elayers[l];
      timed("r.enc", 2.0 * rows * 256.0 * (768 + 256 + 1024) + 4.0 * rows * (double)B * d,
            4.0 * (rows * 256.0 * 12 + 256.0 * 256 * 8), [&] {
        RowGemmParams q = rg();
        q.A = xin; q.a_stats = xs; q.a_ln_g = xg; q.a_ln_b = xb; q.W = W(e.inw); q.bias = W(e.inb); q.out = EQKV;
        q.N = 3 * d; q.K = d; q.ldo = 3 * d; q.n_valid = 3 * d; q.epi = DEC_STORE;
        launch_rowgemm(q, stream);
        launch_dec_attn(nullptr, 0, EQKV, EQKV + d, EQKV + 2 * d, (size_t)3 * d, M * 3 * d, B, B, EATT, rows, d,
                        cfg.n_heads, stream, 3 * d, M);
        q = rg();
        q.A = EATT; q.W = W(e.ow); q.bias = W(e.ob); q.resid = xin; q.r_stats = xs; q.r_ln_g = xg; q.r_ln_b = xb;
        q.out = EY1; q.out_stats = ES1; q.N = d; q.K = d; q.ldo = d; q.n_valid = d; q.epi = DEC_RESADD;
        launch_rowgemm(q, stream);
        q = rg();
        q.A = EY1; q.a_stats = ES1; q.a_ln_g = W(e.n1w); q.a_ln_b = W(e.n1b); q.W = W(e.l1w); q.bias = W(e.l1b);
        q.out = EH; q.N = cfg.d_ff; q.K = d; q.ldo = cfg.d_ff; q.n_valid = cfg.d_ff; q.epi = DEC_RELU;
        launch_rowgemm(q, stream);
        q = rg();
        q.A = EH; q.W = W(e.l2w); q.bias = W(e.l2b); q.resid = EY1; q.r_stats = ES1; q.r_ln_g = W(e.n1w);
        q.r_ln_b = W(e.n1b); q.out = EY2; q.out_stats = ES2; q.N = d; q.K = cfg.d_ff; q.ldo = d; q.n_valid = d;
        q.epi = DEC_RESADD;
        launch_rowgemm(q, stream);
      });
      xin = EY2;
      xs = ES2;
      xg = W(e.n2w);
      xb = W(e.n2b);
    }
    // memory = LN2 of the last layer (materialised for mocr_get_memory) and every decoder
    // layer's cross-attention K/V from it (LayerNorm applied on load)
    launch_ln_rows(xin, xs, xg, xb, MEM, rows, stream);
    const size_t kv_layer = (size_t)cfg.max_batch * M * 2 * d;
    for (int l = 0; l < cfg.n_layers; ++l) {
      const DecLayerW& dl = lay->layers[l];
      RowGemmParams q = rg();
      q.A = xin; q.a_stats = xs; q.a_ln_g = xg; q.a_ln_b = xb; q.W = W(dl.ca_inw) + (size_t)d * d;
      q.bias = W(dl.ca_inb) + d; q.out = MEMKV + l * kv_layer; q.N = 2 * d; q.K = d; q.ldo = 2 * d;
      q.n_valid = 2 * d; q.epi = DEC_STORE;
      timed("crosskv", 2.0 * rows * 512 * 256, 4.0 * (rows * 256.0 + 512 * 256 + rows * 512.0),
            [&] { launch_rowgemm(q, stream); });
    }
    split_memkv24(B);
  }

  // ---------------------------------------------------------------- setup
  void init(const mocr_config& c, int dev) {
    check_config(c);
    cfg = c;
    device = dev;
    MOCR_HIP_CHECK(hipSetDevice(device));
    MOCR_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    lay.reset(new Layout(cfg));

    const size_t B = cfg.max_batch;
    Vpad = (cfg.vocab + 127) / 128 * 128;  // whole logits tiles of up to 128 columns (decwide.hip)
    const size_t d = cfg.d_model, L = cfg.n_layers;
    if (cfg.arch == MOCR_ARCH_RES18TRANS) {
      init_res18();
    } else {
      H1 = cfg.img_h / 4;
      W1 = cfg.img_w / 4;
      int H = H1, Wd = W1, C = kEmbed;
      for (int s = 0; s < kStages; ++s) {
        stage[s] = make_win(H, Wd, C, kHeads[s]);
        const WinGeom& wg = stage[s].win[0];
        szX = std::max(szX, B * H * Wd * C);
        szXW = std::max(szXW, B * wg.nWin * kWinTok * C);
        szQKV = std::max(szQKV, B * wg.nWin * kWinTok * 3 * C);
        szHID = std::max(szHID, B * H * Wd * 4 * C);
        if (s < kStages - 1) {
          const int Ho = (H + 1) / 2, Wo = (Wd + 1) / 2;
          szXW = std::max(szXW, B * Ho * Wo * 4 * C);
          szX = std::max(szX, B * Ho * Wo * 2 * C);
          H = Ho;
          Wd = Wo;
          C *= 2;
        }
      }
      Hm = H;
      Wm = Wd;
      M = Hm * Wm;

      dw = dalloc<float>(lay->total);
      relbias.assign(lay->blocks.size(), nullptr);
      for (size_t i = 0, bi = 0; i < (size_t)kStages; ++i)
        for (int j = 0; j < kDepth[i]; ++j, ++bi) relbias[bi] = dalloc<float>((size_t)kHeads[i] * kWinTok * kWinTok);
      relmask.assign(lay->blocks.size(), nullptr);
      if (cfg.precision != MOCR_PRECISION_FP32)
        for (size_t i = 0, bi = 0; i < (size_t)kStages; ++i)
          for (int j = 0; j < kDepth[i]; ++j, ++bi) relmask[bi] = dalloc<float>((size_t)4 * kHeads[i] * 64 * 64);
      fcw_pad = dalloc<float>((size_t)Vpad * d);
      fcb_pad = dalloc<float>(Vpad);
      kvw_all = dalloc<float>(L * 2 * d * d);
      kvb_all = dalloc<float>(L * 2 * d);

      img = dalloc<float>(B * cfg.img_h * cfg.img_w);
      X = dalloc<float>(szX);
      X2 = dalloc<float>(szX);
      XW = dalloc<float>(szXW);
      ATT = dalloc<float>(szXW);
      QKV = dalloc<float>(szQKV);
      HID = dalloc<float>(szHID);
      MEM = dalloc<float>(B * M * d);
      MEMKV = dalloc<float>(B * M * L * 2 * d);
      if (cfg.precision != MOCR_PRECISION_FP32) {
        const bool x3 = cfg.precision == MOCR_PRECISION_BF16X3;
        XWh = dalloc<uint16_t>(szXW);
        ATTh = dalloc<uint16_t>(szXW);
        HIDh = dalloc<uint16_t>(szHID);
        MEMh = dalloc<uint16_t>(B * M * d);
        dwh = dalloc<uint16_t>(lay->total);
        kvwh = dalloc<uint16_t>(L * 2 * d * d);
        if (x3) {
          XWl = dalloc<uint16_t>(szXW);
          ATTl = dalloc<uint16_t>(szXW);
          HIDl = dalloc<uint16_t>(szHID);
          MEMl = dalloc<uint16_t>(B * M * d);
          dwl = dalloc<uint16_t>(lay->total);
          kvwl = dalloc<uint16_t>(L * 2 * d * d);
        }
      }

    }

    // decoder rows: one per image (greedy) or per hypothesis (beam search)
    const size_t R = B * std::max(1, cfg.max_beam);
    max_rows = (int)R;
    dx = dalloc<float>(R * d);
    dq = dalloc<float>(R * d);
    datt = dalloc<float>(R * d);
    dy_sa = dalloc<float>(R * d);
    dy_ca = dalloc<float>(R * d);
    dy_ff = dalloc<float>(R * d);
    ds_sa = dalloc<float>(R * 32);
    ds_ca = dalloc<float>(R * 32);
    ds_ff = dalloc<float>(R * 32);
    dh = dalloc<float>(R * cfg.d_ff);
    dlogits = dalloc<float>(R * Vpad);
    dpart = dalloc<float>(B * Vpad / 4);
    kcache = dalloc<float>(L * R * cfg.max_pos * d);
    vcache = dalloc<float>(L * R * cfg.max_pos * d);
    if (kv24()) {
      const size_t nkv = (size_t)B * M * L * 2 * d, nc = L * R * cfg.max_pos * d;
      if (kvx16()) {
        MEMKV16 = dalloc<int16_t>(nkv);
        MEMKVS = dalloc<float>((size_t)L * B * 2 * d);
      } else {
        MEMKV24 = dalloc<uint8_t>(3 * nkv);
      }
      if (self16()) {
        kc16 = dalloc<int16_t>(nc);
        vc16 = dalloc<int16_t>(nc);
        ksc16 = dalloc<float>(nc / 32);
        vsc16 = dalloc<float>(nc / 32);
        // zeroed (engine stream): a scale slot is read before the step that writes it (the
        // key loop's masked keys); leftover bytes of a freed engine could be NaN
        MOCR_HIP_CHECK(hipMemsetAsync(ksc16, 0, nc / 32 * sizeof(float), stream));
        MOCR_HIP_CHECK(hipMemsetAsync(vsc16, 0, nc / 32 * sizeof(float), stream));
      } else {
        kc24 = dalloc<uint8_t>(3 * nc);
        vc24 = dalloc<uint8_t>(3 * nc);
      }
    }
    ld_ids = cfg.max_pos + 1;
    if (cfg.max_beam > 0) {
      bscore = dalloc<float>(R);
      bfin = dalloc<int32_t>(R);
      for (int i = 0; i < 2; ++i) {
        bseq[i] = dalloc<int32_t>(R * ld_ids);
        bslot[i] = dalloc<int32_t>(R * ld_ids);
        // engine stream, not the null stream (see init_res18's rzero)
        MOCR_HIP_CHECK(hipMemsetAsync(bseq[i], 0, R * ld_ids * sizeof(int32_t), stream));
        MOCR_HIP_CHECK(hipMemsetAsync(bslot[i], 0, R * ld_ids * sizeof(int32_t), stream));
      }
    }
    if (fold_greedy()) {
      const size_t ff = cfg.d_ff;
      const size_t per = 2 * d * d + 3 * d + ff * 2 * d + 3 * ff + 3 * d * (ff + d) + 9 * d;
      fold_buf = dalloc<float>(per * L);
      fold_floats = per * L;
      if (cfg.precision == MOCR_PRECISION_BF16X3 && dwl) {  // the Swin engine's blob planes exist
        fold_h = dalloc<uint16_t>(per * L);
        fold_l = dalloc<uint16_t>(per * L);
      }
      foldw.resize(L);
      float* f = fold_buf;
      auto take = [&](size_t n) {
        float* o = f;
        f += n;
        return o;
      };
      for (size_t l = 0; l < L; ++l) {
        FoldW& w = foldw[l];
        w.wzq = take(2 * d * d);
        w.bzq = take(d);
        w.sq = take(d);
        w.cq = take(d);
        w.wzh = take(ff * 2 * d);
        w.bzh = take(ff);
        w.sh = take(ff);
        w.ch = take(ff);
        w.wzqkv = take(3 * d * (ff + d));
        w.bzqkv = take(3 * d);
        w.sqkv = take(3 * d);
        w.cqkv = take(3 * d);
      }
      qtab = dalloc<float>((size_t)cfg.vocab * 3 * d);
      qpos = dalloc<float>((size_t)cfg.max_pos * 3 * d);
      dzqkv = dalloc<float>(R * 3 * d);  // rows: images, or hypotheses (beam search)
    }
    ids = dalloc<int32_t>(B * ld_ids);
    feed = dalloc<int32_t>(B * ld_ids);
    forced = dalloc<int32_t>(B * ld_ids);
    finished = dalloc<int32_t>(B);
    logp = dalloc<float>(B * cfg.max_pos);
    st = dalloc<DecodeState>(1);
    MOCR_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&st_host), 2 * sizeof(DecodeState), hipHostMallocDefault));
    for (auto& e : chunk_ev) MOCR_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));  // the setup memsets above
  }

  // [type][h][64 q][64 key] table of the bf16 attention kernel: bias[h][q][key] plus the
  // shifted-window mask (-100 across regions, torchvision shifted_window_attention) of
  // window type (last window row, last window column), -inf on the padded keys 49..63,
  // 0 on the padded query rows.  A window's region ids depend only on whether it is
  // the last one along each axis: shift_region(7 w + p, P, s) = 0 for w < P/7 - 1, and
  // 1 + (p >= 7 - s) for the last window (2 everywhere when s = 0).
  void build_relmask(const std::vector<float>& rb, int h, const WinGeom& wg, float* dst) {
    const bool masked = wg.sh + wg.sw > 0;
    auto reg = [](int p, bool last, int sft) { return sft == 0 ? 2 : (last ? 1 + (p >= kWin - sft) : 0); };
    std::vector<float> t((size_t)4 * h * 64 * 64, 0.f);
    for (int type = 0; type < 4; ++type) {
      const bool ly = type & 2, lx = type & 1;
      for (int hh = 0; hh < h; ++hh)
        for (int q = 0; q < kWinTok; ++q)
          for (int k = 0; k < 64; ++k) {
            float v = -INFINITY;
            if (k < kWinTok) {
              v = rb[((size_t)hh * kWinTok + q) * kWinTok + k];
              if (masked) {
                const int rq = 3 * reg(q / kWin, ly, wg.sh) + reg(q % kWin, lx, wg.sw);
                const int rk = 3 * reg(k / kWin, ly, wg.sh) + reg(k % kWin, lx, wg.sw);
                if (rq != rk) v += -100.0f;
              }
            }
            t[(((size_t)type * h + hh) * 64 + q) * 64 + k] = v;
          }
    }
    MOCR_HIP_CHECK(hipMemcpy(dst, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
  }

  void load_weights(const float* blob, size_t n) {
    if (n != lay->total)
      throw std::runtime_error("weight blob has " + std::to_string(n) + " floats, expected " +
                               std::to_string(lay->total));
    MOCR_HIP_CHECK(hipSetDevice(device));
    MOCR_HIP_CHECK(hipMemcpy(dw, blob, n * sizeof(float), hipMemcpyHostToDevice));
    if (cfg.arch == MOCR_ARCH_RES18TRANS) load_res18(blob);
    // Expanded relative-position bias [h, 49, 49] = table[index(i, j), h]
    // (torchvision _get_relative_position_bias with relative_position_index).
    size_t bi = 0;
    for (int s = 0; s < kStages && cfg.arch == MOCR_ARCH_SWIN; ++s) {
      const int h = kHeads[s];
      for (int j = 0; j < kDepth[s]; ++j, ++bi) {
        const float* table = blob + lay->blocks[bi].table;
        std::vector<float> rb((size_t)h * kWinTok * kWinTok);
        for (int i = 0; i < kWinTok; ++i)
          for (int k = 0; k < kWinTok; ++k) {
            const int dy = i / kWin - k / kWin + kWin - 1;
            const int dx = i % kWin - k % kWin + kWin - 1;
            const int idx = dy * (2 * kWin - 1) + dx;
            for (int hh = 0; hh < h; ++hh) rb[((size_t)hh * kWinTok + i) * kWinTok + k] = table[idx * h + hh];
          }
        MOCR_HIP_CHECK(hipMemcpy(relbias[bi], rb.data(), rb.size() * sizeof(float), hipMemcpyHostToDevice));
        if (relmask[bi]) build_relmask(rb, h, stage[s].win[j & 1], relmask[bi]);
      }
    }
    // Everything below runs on the engine's stream, ordered behind the uploads above: the
    // stream is non-blocking, so null-stream memsets / device-to-device copies (which may
    // return before they complete) would race the split kernels that read them.
    MOCR_HIP_CHECK(hipDeviceSynchronize());
    const size_t d = cfg.d_model, V = cfg.vocab;
    MOCR_HIP_CHECK(hipMemsetAsync(fcw_pad, 0, (size_t)Vpad * d * sizeof(float), stream));
    MOCR_HIP_CHECK(hipMemsetAsync(fcb_pad, 0, (size_t)Vpad * sizeof(float), stream));
    MOCR_HIP_CHECK(hipMemcpyAsync(fcw_pad, dw + lay->fcw, V * d * sizeof(float), hipMemcpyDeviceToDevice, stream));
    MOCR_HIP_CHECK(hipMemcpyAsync(fcb_pad, dw + lay->fcb, V * sizeof(float), hipMemcpyDeviceToDevice, stream));
    for (int l = 0; l < cfg.n_layers; ++l) {
      const DecLayerW& w = lay->layers[l];
      MOCR_HIP_CHECK(hipMemcpyAsync(kvw_all + (size_t)l * 2 * d * d, dw + w.ca_inw + d * d, 2 * d * d * sizeof(float),
                                    hipMemcpyDeviceToDevice, stream));
      MOCR_HIP_CHECK(hipMemcpyAsync(kvb_all + (size_t)l * 2 * d, dw + w.ca_inb + d, 2 * d * sizeof(float),
                                    hipMemcpyDeviceToDevice, stream));
    }
    if (dwh) {
      launch_split_bf16(dw, dwh, dwl, lay->total, stream);
      launch_split_bf16(kvw_all, kvwh, kvwl, (size_t)cfg.n_layers * 2 * d * d, stream);
      MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    }
    if (dwh && cfg.arch != MOCR_ARCH_RES18TRANS) pack_swin_frags();
    if (fold_greedy()) fold_decoder();
    if (fold_wide()) pack_frags();
    MOCR_HIP_CHECK(hipDeviceSynchronize());
    weights_loaded = true;
    encoded = false;
  }

  // Folded greedy-step weights (kernels.h FoldGemmParams), fp64-accumulated on the device.
  // For a LayerNorm (g, b) in front of W x + c: W' = W diag(g), s = W g, c' = W b + c, and
  // W' times the producer's terms: z_q over [SA attn | x] = [W_q' W_o | W_q'] + W_q' b_o;
  // z_h over [CA attn | LN1(y_sa)] = [W_1' W_o | W_1'] + W_1' b_o; the next layer's z_qkv
  // over [hidden | LN2(y_ca)] = [W_in' W_2 | W_in'] + W_in' b_2.  Layer 0's q|k|v of token
  // v at position p: qtab[v] + qpos[p] = W_in emb[v] + b_in + W_in pos[p].
  void fold_decoder() {
    const int d = cfg.d_model, ff = cfg.d_ff, L = cfg.n_layers;
    hipStream_t s = stream;
    for (int l = 0; l < L; ++l) {
      const DecLayerW& w = lay->layers[l];
      FoldW& f = foldw[l];
      const float* wq = W(w.ca_inw);  // q rows of the cross-attention in_proj
      launch_fold_mm(wq, d, W(w.n1w), W(w.sa_ow), d, 1, d, nullptr, nullptr, f.wzq, 2 * d, d, d, s);
      launch_fold_mm(wq, d, W(w.n1w), nullptr, 0, 0, 0, nullptr, nullptr, f.wzq + d, 2 * d, d, d, s);
      launch_fold_mm(wq, d, W(w.n1w), W(w.sa_ob), 1, 0, d, nullptr, nullptr, f.bzq, 1, d, 1, s);
      launch_fold_mm(wq, d, nullptr, W(w.n1w), 1, 0, d, nullptr, nullptr, f.sq, 1, d, 1, s);
      launch_fold_mm(wq, d, nullptr, W(w.n1b), 1, 0, d, W(w.ca_inb), nullptr, f.cq, 1, d, 1, s);
      const float* w1 = W(w.l1w);
      launch_fold_mm(w1, d, W(w.n2w), W(w.ca_ow), d, 1, d, nullptr, nullptr, f.wzh, 2 * d, ff, d, s);
      launch_fold_mm(w1, d, W(w.n2w), nullptr, 0, 0, 0, nullptr, nullptr, f.wzh + d, 2 * d, ff, d, s);
      launch_fold_mm(w1, d, W(w.n2w), W(w.ca_ob), 1, 0, d, nullptr, nullptr, f.bzh, 1, ff, 1, s);
      launch_fold_mm(w1, d, nullptr, W(w.n2w), 1, 0, d, nullptr, nullptr, f.sh, 1, ff, 1, s);
      launch_fold_mm(w1, d, nullptr, W(w.n2b), 1, 0, d, W(w.l1b), nullptr, f.ch, 1, ff, 1, s);
      if (l + 1 < L) {
        const DecLayerW& nx = lay->layers[l + 1];
        const float* wi = W(nx.sa_inw);
        launch_fold_mm(wi, d, W(w.n3w), W(w.l2w), ff, 1, d, nullptr, nullptr, f.wzqkv, ff + d, 3 * d, ff, s);
        launch_fold_mm(wi, d, W(w.n3w), nullptr, 0, 0, 0, nullptr, nullptr, f.wzqkv + ff, ff + d, 3 * d, d, s);
        launch_fold_mm(wi, d, W(w.n3w), W(w.l2b), 1, 0, d, nullptr, nullptr, f.bzqkv, 1, 3 * d, 1, s);
        launch_fold_mm(wi, d, nullptr, W(w.n3w), 1, 0, d, nullptr, nullptr, f.sqkv, 1, 3 * d, 1, s);
        launch_fold_mm(wi, d, nullptr, W(w.n3b), 1, 0, d, W(nx.sa_inb), nullptr, f.cqkv, 1, 3 * d, 1, s);
      }
    }
    const DecLayerW& l0 = lay->layers[0];
    launch_fold_mm(W(lay->emb), d, nullptr, W(l0.sa_inw), 1, d, d, nullptr, W(l0.sa_inb), qtab, 3 * d, cfg.vocab,
                   3 * d, s);
    launch_fold_mm(W(lay->pos), d, nullptr, W(l0.sa_inw), 1, d, d, nullptr, nullptr, qpos, 3 * d, cfg.max_pos, 3 * d, s);
    if (fold_h) launch_split_bf16(fold_buf, fold_h, fold_l, fold_floats, s);
    MOCR_HIP_CHECK(hipStreamSynchronize(s));
  }

  // Fragment-major weights of the wide fold GEMMs and logits (decwide.hip), packed from the
  // fp32 sources after fold_decoder: bf16x3 planes in bf16x3 engines, fp32 otherwise.
  // The buffers are allocated by the first load and repacked in place by later ones: the
  // captured decode graphs hold their addresses.
  void pack_frag(FragW& f, const float* W, int N, int K, bool x3) {
    const size_t n = (size_t)N * K;
    if (x3 && !f.hi) {
      f.hi = dalloc<uint16_t>(n);
      f.lo = dalloc<uint16_t>(n);
      frag_allocs.push_back(f.hi);
      frag_allocs.push_back(f.lo);
    } else if (!x3 && !f.f) {
      f.f = dalloc<float>(n);
      frag_allocs.push_back(f.f);
    }
    launch_frag_pack(W, N, K, f.hi, f.lo, f.f, stream);
  }
  void pack_swin_frags() {
    {  // merge 1: 4 x 96 = 384 channels -> 192 (lngemm384)
      const MergeW& m = lay->merge[0];
      if (!mergepack) {
        mergepack = dalloc<char>((size_t)192 * 384 * 2 * (dwl ? 2 : 1));
        frag_allocs.push_back(mergepack);
      }
      launch_lngemm384_pack(dwh + m.redw, dwl ? dwl + m.redw : nullptr, 192, mergepack, stream);
      if (!mergefrag.hi) {  // merge.hip's registers-resident W (hi / lo; bf16 engines read hi)
        mergefrag.hi = dalloc<uint16_t>((size_t)192 * 384);
        mergefrag.lo = dalloc<uint16_t>((size_t)192 * 384);
        frag_allocs.push_back(mergefrag.hi);
        frag_allocs.push_back(mergefrag.lo);
      }
      launch_frag_pack(W(m.redw), 192, 384, mergefrag.hi, mergefrag.lo, nullptr, stream);
    }
    int nb = 0;
    for (int st = 0; st < kStages; ++st) nb += kDepth[st];
    if (swinfrag.empty()) swinfrag.resize(nb);
    for (int st = 0, bi = 0; st < kStages; ++st) {
      const int C = stage[st].C;  // the fused kernels' W_qkv (+ W_proj at C = 96, 192)
      for (int j = 0; j < kDepth[st]; ++j, ++bi) {
        const SwinBlockW& w = lay->blocks[bi];
        // W_qkv fragments: the fused attention kernels of stages 1-3 (stage 4 only under
        // MOCR_VARIANT_S4_FUSED_ATTN), W_proj at C = 96, 192
        // (W_proj's fragments only when the fused attention that reads them runs)
        const bool need_frag[2] = {attn_fused() && (C != 768 || (cfg.variant & MOCR_VARIANT_S4_FUSED_ATTN)),
                                   attn_fused() && swin_attn_fused_supported(C)};
        for (int m = 0; m < 2; ++m) {
          if (!need_frag[m]) continue;
          FragW& f = swinfrag[bi][m];
          const int N = m == 0 ? 3 * C : C;
          if (!f.hi) {
            f.hi = dalloc<uint16_t>((size_t)N * C);
            f.lo = dalloc<uint16_t>((size_t)N * C);
            frag_allocs.push_back(f.hi);
            frag_allocs.push_back(f.lo);
          }
          launch_frag_pack(W(m == 0 ? w.qkvw : w.projw), N, C, f.hi, f.lo, nullptr, stream, m == 1);
        }
        if (const size_t pb = mlp_pack_bytes(C, dwl != nullptr)) {
          if (mlppack.size() <= (size_t)bi) mlppack.resize(bi + 1, nullptr);
          if (!mlppack[bi]) {
            mlppack[bi] = dalloc<char>(pb);
            frag_allocs.push_back(mlppack[bi]);
          }
          MlpParams mp{};
          mp.C = C;
          mp.w1 = dwh + w.fc1w;
          mp.w1lo = dwl ? dwl + w.fc1w : nullptr;
          mp.w2 = dwh + w.fc2w;
          mp.w2lo = dwl ? dwl + w.fc2w : nullptr;
          if (C == 384) {  // W_proj's chunk images for the block tail kernel (s3_tail_fused)
            mp.wproj = dwh + w.projw;
            mp.wproj_lo = dwl ? dwl + w.projw : nullptr;
          }
          launch_mlp_pack(mp, mlppack[bi], stream);
        }
        // lngemm384's W_qkv image: stage 3's norm1 + qkv runs on it only when its fused
        // attention kernel does not (MOCR_VARIANT_UNFUSED_ATTN)
        if (C == 384 && !attn_fused() && !(cfg.variant & MOCR_VARIANT_UNFUSED_LN_GEMM)) {
          if (lngpack.size() <= (size_t)bi) lngpack.resize(bi + 1, nullptr);
          if (!lngpack[bi]) {
            lngpack[bi] = dalloc<char>((size_t)3 * C * C * 2 * (dwl ? 2 : 1));
            frag_allocs.push_back(lngpack[bi]);
          }
          launch_lngemm384_pack(dwh + w.qkvw, dwl ? dwl + w.qkvw : nullptr, 3 * C, lngpack[bi], stream);
        }
      }
    }
  }
  void pack_frags() {
    const int d = cfg.d_model, ff = cfg.d_ff, L = cfg.n_layers;
    const bool x3 = fold_h != nullptr;
    if (fragw.empty()) fragw.resize(L);
    for (int l = 0; l < L; ++l) {
      const DecLayerW& w = lay->layers[l];
      const FoldW& f = foldw[l];
      pack_frag(fragw[l][0], W(w.sa_ow), d, d, x3);
      pack_frag(fragw[l][1], f.wzq, d, 2 * d, x3);
      pack_frag(fragw[l][2], W(w.ca_ow), d, d, x3);
      pack_frag(fragw[l][3], f.wzh, ff, 2 * d, x3);
      pack_frag(fragw[l][4], W(w.l2w), d, ff, x3);
      if (l + 1 < L) pack_frag(fragw[l][5], f.wzqkv, 3 * d, ff + d, x3);
    }
    pack_frag(frag_logits, fcw_pad, Vpad, d, logits_x3());
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
  }

  void set_images(const float* src, int B, hipMemcpyKind kind) {
    if (B < 1 || B > cfg.max_batch) throw std::runtime_error("batch must be in [1, max_batch]");
    MOCR_HIP_CHECK(hipSetDevice(device));
    MOCR_HIP_CHECK(
        hipMemcpyAsync(img, src, (size_t)B * cfg.img_h * cfg.img_w * sizeof(float), kind, stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    cur_batch = B;
    encoded = false;
  }

  // ---------------------------------------------------------------- timing
  hipEvent_t get_event() {
    if (!event_pool.empty()) {
      hipEvent_t e = event_pool.back();
      event_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    MOCR_HIP_CHECK(hipEventCreate(&e));
    return e;
  }

  template <typename F>
  void timed(const char* name, double flops, double bytes, F&& f) {
    if (!timing) {
      f();
      return;
    }
    TimingRec r{name, get_event(), get_event(), flops, bytes};
    MOCR_HIP_CHECK(hipEventRecord(r.e0, stream));
    f();
    MOCR_HIP_CHECK(hipEventRecord(r.e1, stream));
    pending.push_back(r);
  }

  void flush_timing() {
    for (auto& r : pending) {
      MOCR_HIP_CHECK(hipEventSynchronize(r.e1));
      float ms = 0.f;
      MOCR_HIP_CHECK(hipEventElapsedTime(&ms, r.e0, r.e1));
      mocr_kernel_stat& s = stats[r.name];
      std::strncpy(s.name, r.name.c_str(), sizeof(s.name) - 1);
      s.launches += 1;
      s.total_ms += ms;
      s.flops += r.flops;
      s.bytes += r.bytes;
      event_pool.push_back(r.e0);
      event_pool.push_back(r.e1);
    }
    pending.clear();
  }

  // ---------------------------------------------------------------- encoder
  // A GEMM operand in the engine's precision: fp32, or bf16 hi (+ lo) planes.
  struct Operand {
    const float* f32;
    const uint16_t* hi;
    const uint16_t* lo;
  };
  Operand wop(size_t off) const { return {dw + off, dwh ? dwh + off : nullptr, dwl ? dwl + off : nullptr}; }
  bool bf16_mode() const { return cfg.precision != MOCR_PRECISION_FP32; }
  // Kernel-path variants (include/mathocr.h MOCR_VARIANT_*): the production path fuses
  // norm1 + qkv + W-MSA + proj (wattn.hip) and norm2 + MLP (mlp.hip) in the bf16 modes for
  // the stages those kernels are built for, and runs greedy decoding on the folded step
  // (kernels.h FoldGemmParams).  Beam search always uses the projection+attention kernel
  // (slot-table keys, shared image memory).
  bool attn_fused() const { return !(cfg.variant & MOCR_VARIANT_UNFUSED_ATTN); }
  bool mlp_fused() const { return !(cfg.variant & MOCR_VARIANT_UNFUSED_MLP); }
  bool fold_greedy() const { return !(cfg.variant & MOCR_VARIANT_DEC_UNFOLDED); }
  // wide-tile fold GEMMs and logits (decwide.hip) unless MOCR_VARIANT_DEC_NARROW
  bool fold_wide() const { return fold_greedy() && !(cfg.variant & MOCR_VARIANT_DEC_NARROW); }
  // the folded greedy step of bf16x3 engines streams its K/V as fp24 (common.h) unless
  // MOCR_VARIANT_KV_F32; fp32 engines keep fp32 K/V
  bool kv24() const {
    return fold_greedy() && cfg.precision == MOCR_PRECISION_BF16X3 && !(cfg.variant & MOCR_VARIANT_KV_F32);
  }
  // ... with the cross-attention K/V in int16 and per-column scales, unless
  // MOCR_VARIANT_CROSS_KV_F24 (fp24)
  bool kvx16() const { return kv24() && !(cfg.variant & MOCR_VARIANT_CROSS_KV_F24); }
  // ... and the self-attention cache in int16 with one scale per (row, head, key) over its
  // 32 values (decfold.hip KVF 3), unless MOCR_VARIANT_SELF_KV_F24
  bool self16() const { return kv24() && !(cfg.variant & MOCR_VARIANT_SELF_KV_F24); }
  // beam search on the folded step (int16 or fp32 self-attention cache through slot
  // tables), unless MOCR_VARIANT_BEAM_UNFOLDED or a cache format the slot kernels lack (fp24)
  bool beam_folded() const {
    return fold_greedy() && !(cfg.variant & MOCR_VARIANT_BEAM_UNFOLDED) && (self16() || !kv24());
  }
  // the int16 (or fp24) cross-attention K/V of the B encoded images from MEMKV
  void split_memkv24(int B) {
    if (!kv24()) return;
    const int d = cfg.d_model;
    const size_t kv_layer = (size_t)cfg.max_batch * M * 2 * d;
    if (kvx16()) {
      timed("memkv(i16)", 0, 6.0 * cfg.n_layers * (double)B * M * 2 * d, [&] {
        launch_quant_kv_i16(MEMKV, MEMKV16, MEMKVS, B, M, cfg.n_layers, kv_layer, (size_t)cfg.max_batch * 2 * d,
                            stream);
      });
      return;
    }
    timed("memkv(fp24)", 0, 7.0 * cfg.n_layers * (double)B * M * 2 * d, [&] {
      for (int l = 0; l < cfg.n_layers; ++l)
        launch_split_kv_fp24(MEMKV + l * kv_layer, MEMKV24 + 3 * l * kv_layer, B, M, stream);
    });
  }
  // the wide logits on bf16x3 MFMA (fc_out planes) in bf16x3 engines unless MOCR_VARIANT_LOGITS_F32
  bool logits_x3() const {
    return fold_wide() && cfg.precision == MOCR_PRECISION_BF16X3 && !(cfg.variant & MOCR_VARIANT_LOGITS_F32);
  }
  void fold_gemm(FoldGemmParams& g, hipStream_t s, int layer, int which) {
    if (fold_wide()) {
      g.NY = cfg.d_model;
      const FragW& fy = fragw[layer][2 * which];
      const FragW& fz = fragw[layer][2 * which + 1];
      g.Fy_hi = fy.hi; g.Fy_lo = fy.lo; g.Fy = fy.f;
      g.Fz_hi = fz.hi; g.Fz_lo = fz.lo; g.Fz = fz.f;
      launch_foldwide(g, s);
    } else {
      launch_foldgemm(g, s);
    }
  }
  // stage 3 always (285 vs 301 us per block unfused at B=64, 384²); stage 4 only on request
  // (258 vs 211 us: a window's 64 padded rows re-read all of W_qkv, 1.8 GB from L2 per block,
  // and the padding costs 1.3x the GEMM's MFMA work)
  // stage 3 (C = 384) fused at every batch since its W_qkv fragments are fragment-major
  // (round 4): 8.30 vs 8.93 ms per 512-image encode for lngemm384 + the window attention,
  // bench +1 %, and no fp32 QKV round trip through HBM (profiles/r04/r04x).  Round 3 kept it
  // below 128 images (1054 vs 903 us per block at B = 256 with row-major fragments,
  // profiles/r03/op_times_b256.log).
  bool noproj_fused(int C) const {
    return attn_fused() && swin_attn_noproj_supported(C) && (C != 768 || (cfg.variant & MOCR_VARIANT_S4_FUSED_ATTN));
  }
  // stage 3's kernels for >= 128 images: the unfused attention (above) and mlp.hip's fused
  // C = 384 MLP, which runs 128 rows per workgroup on all 256 CUs (1152 workgroups at
  // B = 256: 989 vs 1298 us per block for ln2 + fc1 + fc2; at B = 64 its 288 workgroups
  // take two rounds, 476 vs 334 us, profiles/r03/mlp384_*.log)
  bool s3_large(int B) const { return B >= 128 || (cfg.variant & MOCR_VARIANT_S3_LARGE_BATCH); }
  // stage 3's block tail at >= 128 images: the attention output
  // projection + residual inside the fused MLP kernel (mlp.hip mlp384_kernel PROJ), which
  // takes O from the fused attention's ATT planes in X's row order
  bool s3_tail_fused(int C, int B) const {
    return C == 384 && bf16_mode() && noproj_fused(C) && s3_large(B) && mlp_fused() && mlp_fused_supported(C) &&
           !(cfg.variant & MOCR_VARIANT_UNFUSED_S3_TAIL);
  }
  int attn_passes() const {
    return cfg.precision == MOCR_PRECISION_FP32 ? 0 : (cfg.precision == MOCR_PRECISION_BF16X3 ? 3 : 1);
  }

  void gemm(const char* name, Operand A, Operand Wt, const float* bias, float* C, uint16_t* Ch, uint16_t* Cl,
            int Mrows, int N, int K, int epi, const WinGeom* wg, long alg_rows, int col_split = 0,
            size_t split_stride = 0, uint8_t* kv24 = nullptr, int kv_M = 0, int16_t* kv16 = nullptr,
            float* kv16_scale = nullptr, size_t kv16_sstride = 0) {
    GemmParams p{};
    p.kv24 = kv24;
    p.kv_M = kv_M;
    p.kv16 = kv16;
    p.kv16_scale = kv16_scale;
    p.kv16_sstride = kv16_sstride;
    if (bf16_mode()) {
      p.A = A.hi;
      p.A_lo = A.lo;
      p.W = Wt.hi;
      p.W_lo = Wt.lo;
      p.C16 = Ch;
      p.C16lo = Cl;
    } else {
      p.A = A.f32;
      p.W = Wt.f32;
    }
    p.bias = bias;
    p.C = C;
    p.M = Mrows;
    p.N = N;
    p.K = K;
    p.lda = K;
    p.ldw = K;
    p.ldc = N;
    p.epi = epi;
    if (wg) p.win = *wg;
    p.col_split = col_split;
    p.split_stride = split_stride;
    const double flops = 2.0 * alg_rows * N * K;
    const double ab = bf16_mode() ? (cfg.precision == MOCR_PRECISION_BF16X3 ? 4.0 : 2.0) : 4.0;
    const double bytes = ab * ((double)alg_rows * K + (double)N * K) +
                         4.0 * (double)alg_rows * N * (epi == EPI_RESADD || epi == EPI_WINRES ? 2 : 1);
    timed(name, flops, bytes, [&] {
      if (bf16_mode())
        launch_gemm_bf16(p, stream);
      else
        launch_gemm_f32(p, stream);
    });
  }

  // stop_after = k >= 0 stops after features[k] (0 = stem, 1..7 = stages/merges) and leaves
  // that NHWC map in X (parity debugging); -1 runs the whole encoder.
  void encode(int B, int stop_after = -1) {
    if (!weights_loaded) throw std::runtime_error("weights not loaded");
    if (B != cur_batch) throw std::runtime_error("batch differs from the uploaded images");
    MOCR_HIP_CHECK(hipSetDevice(device));
    if (cfg.arch == MOCR_ARCH_RES18TRANS) {
      if (stop_after >= 0) throw std::runtime_error("encode_until: Swin only");
      encode_res18(B);
      MOCR_HIP_CHECK(hipStreamSynchronize(stream));
      if (timing) flush_timing();
      encoded = true;
      return;
    }
    const size_t d = cfg.d_model, L = cfg.n_layers;
    timed("stem", 2.0 * B * H1 * W1 * kEmbed * 16, 4.0 * B * (cfg.img_h * cfg.img_w + (double)H1 * W1 * kEmbed),
          [&] { launch_stem(img, W(lay->stem_w), W(lay->stem_b), W(lay->stem_lnw), W(lay->stem_lnb), X, B,
                            cfg.img_h, cfg.img_w, stream); });
    if (stop_after == 0) return finish_partial(0);
    size_t bi = 0;
    static const char* qkv_n[] = {"s1.qkv", "s2.qkv", "s3.qkv", "s4.qkv"};
    static const char* proj_n[] = {"s1.proj", "s2.proj", "s3.proj", "s4.proj"};
    static const char* fc1_n[] = {"s1.fc1", "s2.fc1", "s3.fc1", "s4.fc1"};
    static const char* fc2_n[] = {"s1.fc2", "s2.fc2", "s3.fc2", "s4.fc2"};
    static const char* att_n[] = {"s1.wattn", "s2.wattn", "s3.wattn", "s4.wattn"};
    static const char* mrg_n[] = {"merge1", "merge2", "merge3"};
    static const char* ln1_n[] = {"s1.ln1", "s2.ln1", "s3.ln1", "s4.ln1"};
    static const char* lnqkv_n[] = {"s1.lnqkv", "s2.lnqkv", "s3.lnqkv", "s4.lnqkv"};
    static const char* ln2_n[] = {"s1.ln2", "s2.ln2", "s3.ln2", "s4.ln2"};
    static const char* mlp_n[] = {"s1.mlp", "s2.mlp", "s3.mlp", "s4.mlp"};
    static const char* attn_n[] = {"s1.attn", "s2.attn", "s3.attn", "s4.attn"};
    static const char* mln_n[] = {"merge1.ln", "merge2.ln", "merge3.ln"};
    const bool b16 = bf16_mode();
    // GEMM A operands: fp32 buffers, or their bf16 planes
    float* xw32 = b16 ? nullptr : XW;
    float* att32 = b16 ? nullptr : ATT;
    float* hid32 = b16 ? nullptr : HID;
    const Operand opXW{XW, XWh, XWl}, opATT{ATT, ATTh, ATTl}, opHID{HID, HIDh, HIDl};
    for (int s = 0; s < kStages; ++s) {
      const StageGeom& g = stage[s];
      const int C = g.C;
      const long rows = (long)B * g.H * g.W;
      for (int j = 0; j < kDepth[s]; ++j, ++bi) {
        const SwinBlockW& w = lay->blocks[bi];
        const WinGeom& wg = g.win[j & 1];
        const long wrows = (long)B * wg.nWin * kWinTok;
        if (b16 && attn_fused() && swin_attn_fused_supported(C)) {
          // norm1 + qkv + W-MSA + proj + residual in one kernel (wattn.hip)
          SwinAttnParams ap{};
          ap.X = X;
          ap.ln_g = W(w.n1w);
          ap.ln_b = W(w.n1b);
          ap.wqkv = dwh + w.qkvw;
          ap.wqkv_lo = dwl ? dwl + w.qkvw : nullptr;
          ap.bqkv = W(w.qkvb);
          ap.wproj = dwh + w.projw;
          ap.wproj_lo = dwl ? dwl + w.projw : nullptr;
          ap.wqkv_fm = swinfrag.at(bi)[0].hi;
          ap.wqkv_fm_lo = dwl ? swinfrag[bi][0].lo : nullptr;
          ap.wproj_fm = swinfrag[bi][1].hi;
          ap.wproj_fm_lo = dwl ? swinfrag[bi][1].lo : nullptr;
          ap.bproj = W(w.projb);
          ap.table = relmask[bi];
          ap.B = B;
          ap.C = C;
          ap.heads = g.heads;
          ap.wg = wg;
          timed(attn_n[s], 8.0 * rows * C * C + 4.0 * rows * kWinTok * C, 8.0 * rows * C + (dwl ? 4.0 : 2.0) * 4.0 * C * C,
                [&] { launch_swin_attn_fused(ap, stream); });
        } else if (b16 && noproj_fused(C)) {
          // norm1 + qkv + W-MSA in one kernel writing the ATT planes (wattn.hip), then proj
          SwinAttnParams ap{};
          ap.X = X;
          ap.ln_g = W(w.n1w);
          ap.ln_b = W(w.n1b);
          ap.wqkv = dwh + w.qkvw;
          ap.wqkv_lo = dwl ? dwl + w.qkvw : nullptr;
          ap.wqkv_fm = swinfrag.at(bi)[0].hi;
          ap.wqkv_fm_lo = dwl ? swinfrag[bi][0].lo : nullptr;
          ap.bqkv = W(w.qkvb);
          ap.table = relmask[bi];
          ap.att_hi = ATTh;
          ap.att_lo = dwl ? ATTl : nullptr;
          ap.att_pixel_rows = 1;  // O in X's row order: proj over the image's tokens only
          ap.B = B;
          ap.C = C;
          ap.heads = g.heads;
          ap.wg = wg;
          timed(attn_n[s], 6.0 * rows * C * C + 4.0 * rows * kWinTok * C, 4.0 * rows * C + (dwl ? 4.0 : 2.0) * 3.0 * C * C +
                (dwl ? 4.0 : 2.0) * rows * C, [&] { launch_swin_attn_noproj(ap, stream); });
          if (!s3_tail_fused(C, B))
            gemm(proj_n[s], opATT, wop(w.projw), W(w.projb), X, nullptr, nullptr, (int)rows, C, C, EPI_RESADD, nullptr,
                 rows);
        } else if (b16 && !(cfg.variant & MOCR_VARIANT_WINDOW_ROWS)) {
          // the image's tokens only (stage 4 at 384²: 144 of 196 window slots per image):
          // norm1 and qkv in X's row order, the attention kernel maps window slots to pixels
          // and takes the padded tokens' k / v from the qkv bias, O comes out in X's order,
          // proj is a plain residual-add GEMM (bitwise the window-row sequence below)
          if (C == 384 && s3_large(B) && !(cfg.variant & MOCR_VARIANT_UNFUSED_LN_GEMM)) {
            // norm1 + qkv in one kernel (mlp.hip lngemm384_kernel)
            LnGemm384Params lp{};
            lp.X = X; lp.M = rows; lp.ln_g = W(w.n1w); lp.ln_b = W(w.n1b);
            lp.w = dwh + w.qkvw; lp.wlo = dwl ? dwl + w.qkvw : nullptr; lp.b = W(w.qkvb);
            lp.wpk = lngpack.at(bi);
            lp.out = QKV; lp.N = 3 * C;
            timed(lnqkv_n[s], 6.0 * rows * C * C, 4.0 * rows * C + 12.0 * rows * C + (dwl ? 4.0 : 2.0) * 3.0 * C * C,
                  [&] { launch_lngemm384(lp, stream); });
          } else {
            timed(ln1_n[s], 0, 8.0 * rows * C,
                  [&] { launch_layernorm(X, W(w.n1w), W(w.n1b), xw32, XWh, XWl, (int)rows, C, stream); });
            gemm(qkv_n[s], opXW, wop(w.qkvw), W(w.qkvb), QKV, nullptr, nullptr, (int)rows, 3 * C, C, EPI_STORE,
                 nullptr, rows);
          }
          timed(att_n[s], 4.0 * rows * kWinTok * C, 4.0 * (double)rows * 4 * C, [&] {
            launch_window_attention(QKV, relbias[bi], relmask[bi], att32, ATTh, ATTl, B, C, g.heads, wg,
                                    attn_passes(), stream, W(w.qkvb));
          });
          gemm(proj_n[s], opATT, wop(w.projw), W(w.projb), X, nullptr, nullptr, (int)rows, C, C, EPI_RESADD, nullptr,
               rows);
        } else {
          timed(ln1_n[s], 0, 8.0 * wrows * C,
                [&] { launch_ln_partition(X, W(w.n1w), W(w.n1b), xw32, XWh, XWl, B, C, wg, stream); });
          gemm(qkv_n[s], opXW, wop(w.qkvw), W(w.qkvb), QKV, nullptr, nullptr, (int)wrows, 3 * C, C, EPI_STORE,
               nullptr, rows);
          timed(att_n[s], 4.0 * rows * kWinTok * C, 4.0 * (double)rows * 4 * C, [&] {
            launch_window_attention(QKV, relbias[bi], relmask[bi], att32, ATTh, ATTl, B, C, g.heads, wg,
                                    attn_passes(), stream);
          });
          gemm(proj_n[s], opATT, wop(w.projw), W(w.projb), X, nullptr, nullptr, (int)wrows, C, C, EPI_WINRES, &wg,
               rows);
        }
        if (b16 && mlp_fused() && mlp_fused_supported(C) && (C != 384 || s3_large(B))) {
          // norm2 + fc1 + GELU + fc2 + residual in one kernel (mlp.hip)
          MlpParams mp{};
          mp.X = X;
          mp.M = rows;
          mp.C = C;
          mp.ln_g = W(w.n2w);
          mp.ln_b = W(w.n2b);
          mp.w1 = dwh + w.fc1w;
          mp.w1lo = dwl ? dwl + w.fc1w : nullptr;
          mp.b1 = W(w.fc1b);
          mp.w2 = dwh + w.fc2w;
          mp.w2lo = dwl ? dwl + w.fc2w : nullptr;
          mp.b2 = W(w.fc2b);
          mp.wpack = bi < (int)mlppack.size() ? mlppack[bi] : nullptr;
          const bool tail = s3_tail_fused(C, B);
          if (tail) {  // proj + residual in front of norm2 (the block tail, "s3.tail")
            mp.att_hi = ATTh;
            mp.att_lo = dwl ? ATTl : nullptr;
            mp.wproj = dwh + w.projw;
            mp.wproj_lo = dwl ? dwl + w.projw : nullptr;
            mp.bproj = W(w.projb);
          }
          timed(tail ? "s3.tail" : mlp_n[s], (tail ? 18.0 : 16.0) * rows * C * C,
                (tail ? 12.0 + (dwl ? 4.0 : 2.0) : 8.0) * rows * C + (dwl ? 4.0 : 2.0) * (tail ? 9.0 : 8.0) * C * C,
                [&] { launch_mlp_fused(mp, stream); });
        } else {
          timed(ln2_n[s], 0, 8.0 * rows * C,
                [&] { launch_layernorm(X, W(w.n2w), W(w.n2b), xw32, XWh, XWl, (int)rows, C, stream); });
          gemm(fc1_n[s], opXW, wop(w.fc1w), W(w.fc1b), hid32, HIDh, HIDl, (int)rows, 4 * C, C, EPI_GELU, nullptr,
               rows);
          gemm(fc2_n[s], opHID, wop(w.fc2w), W(w.fc2b), X, nullptr, nullptr, (int)rows, C, 4 * C, EPI_RESADD,
               nullptr, rows);
        }
      }
      if (stop_after == 1 + 2 * s) return finish_partial(1 + 2 * s);
      if (s < kStages - 1) {
        const MergeW& m = lay->merge[s];
        const long orow = (long)B * ((g.H + 1) / 2) * ((g.W + 1) / 2);
        if (b16 && 4 * C == 384 && merge1_supported(g.H, g.W) && !(cfg.variant & MOCR_VARIANT_UNFUSED_LN_GEMM)) {
          // gather + norm + reduction as a stream (merge.hip)
          Merge1Params mp{};
          mp.X = X; mp.B = B; mp.H = g.H; mp.W = g.W;
          mp.ln_g = W(m.nw); mp.ln_b = W(m.nb);
          mp.w_hi = mergefrag.hi; mp.w_lo = dwl ? mergefrag.lo : nullptr;
          mp.out = X2;
          timed(mrg_n[s], 2.0 * orow * 4 * C * 2 * C, 4.0 * (double)B * g.H * g.W * C + 8.0 * orow * C +
                (dwl ? 4.0 : 2.0) * 8.0 * C * C, [&] { launch_merge1(mp, stream); });
        } else if (b16 && 4 * C == 384 && !(cfg.variant & MOCR_VARIANT_UNFUSED_LN_GEMM)) {
          // gather + norm + reduction in one kernel (mlp.hip lngemm384_kernel)
          LnGemm384Params lp{};
          lp.X = X; lp.M = orow; lp.ln_g = W(m.nw); lp.ln_b = W(m.nb);
          lp.w = dwh + m.redw; lp.wlo = dwl ? dwl + m.redw : nullptr; lp.b = nullptr;
          lp.wpk = mergepack;
          lp.out = X2; lp.N = 2 * C; lp.merge_H = g.H; lp.merge_W = g.W;
          timed(mrg_n[s], 2.0 * orow * 4 * C * 2 * C, 4.0 * (double)B * g.H * g.W * C + 8.0 * orow * C +
                (dwl ? 4.0 : 2.0) * 8.0 * C * C, [&] { launch_lngemm384(lp, stream); });
        } else {
          timed(mln_n[s], 0, 8.0 * orow * 4 * C,
                [&] { launch_merge_ln(X, W(m.nw), W(m.nb), xw32, XWh, XWl, B, g.H, g.W, C, stream); });
          gemm(mrg_n[s], opXW, wop(m.redw), nullptr, X2, nullptr, nullptr, (int)orow, 2 * C, 4 * C, EPI_STORE, nullptr,
               orow);
        }
        std::swap(X, X2);
        if (stop_after == 2 + 2 * s) return finish_partial(2 + 2 * s);
      }
    }
    Operand opX{X, nullptr, nullptr};
    if (b16) {
      timed("split(memory)", 0, 8.0 * B * M * kEncDim,
            [&] { launch_split_bf16(X, XWh, XWl, (size_t)B * M * kEncDim, stream); });
      opX = opXW;
    }
    gemm("memproj", opX, wop(lay->projw), W(lay->projb), MEM, MEMh, MEMl, B * M, (int)d, kEncDim, EPI_STORE, nullptr,
         (long)B * M);
    // bf16x3 greedy engines: the epilogue writes the fp24 planes the step streams (no fp32
    // copy unless beam search, whose kernels read fp32, may run on this engine)
    // (int16 K/V: quantised in the epilogue when each 144-row half tile is one image and
    // beam search, whose kernels read fp32, cannot run on this engine; else by a pass over
    // the fp32 output)
    const bool kv_planes = kv24() && bf16_mode() && !kvx16();
    const bool kv16_epi = kvx16() && bf16_mode() && M == 144 && cfg.max_beam == 0;
    const size_t kv_layer = (size_t)cfg.max_batch * M * 2 * d;
    gemm("crosskv", Operand{MEM, MEMh, MEMl}, Operand{kvw_all, kvwh, kvwl}, kvb_all,
         (kv_planes || kv16_epi) && cfg.max_beam == 0 ? nullptr : MEMKV, nullptr, nullptr, B * M, (int)(L * 2 * d),
         (int)d, kv16_epi ? EPI_KV16 : EPI_STORE, nullptr, (long)B * M, (int)(2 * d), kv_layer,
         kv_planes ? MEMKV24 : nullptr, M,
         kv16_epi ? MEMKV16 : nullptr, kv16_epi ? MEMKVS : nullptr, (size_t)cfg.max_batch * 2 * d);
    if (kvx16() && !kv16_epi) split_memkv24(B);
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    if (timing) flush_timing();
    encoded = true;
  }

  void finish_partial(int k) {
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    if (timing) flush_timing();
    partial_stage = k;
    encoded = false;
  }

  size_t stage_elems(int k) const {
    if (k == 0) return (size_t)cur_batch * stage[0].H * stage[0].W * stage[0].C;
    const int s = (k - 1) / 2;
    if (k % 2 == 1) return (size_t)cur_batch * stage[s].H * stage[s].W * stage[s].C;
    return (size_t)cur_batch * stage[s + 1].H * stage[s + 1].W * stage[s + 1].C;
  }

  // ---------------------------------------------------------------- decoder
  // One greedy step t.  Buffers: dx = fed-token embedding (layer-0 input),
  // ysa/yca/yff = pre-LayerNorm sums of the three post-norm sublayers; LN1/LN2/LN3 are
  // applied by their consumers.  stp = stop state (nullptr unless batch-global stop).
  // The decoder layers of step t over `B` decoder rows (images, or hypotheses with beam
  // search: self-attention keys through `slots`, memory row = row / mem_div).
  void record_layers(int B, int t, const DecodeState* stp, const int32_t* slots, int mem_div) {
    const int d = cfg.d_model, L = cfg.n_layers;
    const bool fused = slots != nullptr || mem_div != 1;
    if (!fused && fold_greedy()) return record_layers_fold(B, t, stp);
    const size_t cache_layer = (size_t)max_rows * cfg.max_pos * d;
    const size_t kv_layer = (size_t)cfg.max_batch * M * 2 * d;
    hipStream_t s = stream;
    auto base = [&]() {
      RowGemmParams p{};
      p.B = B;
      p.st = stp;
      p.t = t;
      p.d = d;
      p.max_pos = cfg.max_pos;
      return p;
    };
    auto pa_base = [&]() {
      ProjAttnParams a{};
      a.st = stp;
      a.t = t;
      a.out = datt;
      a.B = B;
      a.d = d;
      a.heads = cfg.n_heads;
      a.max_pos = cfg.max_pos;
      a.mem_div = 1;
      return a;
    };
    for (int l = 0; l < L; ++l) {
      const DecLayerW& w = lay->layers[l];
      const DecLayerW* prev = l ? &lay->layers[l - 1] : nullptr;
      float* kc = kcache + l * cache_layer;
      float* vc = vcache + l * cache_layer;
      // layer input: embedding (l = 0) or LN3 of the previous layer
      const float* xin = l ? dy_ff : dx;
      const float* xin_g = l ? W(prev->n3w) : nullptr;
      const float* xin_b = l ? W(prev->n3b) : nullptr;
      const float* xin_s = l ? ds_ff : nullptr;
      // self-attention block: y_sa = x + SA(x)
      RowGemmParams p = base();
      if (fused) {
        ProjAttnParams a = pa_base();
        a.A = xin; a.a_ln_g = xin_g; a.a_ln_b = xin_b; a.a_stats = xin_s; a.W = W(w.sa_inw); a.bias = W(w.sa_inb);
        a.K = kc; a.V = vc; a.kv_b_stride = (size_t)cfg.max_pos * d; a.kv_row_stride = d; a.n_cached = t;
        a.kcache = kc; a.vcache = vc; a.slot_rows = slots; a.slot_ld = ld_ids;
        launch_dec_projattn(a, true, t + 1, s);
      } else {
        p.A = xin; p.a_ln_g = xin_g; p.a_ln_b = xin_b; p.a_stats = xin_s; p.W = W(w.sa_inw); p.bias = W(w.sa_inb);
        p.out = dq; p.kcache = kc; p.vcache = vc; p.N = 3 * d; p.K = d; p.ldo = d; p.n_valid = 3 * d;
        p.epi = DEC_QKV;
        launch_rowgemm(p, s);
        launch_dec_attn(stp, t, dq, kc, vc, (size_t)cfg.max_pos * d, d, t + 1, t + 1, datt, B, d, cfg.n_heads, s);
      }
      p = base();
      p.A = datt; p.W = W(w.sa_ow); p.bias = W(w.sa_ob); p.out = dy_sa; p.resid = xin; p.r_ln_g = xin_g;
      p.r_ln_b = xin_b; p.r_stats = xin_s; p.out_stats = ds_sa; p.N = d; p.K = d; p.ldo = d; p.n_valid = d;
      p.epi = DEC_RESADD;
      launch_rowgemm(p, s);
      // cross-attention block: y_ca = LN1(y_sa) + MHA(LN1(y_sa), mem)
      const float* memk = MEMKV + l * kv_layer;
      if (fused) {
        ProjAttnParams a = pa_base();
        a.A = dy_sa; a.a_ln_g = W(w.n1w); a.a_ln_b = W(w.n1b); a.a_stats = ds_sa; a.W = W(w.ca_inw);
        a.bias = W(w.ca_inb); a.K = memk; a.V = memk + d; a.kv_b_stride = (size_t)M * 2 * d; a.kv_row_stride = 2 * d;
        a.n_cached = M; a.mem_div = mem_div;
        launch_dec_projattn(a, false, M, s);
      } else {
        p = base();
        p.A = dy_sa; p.a_ln_g = W(w.n1w); p.a_ln_b = W(w.n1b); p.a_stats = ds_sa; p.W = W(w.ca_inw);
        p.bias = W(w.ca_inb);
        p.out = dq; p.N = d; p.K = d; p.ldo = d; p.n_valid = d; p.epi = DEC_STORE;
        launch_rowgemm(p, s);
        launch_dec_attn(stp, t, dq, memk, memk + d, (size_t)M * 2 * d, 2 * d, M, M, datt, B, d, cfg.n_heads, s);
      }
      p = base();
      p.A = datt; p.W = W(w.ca_ow); p.bias = W(w.ca_ob); p.out = dy_ca; p.resid = dy_sa; p.r_ln_g = W(w.n1w);
      p.r_ln_b = W(w.n1b); p.r_stats = ds_sa; p.out_stats = ds_ca; p.N = d; p.K = d; p.ldo = d; p.n_valid = d;
      p.epi = DEC_RESADD;
      launch_rowgemm(p, s);
      // feed-forward block: y_ff = LN2(y_ca) + W2 relu(W1 LN2(y_ca))
      p = base();
      p.A = dy_ca; p.a_ln_g = W(w.n2w); p.a_ln_b = W(w.n2b); p.a_stats = ds_ca; p.W = W(w.l1w); p.bias = W(w.l1b);
      p.out = dh;
      p.N = cfg.d_ff; p.K = d; p.ldo = cfg.d_ff; p.n_valid = cfg.d_ff; p.epi = DEC_RELU;
      launch_rowgemm(p, s);
      p = base();
      p.A = dh; p.W = W(w.l2w); p.bias = W(w.l2b); p.out = dy_ff; p.resid = dy_ca; p.r_ln_g = W(w.n2w);
      p.r_ln_b = W(w.n2b); p.r_stats = ds_ca; p.out_stats = ds_ff; p.N = d; p.K = cfg.d_ff; p.ldo = d;
      p.n_valid = d; p.epi = DEC_RESADD;
      launch_rowgemm(p, s);
    }
  }

  // bf16x3 engines run the fold GEMMs on bf16x3 MFMA: Wy's planes are the blob's (dwh /
  // dwl at the blob offset), Wz's the split of the folded weights
  void fold_planes(FoldGemmParams& g, size_t wy_off) const {
    if (!fold_h) return;
    g.Wy_hi = dwh + wy_off;
    g.Wy_lo = dwl + wy_off;
    if (g.NZ) {
      const size_t zo = (size_t)(g.Wz - fold_buf);
      g.Wz_hi = fold_h + zo;
      g.Wz_lo = fold_l + zo;
    }
  }

  // The folded greedy step (kernels.h FoldGemmParams): per layer 5 dependent kernels --
  // self-attention (q|k|v unfolded from dzqkv: layer 0's from the embedding tables, later
  // layers' from the previous FFN kernel), out_proj + z_q, cross-attention (q unfolded),
  // out_proj + z_h, FFN (hidden unfolded from z_h) + the next layer's z_qkv.
  // slots / mem_div: beam search (rows = hypotheses, self-attention keys through the
  // slot table of step t, memory row = row / mem_div); nullptr / 1 for greedy decoding.
  void record_layers_fold(int B, int t, const DecodeState* stp, const int32_t* slots = nullptr, int mem_div = 1) {
    const int d = cfg.d_model, L = cfg.n_layers;
    const size_t cache_layer = (size_t)max_rows * cfg.max_pos * d;
    const size_t kv_layer = (size_t)cfg.max_batch * M * 2 * d;
    hipStream_t s = stream;
    for (int l = 0; l < L; ++l) {
      const DecLayerW& w = lay->layers[l];
      const FoldW& f = foldw[l];
      const DecLayerW* prev = l ? &lay->layers[l - 1] : nullptr;
      float* kc = kcache + l * cache_layer;
      float* vc = vcache + l * cache_layer;
      // y_sa = x + SA(x): attention, then out_proj + z_q = W_q' y_sa
      FoldAttnParams a{};
      a.st = stp; a.t = t; a.B = B; a.out = datt; a.z = dzqkv; a.z_ld = 3 * d;
      if (l) { a.z_stats = ds_ff; a.s = foldw[l - 1].sqkv; a.c = foldw[l - 1].cqkv; }
      if (!l && sel_prev) {  // step t-1's greedy selection, then q|k|v from the tables
        a.sel_on = 1; a.sel = *sel_prev; a.qtab = qtab; a.qpos = qpos; a.emb = W(lay->emb); a.pos = W(lay->pos);
        a.x = dx;
      }
      a.K = kc; a.V = vc; a.kcache = kc; a.vcache = vc;
      if (kv24()) {  // head-major [rows][8][max_pos][32] per layer
        const size_t o = l * cache_layer;
        if (self16()) {
          a.kc16 = kc16 + o; a.vc16 = vc16 + o; a.ksc = ksc16 + o / 32; a.vsc = vsc16 + o / 32;
        } else {
          a.K24 = a.kc24 = kc24 + 3 * o; a.V24 = a.vc24 = vc24 + 3 * o;
        }
        a.f24_b = (size_t)8 * cfg.max_pos * 32; a.f24_h = (size_t)cfg.max_pos * 32;
      }
      a.kv_b_stride = (size_t)cfg.max_pos * d; a.kv_row_stride = d; a.n = t + 1;
      a.slot_rows = slots; a.slot_ld = ld_ids;
      launch_dec_foldattn(a, true, s);
      FoldGemmParams g{};
      g.B = B; g.t = t; g.st = stp;
      g.A1 = datt; g.K1 = d; g.A2 = l ? dy_ff : dx;
      if (l) { g.a2_stats = ds_ff; g.a2_g = W(prev->n3w); g.a2_b = W(prev->n3b); }
      g.Wy = W(w.sa_ow); g.by = W(w.sa_ob); g.y = dy_sa; g.y_stats = ds_sa;
      g.Wz = f.wzq; g.bz = f.bzq; g.z = dq; g.NZ = d;
      fold_planes(g, w.sa_ow);
      fold_gemm(g, s, l, 0);
      // y_ca = LN1(y_sa) + CA(LN1(y_sa), mem): attention, then out_proj + z_h = W_1' y_ca
      const float* memk = MEMKV + l * kv_layer;
      a = FoldAttnParams{};
      a.st = stp; a.t = t; a.B = B; a.out = datt; a.z = dq; a.z_ld = d; a.z_stats = ds_sa; a.s = f.sq; a.c = f.cq;
      a.K = memk; a.V = memk + d; a.kv_b_stride = (size_t)M * 2 * d; a.kv_row_stride = 2 * d; a.n = M;
      a.mem_div = mem_div;
      if (kv24()) {  // head-major [B][k | v][8][M][32] per layer
        const size_t o = l * kv_layer, ov = o + (size_t)8 * M * 32;
        if (kvx16()) {
          a.K16 = MEMKV16 + o; a.V16 = MEMKV16 + ov;
          a.Ks = MEMKVS + (size_t)l * cfg.max_batch * 2 * d; a.Vs = a.Ks + d; a.s_b = 2 * d;
        } else {
          a.K24 = MEMKV24 + 3 * o; a.V24 = MEMKV24 + 3 * ov;
        }
        a.f24_b = (size_t)2 * 8 * M * 32; a.f24_h = (size_t)M * 32;
      }
      launch_dec_foldattn(a, false, s);
      g = FoldGemmParams{};
      g.B = B; g.t = t; g.st = stp;
      g.A1 = datt; g.K1 = d; g.A2 = dy_sa; g.a2_stats = ds_sa; g.a2_g = W(w.n1w); g.a2_b = W(w.n1b);
      g.Wy = W(w.ca_ow); g.by = W(w.ca_ob); g.y = dy_ca; g.y_stats = ds_ca;
      g.Wz = f.wzh; g.bz = f.bzh; g.z = dh; g.NZ = cfg.d_ff;
      fold_planes(g, w.ca_ow);
      fold_gemm(g, s, l, 1);
      // y_ff = LN2(y_ca) + W_2 relu(unfold(z_h)) + b_2, and the next layer's z_qkv
      g = FoldGemmParams{};
      g.B = B; g.t = t; g.st = stp;
      g.A1 = dh; g.K1 = cfg.d_ff; g.a1_stats = ds_ca; g.a1_s = f.sh; g.a1_c = f.ch;
      g.A2 = dy_ca; g.a2_stats = ds_ca; g.a2_g = W(w.n2w); g.a2_b = W(w.n2b);
      g.Wy = W(w.l2w); g.by = W(w.l2b); g.y = dy_ff; g.y_stats = ds_ff;
      if (l + 1 < L) { g.Wz = f.wzqkv; g.bz = f.bzqkv; g.z = dzqkv; g.NZ = 3 * d; }
      fold_planes(g, w.l2w);
      fold_gemm(g, s, l, 2);
    }
  }

  // Logits of the last layer's LN3 output over `B` rows into `out` (row stride Vpad).
  void record_logits(int B, int t, const DecodeState* stp, float* out, size_t hist_stride, float* part = nullptr) {
    const int d = cfg.d_model, L = cfg.n_layers;
    const DecLayerW& last = lay->layers[L - 1];
    if (part && fold_wide()) {  // the greedy step: fc_out on decwide.hip's tiles
      FoldGemmParams g{};
      g.B = B; g.t = t; g.st = stp; g.K1 = 0; g.NY = 0;
      g.A2 = dy_ff; g.a2_stats = ds_ff; g.a2_g = W(last.n3w); g.a2_b = W(last.n3b);
      // without a logits history the selection reads only the partials: no logits stores
      // (10.4 MB per step at 512 rows)
      g.Wz = fcw_pad; g.bz = fcb_pad; g.z = hist_stride ? out : nullptr; g.NZ = Vpad; g.n_valid = cfg.vocab;
      g.hist_stride = hist_stride;
      g.part = part;
      g.Fz_hi = frag_logits.hi; g.Fz_lo = frag_logits.lo; g.Fz = frag_logits.f;
      launch_foldwide(g, stream);
      return;
    }
    RowGemmParams p{};
    p.B = B;
    p.st = stp;
    p.t = t;
    p.d = d;
    p.max_pos = cfg.max_pos;
    p.A = dy_ff;
    p.a_ln_g = W(last.n3w);
    p.a_ln_b = W(last.n3b);
    p.a_stats = ds_ff;
    p.W = fcw_pad;
    p.bias = fcb_pad;
    p.out = out;
    p.hist_stride = hist_stride;
    p.N = Vpad;
    p.K = d;
    p.ldo = Vpad;
    p.n_valid = cfg.vocab;
    p.epi = DEC_LOGITS;
    p.part = part;
    launch_rowgemm(p, stream);
  }

  // greedy selection of step t (select.h) over the logits slot record_logits writes
  SelectArgs select_args(int t, bool hist, bool use_forced, bool stop_batch) const {
    SelectArgs a{};
    a.st = st; a.t = t; a.logits = hist ? dlogits_hist : dlogits; a.hist_stride = hist ? (size_t)cfg.max_batch * Vpad : 0;
    a.ldl = Vpad; a.V = cfg.vocab; a.ids = ids; a.feed = feed; a.forced = use_forced ? forced : nullptr;
    a.ld_ids = ld_ids; a.logp = logp; a.finished = finished; a.eos = cfg.eos_id; a.stop_batch = stop_batch ? 1 : 0;
    a.part = dpart; a.nparts = Vpad / 16;
    return a;
  }

  // The folded step runs step t-1's selection in step t's first kernel (layer 0's
  // self-attention, decfold.hip): 41 dependent launches per step; only the last step
  // ends with dec_argmax_kernel.
  void record_step(int B, int t, int max_steps, bool hist, bool use_forced, bool stop_batch) {
    const DecodeState* stp = stop_batch ? st : nullptr;
    const bool fold = fold_greedy();
    SelectArgs prev{};
    if (fold && t > 0) {
      prev = select_args(t - 1, hist, use_forced, stop_batch);
      sel_prev = &prev;
    }
    try {
      record_layers(B, t, stp, nullptr, 1);
    } catch (...) {
      sel_prev = nullptr;
      throw;
    }
    sel_prev = nullptr;
    float* out = hist ? dlogits_hist : dlogits;
    const size_t hs = hist ? (size_t)cfg.max_batch * Vpad : 0;
    record_logits(B, t, stp, out, hs, dpart);
    if (!fold || t + 1 >= max_steps)
      launch_dec_argmax(select_args(t, hist, use_forced, stop_batch), t + 1 >= max_steps, B, W(lay->emb), W(lay->pos),
                        dx, cfg.d_model, stream, fold ? qtab : nullptr, fold ? qpos : nullptr,
                        fold ? dzqkv : nullptr);
  }

  BeamParams beam_params(int B, int K, int t, int max_steps, bool stop_batch) {
    BeamParams b{};
    b.st = st;
    b.t = t;
    b.last_step = t + 1 >= max_steps;
    b.stop_batch = stop_batch;
    b.B = B;
    b.K = K;
    b.V = cfg.vocab;
    b.ldl = Vpad;
    b.d = cfg.d_model;
    b.ld = ld_ids;
    b.sos = cfg.sos_id;
    b.eos = cfg.eos_id;
    b.pad = cfg.pad_id;
    b.logits = dlogits;
    b.score = bscore;
    b.fin = bfin;
    b.seq_old = bseq[t & 1];
    b.seq_new = bseq[(t + 1) & 1];
    b.slot_old = bslot[t & 1];
    b.slot_new = bslot[(t + 1) & 1];
    b.emb = W(lay->emb);
    b.pos = W(lay->pos);
    b.x = dx;
    if (beam_folded()) {
      b.qtab = qtab;
      b.qpos = qpos;
      b.z = dzqkv;
    }
    return b;
  }

  // One beam-search step over B images x K hypotheses (oracle/model_ref.py beam_search).
  // Folded (production): the greedy step's kernels over the B*K hypothesis rows, the
  // self-attention through the slot table, the logits on decwide.hip's tiles into the full
  // rows beam_select_kernel reads.  MOCR_VARIANT_BEAM_UNFOLDED: round 2's projection +
  // attention kernels and row GEMMs on fp32 K/V.
  void record_beam_step(int B, int K, int t, int max_steps, bool stop_batch) {
    const DecodeState* stp = stop_batch ? st : nullptr;
    if (beam_folded()) {
      record_layers_fold(B * K, t, stp, bslot[t & 1], K);
      if (fold_wide()) {
        const DecLayerW& last = lay->layers[cfg.n_layers - 1];
        FoldGemmParams g{};
        g.B = B * K; g.t = t; g.st = stp; g.K1 = 0; g.NY = 0;
        g.A2 = dy_ff; g.a2_stats = ds_ff; g.a2_g = W(last.n3w); g.a2_b = W(last.n3b);
        g.Wz = fcw_pad; g.bz = fcb_pad; g.z = dlogits; g.NZ = Vpad; g.n_valid = cfg.vocab;
        g.Fz_hi = frag_logits.hi; g.Fz_lo = frag_logits.lo; g.Fz = frag_logits.f;
        launch_foldwide(g, stream);
      } else {
        record_logits(B * K, t, stp, dlogits, 0);
      }
    } else {
      record_layers(B * K, t, stp, bslot[t & 1], K);
      record_logits(B * K, t, stp, dlogits, 0);
    }
    launch_beam_select(beam_params(B, K, t, max_steps, stop_batch), stream);
  }


  // Graph of steps [c*kDecodeChunk, min(max_steps, (c+1)*kDecodeChunk)), step indices baked in.
  // beam > 0: beam-search steps with that many hypotheses per image.
  hipGraphExec_t graph_for(int B, int c, int max_steps, bool hist, bool use_forced, bool stop_batch, int beam = 0) {
    const int t0 = c * kDecodeChunk;
    const int t1 = std::min(max_steps, t0 + kDecodeChunk);
    const bool ends = t1 == max_steps;  // the last step skips the next embedding
    const int flags = (int)hist | (int)use_forced << 1 | (int)stop_batch << 2 | (int)ends << 3 | beam << 4;
    auto key = std::make_tuple(B, t0 * 1000 + t1, flags);
    auto it = graphs.find(key);
    if (it != graphs.end()) return it->second;
    hipGraph_t g;
    MOCR_HIP_CHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    try {
      for (int t = t0; t < t1; ++t) {
        if (beam)
          record_beam_step(B, beam, t, max_steps, stop_batch);
        else
          record_step(B, t, max_steps, hist, use_forced, stop_batch);
      }
    } catch (...) {
      (void)hipStreamEndCapture(stream, &g);
      throw;
    }
    MOCR_HIP_CHECK(hipStreamEndCapture(stream, &g));
    hipGraphExec_t exec;
    MOCR_HIP_CHECK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
    MOCR_HIP_CHECK(hipGraphDestroy(g));
    graphs[key] = exec;
    return exec;
  }

  // Runs the decode; returns steps run.
  int decode(int max_steps, int stop_mode, const int32_t* forced_host, bool want_logits) {
    if (!encoded) throw std::runtime_error("mocr_decode before mocr_encode");
    if (max_steps < 1 || max_steps > cfg.max_pos) throw std::runtime_error("max_steps must be in [1, max_pos]");
    if (stop_mode != MOCR_STOP_BATCH && stop_mode != MOCR_STOP_NONE) throw std::runtime_error("bad stop_mode");
    MOCR_HIP_CHECK(hipSetDevice(device));
    const int B = cur_batch;
    const bool stop_batch = stop_mode == MOCR_STOP_BATCH;
    if (want_logits && !dlogits_hist) dlogits_hist = dalloc<float>((size_t)cfg.max_pos * cfg.max_batch * Vpad);
    // ids/feed: column 0 = sos, the rest pad (src/inference.py:15)
    std::vector<int32_t> init((size_t)B * ld_ids, cfg.pad_id);
    for (int b = 0; b < B; ++b) init[(size_t)b * ld_ids] = cfg.sos_id;
    MOCR_HIP_CHECK(hipMemcpyAsync(ids, init.data(), init.size() * 4, hipMemcpyHostToDevice, stream));
    if (forced_host) {
      std::vector<int32_t> f((size_t)B * ld_ids, cfg.pad_id);
      for (int b = 0; b < B; ++b)
        std::memcpy(&f[(size_t)b * ld_ids], forced_host + (size_t)b * (max_steps + 1), (max_steps + 1) * 4);
      MOCR_HIP_CHECK(hipMemcpyAsync(forced, f.data(), f.size() * 4, hipMemcpyHostToDevice, stream));
      MOCR_HIP_CHECK(hipMemcpyAsync(feed, f.data(), f.size() * 4, hipMemcpyHostToDevice, stream));
      MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    } else {
      MOCR_HIP_CHECK(hipMemcpyAsync(feed, init.data(), init.size() * 4, hipMemcpyHostToDevice, stream));
      MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    }
    MOCR_HIP_CHECK(hipMemsetAsync(finished, 0, (size_t)B * 4, stream));
    DecodeState h{};
    h.done_step = 0x7fffffff;
    h.batch = B;
    MOCR_HIP_CHECK(hipMemcpyAsync(st, &h, sizeof(h), hipMemcpyHostToDevice, stream));
    const bool fold = fold_greedy();
    launch_dec_embed0(feed, ld_ids, W(lay->emb), W(lay->pos), dx, B, cfg.d_model, stream, fold ? qtab : nullptr,
                      fold ? qpos : nullptr, fold ? dzqkv : nullptr);
    const int chunks = (max_steps + kDecodeChunk - 1) / kDecodeChunk;
    DecodeState hs{};
    hipEvent_t t0 = nullptr;
    if (timing) {
      t0 = get_event();
      MOCR_HIP_CHECK(hipEventRecord(t0, stream));
    }
    // Batch stop: the state after chunk c is copied to a pinned slot behind chunk c, and
    // the host checks chunk c - 1's copy only once chunk c is queued, so the GPU never
    // idles between chunks; a chunk launched after the stop skips every step (dec_skip).
    // Up to kSyncStopRows rows (serving: im2latex.predict, predict.py) the host waits for
    // chunk c's own state before queuing chunk c + 1: a stop then wastes at most the rest
    // of its chunk instead of up to two chunks of early-out launches (B = 1, EOS at step
    // 1: 2.39 ms for the deferred check, tools/stop_batch_probe.py), for a host round trip
    // per chunk.
    const bool sync_stop = stop_batch && B <= kSyncStopRows;
    for (int c = 0; c < chunks; ++c) {
      hipGraphExec_t ge = graph_for(B, c, max_steps, want_logits, forced_host != nullptr, stop_batch);
      const auto h0 = std::chrono::steady_clock::now();
      MOCR_HIP_CHECK(hipGraphLaunch(ge, stream));
      if (timing) {  // host time spent submitting the chunk's graph
        mocr_kernel_stat& hs_ = stats["host.graph_launch"];
        std::strncpy(hs_.name, "host.graph_launch", sizeof(hs_.name) - 1);
        hs_.launches += 1;
        hs_.total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
      }
      if (stop_batch && c + 1 < chunks) {
        MOCR_HIP_CHECK(hipMemcpyAsync(&st_host[c & 1], st, sizeof(DecodeState), hipMemcpyDeviceToHost, stream));
        MOCR_HIP_CHECK(hipEventRecord(chunk_ev[c & 1], stream));
        const int cc = sync_stop ? c : c - 1;  // the chunk whose state is checked now
        if (cc >= 0) {
          MOCR_HIP_CHECK(hipEventSynchronize(chunk_ev[cc & 1]));
          if (st_host[cc & 1].done_step != 0x7fffffff) break;
        }
      }
    }
    MOCR_HIP_CHECK(hipMemcpyAsync(&hs, st, sizeof(hs), hipMemcpyDeviceToHost, stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));  // hs is read below
    const int n = stop_batch && hs.done_step != 0x7fffffff ? hs.done_step + 1 : max_steps;
    if (timing) {
      // the whole graph-captured greedy decode as one record (launches = steps run)
      TimingRec r{"decode.greedy", t0, get_event(), 0.0, 0.0};
      MOCR_HIP_CHECK(hipEventRecord(r.e1, stream));
      for (int t = 0; t < n; ++t) {
        r.flops += decode_step_flops(B, t);
        r.bytes += decode_step_bytes(B, t);
      }
      pending.push_back(r);
      flush_timing();
      stats["decode.greedy"].launches += n - 1;
    }
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    if (hs.bad_rows)
      throw std::runtime_error("decode: " + std::to_string(hs.bad_rows) +
                               " row-steps had non-finite logits (NaN/inf in the encoder memory or weights)");
    return n;
  }

  // Algorithmic work of greedy step t over B rows (as built: fp32, or
  // bf16x3 weight planes (4 B per weight), int16 cross K/V, and the int16 + scales or fp24
  // self-attention cache under kv24()): every decoder
  // weight and fc_out once, the cross-attention K/V of all layers, the self-attention K/V
  // of positions 0..t read and position t written, the logits written.  FLOP: the per-row
  // projections 2*(6 d^2 + 2 d ff) per layer + 2 V d, attention 4 d (keys) per layer.
  double decode_step_bytes(int B, int t) const {
    const double d = cfg.d_model, ff = cfg.d_ff, L = cfg.n_layers, V = cfg.vocab;
    const double weights = L * (6 * d * d + 2 * d * ff) + V * d;
    const double cross = (double)B * M * 2 * d * L;
    const double self_kv = (double)B * (t + 2) * 2 * d * L;
    const double kvb = kv24() ? 3.0 : 4.0, kvx = kvx16() ? 2.0 : kvb;
    const double kvs = self16() ? 2.0 + 4.0 / 32 : kvb;  // int16 + one fp32 scale per 32 values
    return 4.0 * (weights + (double)B * V) + kvx * cross + kvs * self_kv;
  }
  double decode_step_flops(int B, int t) const {
    const double d = cfg.d_model, ff = cfg.d_ff, L = cfg.n_layers, V = cfg.vocab;
    return (double)B * (L * (2 * (6 * d * d + 2 * d * ff) + 4 * d * ((t + 1) + M)) + 2 * V * d);
  }
  void decode_beam_out(int K, int max_steps, int stop_mode, int32_t* ids_out, float* scores_out, int32_t* beam_ids_out,
                       int32_t* n_steps_out) {
    const int n = decode_beam(K, max_steps, stop_mode);
    const int B = cur_batch, ld = ld_ids, Wd = max_steps + 1;
    std::vector<int32_t> seq((size_t)B * K * ld);
    std::vector<float> sc((size_t)B * K);
    MOCR_HIP_CHECK(hipMemcpyAsync(seq.data(), bseq[n & 1], seq.size() * 4, hipMemcpyDeviceToHost, stream));
    MOCR_HIP_CHECK(hipMemcpyAsync(sc.data(), bscore, sc.size() * 4, hipMemcpyDeviceToHost, stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    for (int r = 0; r < B * K; ++r)
      for (int j = 0; j < Wd; ++j) {
        const int32_t v = j <= n ? seq[(size_t)r * ld + j] : cfg.pad_id;
        if (beam_ids_out) beam_ids_out[(size_t)r * Wd + j] = v;
        if (ids_out && r % K == 0) ids_out[(size_t)(r / K) * Wd + j] = v;  // rank 0 = best
      }
    if (scores_out) std::memcpy(scores_out, sc.data(), sc.size() * 4);
    if (n_steps_out) *n_steps_out = n;
  }

  // Beam search over the encoded batch; returns the steps run.  Results stay in
  // bseq[n & 1] (rank order) and bscore.
  int decode_beam(int K, int max_steps, int stop_mode) {
    if (!encoded) throw std::runtime_error("mocr_decode_beam before mocr_encode");
    if (K < 1 || K > cfg.max_beam) throw std::runtime_error("beam must be in [1, max_beam]");
    if (max_steps < 1 || max_steps > cfg.max_pos) throw std::runtime_error("max_steps must be in [1, max_pos]");
    if (stop_mode != MOCR_STOP_BATCH && stop_mode != MOCR_STOP_NONE) throw std::runtime_error("bad stop_mode");
    MOCR_HIP_CHECK(hipSetDevice(device));
    const int B = cur_batch;
    const bool stop_batch = stop_mode == MOCR_STOP_BATCH;
    DecodeState h{};
    h.done_step = 0x7fffffff;
    h.batch = B;
    MOCR_HIP_CHECK(hipMemcpyAsync(st, &h, sizeof(h), hipMemcpyHostToDevice, stream));
    launch_beam_init(beam_params(B, K, -1, max_steps, stop_batch), stream);
    const int chunks = (max_steps + kDecodeChunk - 1) / kDecodeChunk;
    DecodeState hs{};
    for (int c = 0; c < chunks; ++c) {
      MOCR_HIP_CHECK(hipGraphLaunch(graph_for(B, c, max_steps, false, false, stop_batch, K), stream));
      if (stop_batch && c + 1 < chunks) {
        MOCR_HIP_CHECK(hipMemcpyAsync(&hs, st, sizeof(hs), hipMemcpyDeviceToHost, stream));
        MOCR_HIP_CHECK(hipStreamSynchronize(stream));
        if (hs.done_step != 0x7fffffff) break;
      }
    }
    MOCR_HIP_CHECK(hipMemcpyAsync(&hs, st, sizeof(hs), hipMemcpyDeviceToHost, stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
    if (hs.bad_rows)
      throw std::runtime_error("decode: " + std::to_string(hs.bad_rows) +
                               " row-steps had non-finite logits (NaN/inf in the encoder memory or weights)");
    return stop_batch && hs.done_step != 0x7fffffff ? hs.done_step + 1 : max_steps;
  }


  void copy_ids(int32_t* dst, int max_steps, hipMemcpyKind kind) {
    MOCR_HIP_CHECK(hipMemcpy2DAsync(dst, (max_steps + 1) * 4, ids, ld_ids * 4, (max_steps + 1) * 4, cur_batch, kind,
                                    stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(stream));
  }
};

// ====================================================================== C-ABI
namespace {

int fail(mocr_engine* e, const std::exception& ex, int code = -1) {
  if (e) e->err = ex.what();
  g_last_error = ex.what();
  if (auto* he = dynamic_cast<const HipError*>(&ex)) return -1000 - (int)he->code;
  return code;
}

#define MOCR_API_BODY(eng, body)                   \
  try {                                            \
    if (!(eng)) throw std::runtime_error("null engine"); \
    body;                                          \
    return 0;                                      \
  } catch (const std::exception& ex) {             \
    return fail(eng, ex);                          \
  }

}  // namespace

extern "C" {

int mocr_abi_version(void) { return MOCR_ABI_VERSION; }

int mocr_device_count(void) {
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    g_last_error = std::string("hipGetDeviceCount: ") + hipGetErrorString(e);
    return -1000 - (int)e;
  }
  return n;
}

size_t mocr_weight_count(const mocr_config* cfg) {
  try {
    check_config(*cfg);
    return Layout(*cfg).total;
  } catch (const std::exception& ex) {
    g_last_error = ex.what();
    return 0;
  }
}

int mocr_memory_tokens(const mocr_config* cfg) {
  if (cfg->arch == MOCR_ARCH_RES18TRANS) return res_h4(cfg->img_w);  // one token per layer4 column
  int H = cfg->img_h / 4, W = cfg->img_w / 4;
  for (int s = 0; s < kStages - 1; ++s) {
    H = (H + 1) / 2;
    W = (W + 1) / 2;
  }
  return H * W;
}

int mocr_create(const mocr_config* cfg, int hip_device, mocr_engine** out) {
  mocr_engine* e = nullptr;
  try {
    if (!cfg || !out) throw std::runtime_error("null argument");
    e = new mocr_engine();
    e->init(*cfg, hip_device);
    *out = e;
    return 0;
  } catch (const std::exception& ex) {
    int rc = fail(nullptr, ex);
    delete e;
    if (out) *out = nullptr;
    return rc;
  }
}

int mocr_destroy(mocr_engine* eng) {
  delete eng;
  return 0;
}

const char* mocr_last_error(const mocr_engine* eng) { return eng ? eng->err.c_str() : g_last_error.c_str(); }

int mocr_load_weights(mocr_engine* eng, const float* blob, size_t n) { MOCR_API_BODY(eng, eng->load_weights(blob, n)) }

int mocr_set_images(mocr_engine* eng, const float* img_host, int batch) {
  MOCR_API_BODY(eng, eng->set_images(img_host, batch, hipMemcpyHostToDevice))
}

int mocr_set_images_device(mocr_engine* eng, const float* img_dev, int batch) {
  MOCR_API_BODY(eng, eng->set_images(img_dev, batch, hipMemcpyDeviceToDevice))
}

int mocr_encode(mocr_engine* eng, int batch) { MOCR_API_BODY(eng, eng->encode(batch)) }

int mocr_get_memory(mocr_engine* eng, float* host_out) {
  MOCR_API_BODY(eng, {
    if (!eng->encoded) throw std::runtime_error("not encoded");
    MOCR_HIP_CHECK(hipSetDevice(eng->device));
    MOCR_HIP_CHECK(hipMemcpyAsync(host_out, eng->MEM,
                                  (size_t)eng->cur_batch * eng->M * eng->cfg.d_model * sizeof(float),
                                  hipMemcpyDeviceToHost, eng->stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(eng->stream));
  })
}

int mocr_set_encoder_pos(mocr_engine* eng, const float* table, int tokens) {
  MOCR_API_BODY(eng, eng->set_encoder_pos(table, tokens))
}

int mocr_decode_beam(mocr_engine* eng, int beam, int max_steps, int stop_mode, int32_t* ids_out, float* scores_out,
                     int32_t* beam_ids_out, int32_t* n_steps_out) {
  MOCR_API_BODY(eng, eng->decode_beam_out(beam, max_steps, stop_mode, ids_out, scores_out, beam_ids_out, n_steps_out))
}

int mocr_decode(mocr_engine* eng, int max_steps, int stop_mode, const int32_t* forced_ids, int32_t* ids_out,
                int32_t* n_steps_out, float* logp_out, float* logits_out) {
  MOCR_API_BODY(eng, {
    const int n = eng->decode(max_steps, stop_mode, forced_ids, logits_out != nullptr);
    if (n_steps_out) *n_steps_out = n;
    if (ids_out) eng->copy_ids(ids_out, max_steps, hipMemcpyDeviceToHost);
    const int B = eng->cur_batch;
    if (logp_out) {
      MOCR_HIP_CHECK(hipMemcpy2D(logp_out, max_steps * 4, eng->logp, eng->cfg.max_pos * 4, max_steps * 4, B,
                                 hipMemcpyDeviceToHost));
    }
    if (logits_out) {
      const size_t V = eng->cfg.vocab;
      for (int t = 0; t < max_steps; ++t) {
        // hist slot t is [max_batch, Vpad]; out is [B, max_steps, V]
        MOCR_HIP_CHECK(hipMemcpy2D(logits_out + (size_t)t * V, (size_t)max_steps * V * 4,
                                   eng->dlogits_hist + (size_t)t * eng->cfg.max_batch * eng->Vpad,
                                   (size_t)eng->Vpad * 4, V * 4, B, hipMemcpyDeviceToHost));
      }
    }
  })
}

int mocr_decode_device(mocr_engine* eng, int max_steps, int stop_mode, int32_t* ids_dev, int32_t* n_steps_out) {
  MOCR_API_BODY(eng, {
    const int n = eng->decode(max_steps, stop_mode, nullptr, false);
    if (n_steps_out) *n_steps_out = n;
    eng->copy_ids(ids_dev, max_steps, hipMemcpyDeviceToDevice);
  })
}

int mocr_debug_encode_until(mocr_engine* eng, int batch, int k, float* host_out, size_t n) {
  MOCR_API_BODY(eng, {
    if (k < 0 || k > 7) throw std::runtime_error("k must be in [0, 7]");
    eng->encode(batch, k);
    if (n != eng->stage_elems(k)) throw std::runtime_error("wrong output size for stage " + std::to_string(k));
    MOCR_HIP_CHECK(hipMemcpyAsync(host_out, eng->X, n * sizeof(float), hipMemcpyDeviceToHost, eng->stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(eng->stream));
  })
}

int mocr_set_cu_mask(mocr_engine* eng, const uint32_t* mask, int n_words) {
  MOCR_API_BODY(eng, {
    if (n_words < 0 || (n_words > 0 && !mask)) throw std::runtime_error("bad CU mask");
    if (n_words && eng->stream_priority != 0)
      throw std::runtime_error("mocr_set_cu_mask: the stream has a priority (mocr_set_stream_priority); HIP makes a "
                               "stream with a CU mask or a priority, not both: set the priority to 0 first");
    // clearing a mask the stream does not have keeps the stream (and its priority)
    if (!n_words && !eng->stream_cu_masked) return 0;
    MOCR_HIP_CHECK(hipSetDevice(eng->device));
    MOCR_HIP_CHECK(hipStreamSynchronize(eng->stream));
    hipStream_t s = nullptr;
    if (n_words)
      MOCR_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, mask));
    else
      MOCR_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));  // masked: priority is 0
    MOCR_HIP_CHECK(hipStreamDestroy(eng->stream));
    eng->stream = s;
    eng->stream_cu_masked = n_words != 0;
  })
}

int mocr_set_stream_priority(mocr_engine* eng, int priority) {
  MOCR_API_BODY(eng, {
    MOCR_HIP_CHECK(hipSetDevice(eng->device));
    int least = 0;
    int greatest = 0;
    MOCR_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    // priority: 0 normal, > 0 higher (the device's greatest), < 0 lower (its least)
    const int prio = priority > 0 ? greatest : (priority < 0 ? least : 0);
    if (priority != 0 && eng->stream_cu_masked)
      throw std::runtime_error("mocr_set_stream_priority: the stream has a CU mask (mocr_set_cu_mask); HIP makes a "
                               "stream with a CU mask or a priority, not both: clear the mask first");
    // the normal priority on a masked stream: the masked stream already has it (mask kept)
    if (priority == 0 && eng->stream_cu_masked) return 0;
    MOCR_HIP_CHECK(hipStreamSynchronize(eng->stream));
    hipStream_t s = nullptr;
    MOCR_HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio));
    MOCR_HIP_CHECK(hipStreamDestroy(eng->stream));
    eng->stream = s;
    eng->stream_cu_masked = false;
    eng->stream_priority = priority;
  })
}

int mocr_set_timing(mocr_engine* eng, int enabled) {
  MOCR_API_BODY(eng, {
    eng->timing = enabled != 0;
    eng->stats.clear();
  })
}

int mocr_get_timing(mocr_engine* eng, mocr_kernel_stat* out, int max_records) {
  try {
    if (!eng) throw std::runtime_error("null engine");
    int n = 0;
    for (auto& kv : eng->stats) {
      if (n < max_records && out) out[n] = kv.second;
      ++n;
    }
    return n;
  } catch (const std::exception& ex) {
    return fail(eng, ex);
  }
}

}  // extern "C"
