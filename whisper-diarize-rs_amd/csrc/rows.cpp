// Decoder rows forward (rows.h): the one launch sequence behind every decoder pass of libwdr --
// the multi-chain batched step (StepBatcher), a State's own steps and prompt prefills, the DTW
// re-forward and the encode-ahead language detection.  Reference call site: whisper.cpp
// whisper_decode_internal, driven by whisper_full_with_state (src/transcribe.rs:389).
#include "rows.h"
#include "prof.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace wdr {

namespace {
constexpr int kTileRows = 128;   // rows of one MFMA cross-attention tile (4 waves x 32)
constexpr int kNoEnd = 1 << 30;
size_t up16(size_t x) { return (x + 15) & ~size_t(15); }
}  // namespace

RowBatch::RowBatch(int cr, int cl, int cc) : cap_rows(cr), cap_logits(cl), cap_caps(cc) {
  std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
  // worst-case packed size: 5 ints per row, lead / lrow / crow / cstride, tiles, pointers
  bytes_ = up16((size_t)cr * 4) * 5 + up16((size_t)cr * 4) + up16((size_t)cl * 4) + 2 * up16((size_t)cc * 4) +
           up16((size_t)(cr / 8 + 2 + cr / kTileRows + 2) * 16) + up16((size_t)cr * 8) + up16((size_t)cc * 8) + 256;
  WDR_HIP(hipHostMalloc((void**)&h_, bytes_, hipHostMallocDefault));
  d_ = DevMem(bytes_);
  WDR_HIP(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
}

RowBatch::~RowBatch() {
  std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
  if (pending_) (void)hipEventSynchronize(ev_);
  if (ev_) (void)hipEventDestroy(ev_);
  if (h_) (void)hipHostFree(h_);
}

void RowBatch::clear() {
  if (pending_) {
    WDR_HIP(hipEventSynchronize(ev_));
    pending_ = false;
  }
  R = n_logit = n_vgrp = vgrp_max = n_tiles = n_cap = 0;
  tok_.clear(); pos_.clear(); seq_.clear(); grp_.clear(); lend_.clear(); lead_.clear(); lrow_.clear();
  crow_.clear(); cstride_.clear(); tiles_.clear(); xkv_.clear(); cdst_.clear();
}

int RowBatch::add(const RowGroupDesc& g) {
  WDR_CHECK(g.n >= 1 && g.xkv && g.tok, "row batch: empty group");
  WDR_CHECK(R + g.n <= cap_rows, "row batch: rows over capacity");
  const int r0 = R;
  for (int i = 0; i < g.n; ++i) {
    tok_.push_back(g.tok[i]);
    pos_.push_back(g.pos ? g.pos[i] : g.pos0 + i);
    seq_.push_back(g.seq ? g.seq[i] : g.seq0);
    xkv_.push_back(g.xkv);
    grp_.push_back(0);
    lend_.push_back(kNoEnd);
  }
  R += g.n;
  if (g.n <= XATTN_GRP_MAX) {   // VALU group: one-row arithmetic per row
    grp_[r0] = g.n;
    lend_[r0] = g.l_end;
    lead_.push_back(r0);
    n_vgrp++;
    vgrp_max = std::max(vgrp_max, g.n);
  } else {                      // MFMA tiles of <= 128 rows
    for (int t = 0; t < g.n; t += kTileRows) tiles_.push_back(make_int4(r0 + t, std::min(kTileRows, g.n - t), g.l_end, 0));
    n_tiles = (int)tiles_.size();
  }
  int first_logit = -1;
  if (g.logits) {
    first_logit = n_logit;
    for (int i = g.logits == 1 ? g.n - 1 : 0; i < g.n; ++i) lrow_.push_back(r0 + i);
    n_logit = (int)lrow_.size();
    WDR_CHECK(n_logit <= cap_logits, "row batch: logit rows over capacity");
  }
  if (g.cap) {
    for (int i = 0; i < g.n; ++i) {
      crow_.push_back(r0 + i);
      cdst_.push_back(g.cap + (size_t)i * XKV_T);
      cstride_.push_back(g.n * XKV_T);
    }
    n_cap = (int)crow_.size();
    WDR_CHECK(n_cap <= cap_caps, "row batch: capture rows over capacity");
  }
  return first_logit;
}

void RowBatch::upload(RowsIO& io, hipStream_t s, bool copy, bool track) {
  WDR_CHECK(R >= 1, "row batch: no rows");
  // every row's KV-pool sequence inside the pool the tables address (layer stride / sequence
  // stride sequences): a row past it would read / write another chain's cache or past the pool
  if (io.seq_stride > 0 && io.layer_stride > 0) {
    const long long nseq = io.layer_stride / io.seq_stride;
    for (int i = 0; i < R; ++i) WDR_CHECK(seq_[i] >= 0 && seq_[i] < nseq, "row batch: KV sequence outside the pool");
  }
  size_t off = 0;
  auto put = [&](const void* src, size_t n) -> const void* {
    const size_t o = off;
    if (n) memcpy(h_ + o, src, n);
    off = up16(off + n);
    WDR_CHECK(off <= bytes_, "row batch: tables over capacity");
    return (const void*)(d_.as<char>() + o);
  };
  io.tok = (const int*)put(tok_.data(), (size_t)R * 4);
  io.pos = (const int*)put(pos_.data(), (size_t)R * 4);
  io.seq = (const int*)put(seq_.data(), (size_t)R * 4);
  io.grp = (const int*)put(grp_.data(), (size_t)R * 4);
  io.lend = (const int*)put(lend_.data(), (size_t)R * 4);
  io.lead = (const int*)put(lead_.data(), lead_.size() * 4);
  io.lrow = (const int*)put(lrow_.data(), lrow_.size() * 4);
  io.crow = (const int*)put(crow_.data(), crow_.size() * 4);
  io.cstride = (const int*)put(cstride_.data(), cstride_.size() * 4);
  io.tiles = (const int4*)put(tiles_.data(), tiles_.size() * 16);
  io.xkv = (const f16* const*)put(xkv_.data(), (size_t)R * sizeof(void*));
  io.cdst = (float* const*)put(cdst_.data(), cdst_.size() * sizeof(void*));
  io.n_vgrp = n_vgrp;
  io.vgrp_max = std::max(1, vgrp_max);
  io.n_tiles = n_tiles;
  io.n_logit = n_logit;
  io.n_cap = n_cap;
  if (!copy) return;
  WDR_HIP(wdr_memcpy_async(d_.p, h_, off, hipMemcpyHostToDevice, s));
  if (track) {
    WDR_HIP(hipEventRecord(ev_, s));
    pending_ = true;
  }
}

void RowsBufs::alloc(int r, int lr, int d, int H, int V) {
  std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
  rows = r;
  logit_rows = lr;
  xd = DevMem((size_t)r * d * 4);
  hd = DevMem((size_t)r * d * 2);
  qkvd = DevMem((size_t)r * 3 * d * 2);
  attd = DevMem((size_t)r * d * 2);
  qx = DevMem((size_t)r * d * 2);
  mlpd = DevMem((size_t)r * 4 * d * 2);
  part_o = DevMem((size_t)24 * r * H * 64 * 4);   // 24 key chunks (1500 / 64, rounded up)
  part_ml = DevMem((size_t)24 * r * H * sizeof(float2));
  ml = DevMem((size_t)r * H * sizeof(float2));
  logits = DevMem((size_t)std::max(1, lr) * V * 4);
}

RowsIO RowsBufs::io(const Context& ctx, int V) const {
  RowsIO o{};
  o.xd = xd.as<float>();
  o.hd = hd.as<f16>();
  o.qkvd = qkvd.as<f16>();
  o.attd = attd.as<f16>();
  o.qx = qx.as<f16>();
  o.mlpd = mlpd.as<f16>();
  o.part_o = part_o.as<float>();
  o.part_ml = part_ml.as<float2>();
  o.ml = ml.as<float2>();
  o.logits = logits.as<float>();
  o.ldlogits = V;
  o.kc = ctx.kv_k.as<f16>();
  o.vc = ctx.kv_v.as<f16>();
  o.layer_stride = ctx.kv_layer_stride;
  o.seq_stride = ctx.kv_seq_stride;
  return o;
}

void rows_forward(const Context& ctx, const RowsIO& io, int R, hipStream_t s, int l_stop) {
  const Model& md = ctx.model;
  const HParams& hp = md.hp;
  const int d = hp.n_text_state, L = hp.n_text_layer, H = hp.n_text_head;
  const float scale = 1.0f / 8.0f;
  WDR_CHECK(R >= 1 && io.tok && io.xkv, "rows forward: no rows / tables");
  // the projection's input rows LayerNorm(x): inside the row kernel's prologue (every workgroup
  // normalises its own 16- / 32-row tiles into LDS) up to a per-projection row count, above it
  // one k_layernorm launch into io.hd -- the same arithmetic either way (wdr_dbg_proj_ln,
  // test_rows_ln_fused_equals_split).  The thresholds are where the fused form stops being the
  // faster one alone (tools/rows_bench; profiles/r05/rows_ln_fc2.txt, rows_tilings.txt,
  // rows_ln2.txt; the split figures include the LayerNorm launch): the fused prologue caps a
  // workgroup's row tiles (LDS), so its weights are re-read once per 16 (32) rows, and each of the
  // logits' 1621 column workgroups would normalise every row -- xq (N = d) fused 5.2-9.2 vs
  // 6.7-9.4 us at 1-64 rows; qkv fused 6.0-12.2 vs 7.5-12.6 us up to 48 rows, 14.8 / 16.5 vs
  // 12.9 / 13.4 at 56 / 64; fc1 fused 7.3-11.5 vs 8.8-11.6 up to 24 rows, 13.1-16.2 vs 12.2-14.2 at
  // 32-48; the logits split at every count (32 rows: 48.7 vs 83.7 us).
  // WDR_ROWS_LN_FUSE (read once): one threshold for all four (A/B; round 4 fused <= 32 rows).
  static const int ln_env = getenv("WDR_ROWS_LN_FUSE") ? atoi(getenv("WDR_ROWS_LN_FUSE")) : -1;
  const int fuse_qkv = ln_env >= 0 ? ln_env : 48, fuse_xq = ln_env >= 0 ? ln_env : 64,
            fuse_fc1 = ln_env >= 0 ? ln_env : 24, fuse_logits = ln_env >= 0 ? ln_env : 0;
  auto P = [&](const f16* A, int lda, const f16* W, const float* b, void* out, int ldo, int N, int K, int epi,
               const float* lng = nullptr, const float* lnb = nullptr, int fuse_max = 0) {
    ProjArgs a{A, lda, W, K, b, out, ldo, nullptr, 0, R, N, K, epi};
    a.rows_mma = 1;
    if (lng) {
      if (R <= fuse_max) {
        a.ln_x = io.xd;
        a.ldln = d;
        a.ln_g = lng;
        a.ln_b = lnb;
      } else {
        launch_layernorm(io.xd, d, lng, lnb, io.hd, d, R, d, s);
        a.A = io.hd;
        a.lda = d;
      }
    }
    return a;
  };
  launch_embed(md.tok_emb, md.dec_pos, io.tok, io.pos, R, d, io.xd, s);
  const bool any_cap = io.n_cap > 0 && ctx.aheads_per_layer.size() == (size_t)L;
  int cap_slot0 = 0;
  for (int l = 0; l < L; ++l) {
    const DecLayer& e = md.dec[l];
    f16* kc = io.kc + (size_t)l * io.layer_stride;
    f16* vc = io.vc + (size_t)l * io.layer_stride;
    ProjArgs q = P(nullptr, d, e.w_qkv, e.b_qkv, io.qkvd, 3 * d, 3 * d, d, EPI_QKV_CACHE, e.ln1_g, e.ln1_b, fuse_qkv);
    q.kc = kc;
    q.vc = vc;
    q.seq_stride = io.seq_stride;
    q.row_seq = io.seq;
    q.row_pos = io.pos;
    q.d = d;
    launch_proj(q, s);
    // every row's K / V is in the cache before any row attends (rows of one prefill see their
    // predecessors' keys: causal by position)
    DecSelfArgs sa{io.qkvd, 3 * d, kc, vc, io.seq_stride, d, io.seq, io.pos, io.attd, d, scale};
    launch_dec_self_attn(sa, R, H, s);
    launch_proj(P(io.attd, d, e.w_o, e.b_o, io.xd, d, d, d, EPI_F32_RESID), s);
    launch_proj(P(nullptr, d, e.w_xq, e.b_xq, io.qx, d, d, d, EPI_F16, e.ln2_g, e.ln2_b, fuse_xq), s);
    XAttnArgs xa{io.qx, d, nullptr, nullptr, 64, XKV_T, R, H, scale, io.part_o, io.part_ml, io.attd, d};
    xa.row_k = io.xkv;
    xa.layer_off = xkv_k_off(l, H);
    xa.v_off = xkv_v_off(l, H) - xkv_k_off(l, H);
    xa.hs = XKV_HS;
    xa.grp = io.grp;
    xa.lead = io.lead;
    xa.n_grp = io.n_vgrp;
    xa.n_vgrp = io.n_vgrp;
    xa.vgrp_max = io.vgrp_max;
    xa.lend = io.lend;
    xa.layer = l;
    xa.tiles = io.tiles;
    xa.n_tiles = io.n_tiles;
    const bool cap_layer = any_cap && !ctx.aheads_per_layer[l].empty();
    xa.ml_out = cap_layer ? io.ml : nullptr;
    launch_xattn_rows(xa, s);
    if (cap_layer) {
      CaptureRowsArgs ca{io.qx, d, io.xkv, xkv_k_off(l, H), XKV_HS, io.ml,
                         ctx.aheads_dev.as<int>() + ctx.aheads_dev_off[l], io.crow, io.cdst, io.cstride,
                         io.n_cap, cap_slot0, XKV_T, H, scale};
      launch_aheads_capture_rows(ca, (int)ctx.aheads_per_layer[l].size(), s);
    }
    if (ctx.aheads_per_layer.size() == (size_t)L) cap_slot0 += (int)ctx.aheads_per_layer[l].size();
    if (l + 1 >= l_stop) return;   // a DTW pass: nothing after this layer's capture matters
    launch_proj(P(io.attd, d, e.w_xo, e.b_xo, io.xd, d, d, d, EPI_F32_RESID), s);
    launch_proj(P(nullptr, d, e.w_fc1, e.b_fc1, io.mlpd, 4 * d, 4 * d, d, EPI_F16_GELU, e.ln3_g, e.ln3_b, fuse_fc1), s);
    launch_proj(P(io.mlpd, 4 * d, e.w_fc2, e.b_fc2, io.xd, d, d, 4 * d, EPI_F32_RESID), s);
  }
  if (io.n_logit > 0) {
    // final LayerNorm + logits of the logit rows only, gathered by lrow (compact output)
    ProjArgs a{nullptr, d, md.tok_emb, d, nullptr, io.logits, io.ldlogits, nullptr, 0, io.n_logit, hp.n_vocab, d, EPI_F32};
    a.rows_mma = 1;
    if (io.n_logit <= fuse_logits) {
      a.ln_x = io.xd;
      a.ldln = d;
      a.ln_g = md.ln_g;
      a.ln_b = md.ln_b;
      a.row_map = io.lrow;
    } else {
      launch_layernorm_rows(io.xd, d, md.ln_g, md.ln_b, io.hd, d, io.n_logit, d, io.lrow, s);
      a.A = io.hd;
    }
    launch_proj(a, s);
  }
}

void dtw_rows_forward(const Context& ctx, const RowsIO& io, int R, int l_end, hipStream_t s) {
  WDR_CHECK(io.n_cap == R && ctx.aheads_per_layer.size() == (size_t)ctx.model.hp.n_text_layer,
            "DTW rows forward: every row a capture row, alignment heads known");
  WDR_CHECK(l_end >= 1 && l_end <= ctx.model.hp.n_text_layer, "DTW rows forward: bad last layer");
  rows_forward(ctx, io, R, s, l_end);
}

}  // namespace wdr
