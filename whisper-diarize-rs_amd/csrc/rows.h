// Decoder rows: one forward pass of the Whisper decoder over R
// rows that may belong to many sequences -- decode steps of several chains, the beams of a
// segment, a prompt prefill, a DTW re-forward, a language-detection SOT pass -- on ONE set of
// launches per layer.  Every row carries its own token, position, KV-pool sequence and
// cross-K/V slot; the rows of one request form a group sharing the slot.
//
// Arithmetic contract: a row's result depends only on its own inputs and its group's kind, never
// on the other rows of the launch --
//   * projections: the row kernel (launch_proj with rows_mma, k_skinny's fixed k order);
//   * self-attention: one workgroup per (row, head) over that row's cache prefix;
//   * cross-attention: groups of <= XATTN_GRP_MAX rows on the VALU split kernel (a row scored with
//     the one-row arithmetic), larger groups on the MFMA tile kernel, both merged by one combine;
//   * LayerNorm fused into the projection (each workgroup normalises its own row tiles; the
//     k_layernorm alternative has the same arithmetic).
// So batching decode steps with prompt prefills and DTW re-forwards of other chains changes no
// result: decode chains stay bit-identical to one sequential chain.
#pragma once
#include <vector>

#include "whisper.h"

namespace wdr {

// one request's rows
struct RowGroupDesc {
  int n = 0;
  const int* tok = nullptr;             // [n]
  const int* seq = nullptr;             // [n] absolute KV-pool sequences, or null: seq0 for all
  int seq0 = 0;
  const int* pos = nullptr;             // [n] positions, or null: pos0 + i
  int pos0 = 0;
  const f16* xkv = nullptr;             // cross-K/V slot of every row
  int logits = 0;                       // 0 none, 1 the last row, 2 every row
  float* cap = nullptr;                 // DTW capture [n_aheads][n][1500] (device), or null
  int l_end = 1 << 30;                  // first layer whose cross-attention the group skips
};

struct RowsIO;

// Host-side builder of a batch's row tables: pinned staging + a device mirror, uploaded with one
// copy.  The packed layout depends only on the counts (R, groups, tiles, logit rows, capture
// rows), so a graph captured for one batch shape replays for every batch of that shape.
class RowBatch {
 public:
  RowBatch(int cap_rows, int cap_logits, int cap_caps);
  ~RowBatch();
  RowBatch(const RowBatch&) = delete;
  RowBatch& operator=(const RowBatch&) = delete;
  void clear();
  // appends a group; returns the index of its first logit row (or -1)
  int add(const RowGroupDesc& g);
  int R = 0, n_logit = 0, n_vgrp = 0, vgrp_max = 0, n_tiles = 0, n_cap = 0;
  int cap_rows, cap_logits, cap_caps;
  // packs the tables into the pinned staging and points io at their device mirror; copy: also
  // enqueue the copy on s (without: a graph replay whose captured copy node reads the staging).
  // track: record an event after the copy, which the next clear() waits for (a stream that runs
  // behind its host: the staging is not rewritten while a copy from it is pending)
  void upload(RowsIO& io, hipStream_t s, bool copy = true, bool track = false);

 private:
  hipEvent_t ev_ = nullptr;
  bool pending_ = false;
  std::vector<int> tok_, pos_, seq_, grp_, lend_, lead_, lrow_, crow_, cstride_;
  std::vector<int4> tiles_;
  std::vector<const f16*> xkv_;
  std::vector<float*> cdst_;
  char* h_ = nullptr;
  DevMem d_;
  size_t bytes_ = 0;
};

// a rows forward's working set (activations sized for the batch's capacity) and tables
struct RowsIO {
  float* xd; f16* hd; f16* qkvd; f16* attd; f16* qx; f16* mlpd;
  float* part_o; float2* part_ml; float2* ml;
  float* logits; int ldlogits;                       // [n_logit][ldlogits]
  f16* kc; f16* vc; long long layer_stride, seq_stride;   // KV pool (layer 0) and its strides
  // tables (device; RowBatch::upload)
  const int* tok = nullptr; const int* pos = nullptr; const int* seq = nullptr;
  const f16* const* xkv = nullptr;
  const int* grp = nullptr; const int* lead = nullptr; const int* lend = nullptr;
  int n_vgrp = 0, vgrp_max = 1;
  const int4* tiles = nullptr; int n_tiles = 0;
  const int* lrow = nullptr; int n_logit = 0;
  const int* crow = nullptr; float* const* cdst = nullptr; const int* cstride = nullptr; int n_cap = 0;
};

// working-set buffers of a rows forward for up to `rows` rows and `logit_rows` logit rows
struct RowsBufs {
  DevMem xd, hd, qkvd, attd, qx, mlpd, part_o, part_ml, ml, logits;
  int rows = 0, logit_rows = 0;
  void alloc(int rows, int logit_rows, int d, int H, int V);
  RowsIO io(const Context& ctx, int V) const;   // tables unset
};

// embed + every layer + (LayerNorm + logits of the logit rows); capture of DTW rows.  l_stop:
// return after the cross-attention (+ capture) of layer l_stop - 1 (no logits then)
void rows_forward(const Context& ctx, const RowsIO& io, int R, hipStream_t s, int l_stop = 1 << 30);

// the DTW re-forwards of several segments as one pass (the DTW queue, whisper_ctx.cpp, and a
// single chain's own re-forward): every row a capture row, no logits, the pass stopping after
// the cross-attention of the last alignment-head layer (l_end - 1: later layers cannot change a
// captured probability).  The rows arithmetic above -- independent of the row count -- so a
// segment's DTW times do not depend on which other segments share the pass.
void dtw_rows_forward(const Context& ctx, const RowsIO& io, int R, int l_end, hipStream_t s);

}  // namespace wdr
