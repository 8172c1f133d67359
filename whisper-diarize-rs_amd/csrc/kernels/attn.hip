// Attention kernels (SURVEY.md §8(a) a6 encoder self-attention, a9 decoder self- and
// cross-attention, a12 alignment-head capture for DTW).
//
//  * k_flash_attn   — MFMA flash attention for >8 query rows (encoder T=1500, prompt
//    prefill, DTW re-forward).  Swapped product S^T = K.Q^T so that a query's scores live
//    in ONE lane pair (lane, lane^32): the row max / row sum need one lane exchange, and the
//    f32 accumulator tile of S^T is directly the B operand of O^T = V^T.P^T (no LDS round
//    trip for P).  K tile staged row-major (72-half stride: conflict-free ds_read_b128),
//    V staged transposed (68-half stride: conflict-free ds_read_b64).  d_head = 64.
//    Optionally writes each query row's (max, sum) so the DTW capture can materialise the
//    exact softmax of the alignment heads without a second full pass.
//  * k_dec_self_attn — one wave per (decoder row, head) over that row's KV cache.
//  * k_xattn_partial / k_xattn_combine — split-K ("flash decode") cross-attention for the
//    <=8 decoder rows of a step: the 1500 cross keys are split in 128-key chunks over
//    workgroups so every CU streams the cross K/V once for all beams.
//  * k_aheads_capture — softmax(QK^T) of the alignment heads over all 1500 keys.
#include <cstdlib>

#include "../common.h"
#include "kernels.h"
#include "../prof.h"

namespace wdr {


constexpr int FA_KB = 64, FA_KS = 72, FA_VS = 68;

// OCC = waves per SIMD the register budget is held to: 3 (<= 168 VGPRs) or 4 (<= 128), the
// arithmetic identical (WDR_FLASH_OCC, flash_occ below)
template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_flash_attn(FlashArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  __shared__ __attribute__((aligned(16))) f16 Ks[FA_KB * FA_KS];
  __shared__ __attribute__((aligned(16))) f16 Vt[64 * FA_VS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const f16* Q = a.q + b * a.q_bs + h * 64;
  const f16* K = a.k + b * a.k_bs + h * a.k_hs;
  const f16* V = a.v + b * a.v_bs + h * a.v_hs;
  if (a.nsplit > 1) Q = a.q + h * 64;
  const int fr = lane & 31, hh = lane >> 5;
  const int qrow = qb * 128 + wid * 32 + fr;
  const int qrow_c = qrow < a.Tq ? qrow : a.Tq - 1;

  f16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *(const f16x8*)(Q + (long long)qrow_c * a.ldq + 16 * s + 8 * hh);

  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
  float m = -INFINITY, l = 0.f;
  int kmax = a.Tk, kbeg = 0;
  if (a.nsplit > 1) {   // blockIdx.z = key split (n_batch == 1)
    const int ks = ((a.Tk + a.nsplit - 1) / a.nsplit + FA_KB - 1) / FA_KB * FA_KB;
    kbeg = b * ks;
    kmax = min(a.Tk, kbeg + ks);
    Q = a.q + h * 64;
    K = a.k + h * a.k_hs;
    V = a.v + h * a.v_hs;
  }
  if (a.causal) {
    const int last_q = qb * 128 + 127;
    kmax = kmax < last_q + 1 ? kmax : last_q + 1;
  }
  // K / V tiles are register-staged one tile ahead: the loads of tile k0 + 64 are issued right
  // after tile k0 is published to LDS and land while tile k0 is multiplied; they are written to
  // LDS after the next barrier
  // thread t stages keys 2(t/8) and 2(t/8) + 1, dims 8(t%8)..+7: per dim it holds two
  // consecutive keys, so the transposed V image takes 8 packed 4-B writes instead of 16 scalar
  f16x8 kreg[2], vreg[2];
  const int sr = 2 * (tid >> 3), scol = (tid & 7) * 8;
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int key = kt + sr + i;
      key = key < kmax ? key : kmax - 1;
      kreg[i] = *(const f16x8*)(K + (long long)key * a.ldk + scol);
      vreg[i] = *(const f16x8*)(V + (long long)key * a.ldv + scol);
    }
  };
  // scores in log2 units: p = 2^(s * scale * log2(e) - m), one fma + v_exp_f32 per score
  const float sl2 = a.scale * 1.4426950408889634f;
  if (kbeg < kmax) load_tile(kbeg);
  for (int k0 = kbeg; k0 < kmax; k0 += FA_KB) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) *(f16x8*)(Ks + (sr + i) * FA_KS + scol) = kreg[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
      *(f16x2_t*)(Vt + (scol + e) * FA_VS + sr) = (f16x2_t){vreg[0][e], vreg[1][e]};
    }
    __syncthreads();
    if (k0 + FA_KB < kmax) load_tile(k0 + FA_KB);
    f32x16 st[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[t][r] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const f16x8 af = *(const f16x8*)(Ks + (32 * t + fr) * FA_KS + 16 * s + 8 * hh);
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, qf[s], st[t], 0, 0, 0);
      }
    }
    // raw-score max (the scale is positive: max(s) * sl2 is the max of the scaled scores);
    // masking only on the last key tile or under the causal mask (wave-uniform branch)
    float mx = -INFINITY;
    if (!a.causal && k0 + FA_KB <= kmax) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[t][r]);
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
          const bool ok = key < kmax && (!a.causal || key <= qrow);
          st[t][r] = ok ? st[t][r] : -INFINITY;
          mx = fmaxf(mx, st[t][r]);
        }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx == -INFINITY ? -INFINITY : mx * sl2);
    const float alpha = (mnew == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
    const float mu = (mnew == -INFINITY) ? 0.f : mnew;   // masked scores: 2^-inf = 0
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(st[t][r], sl2, -mu));
        st[t][r] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    // rescale only when some row's max moved (alpha == 1 exactly otherwise: the skip is exact);
    // past the first key tiles of a 1500-key row that is rare, and it saves 32 multiplies a tile
    const bool moved = __any(mnew != m);
    m = mnew;
    if (moved) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (f16)st[t][8 * s + j];
        const int kc = 32 * t + 16 * s + 4 * hh;
        f16x8 va0, va1;
        {
          const f16x4 lo = *(const f16x4*)(Vt + (fr)*FA_VS + kc);
          const f16x4 hi = *(const f16x4*)(Vt + (fr)*FA_VS + kc + 8);
          va0 = (f16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
        {
          const f16x4 lo = *(const f16x4*)(Vt + (32 + fr) * FA_VS + kc);
          const f16x4 hi = *(const f16x4*)(Vt + (32 + fr) * FA_VS + kc + 8);
          va1 = (f16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(va0, pb, o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(va1, pb, o1, 0, 0, 0);
      }
  }
  if (a.nsplit > 1) {
    if (qrow < a.Tq) {
      float* po = a.part_o + (((long long)b * a.Tq + qrow) * a.n_head + h) * 64;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        *(float4*)(po + 8 * g + 4 * hh) = make_float4(o0[4 * g], o0[4 * g + 1], o0[4 * g + 2], o0[4 * g + 3]);
        *(float4*)(po + 32 + 8 * g + 4 * hh) = make_float4(o1[4 * g], o1[4 * g + 1], o1[4 * g + 2], o1[4 * g + 3]);
      }
      if (hh == 0) a.part_ml[((long long)b * a.n_head + h) * a.Tq + qrow] = make_float2(m * 0.6931471805599453f, l);
    }
    return;
  }
  if (qrow < a.Tq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    f16* O = a.o + b * a.o_bs + (long long)qrow * a.ldo + h * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f16x4 w0, w1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        w0[e] = (f16)(o0[4 * g + e] * inv);
        w1[e] = (f16)(o1[4 * g + e] * inv);
      }
      *(f16x4*)(O + 8 * g + 4 * hh) = w0;
      *(f16x4*)(O + 32 + 8 * g + 4 * hh) = w1;
    }
    if (a.ml && hh == 0) a.ml[((long long)b * a.n_head + h) * a.Tq + qrow] = make_float2(m * 0.6931471805599453f, l);
  }
}

// merge the key splits: O = sum_c e^{m_c - M} O_c / L, (M, L) kept for the DTW capture
__global__ __launch_bounds__(64) void k_flash_combine(FlashArgs a) {
  const int q = blockIdx.x, h = blockIdx.y, d = threadIdx.x;
  float2 ml = make_float2(-INFINITY, 0.f);
  if (d < a.nsplit) ml = a.part_ml[((long long)d * a.n_head + h) * a.Tq + q];
  const float M = wave_max(ml.x);
  const float w = (d < a.nsplit && ml.x != -INFINITY) ? __expf(ml.x - M) : 0.f;
  const float L = wave_sum(ml.y * w);
  float acc = 0.f;
  for (int c = 0; c < a.nsplit; ++c) acc += a.part_o[(((long long)c * a.Tq + q) * a.n_head + h) * 64 + d] * __shfl(w, c, 64);
  a.o[(long long)q * a.ldo + h * 64 + d] = (f16)(acc / L);
  if (a.ml && d == 0) a.ml[(long long)h * a.Tq + q] = make_float2(M, L);
}

static int flash_occ() {
  static const int v = getenv("WDR_FLASH_OCC") && atoi(getenv("WDR_FLASH_OCC")) == 4 ? 4 : 3;
  return v;
}

void launch_flash_attn(const FlashArgs& a, int n_batch, hipStream_t s) {
  WDR_CHECK(a.Tq > 0 && a.Tk > 0, "attention: empty");
  auto* kfn = flash_occ() == 4 ? k_flash_attn<4> : k_flash_attn<3>;
  if (a.nsplit > 1) {
    WDR_CHECK(n_batch == 1 && !a.causal && a.nsplit <= 64 && a.part_o && a.part_ml, "flash split: bad args");
    wdr_launch(PROF_FLASH, (double)a.n_head * 64 * 2 * (2.0 * a.Tq + 2.0 * a.Tk), (double)a.n_head * a.Tq * a.Tk * 64 * 4,
               kfn, dim3(cdiv(a.Tq, 128), a.n_head, a.nsplit), dim3(256), 0, s, a);
    WDR_KLAUNCH(k_flash_combine, dim3(a.Tq, a.n_head), dim3(64), 0, s, a);
    WDR_HIP(hipGetLastError());
    return;
  }
  dim3 grid(cdiv(a.Tq, 128), a.n_head, n_batch);
  const double pairs = a.causal ? 0.5 * (double)a.Tq * a.Tk : (double)a.Tq * a.Tk;
  wdr_launch(PROF_FLASH, (double)n_batch * a.n_head * 64 * 2 * (2.0 * a.Tq + 2.0 * a.Tk),
             (double)n_batch * a.n_head * pairs * 64 * 4, kfn, grid, dim3(256), 0, s, a);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- decoder self-attention
// one 256-thread workgroup per (decoder row, head) over that row's cache (<= 448 keys):
// keys spread over all 4 waves for the scores, 4 key quarters in parallel for P.V.
__global__ __launch_bounds__(256, 8) void k_dec_self_attn(DecSelfArgs a) {   // <= 64 VGPRs: fits beside an encoder tile
  __shared__ float qs[64];
  __shared__ float sc[448];
  __shared__ float red[2][4];
  __shared__ float po[4][64];
  const int r = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int seq = a.row_seq[r];
  const int nk = a.row_pos[r] + 1;
  if (tid < 64) qs[tid] = (float)a.q[(long long)r * a.ldq + h * 64 + tid];
  __syncthreads();
  const f16* K = a.kc + seq * a.seq_stride + h * 64;
  const f16* V = a.vc + seq * a.seq_stride + h * 64;
  // scores: four lanes per key, each a 16-dim partial dot in dim order, added in a fixed
  // shuffle tree (64 keys per pass; the lane's 16 query values stay in registers)
  float mx = -INFINITY;
  const int kq = tid >> 2, qd = tid & 3;
  float qv[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) qv[e] = qs[qd * 16 + e];
  // two 64-key passes per iteration: both passes' key loads in flight before either is scored
  // (each key's dot is unchanged, so the scores are the same bits)
#pragma unroll 1
  for (int k0 = 0; k0 < nk; k0 += 128) {
    f16x8 kv[2][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int k = k0 + 64 * p + kq;
      const f16* kr = K + (long long)(k < nk ? k : nk - 1) * a.d + qd * 16;
      kv[p][0] = *(const f16x8*)kr;
      kv[p][1] = *(const f16x8*)(kr + 8);
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int k = k0 + 64 * p + kq;
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) t += qv[e] * (float)kv[p][0][e];
#pragma unroll
      for (int e = 0; e < 8; ++e) t += qv[8 + e] * (float)kv[p][1][e];
      t += __shfl_xor(t, 1, 64);
      t += __shfl_xor(t, 2, 64);
      if (k < nk) {
        t *= a.scale;
        if (qd == 0) sc[k] = t;
        mx = fmaxf(mx, t);
      }
    }
  }
  mx = wave_max(mx);
  if (lane == 0) red[0][wid] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  float sum = 0.f;
  for (int k = tid; k < nk; k += 256) {
    const float p = __expf(sc[k] - mx);
    sc[k] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  if (lane == 0) red[1][wid] = sum;
  __syncthreads();
  const float inv = 1.f / (red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  // P.V: wave w takes keys w, w+4, ... in the same order as before, with 16 independent V
  // loads in flight per lane (then 8) instead of one dependent load per key
  float acc = 0.f;
  int k = wid;
#pragma unroll 1
  for (; k + 60 < nk; k += 64) {
    f16 vv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) vv[j] = V[(long long)(k + 4 * j) * a.d + lane];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += (float)(f16)(sc[k + 4 * j] * inv) * (float)vv[j];
  }
#pragma unroll 1
  for (; k + 28 < nk; k += 32) {
    f16 vv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) vv[j] = V[(long long)(k + 4 * j) * a.d + lane];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += (float)(f16)(sc[k + 4 * j] * inv) * (float)vv[j];
  }
  for (; k < nk; k += 4) {
    const float p = (float)(f16)(sc[k] * inv);
    acc += p * (float)V[(long long)k * a.d + lane];
  }
  po[wid][lane] = acc;
  __syncthreads();
  if (tid < 64) a.o[(long long)r * a.ldo + h * 64 + tid] = (f16)(po[0][tid] + po[1][tid] + po[2][tid] + po[3][tid]);
}

void launch_dec_self_attn(const DecSelfArgs& a, int R, int n_head, hipStream_t s) {
  WDR_KLAUNCH(k_dec_self_attn, dim3(R, n_head), dim3(256), 0, s, a);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- decoder cross-attention (split)
//
// One workgroup per (64-key chunk, head, row group): thread t takes key t/4 of the chunk and
// dims 16*(t%4)..+16 (4 threads = one key's 128-B head row: coalesced 16-B loads, all issued up
// front), V goes through LDS, and the four waves share the P.V (16 keys each).  A row group is
// the rows sharing one cross K/V -- the beams of one segment -- whose chunk is fetched once and
// scored row after row with exactly the arithmetic of a single row, so a row's result never
// depends on the group (or batch) it runs in.  ROWS: each group its own cross K/V (row_k: the
// multi-chain batched step), else one group of all R rows on k / v (a State's own step).  The
// 24 chunk partials of each row are merged by k_xattn_combine.
constexpr int XA_KC = 64, XA_NS = 24;

// G: the largest group a launch holds -- 1 for the greedy batched step (every row its own
// group), which keeps the kernel at <= 64 VGPRs so a workgroup still fits on a CU beside an
// encoder GEMM tile (k_gemm4: 2 x 224 of the SIMD's 512)
template <bool ROWS, int G>
__global__ __launch_bounds__(256, 8) void k_xattn_partial(XAttnArgs a) {   // <= 64 VGPRs
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  __shared__ __attribute__((aligned(16))) f16 Vs[XA_KC * 64];
  __shared__ float red[2][G][4];
  __shared__ float ps[G][XA_KC];
  __shared__ float pv[G][4][64];
  const int c = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int r0 = 0, nr = a.R;
  const f16* kb = a.k;
  const f16* vb = a.v;
  if (ROWS) {
    r0 = a.lead ? a.lead[blockIdx.z] : blockIdx.z;
    nr = a.grp ? a.grp[r0] : 1;
    if (nr == 0) return;   // a row of a group led by an earlier row
    if (a.lend && a.layer >= a.lend[r0]) return;   // a DTW re-forward past its last head layer
    kb = a.row_k[r0] + a.layer_off;
    vb = kb + a.v_off;
  }
  const int key0 = c * XA_KC;
  const int kk = tid >> 2, qd = tid & 3;
  const int key = key0 + kk;
  const bool kok = key < a.Tk;
  const long long row = (long long)(kok ? key : a.Tk - 1) * a.ldkv + h * a.hs + qd * 16;
  const f16x8 k0 = *(const f16x8*)(kb + row), k1 = *(const f16x8*)(kb + row + 8);
  const f16x8 v0 = *(const f16x8*)(vb + row), v1 = *(const f16x8*)(vb + row + 8);
  *(f16x8*)(Vs + kk * 64 + qd * 16) = v0;
  *(f16x8*)(Vs + kk * 64 + qd * 16 + 8) = v1;
  // every row of the group is scored with exactly the arithmetic of a single row (the same
  // per-thread partial dot, shuffles and wave reductions), all rows between the same three
  // barriers: a row's result never depends on the group (or batch) it runs in
  float sc[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    if (j >= nr) break;
    const f16* qr = a.q + (long long)(r0 + j) * a.ldq + h * 64 + qd * 16;
    const f16x8 q0 = *(const f16x8*)qr, q1 = *(const f16x8*)(qr + 8);
    float t = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) t += (float)q0[e] * (float)k0[e] + (float)q1[e] * (float)k1[e];
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    sc[j] = kok ? t * a.scale : -INFINITY;
    const float wm = wave_max(sc[j]);
    if (lane == 0) red[0][j][wid] = wm;
  }
  __syncthreads();
  float mx[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    if (j >= nr) break;
    mx[j] = fmaxf(fmaxf(red[0][j][0], red[0][j][1]), fmaxf(red[0][j][2], red[0][j][3]));
    const float p = sc[j] == -INFINITY ? 0.f : __expf(sc[j] - mx[j]);
    const float ws = wave_sum(qd == 0 ? p : 0.f);
    if (qd == 0) ps[j][kk] = p;
    if (lane == 0) red[1][j][wid] = ws;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < G; ++j) {
    if (j >= nr) break;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += (float)(f16)ps[j][wid * 16 + i] * (float)Vs[(wid * 16 + i) * 64 + lane];
    pv[j][wid][lane] = acc;
  }
  __syncthreads();
  for (int e = tid; e < nr * 64; e += 256) {
    const int j = e >> 6, dd = e & 63;
    const long long cr = (long long)c * a.R + r0 + j;
    a.part_o[(cr * a.n_head + h) * 64 + dd] = pv[j][0][dd] + pv[j][1][dd] + pv[j][2][dd] + pv[j][3][dd];
    if (dd == 0)
      a.part_ml[cr * a.n_head + h] = make_float2(mx[j], red[1][j][0] + red[1][j][1] + red[1][j][2] + red[1][j][3]);
  }
}

// The greedy batched step's rows (every row its own group, row_k mode) two heads per workgroup:
// half the workgroups of k_xattn_partial<true, 1>, twice the loads in flight per thread; each
// head's arithmetic is that kernel's, instruction for instruction -- the same bits
__global__ __launch_bounds__(256, 8) void k_xattn_partial2(XAttnArgs a) {   // <= 64 VGPRs
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  __shared__ __attribute__((aligned(16))) f16 Vs[2][XA_KC * 64];
  __shared__ float red[2][2][4];
  __shared__ float ps[2][XA_KC];
  __shared__ float pv[2][4][64];
  const int c = blockIdx.x, h0 = blockIdx.y * 2, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r0 = a.lead ? a.lead[blockIdx.z] : blockIdx.z;
  if (a.grp && a.grp[r0] == 0) return;   // a row of a group led by an earlier row
  if (a.lend && a.layer >= a.lend[r0]) return;   // a DTW re-forward past its last head layer
  const f16* kb = a.row_k[r0] + a.layer_off;
  const f16* vb = kb + a.v_off;
  const int key0 = c * XA_KC;
  const int kk = tid >> 2, qd = tid & 3;
  const int key = key0 + kk;
  const bool kok = key < a.Tk;
  const long long row = (long long)(kok ? key : a.Tk - 1) * a.ldkv + h0 * a.hs + qd * 16;
  const f16x8 ka0 = *(const f16x8*)(kb + row), ka1 = *(const f16x8*)(kb + row + 8);
  const f16x8 kc0 = *(const f16x8*)(kb + row + a.hs), kc1 = *(const f16x8*)(kb + row + a.hs + 8);
  {
    const f16x8 v0 = *(const f16x8*)(vb + row), v1 = *(const f16x8*)(vb + row + 8);
    const f16x8 v2 = *(const f16x8*)(vb + row + a.hs), v3 = *(const f16x8*)(vb + row + a.hs + 8);
    *(f16x8*)(Vs[0] + kk * 64 + qd * 16) = v0;
    *(f16x8*)(Vs[0] + kk * 64 + qd * 16 + 8) = v1;
    *(f16x8*)(Vs[1] + kk * 64 + qd * 16) = v2;
    *(f16x8*)(Vs[1] + kk * 64 + qd * 16 + 8) = v3;
  }
  auto score = [&](int hp, const f16x8& k0, const f16x8& k1) {
    const f16* qr = a.q + (long long)r0 * a.ldq + (h0 + hp) * 64 + qd * 16;
    const f16x8 q0 = *(const f16x8*)qr, q1 = *(const f16x8*)(qr + 8);
    float t = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) t += (float)q0[e] * (float)k0[e] + (float)q1[e] * (float)k1[e];
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    const float sc = kok ? t * a.scale : -INFINITY;
    const float wm = wave_max(sc);
    if (lane == 0) red[hp][0][wid] = wm;
    return sc;
  };
  const float sc0 = score(0, ka0, ka1), sc1 = score(1, kc0, kc1);
  __syncthreads();
  float mx[2];
  const float scs[2] = {sc0, sc1};
#pragma unroll
  for (int hp = 0; hp < 2; ++hp) {
    mx[hp] = fmaxf(fmaxf(red[hp][0][0], red[hp][0][1]), fmaxf(red[hp][0][2], red[hp][0][3]));
    const float p = scs[hp] == -INFINITY ? 0.f : __expf(scs[hp] - mx[hp]);
    const float ws = wave_sum(qd == 0 ? p : 0.f);
    if (qd == 0) ps[hp][kk] = p;
    if (lane == 0) red[hp][1][wid] = ws;
  }
  __syncthreads();
#pragma unroll
  for (int hp = 0; hp < 2; ++hp) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += (float)(f16)ps[hp][wid * 16 + i] * (float)Vs[hp][(wid * 16 + i) * 64 + lane];
    pv[hp][wid][lane] = acc;
  }
  __syncthreads();
  if (tid < 128) {
    const int hp = tid >> 6, dd = tid & 63, h = h0 + hp;
    const long long cr = (long long)c * a.R + r0;
    a.part_o[(cr * a.n_head + h) * 64 + dd] = pv[hp][0][dd] + pv[hp][1][dd] + pv[hp][2][dd] + pv[hp][3][dd];
    if (dd == 0) a.part_ml[cr * a.n_head + h] = make_float2(mx[hp], red[hp][1][0] + red[hp][1][1] + red[hp][1][2] + red[hp][1][3]);
  }
}

template <int NS>
__global__ __launch_bounds__(64) void k_xattn_combine(XAttnArgs a) {
  const int r = blockIdx.x, h = blockIdx.y, d = threadIdx.x;
  float po[NS];
#pragma unroll
  for (int c = 0; c < NS; ++c) po[c] = a.part_o[(((long long)c * a.R + r) * a.n_head + h) * 64 + d];
  float2 ml = make_float2(-INFINITY, 0.f);
  if (d < NS) ml = a.part_ml[((long long)d * a.R + r) * a.n_head + h];
  const float M = wave_max(ml.x);
  const float w = (d < NS && ml.x != -INFINITY) ? __expf(ml.x - M) : 0.f;
  const float L = wave_sum(ml.y * w);
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < NS; ++c) acc += po[c] * __shfl(w, c, 64);
  a.o[(long long)r * a.ldo + h * 64 + d] = (f16)(acc / L);
  if (a.ml_out && d == 0) a.ml_out[(long long)r * a.n_head + h] = make_float2(M, L);
}

// ---------------------------------------------------------------- cross-attention, MFMA row tiles
// The rows of a prompt prefill or a DTW re-forward (more than XATTN_GRP_MAX rows sharing one
// cross-K/V slot): one workgroup per (64-key chunk, head, tile of <= 128 rows); the chunk's K
// and V^T are staged in LDS once and each wave scores 32 rows with k_flash_attn's swapped
// product S^T = K.Q^T (v_mfma_f32_32x32x16_f16: a row's scores depend only on its own query),
// takes the chunk's max / sum per row and P.V (P rounded to f16, as the VALU kernel) into the
// same partial layout as k_xattn_partial, so k_xattn_combine merges both kinds.
__global__ __launch_bounds__(256) void k_xattn_mma(XAttnArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  __shared__ __attribute__((aligned(16))) f16 Ks[FA_KB * FA_KS];
  __shared__ __attribute__((aligned(16))) f16 Vt[64 * FA_VS];
  const int c = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int4 t = a.tiles[blockIdx.z];
  if (a.layer >= t.z) return;   // a DTW re-forward past its last head layer
  const f16* kb = a.row_k[t.x] + a.layer_off + h * a.hs;
  const f16* vb = kb + a.v_off;
  const int key0 = c * FA_KB;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;
    const int r = e >> 3, col = (e & 7) * 8;
    int key = key0 + r;
    key = key < a.Tk ? key : a.Tk - 1;
    const f16x8 kr = *(const f16x8*)(kb + (long long)key * a.ldkv + col);
    const f16x8 vr = *(const f16x8*)(vb + (long long)key * a.ldkv + col);
    *(f16x8*)(Ks + r * FA_KS + col) = kr;
#pragma unroll
    for (int j = 0; j < 8; ++j) Vt[(col + j) * FA_VS + r] = vr[j];
  }
  __syncthreads();
  if (32 * wid >= t.y) return;   // no barrier below: idle waves leave
  const int fr = lane & 31, hh = lane >> 5;
  const int ql = 32 * wid + fr;
  const int qrow = t.x + (ql < t.y ? ql : t.y - 1);
  f16x8 qf[4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) qf[s4] = *(const f16x8*)(a.q + (long long)qrow * a.ldq + h * 64 + 16 * s4 + 8 * hh);
  f32x16 st[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
#pragma unroll
    for (int r = 0; r < 16; ++r) st[u][r] = 0.f;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const f16x8 af = *(const f16x8*)(Ks + (32 * u + fr) * FA_KS + 16 * s4 + 8 * hh);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, qf[s4], st[u], 0, 0, 0);
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = key0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const float sv = key < a.Tk ? st[u][r] * a.scale : -INFINITY;
      st[u][r] = sv;
      mx = fmaxf(mx, sv);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float rs = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = st[u][r] == -INFINITY ? 0.f : __expf(st[u][r] - mx);
      st[u][r] = p;
      rs += p;
    }
  rs += __shfl_xor(rs, 32, 64);
  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      f16x8 pb;
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = (f16)st[u][8 * s2 + j];
      const int kc = 32 * u + 16 * s2 + 4 * hh;
      const f16x4 lo0 = *(const f16x4*)(Vt + fr * FA_VS + kc), hi0 = *(const f16x4*)(Vt + fr * FA_VS + kc + 8);
      const f16x4 lo1 = *(const f16x4*)(Vt + (32 + fr) * FA_VS + kc), hi1 = *(const f16x4*)(Vt + (32 + fr) * FA_VS + kc + 8);
      const f16x8 va0 = {lo0[0], lo0[1], lo0[2], lo0[3], hi0[0], hi0[1], hi0[2], hi0[3]};
      const f16x8 va1 = {lo1[0], lo1[1], lo1[2], lo1[3], hi1[0], hi1[1], hi1[2], hi1[3]};
      o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(va0, pb, o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(va1, pb, o1, 0, 0, 0);
    }
  if (ql >= t.y) return;
  const long long cr = (long long)c * a.R + t.x + ql;
  float* po = a.part_o + (cr * a.n_head + h) * 64;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    *(float4*)(po + 8 * g + 4 * hh) = make_float4(o0[4 * g], o0[4 * g + 1], o0[4 * g + 2], o0[4 * g + 3]);
    *(float4*)(po + 32 + 8 * g + 4 * hh) = make_float4(o1[4 * g], o1[4 * g + 1], o1[4 * g + 2], o1[4 * g + 3]);
  }
  if (hh == 0) a.part_ml[cr * a.n_head + h] = make_float2(mx, rs);
}

void launch_xattn_rows(const XAttnArgs& a, hipStream_t s) {
  WDR_CHECK(cdiv(a.Tk, XA_KC) == XA_NS && XA_KC == FA_KB, "cross-attention rows expect 1500 keys");
  WDR_CHECK(a.row_k && a.R >= 1 && (a.n_vgrp == 0 || (a.grp && a.lead)) && (a.n_tiles == 0 || a.tiles),
            "cross-attention rows: bad tables");
  const double kv = (double)a.Tk * a.n_head * 64 * 2 * 2;
  if (a.n_vgrp > 0) {
    const double flops = (double)a.R * a.Tk * a.n_head * 64 * 4;
    if (a.vgrp_max <= 1 && a.n_head % 2 == 0)
      wdr_launch(PROF_XATTN, a.n_vgrp * kv, flops, k_xattn_partial2, dim3(XA_NS, a.n_head / 2, a.n_vgrp), dim3(256),
                 0, s, a);
    else if (a.vgrp_max <= 1)
      wdr_launch(PROF_XATTN, a.n_vgrp * kv, flops, k_xattn_partial<true, 1>, dim3(XA_NS, a.n_head, a.n_vgrp),
                 dim3(256), 0, s, a);
    else
      wdr_launch(PROF_XATTN, a.n_vgrp * kv, flops, k_xattn_partial<true, XATTN_GRP_MAX>,
                 dim3(XA_NS, a.n_head, a.n_vgrp), dim3(256), 0, s, a);
  }
  if (a.n_tiles > 0)
    wdr_launch(PROF_XATTN, a.n_tiles * kv, (double)a.n_tiles * 128 * a.Tk * a.n_head * 64 * 4, k_xattn_mma,
               dim3(XA_NS, a.n_head, a.n_tiles), dim3(256), 0, s, a);
  WDR_KLAUNCH(k_xattn_combine<XA_NS>, dim3(a.R, a.n_head), dim3(64), 0, s, a);
  WDR_HIP(hipGetLastError());
}

void launch_xattn(const XAttnArgs& a, hipStream_t s) {
  WDR_CHECK(cdiv(a.Tk, XA_KC) == XA_NS, "cross-attention decode expects 1500 keys");
  WDR_CHECK(a.R >= 1 && (a.row_k || a.R <= XATTN_GRP_MAX), "cross-attention decode: R out of range");
  // algorithmic bytes: every group's K/V once
  const int ng = a.row_k ? (a.grp ? a.n_grp : a.R) : 1;
  const double bytes = (double)ng * a.Tk * a.n_head * 64 * 2 * 2, flops = (double)a.R * a.Tk * a.n_head * 64 * 4;
  WDR_CHECK(!a.lead || (a.grp && a.n_grp >= 1 && a.n_grp <= a.R), "cross-attention decode: leaders need groups");
  if (a.row_k && !a.grp && a.n_head % 2 == 0)
    wdr_launch(PROF_XATTN, bytes, flops, k_xattn_partial2, dim3(XA_NS, a.n_head / 2, a.R), dim3(256), 0, s, a);
  else if (a.row_k && !a.grp)
    wdr_launch(PROF_XATTN, bytes, flops, k_xattn_partial<true, 1>, dim3(XA_NS, a.n_head, a.R), dim3(256), 0, s, a);
  else if (a.row_k)
    wdr_launch(PROF_XATTN, bytes, flops, k_xattn_partial<true, XATTN_GRP_MAX>,
               dim3(XA_NS, a.n_head, a.lead ? a.n_grp : a.R), dim3(256), 0, s, a);
  else
    wdr_launch(PROF_XATTN, bytes, flops, k_xattn_partial<false, XATTN_GRP_MAX>, dim3(XA_NS, a.n_head), dim3(256), 0,
               s, a);
  WDR_KLAUNCH(k_xattn_combine<XA_NS>, dim3(a.R, a.n_head), dim3(64), 0, s, a);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- alignment-head capture

__global__ __launch_bounds__(256) void k_aheads_capture(CaptureArgs a) {
  __shared__ float qs[64];
  const int r = blockIdx.x, i = blockIdx.y, tid = threadIdx.x;
  const int h = a.heads[i];
  if (tid < 64) qs[tid] = (float)a.q[(long long)r * a.ldq + h * 64 + tid];
  __syncthreads();
  // identical arithmetic to k_flash_attn's f32 accumulate is not guaranteed; the capture
  // recomputes q.k in f32 from the same f16 operands.
  const float2 ml = a.ml[(long long)h * a.R + r];
  const float inv = 1.f / ml.y;
  float* out = a.out + ((long long)(a.slot0 + i) * a.R + r) * a.Tk;
  for (int key = tid; key < a.Tk; key += 256) {
    const f16* kr = a.k + (long long)key * a.ldk + h * a.hs;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 64; c += 8) {
      const f16x8 kv = *(const f16x8*)(kr + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += qs[c + e] * (float)kv[e];
    }
    out[key] = __expf(s * a.scale - ml.x) * inv;
  }
}

void launch_aheads_capture(const CaptureArgs& a, int n_sel, hipStream_t s) {
  WDR_KLAUNCH(k_aheads_capture, dim3(a.R, n_sel), dim3(256), 0, s, a);
  WDR_HIP(hipGetLastError());
}

// k_aheads_capture for rows of several DTW re-forwards in one batch (rows_forward): each
// capture row reads its own slot and writes its own request's buffer
__global__ __launch_bounds__(256) void k_aheads_capture_rows(CaptureRowsArgs a) {
  __shared__ float qs[64];
  const int j = blockIdx.x, i = blockIdx.y, tid = threadIdx.x;
  const int r = a.crow[j], h = a.heads[i];
  if (tid < 64) qs[tid] = (float)a.q[(long long)r * a.ldq + h * 64 + tid];
  __syncthreads();
  const float2 ml = a.ml[(long long)r * a.n_head + h];
  const float inv = 1.f / ml.y;
  const f16* kb = a.row_k[r] + a.layer_off + h * a.hs;
  float* out = a.cdst[j] + (long long)(a.slot0 + i) * a.cstride[j];
  for (int key = tid; key < a.Tk; key += 256) {
    const f16* kr = kb + (long long)key * 64;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 64; c += 8) {
      const f16x8 kv = *(const f16x8*)(kr + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += qs[c + e] * (float)kv[e];
    }
    out[key] = __expf(s * a.scale - ml.x) * inv;
  }
}

void launch_aheads_capture_rows(const CaptureRowsArgs& a, int n_sel, hipStream_t s) {
  if (a.n_cap <= 0 || n_sel <= 0) return;
  WDR_KLAUNCH(k_aheads_capture_rows, dim3(a.n_cap, n_sel), dim3(256), 0, s, a);
  WDR_HIP(hipGetLastError());
}

}  // namespace wdr
