// Persistent greedy decode step: all decoder layers + the final LayerNorm
// + the logits projection of ONE decoder row in ONE launch of one 256-thread workgroup per CU.
//
// Why: a large-v3 step is a chain of ~290 small dependent kernels (3-13 MB each) whose bodies
// are latency-bound (a 3.3 MB GEMV runs ~4 us where streaming its bytes takes ~0.5 us) and
// whose boundaries cost ~1.2 us each.  Here every workgroup walks the same phase list; before
// it waits for a phase's inputs it issues the loads of its share of that phase's weights, so
// the HBM latency of the weight stream overlaps the dependency edge instead of following it.
//
// Phases of layer l (items are workgroup-sized units of work, item i runs on workgroup i % G):
//   QKV   LN1(x) . Wqkv, 12 items per head (16 rows each); k, v go straight into the cache
//   SELF  per head, on workgroup G-1-h once that head's 12 QKV items are in
//   O     att . Wo + bo added into x (d/8 items)
//   XQ    LN2(x) . Wxq, 8 items per head
//   XATT  (head, 64-key chunk) partials, 24 per head; the chunk's cross K/V are loaded before
//         the wait; the last chunk of a head to finish merges the head's 24 partials
//   XO    xatt . Wxo + bxo added into x
//   FC1   gelu(LN3(x) . Wfc1 + b) (4d/16 items)
//   FC2   mlp . Wfc2 + b added into x (d/4 items)
// then LN(x) . tok_emb^T -> logits (V/16 items, double-buffered weight loads).
//
// Hand-offs (MI355X_MICROARCH.md, hand-off table row 1): producers store every handed-off
// byte with `sc1` stores, every storing wave drains (`s_waitcnt vmcnt(0)`), a workgroup barrier,
// then ONE lane adds to the phase's agent-scope counter; consumers poll with `sc1` loads and
// read every handed-off byte with `sc1` loads.  Counters are zero between launches: the last
// workgroup to finish resets them.  Every wait is bounded; a timeout sets *err, the workgroup
// leaves, and the host resets the counters and raises.  Co-residency is not required for
// progress (items only wait on lower phases, which never wait on later ones).
#include "kernels.h"
#include "../prof.h"

namespace wdr {

namespace {

constexpr unsigned kSpinLimit = 400000;   // ~0.2-0.4 s of polling before a wait gives up
constexpr int kSC1 = 16;                  // buffer cache-policy bit: sc1 (gfx950)
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ f16x8 ld16_sc1(const void* base, int byte_off) {
  const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), byte_off, 0, kSC1);
  return __builtin_bit_cast(f16x8, v);
}
__device__ __forceinline__ float ldf_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stf_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sth_sc1(f16* p, f16 v) {
  __hip_atomic_store((unsigned short*)p, __builtin_bit_cast(unsigned short, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st8_sc1(void* p, unsigned long long v) {
  __hip_atomic_store((unsigned long long*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ float dot8(f16x8 w, f16x8 x, float s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f16x2 wp = {w[2 * q], w[2 * q + 1]};
    f16x2 xp = {x[2 * q], x[2 * q + 1]};
    s = __builtin_amdgcn_fdot2(wp, xp, s, false);
  }
  return s;
}

struct Lds {
  f16 xs[10 * 512 + 8];          // staged activation row (f16), up to K = 4d = 5120
  float red[8];
  int flag;
  float qs[64];
  float sc[448];
  float po[4][64];
  f16 vs[64 * 64];
  float ps[64];
};

// Wait until *c >= target (thread 0 polls, the workgroup joins).  False: gave up or another
// workgroup already failed; the caller leaves.
__device__ bool wg_wait(const unsigned* c, unsigned target, int* err) {
  int ok = 1;
  if (threadIdx.x == 0) {
    unsigned it = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      ++it;
      if (it > kSpinLimit || ((it & 63) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  return __syncthreads_and(ok);
}

// Publish this workgroup's sc1 stores: every wave drains, barrier, one lane adds n.
__device__ void wg_signal(unsigned* c, unsigned n) {
  vm_drain();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Same, and tell the workgroup whether its add completed the count `total`.
__device__ bool wg_signal_last(unsigned* c, unsigned total) {
  vm_drain();
  __syncthreads();
  int last = 0;
  if (threadIdx.x == 0) last = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
  return __syncthreads_or(last);
}

// f16 activation row (written by other workgroups in this launch) -> LDS
__device__ void stage_f16(const f16* src, int n, f16* xs) {
  for (int i = threadIdx.x; i < n / 8; i += 256) *(f16x8*)(xs + i * 8) = ld16_sc1(src, i * 16);
  __syncthreads();
}

// ggml_norm (eps 1e-5) of the f32 residual row x[d], times g plus b, as f16 into LDS
__device__ void stage_ln(const float* x, int d, const float* g, const float* b, Lds& s) {
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const bool on = t * 8 < d;
  float v[8], gg[8], bb[8];
  const int o = on ? t * 8 : 0;
  {
    const f16x8 r0 = ld16_sc1(x, o * 4), r1 = ld16_sc1(x, o * 4 + 16);
    const float4 a0 = __builtin_bit_cast(float4, r0), a1 = __builtin_bit_cast(float4, r1);
    v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
    const float4 g0 = *(const float4*)(g + o), g1 = *(const float4*)(g + o + 4);
    const float4 b0 = *(const float4*)(b + o), b1 = *(const float4*)(b + o + 4);
    gg[0] = g0.x; gg[1] = g0.y; gg[2] = g0.z; gg[3] = g0.w; gg[4] = g1.x; gg[5] = g1.y; gg[6] = g1.z; gg[7] = g1.w;
    bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
  }
  float sm = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) sm += on ? v[e] : 0.f;
  sm = wave_sum(sm);
  if (lane == 0) s.red[wid] = sm;
  __syncthreads();
  const float mean = (s.red[0] + s.red[1] + s.red[2] + s.red[3]) / d;
  float s2 = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float q = v[e] - mean;
    s2 += on ? q * q : 0.f;
  }
  s2 = wave_sum(s2);
  if (lane == 0) s.red[4 + wid] = s2;
  __syncthreads();
  const float scale = 1.0f / sqrtf((s.red[4] + s.red[5] + s.red[6] + s.red[7]) / d + 1e-5f);
  if (on) {
    f16x8 h;
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = (f16)((v[e] - mean) * scale * gg[e] + bb[e]);
    *(f16x8*)(s.xs + t * 8) = h;
  }
  __syncthreads();
}

// RW consecutive weight rows per wave, K split in 512-wide chunks (lane l owns k = 512c + 8l..+8)
template <int RW, int NCH>
struct Rows {
  f16x8 w[RW][NCH];
  __device__ __forceinline__ void load(const f16* W, int K, int N, int n0) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int n = n0 + r < N ? n0 + r : N - 1;
      const f16* wr = W + (size_t)n * K;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int k = c * 512 + lane * 8;
        const f16x8 t = __builtin_nontemporal_load((const f16x8*)(wr + (k < K ? k : K - 8)));
        w[r][c] = k < K ? t : (f16x8){};
      }
    }
  }
  // acc[r] = sum_k W[n0 + r][k] xs[k], reduced over the wave (every lane holds the sums)
  __device__ __forceinline__ void dot(const f16* xs, int K, float (&acc)[RW]) const {
    const int lane = threadIdx.x & 63;
    f16x8 xv[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = c * 512 + lane * 8;
      const f16x8 t = *(const f16x8*)(xs + (k < K ? k : 0));
      xv[c] = k < K ? t : (f16x8){};
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) a = dot8(w[r][c], xv[c], a);
      acc[r] = wave_sum(a);
    }
  }
};

}  // namespace

// counter layout per layer (stride 3H + 6): [0,H) qkv/head, H att, H+1 o, [H+2,2H+2) xq/head,
// [2H+2,3H+2) xatt/head, 3H+2 combined heads, 3H+3 xo, 3H+4 fc1, 3H+5 fc2; then one end counter
template <int ND, int NF>
__global__ __launch_bounds__(256) void k_step(StepArgs a) {
  __shared__ __attribute__((aligned(16))) Lds s;
  const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int d = a.d, H = a.n_head, L = a.L;
  const int CPL = 3 * H + 6;
  const int seq = a.row_seq[0], pos = a.row_pos[0];
  // item counts
  const int n_qkv = 12 * H, n_o = d / 8, n_xa = 24 * H, n_fc1 = (4 * d + 15) / 16, n_fc2 = d / 4;
  const int n_lg = (a.V + 15) / 16;
  // optional timeline (tools/step_probe.py): wall_clock64 of thread 0 per (layer < 4, event)
#define TR(l, e) \
  if (a.trace && tid == 0 && (l) < 4) a.trace[((l) * 16 + (e)) * G + w] = wall_clock64();
#define TRX(e) \
  if (a.trace && tid == 0) a.trace[(e) * G + w] = wall_clock64();
  TRX(64);

  for (int l = 0; l < L; ++l) {
    const StepLayer& ly = a.layers[l];
    unsigned* C = a.ctr + l * CPL;
    const unsigned* Cprev = l > 0 ? a.ctr + (l - 1) * CPL + 3 * H + 5 : nullptr;   // fc2 of layer l-1
    f16* kc = a.kc + l * a.layer_stride + seq * a.seq_stride;
    f16* vc = a.vc + l * a.layer_stride + seq * a.seq_stride;

    // ---------------- QKV: item i -> head h = i / 12, part (q/k/v) = (i % 12) / 4, 16 rows
    {
      const bool has = w < n_qkv;
      Rows<4, ND> R;
      int h = 0, n0 = 0;
      if (has) {
        h = w / 12;
        const int j = w % 12;
        n0 = (j / 4) * d + h * 64 + (j % 4) * 16 + wid * 4;
        R.load(ly.w_qkv, d, 3 * d, n0);
      }
      if (has) {
        if (Cprev && !wg_wait(Cprev, n_fc2, a.err)) return;
        TR(l, 0);
        stage_ln(a.x, d, ly.ln1_g, ly.ln1_b, s);
        float acc[4];
        R.dot(s.xs, d, acc);
        if (lane == 0) {
          f16 o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (f16)(acc[r] + ly.b_qkv[n0 + r]);
          const unsigned long long pk = __builtin_bit_cast(unsigned long long, (f16x4){o[0], o[1], o[2], o[3]});
          if (n0 < d) st8_sc1(a.q + n0, pk);
          else if (n0 < 2 * d) st8_sc1(kc + (size_t)pos * d + n0 - d, pk);
          else st8_sc1(vc + (size_t)pos * d + n0 - 2 * d, pk);
        }
        wg_signal(C + h, 1);
        TR(l, 1);
      }
    }
    // ---------------- SELF attention of head h on workgroup G-1-h (<= 448 cached keys)
    if (w >= G - H) {
      const int h = G - 1 - w;
      if (!wg_wait(C + h, 12, a.err)) return;
      TR(l, 2);
      const int nk = pos + 1;
      const f16* K = kc + h * 64;
      const f16* Vv = vc + h * 64;
      if (tid < 8) {
        const f16x8 qv = ld16_sc1(a.q, (h * 64 + tid * 8) * 2);
#pragma unroll
        for (int e = 0; e < 8; ++e) s.qs[tid * 8 + e] = (float)qv[e];
      }
      __syncthreads();
      float mx = -INFINITY;
      for (int k = tid; k < nk; k += 256) {
        float sc = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const f16x8 kv = ld16_sc1(K, ((size_t)k * d + 8 * c) * 2);
#pragma unroll
          for (int e = 0; e < 8; ++e) sc += s.qs[8 * c + e] * (float)kv[e];
        }
        sc *= a.scale;
        s.sc[k] = sc;
        mx = fmaxf(mx, sc);
      }
      mx = wave_max(mx);
      if (lane == 0) s.red[wid] = mx;
      __syncthreads();
      mx = fmaxf(fmaxf(s.red[0], s.red[1]), fmaxf(s.red[2], s.red[3]));
      float sum = 0.f;
      for (int k = tid; k < nk; k += 256) {
        const float p = __expf(s.sc[k] - mx);
        s.sc[k] = p;
        sum += p;
      }
      sum = wave_sum(sum);
      if (lane == 0) s.red[4 + wid] = sum;
      __syncthreads();
      const float inv = 1.f / (s.red[4] + s.red[5] + s.red[6] + s.red[7]);
      float acc = 0.f;
      const __amdgpu_buffer_rsrc_t vr = rsrc(Vv);
      int k = wid;
      for (; k + 28 < nk; k += 32) {   // 8 independent V loads in flight per lane
        unsigned short vb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) vb[j] = __builtin_amdgcn_raw_buffer_load_b16(vr, ((k + 4 * j) * d + lane) * 2, 0, kSC1);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += (float)(f16)(s.sc[k + 4 * j] * inv) * (float)__builtin_bit_cast(f16, vb[j]);
      }
      for (; k < nk; k += 4) {
        const unsigned short vb = __builtin_amdgcn_raw_buffer_load_b16(vr, (k * d + lane) * 2, 0, kSC1);
        acc += (float)(f16)(s.sc[k] * inv) * (float)__builtin_bit_cast(f16, vb);
      }
      s.po[wid][lane] = acc;
      __syncthreads();
      if (tid < 64) sth_sc1(a.att + h * 64 + tid, (f16)(s.po[0][tid] + s.po[1][tid] + s.po[2][tid] + s.po[3][tid]));
      wg_signal(C + H, 1);
      TR(l, 3);
    }
    // ---------------- O: 8 rows per item (2 per wave), added into x
    {
      const bool has = w < n_o;
      Rows<2, ND> R;
      const int n0 = w * 8 + wid * 2;
      if (has) R.load(ly.w_o, d, d, n0);
      if (has) {
        if (!wg_wait(C + H, H, a.err)) return;
        TR(l, 4);
        stage_f16(a.att, d, s.xs);
        float acc[2];
        R.dot(s.xs, d, acc);
        if (lane == 0) {
          const float x0 = ldf_sc1(a.x + n0), x1 = ldf_sc1(a.x + n0 + 1);
          const float2 o = make_float2(x0 + acc[0] + ly.b_o[n0], x1 + acc[1] + ly.b_o[n0 + 1]);
          st8_sc1(a.x + n0, __builtin_bit_cast(unsigned long long, o));
        }
        wg_signal(C + H + 1, 1);
        TR(l, 5);
      }
    }
    // ---------------- XQ: 8 items per head (2 rows per wave)
    {
      const bool has = w < n_o;
      Rows<2, ND> R;
      const int n0 = w * 8 + wid * 2;
      if (has) R.load(ly.w_xq, d, d, n0);
      if (has) {
        if (!wg_wait(C + H + 1, n_o, a.err)) return;
        TR(l, 6);
        stage_ln(a.x, d, ly.ln2_g, ly.ln2_b, s);
        float acc[2];
        R.dot(s.xs, d, acc);
        if (lane == 0) {
          const f16x2 o = {(f16)(acc[0] + ly.b_xq[n0]), (f16)(acc[1] + ly.b_xq[n0 + 1])};
          __hip_atomic_store((unsigned*)(a.qx + n0), __builtin_bit_cast(unsigned, o), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
        wg_signal(C + H + 2 + (w * 8) / 64, 1);
        TR(l, 7);
      }
    }
    // ---------------- XATT: (head, 64-key chunk) items; cross K/V loaded before the wait
    {
      const f16* xk = a.xkv + xkv_k_off(l, a.n_head);   // head-major slot (common.h)
      const f16* xv = a.xkv + xkv_v_off(l, a.n_head);
      const int kk = tid >> 2, qd = tid & 3;
      f16x8 kr[2][2], vr[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int it = w + u * G;
        if (it < n_xa) {
          const int c = it % 24, h = it / 24;
          const int key = c * 64 + kk;
          const size_t row = (size_t)(key < 1500 ? key : 1499) * 64 + h * XKV_HS + qd * 16;
          kr[u][0] = __builtin_nontemporal_load((const f16x8*)(xk + row));
          kr[u][1] = __builtin_nontemporal_load((const f16x8*)(xk + row + 8));
          vr[u][0] = __builtin_nontemporal_load((const f16x8*)(xv + row));
          vr[u][1] = __builtin_nontemporal_load((const f16x8*)(xv + row + 8));
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int it = w + u * G;
        if (it >= n_xa) break;
        const int c = it % 24, h = it / 24;
        const int key = c * 64 + kk;
        const bool kok = key < 1500;
        if (!wg_wait(C + H + 2 + h, 8, a.err)) return;
        TR(l, 8);
        const f16x8 q0 = ld16_sc1(a.qx, (h * 64 + qd * 16) * 2), q1 = ld16_sc1(a.qx, (h * 64 + qd * 16 + 8) * 2);
        *(f16x8*)(s.vs + kk * 64 + qd * 16) = vr[u][0];
        *(f16x8*)(s.vs + kk * 64 + qd * 16 + 8) = vr[u][1];
        float sc = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) sc += (float)q0[e] * (float)kr[u][0][e] + (float)q1[e] * (float)kr[u][1][e];
        sc += __shfl_xor(sc, 1, 64);
        sc += __shfl_xor(sc, 2, 64);
        sc = kok ? sc * a.scale : -INFINITY;
        const float wm = wave_max(sc);
        if (lane == 0) s.red[wid] = wm;
        __syncthreads();
        const float mx = fmaxf(fmaxf(s.red[0], s.red[1]), fmaxf(s.red[2], s.red[3]));
        const float p = sc == -INFINITY ? 0.f : __expf(sc - mx);
        const float ws = wave_sum(qd == 0 ? p : 0.f);
        if (qd == 0) s.ps[kk] = p;
        if (lane == 0) s.red[4 + wid] = ws;
        __syncthreads();
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += (float)(f16)s.ps[wid * 16 + j] * (float)s.vs[(wid * 16 + j) * 64 + lane];
        s.po[wid][lane] = acc;
        __syncthreads();
        if (tid < 64) {
          stf_sc1(a.part_o + ((size_t)c * H + h) * 64 + tid, s.po[0][tid] + s.po[1][tid] + s.po[2][tid] + s.po[3][tid]);
          if (tid == 0)
            st8_sc1(a.part_ml + (size_t)c * H + h,
                    __builtin_bit_cast(unsigned long long,
                                       make_float2(mx, s.red[4] + s.red[5] + s.red[6] + s.red[7])));
        }
        if (wg_signal_last(C + 2 * H + 2 + h, 24)) {
          // the last chunk of head h merges the 24 partials (as k_xattn_combine<24>)
          if (tid < 64) {
            float po[24];
#pragma unroll
            for (int cc = 0; cc < 24; ++cc) po[cc] = ldf_sc1(a.part_o + ((size_t)cc * H + h) * 64 + tid);
            float2 ml = make_float2(-INFINITY, 0.f);
            if (tid < 24) {
              const unsigned long long r = __hip_atomic_load((const unsigned long long*)(a.part_ml + (size_t)tid * H + h),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              ml = __builtin_bit_cast(float2, r);
            }
            const float M = wave_max(ml.x);
            const float wgt = (tid < 24 && ml.x != -INFINITY) ? __expf(ml.x - M) : 0.f;
            const float Ls = wave_sum(ml.y * wgt);
            float o = 0.f;
#pragma unroll
            for (int cc = 0; cc < 24; ++cc) o += po[cc] * __shfl(wgt, cc, 64);
            sth_sc1(a.xatt + h * 64 + tid, (f16)(o / Ls));
          }
          wg_signal(C + 3 * H + 2, 1);
          TR(l, 9);
        }
      }
    }
    // ---------------- XO: 8 rows per item, added into x
    {
      const bool has = w < n_o;
      Rows<2, ND> R;
      const int n0 = w * 8 + wid * 2;
      if (has) R.load(ly.w_xo, d, d, n0);
      if (has) {
        if (!wg_wait(C + 3 * H + 2, H, a.err)) return;
        TR(l, 10);
        stage_f16(a.xatt, d, s.xs);
        float acc[2];
        R.dot(s.xs, d, acc);
        if (lane == 0) {
          const float x0 = ldf_sc1(a.x + n0), x1 = ldf_sc1(a.x + n0 + 1);
          const float2 o = make_float2(x0 + acc[0] + ly.b_xo[n0], x1 + acc[1] + ly.b_xo[n0 + 1]);
          st8_sc1(a.x + n0, __builtin_bit_cast(unsigned long long, o));
        }
        wg_signal(C + 3 * H + 3, 1);
        TR(l, 11);
      }
    }
    // ---------------- FC1: 16 rows per item (4 per wave), up to two items per workgroup
    {
      Rows<4, ND> R[2];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int it = w + u * G;
        if (it < n_fc1) {
          R[u].load(ly.w_fc1, d, 4 * d, it * 16 + wid * 4);
          cnt++;
        }
      }
      if (cnt) {
        if (!wg_wait(C + 3 * H + 3, n_o, a.err)) return;
        TR(l, 12);
        stage_ln(a.x, d, ly.ln3_g, ly.ln3_b, s);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (u >= cnt) break;
          const int n0 = (w + u * G) * 16 + wid * 4;
          float acc[4];
          R[u].dot(s.xs, d, acc);
          if (lane == 0 && n0 < 4 * d) {
            f16 o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (f16)gelu_tanh(acc[r] + ly.b_fc1[n0 + r]);
            st8_sc1(a.mlp + n0, __builtin_bit_cast(unsigned long long, (f16x4){o[0], o[1], o[2], o[3]}));
          }
        }
        wg_signal(C + 3 * H + 4, cnt);
        TR(l, 13);
      }
    }
    // ---------------- FC2: 4 rows per item (1 per wave, K = 4d), added into x
    {
      Rows<1, NF> R[2];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int it = w + u * G;
        if (it < n_fc2) {
          R[u].load(ly.w_fc2, 4 * d, d, it * 4 + wid);
          cnt++;
        }
      }
      if (cnt) {
        if (!wg_wait(C + 3 * H + 4, n_fc1, a.err)) return;
        TR(l, 14);
        stage_f16(a.mlp, 4 * d, s.xs);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (u >= cnt) break;
          const int n0 = (w + u * G) * 4 + wid;
          float acc[1];
          R[u].dot(s.xs, 4 * d, acc);
          if (lane == 0) stf_sc1(a.x + n0, ldf_sc1(a.x + n0) + acc[0] + ly.b_fc2[n0]);
        }
        wg_signal(C + 3 * H + 5, cnt);
        TR(l, 15);
      }
    }
  }
  // ---------------- final LayerNorm + logits = LN(x) . tok_emb^T (16 rows per item)
  {
    const unsigned* Clast = a.ctr + (L - 1) * CPL + 3 * H + 5;
    Rows<4, ND> R0, R1;
    int it = w;
    if (it < n_lg) R0.load(a.tok_emb, d, a.V, it * 16 + wid * 4);
    if (it < n_lg) {
      if (!wg_wait(Clast, n_fc2, a.err)) return;
      TRX(65);
      stage_ln(a.x, d, a.ln_g, a.ln_b, s);
    }
    auto emit = [&](const Rows<4, ND>& R, int item) {
      const int n0 = item * 16 + wid * 4;
      float acc[4];
      R.dot(s.xs, d, acc);
      if (lane < 4 && n0 + lane < a.V) {
        float v = acc[0];
#pragma unroll
        for (int r = 1; r < 4; ++r)
          if (lane == r) v = acc[r];
        a.logits[n0 + lane] = v;
      }
    };
    // two register sets, static indices: item it computes while item it + G streams in
    while (it < n_lg) {
      if (it + G < n_lg) R1.load(a.tok_emb, d, a.V, (it + G) * 16 + wid * 4);
      emit(R0, it);
      it += G;
      if (it >= n_lg) break;
      if (it + G < n_lg) R0.load(a.tok_emb, d, a.V, (it + G) * 16 + wid * 4);
      emit(R1, it);
      it += G;
    }
  }
  // ---------------- the last workgroup out resets every counter for the next launch
  vm_drain();
  __syncthreads();
  unsigned* Cend = a.ctr + L * CPL;
  int last = 0;
  if (tid == 0) last = __hip_atomic_fetch_add(Cend, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)G - 1;
  TRX(66);
  if (__syncthreads_or(last)) {
    for (int i = tid; i <= L * CPL; i += 256) __hip_atomic_store(a.ctr + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int step_counters(int L, int n_head) { return L * (3 * n_head + 6) + 1; }

bool step_supported(int d, int n_head) {
  return d % 64 == 0 && d / 64 == n_head && d >= 128 && d <= 1280;
}

void launch_step(const StepArgs& a, int n_wg, hipStream_t s) {
  WDR_CHECK(step_supported(a.d, a.n_head), "persistent step: unsupported model width");
  WDR_CHECK(n_wg >= 12 * a.n_head && 2 * n_wg >= 24 * a.n_head && 2 * n_wg >= (4 * a.d + 15) / 16 &&
                2 * n_wg >= a.d / 4 && n_wg >= a.d / 8,
            "persistent step: too few workgroups for the item counts");
  const int nd = cdiv(a.d, 512), nf = cdiv(4 * a.d, 512);
  dim3 g(n_wg), b(256);
#define WDR_ST(ND, NF)                                   \
  if (nd == ND && nf == NF) {                            \
    WDR_KLAUNCH((k_step<ND, NF>), g, b, 0, s, a); \
    WDR_HIP(hipGetLastError());                          \
    return;                                              \
  }
  WDR_ST(1, 1) WDR_ST(1, 3) WDR_ST(1, 4) WDR_ST(2, 6) WDR_ST(2, 8) WDR_ST(3, 10)
#undef WDR_ST
  throw std::runtime_error("persistent step: no instantiation for this width");
}

}  // namespace wdr
