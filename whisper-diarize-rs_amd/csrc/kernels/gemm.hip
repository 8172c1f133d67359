// Projection kernels: the dense contractions of the Whisper encoder / decoder
// (SURVEY.md §8(a) a5-a7, a9, a12).
//
//  * k_gemm  — MFMA GEMM for M > 8 rows (encoder windows, cross-K/V, prompt prefill,
//              DTW re-forward):  C[M][N] = A[M][K] . B[N][K]^T  (+ fused epilogue).
//              f16 operands (what ggml's mul_mat feeds: f16 weights, activations cast to
//              f16), f32 accumulation, v_mfma_f32_32x32x16_f16.  128x128x32 block tile,
//              4 waves of 64x64, register-staged double-buffered LDS, row padding for
//              conflict-free ds_read_b128.  Roofline: MFMA (2.5 PF/s dense f16).
//  * k_gemv  — M <= 8 rows (decoder step, one row per decoder): each wave streams one
//              weight row with 16-B loads, v_dot2_f32_f16, wave-shuffle reduction.
//              Roofline: HBM (bytes = N*K*2 per launch).
#include "../common.h"
#include "../prof.h"

#include <algorithm>

namespace wdr {

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

constexpr int GB_M = 128, GB_N = 128, GB_K = 32;
constexpr int GLDS = GB_K + 8;   // LDS row stride in halfs (80 B): conflict-free b128 fragment reads

template <int EPI>
__device__ __forceinline__ void epi_store(const ProjArgs& a, int row, int col, float v) {
  if (row >= a.M || col >= a.N) return;
  if (a.bias) v += a.bias[col];
  if constexpr (EPI == EPI_F16) {
    ((f16*)a.out)[(size_t)row * a.ldo + col] = (f16)v;
  } else if constexpr (EPI == EPI_F16_GELU) {
    ((f16*)a.out)[(size_t)row * a.ldo + col] = (f16)gelu_tanh(v);
  } else if constexpr (EPI == EPI_F32_RESID) {
    float* o = (float*)a.out + (size_t)row * a.ldo + col;
    *o = *o + v;
  } else if constexpr (EPI == EPI_F32) {
    ((float*)a.out)[(size_t)row * a.ldo + col] = v;
  } else if constexpr (EPI == EPI_F32_GELU_POS) {
    ((float*)a.out)[(size_t)row * a.ldo + col] =
        gelu_tanh(v) + a.pos[(size_t)(row % a.pos_rows) * a.N + col];
  } else {  // EPI_QKV_CACHE
    if (col < a.d) {
      ((f16*)a.out)[(size_t)row * a.ldo + col] = (f16)v;
    } else {
      const long long dst = a.row_seq[row] * a.seq_stride + (long long)a.row_pos[row] * a.d;
      if (col < 2 * a.d) a.kc[dst + col - a.d] = (f16)v;
      else a.vc[dst + col - 2 * a.d] = (f16)v;
    }
  }
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm(ProjArgs a) {
  __shared__ __attribute__((aligned(16))) f16 sA[2][GB_M * GLDS];
  __shared__ __attribute__((aligned(16))) f16 sB[2][GB_N * GLDS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int bn = blockIdx.x, bm = blockIdx.y;
  const int wr = wid >> 1, wc = wid & 1;

  // staging: 512 16-B chunks per operand tile, 2 per thread
  int a_off[2], b_off[2], s_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    const int r = c >> 2, kc = (c & 3) * 8;
    int gm = bm * GB_M + r;
    gm = gm < a.M ? gm : a.M - 1;
    const int gn = bn * GB_N + r;   // N % 128 == 0 (host-checked)
    a_off[i] = gm * a.lda + kc;
    b_off[i] = gn * a.ldb + kc;
    s_off[i] = r * GLDS + kc;
  }
  const int nk = a.K / GB_K;
  f16x8 ra[2], rb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    ra[i] = *(const f16x8*)(a.A + a_off[i]);
    rb[i] = *(const f16x8*)(a.B + b_off[i]);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    *(f16x8*)(&sA[0][s_off[i]]) = ra[i];
    *(f16x8*)(&sB[0][s_off[i]]) = rb[i];
  }
  __syncthreads();

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fk = 8 * (lane >> 5);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int ko = (kt + 1) * GB_K;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ra[i] = *(const f16x8*)(a.A + a_off[i] + ko);
        rb[i] = *(const f16x8*)(a.B + b_off[i] + ko);
      }
    }
    const f16* As = sA[cur];
    const f16* Bs = sB[cur];
#pragma unroll
    for (int ks = 0; ks < GB_K / 16; ++ks) {
      f16x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *(const f16x8*)(As + (wr * 64 + i * 32 + fr) * GLDS + ks * 16 + fk);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[j] = *(const f16x8*)(Bs + (wc * 64 + j * 32 + fr) * GLDS + ks * 16 + fk);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        *(f16x8*)(&sA[cur ^ 1][s_off[i]]) = ra[i];
        *(f16x8*)(&sB[cur ^ 1][s_off[i]]) = rb[i];
      }
    }
    __syncthreads();
  }

  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = bm * GB_M + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = bn * GB_N + wc * 64 + j * 32 + fr;
        epi_store<EPI>(a, row, col, acc[i][j][r]);
      }
}

// ---------------------------------------------------------------- GEMV (M <= 8)
// Grid-stride over output rows (one weight row per wave per iteration), 16-B weight loads,
// v_dot2_f32_f16.  With the fused LayerNorm prologue (LN, K <= 1536) every wave normalises
// its input rows itself, straight into the registers that hold exactly the K-slices its lane
// multiplies (lane l owns k in [512 i + 8 l, +8)): one round of loads, no LDS, no barrier.
template <int NCH>
__device__ __forceinline__ void ln_row_regs(const ProjArgs& a, int r, int lane, f16x8 (&xo)[NCH]) {
  const float* xr = a.ln_x + (size_t)r * a.ldln;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    if (k < a.K) {
      const float4 p0 = *(const float4*)(xr + k), p1 = *(const float4*)(xr + k + 4);
      v[c][0] = p0.x; v[c][1] = p0.y; v[c][2] = p0.z; v[c][3] = p0.w;
      v[c][4] = p1.x; v[c][5] = p1.y; v[c][6] = p1.z; v[c][7] = p1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[c][e];
  }
  s = wave_sum(s);
  const float mean = s / a.K;
  float s2 = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
    if (c * 512 + lane * 8 < a.K)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = v[c][e] - mean;
        s2 += t * t;
      }
  s2 = wave_sum(s2);
  const float scale = 1.0f / sqrtf(s2 / a.K + 1e-5f);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    if (k < a.K) {
      const float4 g0 = *(const float4*)(a.ln_g + k), g1 = *(const float4*)(a.ln_g + k + 4);
      const float4 b0 = *(const float4*)(a.ln_b + k), b1 = *(const float4*)(a.ln_b + k + 4);
      const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) xo[c][e] = (f16)((v[c][e] - mean) * scale * gg[e] + bb[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) xo[c][e] = (f16)0.f;
    }
  }
}

__device__ __forceinline__ float dot8(f16x8 w, f16x8 x, float s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f16x2 wp = {w[2 * q], w[2 * q + 1]};
    f16x2 xp = {x[2 * q], x[2 * q + 1]};
    s = __builtin_amdgcn_fdot2(wp, xp, s, false);
  }
  return s;
}

template <int EPI, int MR>
__device__ __forceinline__ void gemv_store(const ProjArgs& a, float (&acc)[MR], int lane, int n) {
#pragma unroll
  for (int r = 0; r < MR; ++r) acc[r] = wave_sum(acc[r]);
  if (lane < MR && lane < a.M) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < MR; ++r)
      if (r == lane) v = acc[r];
    epi_store<EPI>(a, lane, n, v);
  }
}

// LN prologue, M <= 2, K <= 512*NCH: normalised rows live in registers.
template <int EPI, int MR, int NCH>
__global__ __launch_bounds__(256) void k_gemv_ln(ProjArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // the first weight row is requested before the LayerNorm so its latency overlaps the norm
  int n = blockIdx.x * 4 + wid;
  f16x8 wv[NCH];
  if (n < a.N) {
    const f16* w = a.B + (size_t)n * a.ldb;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = c * 512 + lane * 8;
      wv[c] = k < a.K ? *(const f16x8*)(w + k) : (f16x8){};
    }
  }
  f16x8 xr[MR][NCH];
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    if (r < a.M) ln_row_regs<NCH>(a, r, lane, xr[r]);
  }
  for (; n < a.N; n += gridDim.x * 4) {
    if (n != blockIdx.x * 4 + wid) {
      const f16* w = a.B + (size_t)n * a.ldb;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int k = c * 512 + lane * 8;
        wv[c] = k < a.K ? *(const f16x8*)(w + k) : (f16x8){};
      }
    }
    float acc[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      acc[r] = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc[r] = dot8(wv[c], xr[r][c], acc[r]);
    }
    gemv_store<EPI, MR>(a, acc, lane, n);
  }
}

// No-LN GEMV for M <= 2 with K = 512*NCH exactly: every weight and activation load of the
// row is issued before the first dot product (K = 5120 keeps 10 KB per wave in flight).
template <int EPI, int MR, int NCH>
__global__ __launch_bounds__(256) void k_gemv_nc(ProjArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int n = blockIdx.x * 4 + wid; n < a.N; n += gridDim.x * 4) {
    const f16* w = a.B + (size_t)n * a.ldb + lane * 8;
    f16x8 wv[NCH], xv[MR][NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) wv[c] = *(const f16x8*)(w + c * 512);
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c) xv[r][c] = *(const f16x8*)(a.A + (size_t)r * a.lda + c * 512 + lane * 8);
    float acc[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      acc[r] = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc[r] = dot8(wv[c], xv[r][c], acc[r]);
    }
    gemv_store<EPI, MR>(a, acc, lane, n);
  }
}

// General GEMV (optional LN prologue through LDS for 2 < M <= 8).
template <int EPI, int MR, bool LN>
__global__ __launch_bounds__(256) void k_gemv(ProjArgs a) {
  extern __shared__ __attribute__((aligned(16))) f16 xs[];   // [MR][K] when LN
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if constexpr (LN) {
    for (int r = wid; r < a.M; r += 4) {
      f16x8 t[3];
      ln_row_regs<3>(a, r, lane, t);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int k = c * 512 + lane * 8;
        if (k < a.K) *(f16x8*)(xs + r * a.K + k) = t[c];
      }
    }
    __syncthreads();
  }
  for (int n = blockIdx.x * 4 + wid; n < a.N; n += gridDim.x * 4) {
    const f16* w = a.B + (size_t)n * a.ldb;
    float acc[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) acc[r] = 0.f;
#pragma unroll 4
    for (int k = lane * 8; k < a.K; k += 512) {
      const f16x8 wv = *(const f16x8*)(w + k);
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        if (r < a.M) {
          const f16x8 xv = LN ? *(const f16x8*)(xs + r * a.K + k) : *(const f16x8*)(a.A + (size_t)r * a.lda + k);
          acc[r] = dot8(wv, xv, acc[r]);
        }
      }
    }
    gemv_store<EPI, MR>(a, acc, lane, n);
  }
}

// ---------------------------------------------------------------- skinny MFMA GEMM (8 < M <= 64)
// Prompt prefill / DTW re-forward rows.  A workgroup owns 16*NT output columns for ALL rows;
// its 4 waves split K (interleaved 32-wide steps), stream the weight fragments straight from
// HBM into v_mfma_f32_16x16x32_f16 (B operand = 16 contiguous bytes of one weight row per
// lane) and reduce through LDS.  N/16 workgroups instead of N/128 keep every CU streaming.
template <int EPI, int MT, int NT>
__global__ __launch_bounds__(256) void k_skinny(ProjArgs a) {
  __shared__ float red[4][MT][NT][4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16 * NT;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const f16* arow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int m = i * 16 + fr;
    m = m < a.M ? m : a.M - 1;
    arow[i] = a.A + (size_t)m * a.lda + fk;
  }
  const f16* brow[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    int n = n0 + j * 16 + fr;
    n = n < a.N ? n : a.N - 1;
    brow[j] = a.B + (size_t)n * a.ldb + fk;
  }
  for (int k = wid * 32; k < a.K; k += 128) {
    f16x8 bf[NT], af[MT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bf[j] = *(const f16x8*)(brow[j] + k);
#pragma unroll
    for (int i = 0; i < MT; ++i) af[i] = *(const f16x8*)(arow[i] + k);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wid][i][j][r][lane] = acc[i][j][r];
  __syncthreads();
  for (int e = threadIdx.x; e < MT * NT * 4 * 64; e += 256) {
    const int l = e & 63, r = (e >> 6) & 3, j = (e >> 8) % NT, i = (e >> 8) / NT;
    const float v = red[0][i][j][r][l] + red[1][i][j][r][l] + red[2][i][j][r][l] + red[3][i][j][r][l];
    const int row = i * 16 + (l >> 4) * 4 + r, col = n0 + j * 16 + (l & 15);
    epi_store<EPI>(a, row, col, v);
  }
}

template <int EPI>
static void launch_epi(const ProjArgs& a, hipStream_t s) {
  const int ob = (EPI == EPI_F32_RESID || EPI == EPI_F32 || EPI == EPI_F32_GELU_POS) ? 4 : 2;
  const double bytes = (double)a.N * a.K * 2 + (double)a.M * a.K * 2 + (double)a.M * a.N * ob;
  const double flops = 2.0 * a.M * a.N * a.K;
  if (a.M <= 8) {
    const int nwg = std::min(cdiv(a.N, 4), 1024);
    dim3 grid(nwg), blk(256);
    const bool ln = a.ln_x != nullptr;
    if (ln && a.M <= 2 && a.K <= 1536) {
      const int nch = cdiv(a.K, 512);
#define WDR_GLN(MR, NCH) wdr_launch(PROF_GEMV, bytes, flops, k_gemv_ln<EPI, MR, NCH>, grid, blk, 0, s, a);
      if (a.M == 1) {
        if (nch == 1) { WDR_GLN(1, 1) } else if (nch == 2) { WDR_GLN(1, 2) } else { WDR_GLN(1, 3) }
      } else {
        if (nch == 1) { WDR_GLN(2, 1) } else if (nch == 2) { WDR_GLN(2, 2) } else { WDR_GLN(2, 3) }
      }
#undef WDR_GLN
    } else if (!ln && a.M <= 2 && a.K % 512 == 0 && a.K <= 5120) {
      const int nch = a.K / 512;
#define WDR_GNC(MR, NCH) wdr_launch(PROF_GEMV, bytes, flops, k_gemv_nc<EPI, MR, NCH>, grid, blk, 0, s, a);
#define WDR_GNC_M(MR)                                                          \
  switch (nch) {                                                               \
    case 1: WDR_GNC(MR, 1) break;                                              \
    case 2: WDR_GNC(MR, 2) break;                                              \
    case 3: WDR_GNC(MR, 3) break;                                              \
    case 4: WDR_GNC(MR, 4) break;                                              \
    case 6: WDR_GNC(MR, 6) break;                                              \
    case 8: WDR_GNC(MR, 8) break;                                              \
    case 10: WDR_GNC(MR, 10) break;                                            \
    default: wdr_launch(PROF_GEMV, bytes, flops, k_gemv<EPI, MR, false>, grid, blk, 0, s, a); \
  }
      if (a.M == 1) { WDR_GNC_M(1) } else { WDR_GNC_M(2) }
#undef WDR_GNC_M
#undef WDR_GNC
    } else {
      const uint32_t lds = ln ? (uint32_t)a.M * a.K * 2 : 0;
#define WDR_GEMV(MR)                                                                          \
  if (ln) wdr_launch(PROF_GEMV, bytes, flops, k_gemv<EPI, MR, true>, grid, blk, lds, s, a);  \
  else wdr_launch(PROF_GEMV, bytes, flops, k_gemv<EPI, MR, false>, grid, blk, 0, s, a);
      if (a.M <= 1) { WDR_GEMV(1) }
      else if (a.M <= 2) { WDR_GEMV(2) }
      else if (a.M <= 4) { WDR_GEMV(4) }
      else { WDR_GEMV(8) }
#undef WDR_GEMV
    }
  } else if (a.M <= 64) {
    const bool wide = a.N >= 4096;
    dim3 grid(cdiv(a.N, wide ? 32 : 16)), blk(256);
    const int mt = cdiv(a.M, 16);
#define WDR_SK(MTV)                                                                            \
  if (wide) wdr_launch(PROF_SKINNY, bytes, flops, k_skinny<EPI, MTV, 2>, grid, blk, 0, s, a);  \
  else wdr_launch(PROF_SKINNY, bytes, flops, k_skinny<EPI, MTV, 1>, grid, blk, 0, s, a);
    if (mt == 1) { WDR_SK(1) }
    else if (mt == 2) { WDR_SK(2) }
    else if (mt == 3) { WDR_SK(3) }
    else { WDR_SK(4) }
#undef WDR_SK
  } else {
    dim3 grid(a.N / GB_N, cdiv(a.M, GB_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm<EPI>, grid, dim3(256), 0, s, a);
  }
}

void launch_proj(const ProjArgs& a, hipStream_t s) {
  WDR_CHECK(a.M > 0 && a.K > 0 && a.N > 0, "projection: empty shape");
  WDR_CHECK(a.K % 8 == 0 && a.lda % 8 == 0 && a.ldb % 8 == 0, "projection: K/lda/ldb must be multiples of 8");
  if (a.M > 64) {
    WDR_CHECK(a.N % GB_N == 0, "gemm: N must be a multiple of 128");
    WDR_CHECK(a.K % GB_K == 0, "gemm: K must be a multiple of 32");
  } else if (a.M > 8) {
    WDR_CHECK(a.K % 32 == 0, "skinny gemm: K must be a multiple of 32");
  } else if (a.ln_x) {
    WDR_CHECK(a.K <= 1536 && a.K % 8 == 0, "gemv LN prologue: K must be <= 1536");
  }
  WDR_CHECK(a.epi != EPI_QKV_CACHE || (a.kc && a.vc && a.row_seq && a.row_pos && a.d > 0), "qkv-cache epilogue args");
  switch (a.epi) {
    case EPI_F16: launch_epi<EPI_F16>(a, s); break;
    case EPI_F16_GELU: launch_epi<EPI_F16_GELU>(a, s); break;
    case EPI_F32_RESID: launch_epi<EPI_F32_RESID>(a, s); break;
    case EPI_F32: launch_epi<EPI_F32>(a, s); break;
    case EPI_F32_GELU_POS: launch_epi<EPI_F32_GELU_POS>(a, s); break;
    case EPI_QKV_CACHE: launch_epi<EPI_QKV_CACHE>(a, s); break;
    default: throw std::runtime_error("projection: bad epilogue");
  }
  WDR_HIP(hipGetLastError());
}

}  // namespace wdr
