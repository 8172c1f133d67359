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
  } else {  // EPI_F32_GELU_POS
    ((float*)a.out)[(size_t)row * a.ldo + col] =
        gelu_tanh(v) + a.pos[(size_t)(row % a.pos_rows) * a.N + col];
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
template <int EPI, int MR>
__global__ __launch_bounds__(256) void k_gemv(ProjArgs a) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= a.N) return;
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
        const f16x8 xv = *(const f16x8*)(a.A + (size_t)r * a.lda + k);
        float s = acc[r];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f16x2 wp = {wv[2 * q], wv[2 * q + 1]};
          f16x2 xp = {xv[2 * q], xv[2 * q + 1]};
          s = __builtin_amdgcn_fdot2(wp, xp, s, false);
        }
        acc[r] = s;
      }
    }
  }
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

template <int EPI>
static void launch_epi(const ProjArgs& a, hipStream_t s) {
  if (a.M <= 8) {
    dim3 grid(cdiv(a.N, 4));
    if (a.M <= 1)
      hipLaunchKernelGGL((k_gemv<EPI, 1>), grid, dim3(256), 0, s, a);
    else if (a.M <= 2)
      hipLaunchKernelGGL((k_gemv<EPI, 2>), grid, dim3(256), 0, s, a);
    else if (a.M <= 4)
      hipLaunchKernelGGL((k_gemv<EPI, 4>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((k_gemv<EPI, 8>), grid, dim3(256), 0, s, a);
  } else {
    dim3 grid(a.N / GB_N, cdiv(a.M, GB_M));
    hipLaunchKernelGGL((k_gemm<EPI>), grid, dim3(256), 0, s, a);
  }
}

void launch_proj(const ProjArgs& a, hipStream_t s) {
  WDR_CHECK(a.M > 0 && a.K > 0 && a.N > 0, "projection: empty shape");
  WDR_CHECK(a.K % 8 == 0 && a.lda % 8 == 0 && a.ldb % 8 == 0, "projection: K/lda/ldb must be multiples of 8");
  if (a.M > 8) {
    WDR_CHECK(a.N % GB_N == 0, "gemm: N must be a multiple of 128");
    WDR_CHECK(a.K % GB_K == 0, "gemm: K must be a multiple of 32");
  }
  switch (a.epi) {
    case EPI_F16: launch_epi<EPI_F16>(a, s); break;
    case EPI_F16_GELU: launch_epi<EPI_F16_GELU>(a, s); break;
    case EPI_F32_RESID: launch_epi<EPI_F32_RESID>(a, s); break;
    case EPI_F32: launch_epi<EPI_F32>(a, s); break;
    case EPI_F32_GELU_POS: launch_epi<EPI_F32_GELU_POS>(a, s); break;
    default: throw std::runtime_error("projection: bad epilogue");
  }
  WDR_HIP(hipGetLastError());
}

}  // namespace wdr
