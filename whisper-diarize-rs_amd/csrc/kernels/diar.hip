// Diarization kernels: pyannote segmentation-3.0, Kaldi fbank,
// CAM++.  Mirrors oracle/diarize.py.  Both models run in f32 (the reference runs them in
// ONNX Runtime f32 on the CPU), so the contractions use an f32 LDS-tiled GEMM rather than
// the f16 MFMA path: the argmax of the 7 powerset classes and the cosine thresholds of the
// speaker search are what parity is judged on.
//
// Activations are time-major [T][C] (row = frame) so a 1x1 conv is a plain GEMM, a k-tap
// conv is a GEMM over an im2col of neighbouring rows, and the CAM dense blocks append their
// 32 new channels as a column range of one [T][C_max] buffer (the concat costs nothing).
//
//  k_gemm32        C = act(affine(A' . B^T) [+ C]), A' = optional per-column affine+ReLU of A
//                  (the BN-ReLU that precedes every CAM linear), 64x64x16 tiles, 4x4 per thread.
//  k_im2col_1d     k-tap / strided / dilated conv rows over [T][C] (c-major taps as torch).
//  k_im2col_2d     3x3 (or 1x1) conv over [T][F][C] with a frequency stride (FCM front-end).
//  k_maxpool3 / k_inorm   maxpool-3, InstanceNorm(affine) + LeakyReLU (SincNet; double sums).
//  k_lstm_scan     one workgroup per (window, direction): the 4 gate rows of a hidden unit in
//                  registers (f32, 4 threads per unit), h in LDS, one barrier per step.
//  k_logsoftmax7   log-softmax over 7 classes + pyannote-rs find_max_index (last max).
//  k_fbank         Kaldi fbank frame: DC removal, pre-emphasis, Povey, 512-pt power, mel, log.
//  k_colstats      per-utterance mean subtraction (CMN); stats pooling (mean, unbiased std).
//  k_cam_context   CAM context rows: global mean + 100-frame segment means.
//  k_cam_gate      out = y * m[segment] into the dense block's column range.
#include <atomic>

#include "../common.h"
#include "kernels.h"
#include "../prof.h"

namespace wdr {

__device__ __forceinline__ float act_apply(float v, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_LRELU: return v >= 0.f ? v : v * 0.01f;
    case ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
    case ACT_ABS: return fabsf(v);
    default: return v;
  }
}

// ---------------------------------------------------------------- f32 GEMM
constexpr int G_BM = 64, G_BN = 64, G_BK = 16;

__global__ __launch_bounds__(256) void k_gemm32(Gemm32Args a) {
  __shared__ float As[G_BK][G_BM + 4];
  __shared__ float Bs[G_BK][G_BN + 4];
  const int tid = threadIdx.x;
  const int m0 = blockIdx.y * G_BM, n0 = blockIdx.x * G_BN;
  const int tm = (tid >> 4) * 4, tn = (tid & 15) * 4;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < a.K; k0 += G_BK) {
    // 64 x 16 tiles: each thread loads 4 elements of A and 4 of B
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + r * 256;
      const int row = e >> 4, kk = e & 15;
      const int gk = k0 + kk;
      float va = 0.f, vb = 0.f;
      if (m0 + row < a.M && gk < a.K) {
        va = a.A[(long long)(m0 + row) * a.lda + gk];
        if (a.pro_scale) va = fmaxf(va * a.pro_scale[gk] + a.pro_shift[gk], 0.f);
      }
      if (n0 + row < a.N && gk < a.K) vb = a.B[(long long)(n0 + row) * a.ldb + gk];
      As[kk][row] = va;
      Bs[kk][row] = vb;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < G_BK; ++kk) {
      const float4 av = *reinterpret_cast<const float4*>(&As[kk][tm]);
      const float4 bv = *reinterpret_cast<const float4*>(&Bs[kk][tn]);
      const float ar[4] = {av.x, av.y, av.z, av.w}, br[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += ar[i] * br[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + tm + i;
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tn + j;
      if (n >= a.N) continue;
      float v = acc[i][j];
      if (a.bias) v += a.bias[n];
      if (a.scale) v = v * a.scale[n] + a.shift[n];
      float* c = a.C + (long long)m * a.ldc + n;
      if (a.accum) v += *c;
      *c = act_apply(v, a.act);
    }
  }
}

// ---------------------------------------------------------------- f32 MFMA GEMM
// The same contraction on the matrix cores: v_mfma_f32_32x32x2_f32 (exact f32 products, one
// fma per k in k order -- the arithmetic of k_gemm32's per-thread fma chain), 4 waves of 32 x 32
// output tiles arranged WM x WN (64 x 64, or 128 x 32 for narrow N), BK 16 k-major LDS tiles
// with the next tile's loads in flight (registers) during the current tile's MFMAs.
template <int WM, int WN>
__global__ __launch_bounds__(256) void k_gemm32m(Gemm32Args a) {
  constexpr int BM = 32 * WM, BN = 32 * WN, BK = 16;
  constexpr int LA = BM * BK / 256, LB = BN * BK / 256;   // elements staged per thread
  __shared__ float As[BK][BM + 4];
  __shared__ float Bs[BK][BN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  float ra[LA], rb[LB];
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < LA; ++r) {
      const int e = tid + r * 256, row = e >> 4, kk = e & 15, gk = k0 + kk;
      float va = 0.f;
      if (m0 + row < a.M && gk < a.K) {
        va = a.A[(long long)(m0 + row) * a.lda + gk];
        if (a.pro_scale) va = fmaxf(va * a.pro_scale[gk] + a.pro_shift[gk], 0.f);
      }
      ra[r] = va;
    }
#pragma unroll
    for (int r = 0; r < LB; ++r) {
      const int e = tid + r * 256, row = e >> 4, kk = e & 15, gk = k0 + kk;
      rb[r] = (n0 + row < a.N && gk < a.K) ? a.B[(long long)(n0 + row) * a.ldb + gk] : 0.f;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int r = 0; r < LA; ++r) {
      const int e = tid + r * 256;
      As[e & 15][e >> 4] = ra[r];
    }
#pragma unroll
    for (int r = 0; r < LB; ++r) {
      const int e = tid + r * 256;
      Bs[e & 15][e >> 4] = rb[r];
    }
  };
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  load(0);
  const int fi = lane & 31, fk = lane >> 5;
  for (int k0 = 0; k0 < a.K; k0 += BK) {
    store();
    __syncthreads();
    if (k0 + BK < a.K) load(k0 + BK);   // next tile's loads overlap this tile's MFMAs
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[kk + fk][wr * 32 + fi], Bs[kk + fk][wc * 32 + fi], acc, 0, 0, 0);
    __syncthreads();
  }
  const int n = n0 + wc * 32 + fi;
  if (n >= a.N) return;
  const float bias = a.bias ? a.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * fk;
    if (m >= a.M) continue;
    float v = acc[r];
    if (a.bias) v += bias;
    if (a.scale) v = v * a.scale[n] + a.shift[n];
    float* c = a.C + (long long)m * a.ldc + n;
    if (a.accum) v += *c;
    *c = act_apply(v, a.act);
  }
}

// the f32 MFMA kernel (default) or the VALU one: WDR_GEMM32=0 at load, or wdr_dbg_set_gemm32
// (tests/test_gpu_diarize.py compares both within one process)
static std::atomic<int> g_gemm32_mfma{[] {
  const char* e = getenv("WDR_GEMM32");
  return e && atoi(e) == 0 ? 0 : 1;
}()};
void set_gemm32_mfma(bool on) { g_gemm32_mfma.store(on ? 1 : 0); }
static bool gemm32_mfma() { return g_gemm32_mfma.load(std::memory_order_relaxed) != 0; }

void launch_gemm32(const Gemm32Args& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return;
  if (gemm32_mfma()) {
    // 128 x 32 tiles where they waste fewer columns than 64 x 64 (N = 7, 32, 80), else 64 x 64
    const int w64 = cdiv(a.N, 64) * 64 - a.N, w32 = cdiv(a.N, 32) * 32 - a.N;
    if (w32 < w64 || a.N <= 32) {
      WDR_CHECK(cdiv(a.M, 128) <= 65535, "gemm32: too many row tiles");
      WDR_KLAUNCH((k_gemm32m<4, 1>), dim3(cdiv(a.N, 32), cdiv(a.M, 128)), dim3(256), 0, s, a);
    } else {
      WDR_CHECK(cdiv(a.M, 64) <= 65535, "gemm32: too many row tiles");
      WDR_KLAUNCH((k_gemm32m<2, 2>), dim3(cdiv(a.N, 64), cdiv(a.M, 64)), dim3(256), 0, s, a);
    }
  } else {
    WDR_CHECK(cdiv(a.M, G_BM) <= 65535, "gemm32: too many row tiles");
    WDR_KLAUNCH(k_gemm32, dim3(cdiv(a.N, G_BN), cdiv(a.M, G_BM)), dim3(256), 0, s, a);
  }
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- im2col
// col[t][c*k + j] = X[t*stride + j*dil - pad][c]  (zero outside [0, T))
__global__ void k_im2col_1d(const float* X, int ldx, int T, int C, int k, int stride, int dil, int pad, int To,
                            float* col) {
  const long long total = (long long)To * C * k;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / (C * k));
    const int r = (int)(i - (long long)t * C * k);
    const int c = r / k, j = r - c * k;
    const int u = t * stride + j * dil - pad;
    col[i] = (u >= 0 && u < T) ? X[(long long)u * ldx + c] : 0.f;
  }
}

void launch_im2col_1d(const float* X, int ldx, int T, int C, int k, int stride, int dil, int pad, int To, float* col,
                      hipStream_t s) {
  const long long total = (long long)To * C * k;
  if (total <= 0) return;
  const int grid = (int)std::min<long long>(cdiv((int)std::min<long long>(total, 1ll << 30), 256), 8192);
  WDR_KLAUNCH(k_im2col_1d, dim3(grid), dim3(256), 0, s, X, ldx, T, C, k, stride, dil, pad, To, col);
  WDR_HIP(hipGetLastError());
}

// X [T][F][C] -> col [(t*Fo + f)][c*kf*kt + a*kt + b] = X[t + b - pt][f*sf + a - pf][c]
__global__ void k_im2col_2d(const float* X, int T, int F, int C, int kf, int kt, int sf, int Fo, float* col) {
  const int pf = (kf - 1) / 2, pt = (kt - 1) / 2;
  const int K = C * kf * kt;
  const long long total = (long long)T * Fo * K;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / K;
    const int r = (int)(i - row * K);
    const int t = (int)(row / Fo), f = (int)(row - (long long)t * Fo);
    const int c = r / (kf * kt), q = r - c * kf * kt;
    const int aa = q / kt, bb = q - aa * kt;
    const int tt = t + bb - pt, ff = f * sf + aa - pf;
    col[i] = (tt >= 0 && tt < T && ff >= 0 && ff < F) ? X[((long long)tt * F + ff) * C + c] : 0.f;
  }
}

void launch_im2col_2d(const float* X, int T, int F, int C, int kf, int kt, int sf, int Fo, float* col, hipStream_t s) {
  const long long total = (long long)T * Fo * C * kf * kt;
  if (total <= 0) return;
  const int grid = (int)std::min<long long>((total + 255) / 256, 8192);
  WDR_KLAUNCH(k_im2col_2d, dim3(grid), dim3(256), 0, s, X, T, F, C, kf, kt, sf, Fo, col);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- SincNet pool + InstanceNorm
// x [B][T][C] (batch stride bs) -> maxpool 3 over T -> y [B][To][C]; then per (b, c) mean/var
// over To (double sums) -> y = lrelu((y - m) / sqrt(v + eps) * g + beta)
__global__ void k_maxpool3(const float* x, long long bs, int T, int C, float* y, long long ybs) {
  const int To = T / 3;
  const int b = blockIdx.y;
  const long long total = (long long)To * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / C), c = (int)(i - (long long)t * C);
    const float* p = x + b * bs + (long long)(3 * t) * C + c;
    y[b * ybs + i] = fmaxf(fmaxf(p[0], p[C]), p[2 * C]);
  }
}

__global__ __launch_bounds__(256) void k_inorm(float* y, long long bs, int T, int C, const float* g, const float* beta,
                                               int act) {
  const int c = blockIdx.x, b = blockIdx.y;
  float* p = y + b * bs + c;
  double s = 0.0;
  for (int t = threadIdx.x; t < T; t += 256) s += p[(long long)t * C];
  __shared__ double red[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / T;
  __syncthreads();
  double v = 0.0;
  for (int t = threadIdx.x; t < T; t += 256) {
    const double d = p[(long long)t * C] - mean;
    v += d * d;
  }
  v = wave_sum_d(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double var = (red[0] + red[1] + red[2] + red[3]) / T;
  const double inv = 1.0 / sqrt(var + 1e-5);
  const float gg = g[c], bb = beta[c];
  for (int t = threadIdx.x; t < T; t += 256) {
    const float val = (float)(((double)p[(long long)t * C] - mean) * inv) * gg + bb;
    p[(long long)t * C] = act_apply(val, act);
  }
}

void launch_maxpool3(const float* x, long long bs, int T, int C, int B, float* y, long long ybs, hipStream_t s) {
  const long long total = (long long)(T / 3) * C;
  if (total <= 0 || B <= 0) return;
  WDR_KLAUNCH(k_maxpool3, dim3((unsigned)std::min<long long>((total + 255) / 256, 2048), B), dim3(256), 0, s, x,
                     bs, T, C, y, ybs);
  WDR_HIP(hipGetLastError());
}

void launch_inorm(float* y, long long bs, int T, int C, int B, const float* g, const float* beta, int act,
                  hipStream_t s) {
  if (B <= 0 || C <= 0) return;
  WDR_KLAUNCH(k_inorm, dim3(C, B), dim3(256), 0, s, y, bs, T, C, g, beta, act);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- LSTM scan
// xg [B][T][ldxg] holds W_ih x + b_ih for both directions (dir d at column offset d*512);
// out [B][T][ldo] receives h of direction d at column offset d*128.  whh/bhh [2][512][128]/[2][512].
constexpr int kLP = 4;   // threads per hidden unit (each holds 32 of the 128 W_hh columns)

__global__ __launch_bounds__(512) void k_lstm_scan(const float* __restrict__ xg, long long xbs, int ldxg, int T,
                                                   const float* __restrict__ whh, const float* __restrict__ bhh,
                                                   float* __restrict__ out, long long obs, int ldo) {
  __shared__ float hs[2][128];
  const int b = blockIdx.x, dir = blockIdx.y;
  const int tid = threadIdx.x, u = tid / kLP, part = tid % kLP;
  constexpr int KC = 128 / kLP;
  const float* W = whh + (size_t)dir * 512 * 128;
  float4 w[4][KC / 4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int q = 0; q < KC / 4; ++q)
      w[g][q] = reinterpret_cast<const float4*>(W + (size_t)(g * 128 + u) * 128 + part * KC)[q];
  float bh[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bh[g] = bhh[dir * 512 + g * 128 + u];
  if (tid < 128) hs[0][tid] = 0.f;
  float c = 0.f;
  const float* xb = xg + b * xbs + dir * 512;
  float* ob = out + b * obs + dir * 128;
  // W_ih x + b_ih of the next kLPF steps in flight (registers), one LDS-only barrier per step:
  // the arithmetic of every step is unchanged (round 6: a one-step lookahead behind
  // __syncthreads waited for each step's load)
  constexpr int kLPF = 8;
  float pf[kLPF][4];
#pragma unroll
  for (int q = 0; q < kLPF; ++q) {
    const int tq = dir ? T - 1 - q : q;
#pragma unroll
    for (int g = 0; g < 4; ++g) pf[q][g] = q < T ? xb[(long long)tq * ldxg + g * 128 + u] : 0.f;
  }
  __syncthreads();
  for (int s0 = 0; s0 < T; s0 += kLPF) {
#pragma unroll
    for (int q = 0; q < kLPF; ++q) {
      const int s = s0 + q;
      if (s >= T) break;
      const int t = dir ? T - 1 - s : s;
      float cur[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) cur[g] = pf[q][g];
      if (s + kLPF < T) {
        const int tn = dir ? t - kLPF : t + kLPF;
#pragma unroll
        for (int g = 0; g < 4; ++g) pf[q][g] = xb[(long long)tn * ldxg + g * 128 + u];
      }
      const float* h = hs[s & 1] + part * KC;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int qq = 0; qq < KC / 4; ++qq) {
        const float4 hv = *reinterpret_cast<const float4*>(h + qq * 4);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          acc[g] += w[g][qq].x * hv.x + w[g][qq].y * hv.y + w[g][qq].z * hv.z + w[g][qq].w * hv.w;
      }
      float pre[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        acc[g] += __shfl_xor(acc[g], 1, 64);
        acc[g] += __shfl_xor(acc[g], 2, 64);
        pre[g] = cur[g] + (acc[g] + bh[g]);
      }
      const float ig = 1.f / (1.f + expf(-pre[0])), fg = 1.f / (1.f + expf(-pre[1]));
      const float gg = tanhf(pre[2]), og = 1.f / (1.f + expf(-pre[3]));
      c = fg * c + ig * gg;
      const float hn = og * tanhf(c);
      if (part == 0) {
        hs[(s + 1) & 1][u] = hn;
        ob[(long long)t * ldo + u] = hn;
      }
      lds_barrier();
    }
  }
}

void launch_lstm_scan(const float* xg, long long xbs, int ldxg, int T, int B, const float* whh, const float* bhh,
                      float* out, long long obs, int ldo, hipStream_t s) {
  if (B <= 0) return;
  WDR_KLAUNCH(k_lstm_scan, dim3(B, 2), dim3(128 * kLP), 0, s, xg, xbs, ldxg, T, whh, bhh, out, obs, ldo);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- classifier output
__global__ void k_logsoftmax7(float* z, int rows, int* cls) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float* p = z + (long long)r * 7;
  float m = p[0];
  int bi = 0;
  for (int i = 1; i < 7; ++i) {
    m = fmaxf(m, p[i]);
  }
  float s = 0.f;
  for (int i = 0; i < 7; ++i) s += expf(p[i] - m);
  const float ls = logf(s);
  float best = 0.f;
  for (int i = 0; i < 7; ++i) {
    const float v = p[i] - m - ls;
    p[i] = v;
    if (i == 0 || !(v < best)) {   // Iterator::max_by: the last maximal element wins
      best = v;
      bi = i;
    }
  }
  cls[r] = bi;
}

void launch_logsoftmax7(float* z, int rows, int* cls, hipStream_t s) {
  if (rows <= 0) return;
  WDR_KLAUNCH(k_logsoftmax7, dim3(cdiv(rows, 256)), dim3(256), 0, s, z, rows, cls);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- Kaldi fbank
// one workgroup (256 threads) per frame; tables: povey [400], cos/sin [512] (2 pi j / 512),
// banks [80][256] dense.
__global__ __launch_bounds__(256) void k_fbank(const float* x, int T, const float* povey, const float* cos_t,
                                               const float* sin_t, const float* banks, float* out) {
  __shared__ float fr[512];
  __shared__ float pw[256];
  __shared__ float cs[512], sn[512];   // the twiddles in LDS: the DFT's 400 dependent-index reads
  __shared__ double red[4];
  const int t = blockIdx.x, tid = threadIdx.x;
  const float* src = x + (long long)t * 160;
  for (int i = tid; i < 512; i += 256) {
    cs[i] = cos_t[i];
    sn[i] = sin_t[i];
  }
  double s = 0.0;
  for (int i = tid; i < 400; i += 256) s += src[i];
  s = wave_sum_d(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  const float mean = (float)((red[0] + red[1] + red[2] + red[3]) / 400.0);
  // DC removal, pre-emphasis (x[i] - 0.97 x[i-1], x[0] - 0.97 x[0]), Povey window
  for (int i = tid; i < 512; i += 256) {
    float v = 0.f;
    if (i < 400) {
      const float cur = src[i] - mean;
      const float prev = i > 0 ? src[i - 1] - mean : cur;
      v = (cur - 0.97f * prev) * povey[i];
    }
    fr[i] = v;
  }
  __syncthreads();
  // power spectrum bins 0..255 (the Nyquist bin is not used by the mel banks)
  {
    const int kb = tid;
    float re = 0.f, im = 0.f;
    int idx = 0;
    for (int j = 0; j < 400; ++j) {
      const float v = fr[j];
      re += v * cs[idx];
      im -= v * sn[idx];
      idx = (idx + kb) & 511;
    }
    pw[kb] = re * re + im * im;
  }
  __syncthreads();
  if (tid < 80) {
    const float* bk = banks + tid * 256;
    float e = 0.f;
    for (int i = 0; i < 256; ++i) e += bk[i] * pw[i];
    out[(long long)t * 80 + tid] = logf(fmaxf(e, 1.1920928955078125e-07f));
  }
}

void launch_fbank(const float* x, int T, const float* povey, const float* cos_t, const float* sin_t, const float* banks,
                  float* out, hipStream_t s) {
  if (T <= 0) return;
  WDR_KLAUNCH(k_fbank, dim3(T), dim3(256), 0, s, x, T, povey, cos_t, sin_t, banks, out);
  WDR_HIP(hipGetLastError());
}

// column statistics over T rows of [T][C] (ld): mode 0 -> subtract the mean in place (CMN);
// mode 1 -> stats pooling: out[c] = mean, out[C + c] = unbiased std (NaN when T == 1)
__global__ __launch_bounds__(256) void k_colstats(float* x, int ld, int T, int C, int mode, float* out) {
  const int c = blockIdx.x;
  __shared__ double red[4];
  double s = 0.0;
  for (int t = threadIdx.x; t < T; t += 256) s += x[(long long)t * ld + c];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / T;
  if (mode == 0) {
    const float mf = (float)mean;
    for (int t = threadIdx.x; t < T; t += 256) x[(long long)t * ld + c] -= mf;
    return;
  }
  __syncthreads();
  double v = 0.0;
  for (int t = threadIdx.x; t < T; t += 256) {
    const double d = x[(long long)t * ld + c] - mean;
    v += d * d;
  }
  v = wave_sum_d(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[c] = (float)mean;
    out[C + c] = T > 1 ? (float)sqrt((red[0] + red[1] + red[2] + red[3]) / (T - 1)) : __builtin_nanf("");
  }
}

void launch_colstats(float* x, int ld, int T, int C, int mode, float* out, hipStream_t s) {
  if (T <= 0 || C <= 0) return;
  WDR_KLAUNCH(k_colstats, dim3(C), dim3(256), 0, s, x, ld, T, C, mode, out);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- CAM layer helpers
// ctx rows: out[s][c] = mean_t h[t][c] + mean_{t in segment s} h[t][c]   (nseg = ceil(T/100))
__global__ __launch_bounds__(256) void k_cam_context(const float* h, int ldh, int T, int C, float* out) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  double tot = 0.0;
  for (int t = lane; t < T; t += 64) tot += h[(long long)t * ldh + c];
  tot = wave_sum_d(tot);
  const float gm = (float)(tot / T);
  const int nseg = (T + 99) / 100;
  for (int sgi = 0; sgi < nseg; ++sgi) {
    const int t0 = sgi * 100, t1 = min(T, t0 + 100);
    double s = 0.0;
    for (int t = t0 + lane; t < t1; t += 64) s += h[(long long)t * ldh + c];
    s = wave_sum_d(s);
    if (lane == 0) out[(long long)sgi * C + c] = gm + (float)(s / (t1 - t0));
  }
}

__global__ void k_cam_gate(const float* y, int ldy, const float* m, int T, int G, float* out, int ldo) {
  const long long total = (long long)T * G;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / G), j = (int)(i - (long long)t * G);
    out[(long long)t * ldo + j] = y[(long long)t * ldy + j] * m[(long long)(t / 100) * G + j];
  }
}

void launch_cam_context(const float* h, int ldh, int T, int C, float* out, hipStream_t s) {
  if (T <= 0) return;
  WDR_KLAUNCH(k_cam_context, dim3(cdiv(C, 4)), dim3(256), 0, s, h, ldh, T, C, out);
  WDR_HIP(hipGetLastError());
}

void launch_cam_gate(const float* y, int ldy, const float* m, int T, int G, float* out, int ldo, hipStream_t s) {
  const long long total = (long long)T * G;
  if (total <= 0) return;
  WDR_KLAUNCH(k_cam_gate, dim3((unsigned)std::min<long long>((total + 255) / 256, 4096)), dim3(256), 0, s, y, ldy,
                     m, T, G, out, ldo);
  WDR_HIP(hipGetLastError());
}


// ---------------------------------------------------------------- batched CAM++ (several utterances)
// Utterance b's rows are [off[b], off[b] + len[b]) of a concatenated [rows][...] buffer (CamModel
// embed_batch).  Each kernel below does, per utterance, exactly the arithmetic of its
// single-utterance form above, so every embedding is bit-identical to a one-utterance run.
__device__ __forceinline__ int seg_of(const int* off, int B, int r) {
  int lo = 0, hi = B - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= r) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// A block per RB consecutive output rows (t, f): each row's utterance lookup and position once,
// into LDS; the rows' taps are read channel-fastest (C = 32 consecutive floats of one (t, f)
// position: coalesced) into an LDS image of the block's RB * K columns, which is then written as
// one contiguous run of the col buffer, every lane busy.  The wave-per-row form left 55 of 64 lanes
// idle on the 1-channel stem (K = 9), read tap-fastest and split columns by runtime divisions.
// Alone, 16 000 frames (tools/im2col_bench, profiles/r06/im2col_bench.txt): stem 336 -> 25 us,
// 1x1 shortcut 198 -> 50 us, 3x3 blocks 8-15 % faster (1.4-1.9 TB/s written).  The same values in
// the same places as the one-utterance k_im2col_2d (column c * KF * KT + aa * KT + bb).
template <int C, int KF, int KT>
__global__ __launch_bounds__(256) void k_im2col_2d_b(const float* X, SegRows sr, int Ttot, int F, int sf, int Fo,
                                                     float* col) {
  constexpr int KQ = KF * KT, K = C * KQ, RB = K >= 64 ? 32 : 256;
  constexpr int PF = (KF - 1) / 2, PT = (KT - 1) / 2;
  __shared__ int s_t[RB], s_T[RB], s_o[RB], s_f[RB];
  __shared__ float s_col[RB * K];
  const int nrows = Ttot * Fo;
  for (int r0 = blockIdx.x * RB; r0 < nrows; r0 += gridDim.x * RB) {
    for (int rl = threadIdx.x; rl < RB; rl += 256) {
      const int row = r0 + rl;
      if (row < nrows) {
        const int tg = row / Fo;
        const int b = seg_of(sr.off, sr.B, tg);
        s_t[rl] = tg - sr.off[b];
        s_T[rl] = sr.len[b];
        s_o[rl] = sr.off[b];
        s_f[rl] = row - tg * Fo;
      }
    }
    __syncthreads();
    const int n = min(RB, nrows - r0) * K;
    for (int e = threadIdx.x; e < n; e += 256) {   // channel-fastest reads
      const int rl = e / K, r = e - rl * K;
      const int q = r / C, c = r - q * C;
      const int aa = q / KT, bb = q - aa * KT;
      const int tt = s_t[rl] + bb - PT, ff = s_f[rl] * sf + aa - PF;
      s_col[rl * K + c * KQ + q] =
          (tt >= 0 && tt < s_T[rl] && ff >= 0 && ff < F) ? X[((long long)(s_o[rl] + tt) * F + ff) * C + c] : 0.f;
    }
    __syncthreads();
    float* dst = col + (long long)r0 * K;
    for (int e = threadIdx.x; e < n; e += 256) dst[e] = s_col[e];
    __syncthreads();
  }
}

void launch_im2col_2d_b(const float* X, const SegRows& sr, int Ttot, int F, int C, int kf, int kt, int sf, int Fo,
                        float* col, hipStream_t s) {
  const long long rows = (long long)Ttot * Fo;
  if (rows <= 0 || C * kf * kt <= 0) return;
  WDR_CHECK(rows < (1ll << 31) && rows * C * kf * kt < (1ll << 40), "im2col 2d: too many rows");
  auto go = [&](auto kern, int rb) {
    const int grid = (int)std::min<long long>((rows + rb - 1) / rb, 8192);
    WDR_KLAUNCH(kern, dim3(grid), dim3(256), 0, s, X, sr, Ttot, F, sf, Fo, col);
  };
  if (C == 1 && kf == 3 && kt == 3) go(k_im2col_2d_b<1, 3, 3>, 256);
  else if (C == 32 && kf == 3 && kt == 3) go(k_im2col_2d_b<32, 3, 3>, 32);
  else if (C == 32 && kf == 1 && kt == 1) go(k_im2col_2d_b<32, 1, 1>, 256);
  else WDR_CHECK(false, "im2col 2d: shape without an instantiation (CAM++ FCM: C 1 / 32, 3x3 / 1x1)");
  WDR_HIP(hipGetLastError());
}

// col[u][c*k + j] = X[in.off[b] + u_local*stride + j*dil - pad][c] within utterance b's input rows
__global__ __launch_bounds__(256) void k_im2col_1d_b(const float* X, int ldx, SegRows in, SegRows out, int Ttot_out,
                                                     int C, int k, int stride, int dil, int pad, float* col) {
  // one wave per output row, as k_im2col_2d_b
  const int K = C * k;
  const int lane = threadIdx.x & 63;
  for (int tg = blockIdx.x * 4 + (threadIdx.x >> 6); tg < Ttot_out; tg += gridDim.x * 4) {
    const int b = seg_of(out.off, out.B, tg);
    const int t = tg - out.off[b], L = in.len[b], o = in.off[b];
    float* dst = col + (long long)tg * K;
    for (int r = lane; r < K; r += 64) {
      const int c = r / k, j = r - c * k;
      const int u = t * stride + j * dil - pad;
      dst[r] = (u >= 0 && u < L) ? X[(long long)(o + u) * ldx + c] : 0.f;
    }
  }
}

void launch_im2col_1d_b(const float* X, int ldx, const SegRows& in, const SegRows& out, int Ttot_out, int C, int k,
                        int stride, int dil, int pad, float* col, hipStream_t s) {
  if (Ttot_out <= 0 || C * k <= 0) return;
  const int grid = std::min((Ttot_out + 3) / 4, 16384);
  WDR_KLAUNCH(k_im2col_1d_b, dim3(grid), dim3(256), 0, s, X, ldx, in, out, Ttot_out, C, k, stride, dil, pad,
                     col);
  WDR_HIP(hipGetLastError());
}

// k_colstats per utterance (blockIdx.y): CMN in place, or stats pooling into out[b][2C]
__global__ __launch_bounds__(256) void k_colstats_b(float* xall, int ld, SegRows sr, int C, int mode, float* outall) {
  const int c = blockIdx.x, b = blockIdx.y;
  const int T = sr.len[b];
  float* x = xall + (long long)sr.off[b] * ld;
  float* out = outall ? outall + (long long)b * 2 * C : nullptr;
  __shared__ double red[4];
  double s = 0.0;
  for (int t = threadIdx.x; t < T; t += 256) s += x[(long long)t * ld + c];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / T;
  if (mode == 0) {
    const float mf = (float)mean;
    for (int t = threadIdx.x; t < T; t += 256) x[(long long)t * ld + c] -= mf;
    return;
  }
  __syncthreads();
  double v = 0.0;
  for (int t = threadIdx.x; t < T; t += 256) {
    const double d = x[(long long)t * ld + c] - mean;
    v += d * d;
  }
  v = wave_sum_d(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[c] = (float)mean;
    out[C + c] = T > 1 ? (float)sqrt((red[0] + red[1] + red[2] + red[3]) / (T - 1)) : __builtin_nanf("");
  }
}

void launch_colstats_b(float* x, int ld, const SegRows& sr, int C, int mode, float* out, hipStream_t s) {
  if (sr.B <= 0 || C <= 0) return;
  WDR_KLAUNCH(k_colstats_b, dim3(C, sr.B), dim3(256), 0, s, x, ld, sr, C, mode, out);
  WDR_HIP(hipGetLastError());
}

// k_cam_context per utterance (blockIdx.y); its context rows start at ctx_off[b]
__global__ __launch_bounds__(256) void k_cam_context_b(const float* hall, int ldh, SegRows sr, const int* ctx_off, int C,
                                                       float* outall) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, b = blockIdx.y;
  if (c >= C) return;
  const int T = sr.len[b];
  const float* h = hall + (long long)sr.off[b] * ldh;
  float* out = outall + (long long)ctx_off[b] * C;
  double tot = 0.0;
  for (int t = lane; t < T; t += 64) tot += h[(long long)t * ldh + c];
  tot = wave_sum_d(tot);
  const float gm = (float)(tot / T);
  const int nseg = (T + 99) / 100;
  for (int sgi = 0; sgi < nseg; ++sgi) {
    const int t0 = sgi * 100, t1 = min(T, t0 + 100);
    double s = 0.0;
    for (int t = t0 + lane; t < t1; t += 64) s += h[(long long)t * ldh + c];
    s = wave_sum_d(s);
    if (lane == 0) out[(long long)sgi * C + c] = gm + (float)(s / (t1 - t0));
  }
}

void launch_cam_context_b(const float* h, int ldh, const SegRows& sr, const int* ctx_off, int C, float* out,
                          hipStream_t s) {
  if (sr.B <= 0) return;
  WDR_KLAUNCH(k_cam_context_b, dim3(cdiv(C, 4), sr.B), dim3(256), 0, s, h, ldh, sr, ctx_off, C, out);
  WDR_HIP(hipGetLastError());
}

__global__ void k_cam_gate_b(const float* y, int ldy, const float* m, SegRows sr, const int* ctx_off, int Ttot, int G,
                             float* out, int ldo) {
  const long long total = (long long)Ttot * G;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int tg = (int)(i / G), j = (int)(i - (long long)tg * G);
    const int b = seg_of(sr.off, sr.B, tg);
    const int t = tg - sr.off[b];
    out[(long long)tg * ldo + j] = y[(long long)tg * ldy + j] * m[(long long)(ctx_off[b] + t / 100) * G + j];
  }
}

void launch_cam_gate_b(const float* y, int ldy, const float* m, const SegRows& sr, const int* ctx_off, int Ttot, int G,
                       float* out, int ldo, hipStream_t s) {
  const long long total = (long long)Ttot * G;
  if (total <= 0) return;
  WDR_KLAUNCH(k_cam_gate_b, dim3((unsigned)std::min<long long>((total + 255) / 256, 8192)), dim3(256), 0, s, y,
                     ldy, m, sr, ctx_off, Ttot, G, out, ldo);
  WDR_HIP(hipGetLastError());
}
}  // namespace wdr

namespace wdr {

__global__ void k_i16_scale(const int16_t* in, long long n, float scale, float* out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = (float)in[i] * scale;
}

void launch_i16_scale(const int16_t* in, long long n, float scale, float* out, hipStream_t s) {
  if (n <= 0) return;
  WDR_KLAUNCH(k_i16_scale, dim3((unsigned)std::min<long long>((n + 255) / 256, 8192)), dim3(256), 0, s, in, n,
                     scale, out);
  WDR_HIP(hipGetLastError());
}

}  // namespace wdr
