// Silero VAD v5.1.2 forward as whisper.cpp runs it (reference call
// site src/vad.rs:15-31).  Mirrors oracle/vad.py.
//
//  k_vad_front   every 512-sample chunk independently (one workgroup per chunk): reflect pad
//                64|64, STFT-as-conv (258 x 256 basis, hop 128, 4 frames) + magnitude, the four
//                conv+ReLU layers and the LSTM input projection W_ih x + b_ih.  All inputs of a
//                conv / mul_mat are rounded to f16 (ggml im2col is f16), f16 weights, f32 sums.
//                Output xg [chunks][512] f32 -- the only HBM traffic that scales with audio.
//  k_vad_lstm    the recurrence: ONE workgroup scans all chunks (state carried across the
//                file).  Thread pair (2u, 2u+1) owns hidden unit u: each thread holds half of
//                the four W_hh rows of u in registers (4 x 64 f16) and dots them with the
//                f16 hidden state in LDS (double-buffered, one barrier per step); the pair
//                combines with one shuffle and both update (c, h) redundantly.  xg is
//                prefetched kPF steps ahead.  Latency-bound chain: reported in us/step.
//  k_vad_head    p = sigmoid(w_o . f16(relu(h)) + b_o), one wave per chunk.
#include "../common.h"
#include "kernels.h"
#include "../prof.h"

namespace wdr {

__device__ __forceinline__ float r16(float v) { return (float)(f16)v; }

__global__ __launch_bounds__(256) void k_vad_front(const float* __restrict__ x, long long n, VadWeights w,
                                                   float* __restrict__ xg) {
  __shared__ float fr[640];
  __shared__ float mag[129 * 4];
  __shared__ float c0[128 * 4];
  __shared__ float c1[64 * 2];
  __shared__ float c2[64];
  __shared__ float c3[128];
  const int tid = threadIdx.x;
  const long long chunk = blockIdx.x;
  const long long base = chunk * 512;
  for (int i = tid; i < 640; i += 256) {
    int j = i - 64;
    if (j < 0) j = -j;
    if (j >= 512) j = 1022 - j;
    const long long s = base + j;
    fr[i] = r16(s < n ? x[s] : 0.f);
  }
  __syncthreads();
  // STFT magnitude: pair p -> (frame f, bin k); rows k (real) and 129 + k (imag)
  for (int p = tid; p < 516; p += 256) {
    const int f = p / 129, k = p - f * 129;
    const f16x8* br = reinterpret_cast<const f16x8*>(w.stft + (size_t)k * 256);
    const f16x8* bi = reinterpret_cast<const f16x8*>(w.stft + (size_t)(129 + k) * 256);
    const float* xs = fr + 128 * f;
    float re = 0.f, im = 0.f;
#pragma unroll 4
    for (int q = 0; q < 32; ++q) {
      const f16x8 a = br[q], b = bi[q];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = xs[q * 8 + e];
        re += (float)a[e] * v;
        im += (float)b[e] * v;
      }
    }
    mag[k * 4 + f] = r16(sqrtf(re * re + im * im));
  }
  __syncthreads();
  // conv0 129 -> 128, k3 s1 p1, T 4 -> 4
  for (int q = tid; q < 512; q += 256) {
    const int o = q >> 2, t = q & 3;
    const f16* wr = w.c0w + (size_t)o * 387;
    float acc = 0.f;
    for (int c = 0; c < 129; ++c) {
#pragma unroll
      for (int kk = 0; kk < 3; ++kk) {
        const int u = t + kk - 1;
        if (u >= 0 && u < 4) acc += (float)wr[c * 3 + kk] * mag[c * 4 + u];
      }
    }
    c0[o * 4 + t] = r16(fmaxf(acc + w.c0b[o], 0.f));
  }
  __syncthreads();
  // conv1 128 -> 64, k3 s2 p1, T 4 -> 2: two threads per output (channel halves)
  {
    const int q = tid >> 1, part = tid & 1;
    const int o = q >> 1, t = q & 1;
    const f16* wr = w.c1w + (size_t)o * 384;
    float acc = 0.f;
    for (int c = part * 64; c < part * 64 + 64; ++c) {
#pragma unroll
      for (int kk = 0; kk < 3; ++kk) {
        const int u = 2 * t + kk - 1;
        if (u >= 0 && u < 4) acc += (float)wr[c * 3 + kk] * c0[c * 4 + u];
      }
    }
    acc += __shfl_xor(acc, 1, 64);
    if (part == 0) c1[o * 2 + t] = r16(fmaxf(acc + w.c1b[o], 0.f));
  }
  __syncthreads();
  // conv2 64 -> 64, k3 s2 p1, T 2 -> 1: four threads per output
  {
    const int o = tid >> 2, part = tid & 3;
    const f16* wr = w.c2w + (size_t)o * 192;
    float acc = 0.f;
    for (int c = part * 16; c < part * 16 + 16; ++c) {
      acc += (float)wr[c * 3 + 1] * c1[c * 2 + 0];
      acc += (float)wr[c * 3 + 2] * c1[c * 2 + 1];
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if (part == 0) c2[o] = r16(fmaxf(acc + w.c2b[o], 0.f));
  }
  __syncthreads();
  // conv3 64 -> 128, k3 s1 p1, T 1 -> 1 (only the centre tap sees data): two threads per output
  {
    const int o = tid >> 1, part = tid & 1;
    const f16* wr = w.c3w + (size_t)o * 192;
    float acc = 0.f;
    for (int c = part * 32; c < part * 32 + 32; ++c) acc += (float)wr[c * 3 + 1] * c2[c];
    acc += __shfl_xor(acc, 1, 64);
    if (part == 0) c3[o] = r16(fmaxf(acc + w.c3b[o], 0.f));
  }
  __syncthreads();
  // LSTM input projection: 512 gate rows, K = 128
  for (int r = tid; r < 512; r += 256) {
    const f16x8* wr = reinterpret_cast<const f16x8*>(w.wih + (size_t)r * 128);
    float acc = 0.f;
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      const f16x8 a = wr[q];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += (float)a[e] * c3[q * 8 + e];
    }
    xg[chunk * 512 + r] = acc + w.bih[r];
  }
}

__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }

constexpr int kPF = 8;   // xg prefetch depth (steps)

__global__ __launch_bounds__(256) void k_vad_lstm(const float* __restrict__ xg, long long n_steps, VadWeights w,
                                                  float* __restrict__ hout) {
  __shared__ f16 hs[2][128];
  const int tid = threadIdx.x;
  const int u = tid >> 1, part = tid & 1;
  // W_hh rows g*128 + u, columns [part*64, part*64 + 64) in registers
  f16x8 W[4][8];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int q = 0; q < 8; ++q)
      W[g][q] = reinterpret_cast<const f16x8*>(w.whh + (size_t)(g * 128 + u) * 128 + part * 64)[q];
  float bhh[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bhh[g] = w.bhh[g * 128 + u];
  if (tid < 128) hs[0][tid] = (f16)0.f;
  float c = 0.f;
  float pf[kPF][4];
#pragma unroll
  for (int s = 0; s < kPF; ++s)
#pragma unroll
    for (int g = 0; g < 4; ++g) pf[s][g] = s < n_steps ? xg[(long long)s * 512 + g * 128 + u] : 0.f;
  __syncthreads();
  for (long long t0 = 0; t0 < n_steps; t0 += kPF) {
#pragma unroll
    for (int s = 0; s < kPF; ++s) {
      const long long t = t0 + s;
      if (t >= n_steps) break;
      const f16* hcur = hs[s & 1];
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const f16x8 hv = *reinterpret_cast<const f16x8*>(hcur + part * 64 + q * 8);
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[g] += (float)W[g][q][e] * (float)hv[e];
      }
      float pre[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        acc[g] += __shfl_xor(acc[g], 1, 64);
        pre[g] = pf[s][g] + (acc[g] + bhh[g]);
        const long long tn = t + kPF;
        pf[s][g] = tn < n_steps ? xg[tn * 512 + g * 128 + u] : 0.f;
      }
      const float ig = sigm(pre[0]), fg = sigm(pre[1]), gg = tanhf(pre[2]), og = sigm(pre[3]);
      c = fg * c + ig * gg;
      const float h = og * tanhf(c);
      if (part == 0) {
        hs[(s + 1) & 1][u] = (f16)h;
        hout[t * 128 + u] = h;
      }
      // LDS-only: the xg prefetch kPF steps ahead stays in flight (round 6; measured unchanged
      // here, 1.77 us per chunk -- the step's own dependent FMA / transcendental chain on one wave
      // per SIMD is the cost -- while the same change took pyannote's BiLSTM scans, k_lstm_scan,
      // from 45 to 12 ms of GPU time per hour)
      lds_barrier();
    }
  }
}

__global__ __launch_bounds__(256) void k_vad_head(const float* __restrict__ hout, long long n_steps, VadWeights w,
                                                  float* __restrict__ probs) {
  const long long t = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= n_steps) return;
  float acc = 0.f;
  for (int k = lane; k < 128; k += 64) acc += r16(fmaxf(hout[t * 128 + k], 0.f)) * (float)w.wo[k];
  acc = wave_sum(acc);
  if (lane == 0) probs[t] = sigm(acc + w.bo[0]);
}

void launch_vad(const float* x, long long n, const VadWeights& w, float* xg, float* hout, float* probs,
                hipStream_t s) {
  const long long nc = (n + 511) / 512;
  if (nc <= 0) return;
  WDR_CHECK(nc < (1ll << 31), "VAD: input too long");
  WDR_KLAUNCH(k_vad_front, dim3((unsigned)nc), dim3(256), 0, s, x, n, w, xg);
  WDR_HIP(hipGetLastError());
  WDR_KLAUNCH(k_vad_lstm, dim3(1), dim3(256), 0, s, xg, nc, w, hout);
  WDR_HIP(hipGetLastError());
  WDR_KLAUNCH(k_vad_head, dim3((unsigned)((nc + 3) / 4)), dim3(256), 0, s, hout, nc, w, probs);
  WDR_HIP(hipGetLastError());
}

}  // namespace wdr
