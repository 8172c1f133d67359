// Decode-GEMV microbenchmark (large-v3 decoder shapes, M = 1): per-launch time of the
// production launch_proj path vs. experimental kernels, each replayed from a hipGraph of
// 32 launches over 32 distinct weight copies (> the 256 MiB Infinity Cache, like the 32
// decoder layers).  Build: make -C whisper-diarize-rs_amd gemv_bench ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../whisper-diarize-rs_amd/csrc/common.h"

using namespace wdr;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);          \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// pure streaming read of `n16` halves per launch: the bandwidth floor for the same bytes
__global__ __launch_bounds__(256) void k_stream(const f16x8* w, long long n8, float* out) {
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const f16x8 v = w[i];
    acc += (float)v[0] + (float)v[7];
  }
  if (acc == 12345.f) out[0] = acc;
}

__global__ void k_null(float* out) {
  if (threadIdx.x == 9999) out[0] = 1.f;
}

// experimental: each wave computes R rows; all loads issued before the first FMA
__device__ __forceinline__ float dot8x(f16x8 a, f16x8 b, float acc) {
#pragma unroll
  for (int i = 0; i < 8; ++i) acc += (float)a[i] * (float)b[i];
  return acc;
}
template <int R, int NCH>
__global__ __launch_bounds__(256) void k_gemv_rows(const f16* __restrict__ W, int K, int N,
                                                   const f16* __restrict__ x, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wid) * R;
  f16x8 wv[R][NCH], xv[NCH];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = c * 512 + lane * 8;
      wv[r][c] = (n0 + r < N && k < K) ? *(const f16x8*)(W + (size_t)(n0 + r) * K + k) : (f16x8){};
    }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    xv[c] = k < K ? *(const f16x8*)(x + k) : (f16x8){};
  }
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r] = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) acc[r] = dot8x(wv[r][c], xv[c], acc[r]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc[r] += __shfl_xor(acc[r], o, 64);
  }
  if (lane < R && n0 + lane < N) {
    float v = acc[0];
#pragma unroll
    for (int r = 1; r < R; ++r)
      if (lane == r) v = acc[r];
    out[n0 + lane] = v;
  }
}

// experimental: split K across the 4 waves of a WG (each wave 1/4 of K for RW rows), LDS reduce
template <int RW, int KPW>   // KPW = halves per wave per row / 512
__global__ __launch_bounds__(256) void k_gemv_splitk(const f16* __restrict__ W, int K, int N,
                                                     const f16* __restrict__ x, float* __restrict__ out) {
  __shared__ float red[4][RW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * RW;
  const int kb = wid * KPW * 512;
  f16x8 wv[RW][KPW], xv[KPW];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int c = 0; c < KPW; ++c) {
      const int k = kb + c * 512 + lane * 8;
      wv[r][c] = (n0 + r < N && k < K) ? *(const f16x8*)(W + (size_t)(n0 + r) * K + k) : (f16x8){};
    }
#pragma unroll
  for (int c = 0; c < KPW; ++c) {
    const int k = kb + c * 512 + lane * 8;
    xv[c] = k < K ? *(const f16x8*)(x + k) : (f16x8){};
  }
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < KPW; ++c) a = dot8x(wv[r][c], xv[c], a);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (lane == 0) red[wid][r] = a;
  }
  __syncthreads();
  if (threadIdx.x < RW && n0 + threadIdx.x < N)
    out[n0 + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

struct Shape {
  const char* name;
  int N, K, epi;
  bool ln;
};

template <typename F>
static float time_graph(F launch_all, hipStream_t s, int reps) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  launch_all();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return ms / reps;
}

int main() {
  const int L = 32, d = 1280;
  Shape shapes[] = {{"qkv  3d x d  +LN", 3 * d, d, EPI_F16, true},   {"o    d x d  resid", d, d, EPI_F32_RESID, false},
                    {"xq   d x d  +LN", d, d, EPI_F16, true},        {"fc1 4d x d  +LN gelu", 4 * d, d, EPI_F16_GELU, true},
                    {"fc2  d x 4d resid", d, 4 * d, EPI_F32_RESID, false}};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  float *xf, *out, *g, *b;
  f16* x16;
  CK(hipMalloc(&xf, 8 * 4 * d * 4));
  CK(hipMalloc(&out, 8 * 4 * d * 4 * 16));
  CK(hipMalloc(&g, 4 * d * 4));
  CK(hipMalloc(&b, 4 * d * 4));
  CK(hipMalloc(&x16, 8 * 4 * d * 2));
  CK(hipMemset(xf, 0, 8 * 4 * d * 4));
  CK(hipMemset(x16, 0, 8 * 4 * d * 2));
  CK(hipMemset(g, 0, 4 * d * 4));
  CK(hipMemset(b, 0, 4 * d * 4));
  float* bias;
  CK(hipMalloc(&bias, 4 * d * 4));
  CK(hipMemset(bias, 0, 4 * d * 4));
  {
    // empty kernel in a graph: the per-launch floor
    float t = time_graph([&] { for (int l = 0; l < L; ++l) hipLaunchKernelGGL(k_null, dim3(256), dim3(256), 0, s, out); },
                         s, 50);
    printf("%-22s %8.2f us/launch\n", "null kernel 256 WGs", t * 1e3 / L);
  }
  if (const char* gr = getenv("GB_ROWS")) {
    // multi-row decode-step GEMVs (the batched step's projections after k_ln_rows): launch_proj
    // with step_rows, M rows, no LN prologue; run under WDR_MGEMV_STAGED / WDR_MGEMV_R variants
    const int M = atoi(gr);
    f16* xa;
    CK(hipMalloc(&xa, (size_t)16 * 4 * d * 2));
    CK(hipMemset(xa, 0, (size_t)16 * 4 * d * 2));
    float* o32;
    CK(hipMalloc(&o32, (size_t)16 * 4 * d * 4));
    CK(hipMemset(o32, 0, (size_t)16 * 4 * d * 4));
    for (const Shape& sh : shapes) {
      const size_t wel = (size_t)sh.N * sh.K;
      std::vector<f16*> W(L);
      for (int l = 0; l < L; ++l) {
        CK(hipMalloc(&W[l], wel * 2));
        CK(hipMemset(W[l], 0, wel * 2));
      }
      const double mb = wel * 2 / 1e6;
      float t = time_graph([&] {
        for (int l = 0; l < L; ++l) {
          ProjArgs a{xa, sh.K, W[l], sh.K, bias, o32, sh.N, nullptr, 0, M, sh.N, sh.K,
                     sh.epi == EPI_QKV_CACHE ? EPI_F16 : sh.epi};
          a.step_rows = 1;
          launch_proj(a, s);
        }
      }, s, 20);
      printf("M=%-2d %-22s %8.2f us  %7.2f TB/s\n", M, sh.name, t * 1e3 / L, mb / (t * 1e3 / L));
      for (int l = 0; l < L; ++l) CK(hipFree(W[l]));
    }
    return 0;
  }
  for (const Shape& sh : shapes) {
    const size_t wel = (size_t)sh.N * sh.K;
    std::vector<f16*> W(L);
    for (int l = 0; l < L; ++l) {
      CK(hipMalloc(&W[l], wel * 2));
      CK(hipMemset(W[l], 0, wel * 2));
    }
    const double mb = wel * 2 / 1e6;
    printf("== %s  (%.2f MB)\n", sh.name, mb);
    for (int grid : {256, 512, 1024, 2048}) {
      float t = time_graph([&] {
        for (int l = 0; l < L; ++l)
          hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, s, (const f16x8*)W[l], (long long)(wel / 8), out);
      }, s, 20);
      printf("   stream grid %-5d   %8.2f us  %7.2f TB/s\n", grid, t * 1e3 / L, mb / (t * 1e3 / L));
    }
    {
      float t = time_graph([&] {
        for (int l = 0; l < L; ++l) {
          ProjArgs a{x16, sh.K, W[l], sh.K, bias, out, sh.N, nullptr, 0, 1, sh.N, sh.K, sh.epi};
          if (sh.ln) { a.ln_x = xf; a.ldln = sh.K; a.ln_g = g; a.ln_b = b; }
          if (sh.epi == EPI_QKV_CACHE) a.epi = EPI_F16;
          launch_proj(a, s);
        }
      }, s, 20);
      printf("   launch_proj         %8.2f us  %7.2f TB/s\n", t * 1e3 / L, mb / (t * 1e3 / L));
    }
#define ROWS(R, NCH)                                                                                              \
    {                                                                                                             \
      float t = time_graph([&] {                                                                                  \
        for (int l = 0; l < L; ++l)                                                                               \
          hipLaunchKernelGGL((k_gemv_rows<R, NCH>), dim3((sh.N + 4 * R - 1) / (4 * R)), dim3(256), 0, s, W[l], sh.K, \
                             sh.N, x16, out);                                                                     \
      }, s, 20);                                                                                                  \
      printf("   rows R=%d            %8.2f us  %7.2f TB/s\n", R, t * 1e3 / L, mb / (t * 1e3 / L));          \
    }
    if (sh.K == d) {
      ROWS(1, 3) ROWS(2, 3) ROWS(4, 3)
    } else {
      ROWS(1, 10) ROWS(2, 10)
    }
#define SPLITK(RW, KPW)                                                                                     \
    {                                                                                                       \
      float t = time_graph([&] {                                                                            \
        for (int l = 0; l < L; ++l)                                                                         \
          hipLaunchKernelGGL((k_gemv_splitk<RW, KPW>), dim3((sh.N + RW - 1) / RW), dim3(256), 0, s, W[l], sh.K, \
                             sh.N, x16, out);                                                               \
      }, s, 20);                                                                                            \
      printf("   splitk RW=%d KPW=%d     %8.2f us  %7.2f TB/s\n", RW, KPW, t * 1e3 / L, mb / (t * 1e3 / L)); \
    }
    if (sh.K == d) {
      SPLITK(2, 1) SPLITK(4, 1) SPLITK(8, 1)
    } else {
      SPLITK(2, 3) SPLITK(4, 3) SPLITK(8, 3)
    }
    for (int l = 0; l < L; ++l) CK(hipFree(W[l]));
  }
  return 0;
}
