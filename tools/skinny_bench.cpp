// Prefill / DTW re-forward projection microbenchmark (large-v3 decoder shapes, 8 < M <= 64
// rows): per-launch time of the production launch_proj path vs experimental kernels, each
// replayed from a hipGraph of 32 launches over 32 distinct weight copies (> the 256 MiB
// Infinity Cache, like the 32 decoder layers).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/skinny_bench.cpp -Lwhisper-diarize-rs_amd -lwdr
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>

#include "../whisper-diarize-rs_amd/csrc/common.h"
#include "../whisper-diarize-rs_amd/csrc/kernels/kernels.h"

using namespace wdr;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);          \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void k_stream(const f16x8* w, long long n8, float* out) {
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const f16x8 v = w[i];
    acc += (float)v[0] + (float)v[7];
  }
  if (acc == 12345.f) out[0] = acc;
}

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

struct Shape {
  const char* name;
  int N, K, epi;
};

int main() {
  const int L = 32, d = 1280;
  Shape shapes[] = {{"qkv  3d x d", 3 * d, d, EPI_F16}, {"o    d x d  resid", d, d, EPI_F32_RESID},
                    {"fc1 4d x d  gelu", 4 * d, d, EPI_F16_GELU}, {"fc2  d x 4d resid", d, 4 * d, EPI_F32_RESID}};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  float *out, *bias, *xf, *g, *b;
  f16 *x16, *h16;
  CK(hipMalloc(&out, 64 * 4 * d * 4));
  CK(hipMalloc(&bias, 4 * d * 4));
  CK(hipMalloc(&x16, 64 * 4 * d * 2));
  CK(hipMalloc(&h16, 64 * 4 * d * 2));
  CK(hipMalloc(&xf, 64 * d * 4));
  CK(hipMalloc(&g, d * 4));
  CK(hipMalloc(&b, d * 4));
  CK(hipMemset(out, 0, 64 * 4 * d * 4));
  CK(hipMemset(bias, 0, 4 * d * 4));
  CK(hipMemset(x16, 0, 64 * 4 * d * 2));
  CK(hipMemset(xf, 0, 64 * d * 4));
  CK(hipMemset(g, 0, d * 4));
  CK(hipMemset(b, 0, d * 4));
  for (int M : {24, 40, 64}) {
    float t = time_graph([&] {
      for (int l = 0; l < L; ++l) launch_layernorm(xf, d, g, b, h16, d, M, d, s);
    }, s, 20);
    printf("M=%2d layernorm           %8.2f us\n", M, t * 1e3 / L);
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

    {
      float t = time_graph([&] {
        for (int l = 0; l < L; ++l)
          hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, s, (const f16x8*)W[l], (long long)(wel / 8), out);
      }, s, 20);
      printf("   stream                %8.2f us  %7.2f TB/s\n", t * 1e3 / L, mb / (t * 1e3 / L) / 1e3);
    }
    for (int M : {24, 40, 64}) {
      float t = time_graph([&] {
        for (int l = 0; l < L; ++l) {
          ProjArgs a{x16, sh.K, W[l], sh.K, bias, out, sh.N, nullptr, 0, M, sh.N, sh.K, sh.epi};
          launch_proj(a, s);
        }
      }, s, 20);
      printf("   M=%2d launch_proj      %8.2f us  %7.2f TB/s\n", M, t * 1e3 / L, mb / (t * 1e3 / L) / 1e3);
      setenv("WDR_SKINNY_MSPLIT", "0", 1);
      const float t0 = time_graph([&] {
        for (int l = 0; l < L; ++l) {
          ProjArgs a{x16, sh.K, W[l], sh.K, bias, out, sh.N, nullptr, 0, M, sh.N, sh.K, sh.epi};
          launch_proj(a, s);
        }
      }, s, 20);
      unsetenv("WDR_SKINNY_MSPLIT");
      printf("   M=%2d no row split     %8.2f us\n", M, t0 * 1e3 / L);
    }
    for (int l = 0; l < L; ++l) CK(hipFree(W[l]));
  }
  return 0;
}
