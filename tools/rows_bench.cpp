// Decoder-row projection microbenchmark (large-v3 decoder shapes): the row kernel
// (ProjArgs::rows_mma: k_skinny's arithmetic for any row count, LayerNorm fused up to 32 rows),
// per launch, replayed from a hipGraph of 32 launches over RB_COPIES distinct weight copies
// (default 32: > the 256 MiB Infinity Cache, HBM-bound; RB_COPIES=1: the weights served from
// cache, the latency floor of the launch chain).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/rows_bench.cpp -Lwhisper-diarize-rs_amd -lwdr \
//          -Wl,-rpath,'$ORIGIN/../whisper-diarize-rs_amd' -o tools/rows_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

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
  bool ln;
};

int main(int argc, char** argv) {
  const int L = getenv("RB_LAYERS") ? atoi(getenv("RB_LAYERS")) : 32, d = 1280, MX = 256;
  const int copies = getenv("RB_COPIES") ? atoi(getenv("RB_COPIES")) : L;
  // rows_forward fuses the LayerNorm into the row kernel up to a per-projection row count (qkv 48,
  // xq 64, fc1 24, logits never: csrc/rows.cpp); RB_LN_FUSE: one threshold for all
  const int ln_env = getenv("RB_LN_FUSE") ? atoi(getenv("RB_LN_FUSE")) : -1;
  Shape shapes[] = {{"qkv  +LN", 3 * d, d, EPI_F16, true},        {"o    resid", d, d, EPI_F32_RESID, false},
                    {"xq   +LN", d, d, EPI_F16, true},            {"fc1  +LN gelu", 4 * d, d, EPI_F16_GELU, true},
                    {"fc2  resid", d, 4 * d, EPI_F32_RESID, false}, {"logits +LN", 51866, d, EPI_F32, true}};
  std::vector<int> Ms = {1, 8, 16, 24, 32, 40, 48, 56, 64, 128};
  if (argc > 1) {
    Ms.clear();
    for (int i = 1; i < argc; ++i) Ms.push_back(atoi(argv[i]));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  float *xf, *out, *g, *b, *bias;
  f16 *xa, *hd;
  CK(hipMalloc(&xf, (size_t)MX * 4 * d * 4));
  CK(hipMalloc(&out, (size_t)MX * 51866 * 4));
  CK(hipMalloc(&g, 4 * d * 4));
  CK(hipMalloc(&b, 4 * d * 4));
  CK(hipMalloc(&bias, 51866 * 4));
  CK(hipMalloc(&xa, (size_t)MX * 4 * d * 2));
  CK(hipMalloc(&hd, (size_t)MX * 4 * d * 2));
  CK(hipMemset(xf, 0, (size_t)MX * 4 * d * 4));
  CK(hipMemset(out, 0, (size_t)MX * 51866 * 4));
  CK(hipMemset(g, 0, 4 * d * 4));
  CK(hipMemset(b, 0, 4 * d * 4));
  CK(hipMemset(bias, 0, 51866 * 4));
  CK(hipMemset(xa, 0, (size_t)MX * 4 * d * 2));
  printf("%-14s %4s %10s   (us per launch incl. LN launch; TB/s of the weights)\n", "shape", "M", "rows");
  for (const Shape& sh : shapes) {
    const size_t wel = (size_t)sh.N * sh.K;
    const int nl = sh.N > 10000 ? 4 : L;   // the logits weights once per step
    const int nw = std::max(1, std::min(nl, copies));
    std::vector<f16*> W(nw);
    for (int l = 0; l < nw; ++l) {
      CK(hipMalloc(&W[l], wel * 2));
      CK(hipMemset(W[l], 0, wel * 2));
    }
    const double mb = wel * 2 / 1e6;
    for (int M : Ms) {
      const float tr = time_graph([&] {
        for (int l = 0; l < nl; ++l) {
          ProjArgs a{xa, sh.K, W[l % nw], sh.K, bias, out, sh.N, nullptr, 0, M, sh.N, sh.K, sh.epi};
          a.rows_mma = 1;
          if (sh.ln) {
            const int ln_fuse = ln_env >= 0 ? ln_env : sh.N == 3 * d ? 48 : sh.N == d ? 64 : sh.N == 4 * d ? 24 : 0;
            if (M <= ln_fuse) {
              a.ln_x = xf; a.ldln = sh.K; a.ln_g = g; a.ln_b = b;
            } else {
              launch_layernorm(xf, d, g, b, hd, d, M, d, s);
              a.A = hd;
            }
          }
          launch_proj(a, s);
        }
      }, s, 10);
      const double ur = tr * 1e3 / nl;
      printf("%-14s %4d %7.2f us   %5.2f TB/s\n", sh.name, M, ur, mb / ur);
      fflush(stdout);
    }
    for (int l = 0; l < nw; ++l) CK(hipFree(W[l]));
  }
  return 0;
}
