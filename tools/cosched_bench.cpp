// Co-scheduling probe: how much a decode-step-like chain of dependent kernels slows down beside
// the encoder's GEMMs, and why.  The chain (hipGraph, replayed): 32 layers x {qkv, o, xq, fc1
// GELU, fc2} as rows_forward issues them at R rows (large-v3 shapes, 32 distinct weight copies,
// LayerNorm fused into qkv / xq / fc1), or 160 tiny dependent k_layernorm
// launches ("tiny": boundary + latency only).  The load: a queue of encoder projections (M = 6000: qkv, o, fc1, fc2) on a
// stream of its own, either CU-masked as the pipeline's encode-ahead streams (32 CUs, 4 per
// XCD, left free) or on all CUs.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/cosched_bench.cpp -Lwhisper-diarize-rs_amd -lwdr \
//          -Wl,-rpath,'$ORIGIN/../whisper-diarize-rs_amd' -o tools/cosched_bench
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
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

static hipStream_t masked_stream(int n_res) {
  std::vector<uint32_t> mask(8, 0u);
  std::vector<char> res(256, 0);
  for (int x = 0; x < 8; ++x)
    for (int j = 0; j < n_res / 8; ++j) res[32 * x + 8 * j + x] = 1;
  for (int c = 0; c < 256; ++c)
    if (!res[c]) mask[c / 32] |= 1u << (c % 32);
  hipStream_t s;
  CK(hipExtStreamCreateWithCUMask(&s, 8, mask.data()));
  return s;
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 16;
  const int d = 1280, L = 32, ME = 6000;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  if (ncu != 256) {
    printf("expects 256 CUs (MI355X), found %d\n", ncu);
    return 1;
  }
  hipStream_t s, se_mask, se_all;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  se_mask = masked_stream(32);
  CK(hipStreamCreateWithFlags(&se_all, hipStreamNonBlocking));
  // decode chain buffers
  float *xf, *g, *b, *bias;
  f16 *hq, *att, *mlp;
  CK(hipMalloc(&xf, (size_t)R * d * 4));
  CK(hipMalloc(&g, 4 * d * 4));
  CK(hipMalloc(&b, 4 * d * 4));
  CK(hipMalloc(&bias, 4 * d * 4));
  CK(hipMalloc(&hq, (size_t)R * 3 * d * 2));
  CK(hipMalloc(&att, (size_t)R * d * 2));
  CK(hipMalloc(&mlp, (size_t)R * 4 * d * 2));
  CK(hipMemset(xf, 0, (size_t)R * d * 4));
  CK(hipMemset(g, 0, 4 * d * 4));
  CK(hipMemset(b, 0, 4 * d * 4));
  CK(hipMemset(bias, 0, 4 * d * 4));
  CK(hipMemset(hq, 0, (size_t)R * 3 * d * 2));
  CK(hipMemset(att, 0, (size_t)R * d * 2));
  CK(hipMemset(mlp, 0, (size_t)R * 4 * d * 2));
  struct LW {
    f16 *qkv, *o, *xq, *fc1, *fc2;
  };
  std::vector<LW> W(L);
  for (auto& w : W) {
    CK(hipMalloc(&w.qkv, (size_t)3 * d * d * 2));
    CK(hipMalloc(&w.o, (size_t)d * d * 2));
    CK(hipMalloc(&w.xq, (size_t)d * d * 2));
    CK(hipMalloc(&w.fc1, (size_t)4 * d * d * 2));
    CK(hipMalloc(&w.fc2, (size_t)4 * d * d * 2));
    CK(hipMemset(w.qkv, 0, (size_t)3 * d * d * 2));
    CK(hipMemset(w.o, 0, (size_t)d * d * 2));
    CK(hipMemset(w.xq, 0, (size_t)d * d * 2));
    CK(hipMemset(w.fc1, 0, (size_t)4 * d * d * 2));
    CK(hipMemset(w.fc2, 0, (size_t)4 * d * d * 2));
  }
  auto P = [&](const f16* A, int lda, const f16* Wt, void* out, int ldo, int N, int K, int epi, bool ln) {
    ProjArgs a{A, lda, Wt, K, bias, out, ldo, nullptr, 0, R, N, K, epi};
    a.rows_mma = 1;
    if (ln) {
      if (R <= 32) {
        a.ln_x = xf; a.ldln = d; a.ln_g = g; a.ln_b = b;
      } else {
        launch_layernorm(xf, d, g, b, att, d, R, d, s);
        a.A = att;
        a.lda = d;
      }
    }
    launch_proj(a, s);
  };
  // the decoder layer's projections as rows_forward runs them (attention left out): 5 launches
  // per layer, LayerNorm fused into qkv / xq / fc1 up to 32 rows
  auto chain = [&] {
    for (int l = 0; l < L; ++l) {
      P(nullptr, d, W[l].qkv, hq, 3 * d, 3 * d, d, EPI_F16, true);
      P(att, d, W[l].o, xf, d, d, d, EPI_F32_RESID, false);
      P(nullptr, d, W[l].xq, hq, d, d, d, EPI_F16, true);
      P(nullptr, d, W[l].fc1, mlp, 4 * d, 4 * d, d, EPI_F16_GELU, true);
      P(mlp, 4 * d, W[l].fc2, xf, d, d, 4 * d, EPI_F32_RESID, false);
    }
  };
  auto tiny = [&] {
    for (int i = 0; i < 160; ++i) launch_layernorm(xf, d, g, b, att, d, R, d, s);
  };
  auto capture = [&](auto fn) {
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    fn();
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    return ge;
  };
  hipGraphExec_t g_chain = capture(chain), g_tiny = capture(tiny);
  // encoder load
  f16 *ea, *ew1, *ew2, *eo16;
  float* eo32;
  CK(hipMalloc(&ea, (size_t)ME * 4 * d * 2));
  CK(hipMalloc(&ew1, (size_t)4 * d * d * 2));
  CK(hipMalloc(&ew2, (size_t)4 * d * d * 2));
  CK(hipMalloc(&eo16, (size_t)ME * 4 * d * 2));
  CK(hipMalloc(&eo32, (size_t)ME * d * 4));
  CK(hipMemset(ea, 0, (size_t)ME * 4 * d * 2));
  CK(hipMemset(ew1, 0, (size_t)4 * d * d * 2));
  CK(hipMemset(ew2, 0, (size_t)4 * d * d * 2));
  auto enc_burst = [&](hipStream_t es, int reps) {
    for (int r = 0; r < reps; ++r) {
      ProjArgs q{ea, d, ew1, d, bias, eo16, 3 * d, nullptr, 0, ME, 3 * d, d, EPI_F16};
      launch_proj(q, es);
      ProjArgs o{ea, d, ew1, d, bias, eo32, d, nullptr, 0, ME, d, d, EPI_F32_RESID};
      launch_proj(o, es);
      ProjArgs f1{ea, d, ew1, d, bias, eo16, 4 * d, nullptr, 0, ME, 4 * d, d, EPI_F16_GELU};
      launch_proj(f1, es);
      ProjArgs f2{ea, 4 * d, ew2, 4 * d, bias, eo32, d, nullptr, 0, ME, d, 4 * d, EPI_F32_RESID};
      launch_proj(f2, es);
    }
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_graph = [&](hipGraphExec_t ge, int reps) {
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
  };
  auto time_enc = [&](hipStream_t es) {
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    CK(hipEventRecord(a, es));
    enc_burst(es, 20);
    CK(hipEventRecord(z, es));
    CK(hipEventSynchronize(z));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, z));
    return ms / 20;
  };
  CK(hipDeviceSynchronize());
  printf("R=%d\n", R);
  printf("encoder layer (qkv+o+fc1+fc2, M=6000) alone: masked %.3f ms, all CUs %.3f ms\n", time_enc(se_mask),
         time_enc(se_all));
  const char* names[2] = {"chain (160 rows launches)", "tiny (160 k_layernorm)"};
  hipGraphExec_t gs[2] = {g_chain, g_tiny};
  for (int k = 0; k < 2; ++k) {
    const float alone = time_graph(gs[k], 10);
    // beside the encoder: enough encoder work queued to outlast the replays
    enc_burst(se_mask, 150);
    const float masked = time_graph(gs[k], 10);
    CK(hipDeviceSynchronize());
    enc_burst(se_all, 150);
    const float all = time_graph(gs[k], 10);
    CK(hipDeviceSynchronize());
    const int nl = k == 0 ? 5 * L : 160;
    printf("%-30s alone %.3f ms (%.2f us/launch)  beside masked encoder %.3f ms (x%.2f)  beside unmasked %.3f ms "
           "(x%.2f)\n", names[k], alone, alone * 1e3 / nl, masked, masked / alone, all, all / alone);
    fflush(stdout);
  }
  return 0;
}
