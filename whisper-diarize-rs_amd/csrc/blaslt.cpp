// Encoder projections on the vendor GEMM library (hipBLASLt) -- an A/B seam (WDR_ENC_BLASLT=1)
// beside the hand-written MFMA GEMMs (kernels/gemm.hip), to measure in the pipeline what the
// library's ~1.5x faster tiles (profiles/r02/hipblaslt_reference_rate.txt) are worth.  Plain
// GEMMs only: bias (f16 out), bias + GELU (f16 out), and the residual update out32 += acc + bias
// (C = D f32, beta 1); the other epilogues stay on the MFMA kernels.  No workspace, so the call
// needs no per-stream scratch and captures into the encode-ahead hipGraphs.
#include "blaslt.h"

#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>

namespace wdr {

#define WDR_BLT(call)                                                                        \
  do {                                                                                       \
    hipblasStatus_t st_ = (call);                                                            \
    if (st_ != HIPBLAS_STATUS_SUCCESS)                                                       \
      throw std::runtime_error(std::string("hipBLASLt error ") + std::to_string((int)st_) + \
                               " at " __FILE__ ":" + std::to_string(__LINE__) + " (" #call ")"); \
  } while (0)

bool enc_blaslt_on() {
  static const bool on = getenv("WDR_ENC_BLASLT") && atoi(getenv("WDR_ENC_BLASLT")) != 0;
  return on;
}

namespace {
struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
};
struct Dev {
  hipblasLtHandle_t h = nullptr;
  std::map<std::tuple<int, int, int, int, int, int, int>, Plan> plans;   // M N K epi lda ldb ldo
};
std::mutex g_mu;
std::map<int, Dev> g_dev;
}  // namespace

bool blaslt_proj(const ProjArgs& a, hipStream_t s) {
  if (a.epi != EPI_F16 && a.epi != EPI_F16_GELU && a.epi != EPI_F32_RESID) return false;
  if (a.A8 || a.ln_x || a.row_map || !a.A || !a.B || !a.bias) return false;
  int dev = 0;
  WDR_HIP(hipGetDevice(&dev));
  Plan* p = nullptr;
  hipblasLtHandle_t h = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    Dev& D = g_dev[dev];
    if (!D.h) WDR_BLT(hipblasLtCreate(&D.h));
    h = D.h;
    auto key = std::make_tuple(a.M, a.N, a.K, a.epi, a.lda, a.ldb, a.ldo);
    auto it = D.plans.find(key);
    if (it == D.plans.end()) {
      Plan q;
      // column-major view: D[N x M] (ld = ldo) = W^T-view (K x N, ld = ldb) op T  x  A-view (K x M, ld = lda)
      WDR_BLT(hipblasLtMatmulDescCreate(&q.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
      const int32_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
      WDR_BLT(hipblasLtMatmulDescSetAttribute(q.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT)));
      WDR_BLT(hipblasLtMatmulDescSetAttribute(q.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN)));
      const uint32_t epi = a.epi == EPI_F16_GELU ? HIPBLASLT_EPILOGUE_GELU_BIAS : HIPBLASLT_EPILOGUE_BIAS;
      WDR_BLT(hipblasLtMatmulDescSetAttribute(q.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
      const int32_t bt = HIP_R_32F;
      WDR_BLT(hipblasLtMatmulDescSetAttribute(q.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
      const hipDataType ot = a.epi == EPI_F32_RESID ? HIP_R_32F : HIP_R_16F;
      WDR_BLT(hipblasLtMatrixLayoutCreate(&q.la, HIP_R_16F, a.K, a.N, a.ldb));
      WDR_BLT(hipblasLtMatrixLayoutCreate(&q.lb, HIP_R_16F, a.K, a.M, a.lda));
      WDR_BLT(hipblasLtMatrixLayoutCreate(&q.lc, ot, a.N, a.M, a.ldo));
      hipblasLtMatmulPreference_t pref;
      WDR_BLT(hipblasLtMatmulPreferenceCreate(&pref));
      const uint64_t ws = 0;
      WDR_BLT(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
      hipblasLtMatmulHeuristicResult_t res[1];
      int n = 0;
      WDR_BLT(hipblasLtMatmulAlgoGetHeuristic(h, q.desc, q.la, q.lb, q.lc, q.lc, pref, 1, res, &n));
      (void)hipblasLtMatmulPreferenceDestroy(pref);
      WDR_CHECK(n > 0, "hipBLASLt: no algorithm for an encoder projection");
      q.algo = res[0].algo;
      it = D.plans.emplace(key, q).first;
    }
    p = &it->second;
  }
  // the bias pointer is per call (one descriptor per shape, set under the lock before the launch)
  std::lock_guard<std::mutex> g(g_mu);
  const void* bias = a.bias;
  WDR_BLT(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  const float alpha = 1.f, beta = a.epi == EPI_F32_RESID ? 1.f : 0.f;
  WDR_BLT(hipblasLtMatmul(h, p->desc, &alpha, a.B, p->la, a.A, p->lb, &beta, a.out, p->lc, a.out, p->lc, &p->algo,
                          nullptr, 0, s));
  return true;
}

void blaslt_prewarm(int d, const int* Ms, int nM, hipStream_t s) {
  if (!enc_blaslt_on()) return;
  const int shapes[4][3] = {{3 * d, d, EPI_F16}, {d, d, EPI_F32_RESID}, {4 * d, d, EPI_F16_GELU}, {d, 4 * d, EPI_F32_RESID}};
  int mmax = 0;
  for (int i = 0; i < nM; ++i) mmax = std::max(mmax, Ms[i]);
  void *A = nullptr, *W = nullptr, *O = nullptr, *b = nullptr;
  WDR_HIP(hipMalloc(&A, (size_t)mmax * 4 * d * 2));
  WDR_HIP(hipMalloc(&W, (size_t)4 * d * d * 2));
  WDR_HIP(hipMalloc(&O, (size_t)mmax * 4 * d * 4));
  WDR_HIP(hipMalloc(&b, (size_t)4 * d * 4));
  WDR_HIP(hipMemsetAsync(A, 0, (size_t)mmax * 4 * d * 2, s));
  WDR_HIP(hipMemsetAsync(W, 0, (size_t)4 * d * d * 2, s));
  WDR_HIP(hipMemsetAsync(b, 0, (size_t)4 * d * 4, s));
  for (int i = 0; i < nM; ++i)
    for (auto& sh : shapes) {
      ProjArgs a{(const f16*)A, sh[1], (const f16*)W, sh[1], (const float*)b, O, sh[0], nullptr, 0, Ms[i], sh[0], sh[1], sh[2]};
      WDR_CHECK(blaslt_proj(a, s), "hipBLASLt prewarm");
    }
  WDR_HIP(hipStreamSynchronize(s));
  (void)hipFree(A);
  (void)hipFree(W);
  (void)hipFree(O);
  (void)hipFree(b);
}

}  // namespace wdr
