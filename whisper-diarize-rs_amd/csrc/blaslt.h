// Encoder projections on hipBLASLt (A/B seam, csrc/blaslt.cpp).
#pragma once
#include "common.h"

namespace wdr {
// WDR_ENC_BLASLT=1
bool enc_blaslt_on();
// false when the projection's epilogue / operands are not a plain GEMM the library takes
bool blaslt_proj(const ProjArgs& a, hipStream_t s);
// plans and kernels of the encoder shapes (rows Ms) built before any graph capture
void blaslt_prewarm(int d, const int* Ms, int nM, hipStream_t s);
}  // namespace wdr
