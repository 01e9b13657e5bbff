// Declarations of the experimental prefill GEMM (prefill_gemm.hip in this directory; not part of _C.so:
// slower than hipBLASLt at every measured shape, profiles/prefill_gemm_custom_r2.jsonl).
#pragma once
#include "common.h"

enum { PGEMM_EPI_BF16 = 0 };
struct PgemmEpi {
  bf16* y = nullptr;  // BF16: [M, ldy]
  long long ldy = 0;
};
void launch_pgemm(int epi, const bf16* X, const bf16* W, int M, int N, int K, const PgemmEpi& e, hipStream_t s);
void set_pgemm_variant(int v);  // 0: 8-wave ring, 1: 4-wave 128x128, 10/11: diagnostics
