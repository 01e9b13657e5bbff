// C entry points over csrc/kernels/prefill_gemm.hip for the standalone kernel bench (bench_pgemm.py):
// build: see bench_pgemm.py (hipcc -I csrc/kernels prefill_gemm.hip pgemm_capi.hip)
#include "pgemm.h"

extern "C" int pg_bf16(const void* X, const void* W, void* Y, int M, int N, int K, hipStream_t s) {
  PgemmEpi e;
  e.y = (bf16*)Y;
  e.ldy = N;
  launch_pgemm(PGEMM_EPI_BF16, (const bf16*)X, (const bf16*)W, M, N, K, e, s);
  return (int)hipGetLastError();
}

extern "C" void pg_variant(int v) { set_pgemm_variant(v); }
