// Probe: every hipBLASLt solution for the Llama-3-8B prefill projections vs the library's heuristic pick.
//
// Y[M, N] = X[M, K] . W[N, K]^T as the column-major "TN" GEMM m = N, n = M, k = K (the layout torch.matmul hands
// hipBLASLt).  Weights rotate over >= 1 GiB of copies so every call reads them from HBM, as in a prefill step.
// For each (projection, M, output type): the heuristic's first algorithm, then every algorithm getAllAlgos
// returns that supports the problem; one JSON line with both times and the best algorithm's index.
//
//   hipcc -O2 --offload-arch=gfx950 bench/kernels/blaslt_algos.cpp -lhipblaslt -o /tmp/blaslt_algos
//   /tmp/blaslt_algos [max_algos] [shape] [M] [out: bf16|f32] [layout: tn|nn]
//   (layout nn: the weights stored transposed, [K][N] row-major, i.e. the N x K column-major A operand)
//   (operands: random bf16 in [-1, 1): data-dependent MFMA power draw moves the clock, so constant fills
//   overstate throughput)
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    auto _e = (x);                                                              \
    if ((int)_e != 0) {                                                         \
      fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)_e);     \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

struct Shape {
  const char* name;
  int N, K;
};

static float time_algo(hipblasLtHandle_t h, hipblasLtMatmulDesc_t desc, const std::vector<void*>& Ws, void* X, void* Y,
                       hipblasLtMatrixLayout_t la, hipblasLtMatrixLayout_t lb, hipblasLtMatrixLayout_t lc,
                       const hipblasLtMatmulAlgo_t* algo, void* ws, size_t wsz, hipStream_t s, int reps) {
  const float alpha = 1.f, beta = 0.f;
  for (int i = 0; i < 2; ++i)
    if (hipblasLtMatmul(h, desc, &alpha, Ws[i % Ws.size()], la, X, lb, &beta, Y, lc, Y, lc, algo, ws, wsz, s) != 0)
      return -1.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, s));
    hipblasLtMatmul(h, desc, &alpha, Ws[(r + 2) % Ws.size()], la, X, lb, &beta, Y, lc, Y, lc, algo, ws, wsz, s);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1000.f);
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

static void fill_random(void* dst, size_t bytes, unsigned seed) {
  std::vector<unsigned short> h(bytes / 2);
  unsigned x = seed * 2654435761u + 12345u;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    const float f = (float)(x >> 8) / (float)(1u << 24) * 2.f - 1.f;
    unsigned u;
    memcpy(&u, &f, 4);
    v = (unsigned short)(u >> 16);
  }
  CK(hipMemcpy(dst, h.data(), bytes, hipMemcpyHostToDevice));
}

int main(int argc, char** argv) {
  const int max_algos = argc > 1 ? atoi(argv[1]) : 400;
  const std::string only = argc > 2 ? argv[2] : "";
  const int only_m = argc > 3 ? atoi(argv[3]) : 0;
  const std::string only_out = argc > 4 ? argv[4] : "";
  const bool nn = argc > 5 && std::string(argv[5]) == "nn";
  const Shape shapes[] = {{"qkv", 6144, 4096}, {"o", 4096, 4096}, {"gate_up", 28672, 4096}, {"down", 4096, 14336}};
  const int Ms[] = {512, 768, 1024, 1280};
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const size_t wsz = 128ull << 20;
  void* ws;
  CK(hipMalloc(&ws, wsz));
  for (const Shape& sh : shapes) {
    if (!only.empty() && only != sh.name) continue;
    const size_t wbytes = (size_t)sh.N * sh.K * 2;
    const int copies = std::max<int>(2, (int)((1ull << 30) / wbytes) + 1);
    std::vector<void*> Ws(copies);
    for (size_t i = 0; i < Ws.size(); ++i) {
      CK(hipMalloc(&Ws[i], wbytes));
      fill_random(Ws[i], wbytes, 7 + (unsigned)i);
    }
    for (int M : Ms) {
      if (only_m && M != only_m) continue;
      void *X, *Y;
      CK(hipMalloc(&X, (size_t)M * sh.K * 2));
      fill_random(X, (size_t)M * sh.K * 2, 3);
      CK(hipMalloc(&Y, (size_t)M * sh.N * 4));
      for (int outf = 0; outf < 2; ++outf) {  // 0: bf16 output, 1: fp32 output
        if (!only_out.empty() && only_out != (outf ? "f32" : "bf16")) continue;
        const hipDataType tD = outf ? HIP_R_32F : HIP_R_16BF;
        hipblasLtMatmulDesc_t desc;
        CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
        hipblasOperation_t ta = nn ? HIPBLAS_OP_N : HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
        hipblasLtMatrixLayout_t la, lb, lc;
        if (nn) CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, sh.N, sh.K, sh.N));
        else CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, sh.K, sh.N, sh.K));
        CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, sh.K, M, sh.K));
        CK(hipblasLtMatrixLayoutCreate(&lc, tD, sh.N, M, sh.N));
        hipblasLtMatmulPreference_t pref;
        CK(hipblasLtMatmulPreferenceCreate(&pref));
        uint64_t wl = wsz;
        CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wl, sizeof(wl)));
        hipblasLtMatmulHeuristicResult_t heur[1];
        int got = 0;
        CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 1, heur, &got));
        const float t_def = got ? time_algo(h, desc, Ws, X, Y, la, lb, lc, &heur[0].algo, ws, wsz, s, 9) : -1.f;
        const int def_idx = got ? hipblaslt_ext::getIndexFromAlgo(heur[0].algo) : -1;
        std::vector<hipblasLtMatmulHeuristicResult_t> all;
        hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, HIP_R_16BF, HIP_R_16BF, tD, tD,
                                   HIPBLAS_COMPUTE_32F, all);
        float best = 1e30f;
        int best_idx = -1, tried = 0;
        std::string best_name;
        for (auto& r : all) {
          if (tried >= max_algos) break;
          size_t need = 0;
          const float one = 1.f, zero = 0.f;
          if (hipblaslt_ext::matmulIsAlgoSupported(h, desc, &one, la, lb, &zero, lc, lc, r.algo, need) != 0 ||
              need > wsz)
            continue;
          if (++tried % 2000 == 0) {
            fprintf(stderr, "%s M=%d: %d algos timed, best %.2f us\n", sh.name, M, tried, best);
            fflush(stderr);
          }
          const float t = time_algo(h, desc, Ws, X, Y, la, lb, lc, &r.algo, ws, wsz, s, 5);
          if (t > 0 && t < best) {
            best = t;
            best_idx = hipblaslt_ext::getIndexFromAlgo(r.algo);
            best_name = hipblaslt_ext::getKernelNameFromAlgo(h, r.algo);
          }
        }
        // re-time the best one like the default (9 reps)
        double flops = 2.0 * M * sh.N * sh.K;
        printf("{\"layout\": \"%s\", \"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"out\": \"%s\", \"default_us\": %.2f, "
               "\"default_index\": %d, \"default_tflops\": %.1f, \"best_us\": %.2f, \"best_index\": %d, "
               "\"best_tflops\": %.1f, \"algos_tried\": %d, \"algos_listed\": %zu, \"best_kernel\": \"%s\"}\n",
               nn ? "nn" : "tn", sh.name, M, sh.N, sh.K, outf ? "f32" : "bf16", t_def, def_idx, flops / t_def / 1e6, best, best_idx,
               flops / best / 1e6, tried, all.size(), best_name.substr(0, 90).c_str());
        fflush(stdout);
        CK(hipblasLtMatmulPreferenceDestroy(pref));
        CK(hipblasLtMatrixLayoutDestroy(la));
        CK(hipblasLtMatrixLayoutDestroy(lb));
        CK(hipblasLtMatrixLayoutDestroy(lc));
        CK(hipblasLtMatmulDescDestroy(desc));
      }
      CK(hipFree(X));
      CK(hipFree(Y));
    }
    for (auto& w : Ws) CK(hipFree(w));
  }
  CK(hipFree(ws));
  CK(hipblasLtDestroy(h));
  return 0;
}
