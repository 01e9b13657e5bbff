// Probe of the /opt/rocm hipBLASLt build (standalone, outside torch): for every (N x K projection, M rows) the
// best supported solution of the TN problem y[M][N] = x[M][K] . W[N][K]^T, bf16 in / bf16 out.  The serving
// process calls torch's bundled hipBLASLt instead (its symbols win in the process), which numbers and ships a
// different, smaller solution set: the runtime table comes from bench/kernels/blaslt_tune.py, in-process.  This
// probe's results (profiles/r4/blaslt_tune_8b_rocm_lib.jsonl) show what the newer library would give.
//
//   hipcc -O2 --offload-arch=gfx950 bench/kernels/blaslt_tune.cpp -lhipblaslt -o bench/kernels/blaslt_tune
//   bench/kernels/blaslt_tune 6144x4096,4096x4096,28672x4096,4096x14336 256,512,768 > table.jsonl
//
// Screening: every supported solution timed over 3 calls (weights rotating over >= 1 GiB of copies, so each call
// reads them from HBM as in a prefill step; random bf16 operands, since data-dependent MFMA power moves the clock);
// the 6 fastest are re-timed over 11 calls next to the heuristic's pick.  One JSON line per (N, K, M).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    auto _e = (x);                                                          \
    if ((int)_e != 0) {                                                     \
      fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)_e); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

struct Prob {
  hipblasLtHandle_t h;
  hipblasLtMatmulDesc_t desc;
  hipblasLtMatrixLayout_t la, lb, lc;
  std::vector<void*> Ws;
  void *X, *Y, *ws;
  size_t wsz;
  hipStream_t s;
};

static float time_algo(Prob& p, const hipblasLtMatmulAlgo_t* algo, int reps) {
  const float alpha = 1.f, beta = 0.f;
  for (int i = 0; i < 2; ++i)
    if (hipblasLtMatmul(p.h, p.desc, &alpha, p.Ws[i % p.Ws.size()], p.la, p.X, p.lb, &beta, p.Y, p.lc, p.Y, p.lc, algo,
                        p.ws, p.wsz, p.s) != 0)
      return -1.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, p.s));
    hipblasLtMatmul(p.h, p.desc, &alpha, p.Ws[(r + 2) % p.Ws.size()], p.la, p.X, p.lb, &beta, p.Y, p.lc, p.Y, p.lc,
                    algo, p.ws, p.wsz, p.s);
    CK(hipEventRecord(e1, p.s));
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

static std::vector<std::string> split(const std::string& s, char c) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, c))
    if (!item.empty()) out.push_back(item);
  return out;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: blaslt_tune NxK[,NxK...] M[,M...]\n");
    return 2;
  }
  std::vector<std::pair<int, int>> shapes;
  for (auto& t : split(argv[1], ',')) {
    const auto nk = split(t, 'x');
    shapes.emplace_back(atoi(nk[0].c_str()), atoi(nk[1].c_str()));
  }
  std::vector<int> Ms;
  for (auto& t : split(argv[2], ',')) Ms.push_back(atoi(t.c_str()));

  Prob p;
  CK(hipblasLtCreate(&p.h));
  CK(hipStreamCreate(&p.s));
  p.wsz = 64ull << 20;  // the runtime's workspace (csrc/kernels/blaslt.hip)
  CK(hipMalloc(&p.ws, p.wsz));
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  for (auto [N, K] : shapes) {
    const size_t wbytes = (size_t)N * K * 2;
    p.Ws.assign(std::max<int>(2, (int)((1ull << 30) / wbytes) + 1), nullptr);
    for (size_t i = 0; i < p.Ws.size(); ++i) {
      CK(hipMalloc(&p.Ws[i], wbytes));
      fill_random(p.Ws[i], wbytes, 7 + (unsigned)i);
    }
    for (int M : Ms) {
      CK(hipMalloc(&p.X, (size_t)M * K * 2));
      fill_random(p.X, (size_t)M * K * 2, 3);
      CK(hipMalloc(&p.Y, (size_t)M * N * 2));
      CK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
      CK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
      CK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
      CK(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, K));
      CK(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, K));
      CK(hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, N, M, N));
      hipblasLtMatmulPreference_t pref;
      CK(hipblasLtMatmulPreferenceCreate(&pref));
      uint64_t wl = p.wsz;
      CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wl, sizeof(wl)));
      hipblasLtMatmulHeuristicResult_t heur[1];
      int got = 0;
      CK(hipblasLtMatmulAlgoGetHeuristic(p.h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, heur, &got));
      const float t_def = got ? time_algo(p, &heur[0].algo, 11) : -1.f;
      const int def_idx = got ? hipblaslt_ext::getIndexFromAlgo(heur[0].algo) : -1;
      std::vector<hipblasLtMatmulHeuristicResult_t> all;
      hipblaslt_ext::getAllAlgos(p.h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, HIP_R_16BF, HIP_R_16BF,
                                 HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all);
      std::vector<std::pair<float, size_t>> screen;
      for (size_t i = 0; i < all.size(); ++i) {
        size_t need = 0;
        const float one = 1.f, zero = 0.f;
        if (hipblaslt_ext::matmulIsAlgoSupported(p.h, p.desc, &one, p.la, p.lb, &zero, p.lc, p.lc, all[i].algo,
                                                 need) != 0 ||
            need > p.wsz)
          continue;
        const float t = time_algo(p, &all[i].algo, 3);
        if (t > 0) screen.emplace_back(t, i);
        if (screen.size() % 500 == 0) {
          fprintf(stderr, "%dx%d M=%d: %zu screened\n", N, K, M, screen.size());
          fflush(stderr);
        }
      }
      std::sort(screen.begin(), screen.end());
      float best = t_def;
      int best_idx = def_idx;
      for (size_t j = 0; j < screen.size() && j < 6; ++j) {
        const float t = time_algo(p, &all[screen[j].second].algo, 11);
        if (t > 0 && t < best) {
          best = t;
          best_idx = hipblaslt_ext::getIndexFromAlgo(all[screen[j].second].algo);
        }
      }
      printf("{\"N\": %d, \"K\": %d, \"M\": %d, \"out\": \"bf16\", \"index\": %d, \"us\": %.2f, \"default_index\": %d, "
             "\"default_us\": %.2f, \"supported\": %zu}\n",
             N, K, M, best_idx, best, def_idx, t_def, screen.size());
      fflush(stdout);
      CK(hipblasLtMatmulPreferenceDestroy(pref));
      CK(hipblasLtMatrixLayoutDestroy(p.la));
      CK(hipblasLtMatrixLayoutDestroy(p.lb));
      CK(hipblasLtMatrixLayoutDestroy(p.lc));
      CK(hipblasLtMatmulDescDestroy(p.desc));
      CK(hipFree(p.X));
      CK(hipFree(p.Y));
    }
    for (auto& w : p.Ws) CK(hipFree(w));
  }
  CK(hipFree(p.ws));
  CK(hipblasLtDestroy(p.h));
  return 0;
}
