// Prefill projections on hipBLASLt with a TUNED solution per (N, K, M bucket) instead of the library heuristic.
//
// y[M][N] = x[M][K] . W[N][K]^T (bf16 in, bf16 or fp32 out) as the column-major "TN" matmul m = N, n = M, k = K.
// The heuristic's first pick is 12-30 % off the best supported solution for the Llama-3-8B prefill shapes at
// 512-768 rows (profiles/r4/blaslt_layout.jsonl: o 43.3 -> 30.8 us, down 102.7 -> 86.8, qkv 50.9 -> 42.0 at 768
// rows); the per-shape best solution index comes from an offline sweep on this library build
// (bench/kernels/blaslt_tune.cpp -> symmetry_amd/ops/blaslt_table.json) and is checked against the problem
// (matmulIsAlgoSupported) on first use.  Descriptors, the resolved algorithm and a fixed workspace are cached per
// (device, problem), so a call is one hipblasLtMatmul on the caller's stream (hipGraph-capturable once the
// problem has been seen outside a capture).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "launchers.h"

namespace {

constexpr size_t kWorkspace = 64ull << 20;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool ok = false;
};

struct DevState {
  hipblasLtHandle_t handle = nullptr;
  void* ws = nullptr;
  std::map<std::tuple<int, int, int, int, int>, Plan> plans;  // (M, N, K, out_f32, algo index)
  std::vector<hipblasLtMatmulHeuristicResult_t> all_bf16, all_f32;
};

std::mutex g_mu;
std::map<int, DevState> g_dev;

DevState* dev_state() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  DevState& d = g_dev[dev];
  if (!d.handle && hipblasLtCreate(&d.handle) != HIPBLAS_STATUS_SUCCESS) return nullptr;
  if (!d.ws && hipMalloc(&d.ws, kWorkspace) != hipSuccess) {
    d.ws = nullptr;
    (void)hipGetLastError();
    return nullptr;
  }
  return &d;
}

bool make_plan(DevState& d, Plan& p, int M, int N, int K, int out_f32, int index) {
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const hipDataType tD = out_f32 ? HIP_R_32F : HIP_R_16BF;
  if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, K) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, K) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lc, tD, N, M, N) != HIPBLAS_STATUS_SUCCESS)
    return false;
  // the solution by index among every TN bf16 solution of this output type (getAlgosFromIndex alone finds
  // nothing until the library has loaded that problem type's solutions: getAllAlgos does, once per type)
  std::vector<hipblasLtMatmulHeuristicResult_t>& all = out_f32 ? d.all_f32 : d.all_bf16;
  if (all.empty())
    hipblaslt_ext::getAllAlgos(d.handle, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, HIP_R_16BF, HIP_R_16BF, tD,
                               tD, HIPBLAS_COMPUTE_32F, all);
  hipblasLtMatmulAlgo_t* found = nullptr;
  for (auto& r : all)
    if (hipblaslt_ext::getIndexFromAlgo(r.algo) == index) {
      found = &r.algo;
      break;
    }
  if (!found) {
    if (getenv("SYMMETRY_BLASLT_DEBUG")) fprintf(stderr, "blaslt: index %d not among %zu solutions\n", index, all.size());
    return false;
  }
  hipblasLtMatmulAlgo_t algo = *found;
  const float one = 1.f, zero = 0.f;
  size_t need = 0;
  const hipblasStatus_t ss =
      hipblaslt_ext::matmulIsAlgoSupported(d.handle, p.desc, &one, p.la, p.lb, &zero, p.lc, p.lc, algo, need);
  if (ss != HIPBLAS_STATUS_SUCCESS || need > kWorkspace) {
    if (getenv("SYMMETRY_BLASLT_DEBUG"))
      fprintf(stderr, "blaslt: index %d (%d x %d x %d): supported %d, workspace %zu\n", index, M, N, K, (int)ss, need);
    return false;
  }
  p.algo = algo;
  return true;
}

}  // namespace

// 0: enqueued; 1: the solution does not support this problem (the caller falls back to the library heuristic);
// -1: hipBLASLt error.
int launch_blaslt_gemm(const void* x, const void* w, void* y, int out_f32, int M, int N, int K, int algo_index,
                       hipStream_t s) {
  Plan* p = nullptr;
  DevState* d = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    d = dev_state();
    if (!d) return -1;
    auto key = std::make_tuple(M, N, K, out_f32, algo_index);
    auto it = d->plans.find(key);
    if (it == d->plans.end()) {
      Plan np;
      np.ok = make_plan(*d, np, M, N, K, out_f32, algo_index);
      it = d->plans.emplace(key, np).first;
    }
    p = &it->second;
  }
  if (!p->ok) return 1;
  const float alpha = 1.f, beta = 0.f;
  const hipblasStatus_t st = hipblasLtMatmul(d->handle, p->desc, &alpha, w, p->la, x, p->lb, &beta, y, p->lc, y, p->lc,
                                             &p->algo, d->ws, kWorkspace, s);
  return st == HIPBLAS_STATUS_SUCCESS ? 0 : -1;
}

// Offline sweep (bench/kernels/blaslt_tune.py) IN this process's hipBLASLt -- the library torch loads, whose
// solution indices are the ones launch_blaslt_gemm resolves (the /opt/rocm build numbers them differently).
// Every supported TN bf16 solution is timed over 3 calls (weights rotating over the nw copies in ws), the 6
// fastest again over 11 calls next to the heuristic's pick.  out: {best index, default index, supported count};
// us: {best, default}.  Returns 0, or -1 on a hipBLASLt / HIP error.
int blaslt_tune(const void* x, const void* const* ws, int nw, void* y, int out_f32, int M, int N, int K, int* out,
                float* us, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  DevState* d = dev_state();
  if (!d) return -1;
  Plan p;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return -1;
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const hipDataType tD = out_f32 ? HIP_R_32F : HIP_R_16BF;
  hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, K);
  hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, K);
  hipblasLtMatrixLayoutCreate(&p.lc, tD, N, M, N);
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1;
  const float alpha = 1.f, beta = 0.f;
  auto run = [&](const hipblasLtMatmulAlgo_t* algo, int r) {
    return hipblasLtMatmul(d->handle, p.desc, &alpha, ws[r % nw], p.la, x, p.lb, &beta, y, p.lc, y, p.lc, algo, d->ws,
                           kWorkspace, s);
  };
  auto timed = [&](const hipblasLtMatmulAlgo_t* algo, int reps) -> float {
    for (int i = 0; i < 2; ++i)
      if (run(algo, i) != HIPBLAS_STATUS_SUCCESS) return -1.f;
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      hipEventRecord(e0, s);
      run(algo, r + 2);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      t.push_back(ms * 1000.f);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t wl = kWorkspace;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wl, sizeof(wl));
  hipblasLtMatmulHeuristicResult_t heur[1];
  int got = 0;
  hipblasLtMatmulAlgoGetHeuristic(d->handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, heur, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  us[1] = got ? timed(&heur[0].algo, 11) : -1.f;
  out[1] = got ? hipblaslt_ext::getIndexFromAlgo(heur[0].algo) : -1;
  std::vector<hipblasLtMatmulHeuristicResult_t>& all = out_f32 ? d->all_f32 : d->all_bf16;
  if (all.empty())
    hipblaslt_ext::getAllAlgos(d->handle, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, HIP_R_16BF, HIP_R_16BF, tD,
                               tD, HIPBLAS_COMPUTE_32F, all);
  std::vector<std::pair<float, size_t>> screen;
  for (size_t i = 0; i < all.size(); ++i) {
    size_t need = 0;
    const float one = 1.f, zero = 0.f;
    if (hipblaslt_ext::matmulIsAlgoSupported(d->handle, p.desc, &one, p.la, p.lb, &zero, p.lc, p.lc, all[i].algo,
                                             need) != HIPBLAS_STATUS_SUCCESS ||
        need > kWorkspace)
      continue;
    const float t = timed(&all[i].algo, 3);
    if (t > 0) screen.emplace_back(t, i);
  }
  std::sort(screen.begin(), screen.end());
  us[0] = us[1];
  out[0] = out[1];
  for (size_t j = 0; j < screen.size() && j < 6; ++j) {
    const float t = timed(&all[screen[j].second].algo, 11);
    if (t > 0 && (us[0] < 0 || t < us[0])) {
      us[0] = t;
      out[0] = hipblaslt_ext::getIndexFromAlgo(all[screen[j].second].algo);
    }
  }
  out[2] = (int)screen.size();
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipblasLtMatrixLayoutDestroy(p.la);
  hipblasLtMatrixLayoutDestroy(p.lb);
  hipblasLtMatrixLayoutDestroy(p.lc);
  hipblasLtMatmulDescDestroy(p.desc);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
