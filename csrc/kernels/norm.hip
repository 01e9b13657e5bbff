// K1: RMSNorm with fused residual add / embedding gather / split-K reduce.
//
//   mode 0 (norm):      out = rmsnorm(x) * w                 x: LinOut (bf16 or fp32 slabs)
//   mode 1 (add_norm):  residual += delta; out = rmsnorm(residual) * w
//   mode 2 (embed_norm): residual = table[tok]; out = rmsnorm(residual) * w, tok = src[row] >= 0 ?
//                        prev[src[row]] : ids[row] (src/prev optional: a pipelined decode row's token is the
//                        previous step's on-device sample)
//
// The residual stream is kept in fp32 ([T][d]) for accuracy; activations fed
// to the projections are bf16.  One 256-thread workgroup per row, 16 B per
// lane per access (8 bf16 / 2x4 fp32), the row held in registers between the
// sum-of-squares and the scale pass, so each byte is read once (memory bound:
// SURVEY.md §2.6 K1).  The split-K partial slabs of the skinny decode GEMM are
// summed here, which removes the GEMM's own reduce launch.
#include <stdlib.h>

#include "common.h"
#include "launchers.h"

namespace {

template <int NT, int MAXV, int MODE>
__global__ __launch_bounds__(NT) void rms_norm_kernel(LinOut x, const int* __restrict__ ids,
                                                      const bf16* __restrict__ table,
                                                      float* __restrict__ residual,
                                                      const bf16* __restrict__ w,
                                                      bf16* __restrict__ out, int d, float eps,
                                                      const int* __restrict__ src, const int* __restrict__ prev) {
  __shared__ float scratch[NT / 64];
  const int row = blockIdx.x;
  const int nvec = d >> 3;
  const long long rbase = (long long)row * d;
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = threadIdx.x + k * NT;
    if (vi < nvec) {
      const long long off = rbase + vi * 8;
      if constexpr (MODE == 0) {
        linout_load8(x, off, v[k]);
      } else if constexpr (MODE == 1) {
        float r[8];
        load8f(residual + off, r);
        linout_load8(x, off, v[k]);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[k][i] += r[i];
        store8f(residual + off, v[k]);
      } else {
        const int sr = src ? src[row] : -1;
        const long long tok = sr >= 0 ? prev[sr] : ids[row];
        load8(table + tok * d + vi * 8, v[k]);
        store8f(residual + off, v[k]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[k][i] * v[k][i];
    }
  }
  ss = block_sum<NT>(ss, scratch);
  const float inv = rsqrtf(ss / (float)d + eps);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = threadIdx.x + k * NT;
    if (vi < nvec) {
      float g[8];
      load8(w + vi * 8, g);
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] *= v[k][i] * inv;
      store8(out + rbase + vi * 8, g);
    }
  }
}

template <int MODE>
void launch_mode(LinOut x, const int* ids, const bf16* table, float* residual, const bf16* w, bf16* out,
                 int T, int d, float eps, hipStream_t s, const int* src = nullptr, const int* prev = nullptr) {
  constexpr int NT = 256;
  const int nvec = d / 8;
  dim3 grid(T);
  // rows of <= 4096 elements: 512 threads per row, one 8-element vector each (64-client decode step
  // 4.680 -> 4.608 ms, profiles/norm_wide_ab_r2.jsonl); SYMMETRY_NORM_WIDE=0: 256 threads, 2 vectors
  static const bool wide = [] {
    const char* e = getenv("SYMMETRY_NORM_WIDE");
    return !(e && e[0] == '0');
  }();
  if (wide && nvec <= 512) {
    rms_norm_kernel<512, 1, MODE><<<grid, 512, 0, s>>>(x, ids, table, residual, w, out, d, eps, src, prev);
  } else if (nvec <= NT * 2) {
    rms_norm_kernel<NT, 2, MODE><<<grid, NT, 0, s>>>(x, ids, table, residual, w, out, d, eps, src, prev);
  } else if (nvec <= NT * 4) {
    rms_norm_kernel<NT, 4, MODE><<<grid, NT, 0, s>>>(x, ids, table, residual, w, out, d, eps, src, prev);
  } else {
    rms_norm_kernel<NT, 8, MODE><<<grid, NT, 0, s>>>(x, ids, table, residual, w, out, d, eps, src, prev);
  }
}

}  // namespace

void launch_rms_norm(LinOut x, const bf16* w, bf16* out, int T, int d, float eps, hipStream_t s) {
  launch_mode<0>(x, nullptr, nullptr, nullptr, w, out, T, d, eps, s);
}

void launch_add_rms_norm(LinOut delta, float* residual, const bf16* w, bf16* out, int T, int d, float eps,
                         hipStream_t s) {
  launch_mode<1>(delta, nullptr, nullptr, residual, w, out, T, d, eps, s);
}

void launch_embed_rms_norm(const int* ids, const bf16* table, float* residual, const bf16* w, bf16* out, int T,
                           int d, float eps, hipStream_t s, const int* src, const int* prev) {
  LinOut none{nullptr, 0, 1, 0};
  launch_mode<2>(none, ids, table, residual, w, out, T, d, eps, s, src, prev);
}

// rownorm: out = xw * rsqrt(sum(ss[m][:]) / d + eps)  -- materialises a normalised activation from the
// deferred-RMSNorm residual state (xw, ss) for consumers that are not fused decode GEMMs (MoE).
namespace {
__global__ __launch_bounds__(256) void rownorm_kernel(const bf16* __restrict__ xw, const float* __restrict__ ss,
                                                      int ss_tiles, float eps, bf16* __restrict__ out, int d) {
  __shared__ float scratch[4];
  const int row = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < ss_tiles; i += 256) s += ss[(long long)row * ss_tiles + i];
  s = block_sum<256>(s, scratch);
  const float r = rsqrtf(s / (float)d + eps);
  for (int vi = threadIdx.x; vi < d / 8; vi += 256) {
    float v[8];
    load8(xw + (long long)row * d + vi * 8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= r;
    store8(out + (long long)row * d + vi * 8, v);
  }
}
}  // namespace

void launch_rownorm(const bf16* xw, const float* ss, int ss_tiles, float eps, bf16* out, int T, int d, hipStream_t s) {
  if (T == 0) return;
  rownorm_kernel<<<T, 256, 0, s>>>(xw, ss, ss_tiles, eps, out, d);
}
