// K7: SwiGLU, out[t][f] = silu(gu[t][f]) * gu[t][F + f], gate and up
// concatenated along N by the fused gate_up projection.  Consumes a LinOut,
// so the split-K slabs of the decode gate_up GEMM are summed here.
// Memory bound: 8 elements (16 B of bf16 output) per lane per item.
#include "common.h"
#include "launchers.h"

namespace {

__global__ __launch_bounds__(256) void swiglu_kernel(LinOut gu, bf16* __restrict__ out, int T, int F, int ilv) {
  const long long items = (long long)T * (F / 8);
  for (long long it = blockIdx.x * 256LL + threadIdx.x; it < items; it += (long long)gridDim.x * 256) {
    const long long t = it / (F / 8);
    const int f0 = (int)(it % (F / 8)) * 8;
    float g[8], u[8];
    // ilv: gate/up interleaved per 16 columns (decode layout): gate f0.. at 2*f0, up at 2*f0 + 8
    linout_load8(gu, t * 2 * F + (ilv ? 2 * f0 : f0), g);
    linout_load8(gu, t * 2 * F + (ilv ? 2 * f0 + 8 : F + f0), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = silu(g[j]) * u[j];
    store8(out + t * F + f0, g);
  }
}

}  // namespace

void launch_swiglu(LinOut gu, bf16* out, int T, int F, hipStream_t s, int interleaved) {
  const long long items = (long long)T * (F / 8);
  if (items == 0) return;
  const int grid = (int)std::min<long long>((items + 255) / 256, 2048);
  swiglu_kernel<<<grid, 256, 0, s>>>(gu, out, T, F, interleaved);
}
