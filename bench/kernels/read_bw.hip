// Read-bandwidth probe for the decode weight stream (no MFMA): each wave streams its slice of a
// preshuffled weight (1 KB per load instruction, U loads in flight) and folds it into a checksum.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC read_bw.hip -o read_bw.so ; driven by read_bw.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int U>
__global__ __launch_bounds__(256) void read_kernel(const uint4* __restrict__ w, long long n16_per_wave,
                                                   unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint4* p = w + wave * n16_per_wave + lane;
  unsigned acc = 0;
  for (long long i = 0; i < n16_per_wave; i += 64 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[i + 64 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads live
}

extern "C" int run_read(const void* w, long long bytes, int waves, int u, void* sink, hipStream_t s) {
  const long long per_wave = bytes / 16 / waves;
  const int blocks = waves / 4;
  switch (u) {
    case 2: read_kernel<2><<<blocks, 256, 0, s>>>((const uint4*)w, per_wave, (unsigned*)sink); break;
    case 4: read_kernel<4><<<blocks, 256, 0, s>>>((const uint4*)w, per_wave, (unsigned*)sink); break;
    case 8: read_kernel<8><<<blocks, 256, 0, s>>>((const uint4*)w, per_wave, (unsigned*)sink); break;
    default: read_kernel<16><<<blocks, 256, 0, s>>>((const uint4*)w, per_wave, (unsigned*)sink); break;
  }
  return (int)hipGetLastError();
}
