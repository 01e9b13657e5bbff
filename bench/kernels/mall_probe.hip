// Infinity-Cache (MALL) probe for the decode step: can the idle HBM time of a latency-bound launch
// (decode attention) pull the NEXT launch's weights into the 256 MiB Infinity Cache, and how fast
// does a weight stream run when it is served from there?
//
// Kernels (each a distinct symbol so rocprofv3 --kernel-trace separates them):
//   flush_kernel     streams a large buffer (evicts W from the Infinity Cache)
//   stream_kernel    the consumer: streams W once (stand-in for the O-projection weight read)
//   spin_kernel      latency-bound stand-in for decode attention: `busy` workgroups spin for `ticks`
//                    of the 100 MHz realtime clock; with `pf_blocks` > 0 the launch carries that many
//                    extra workgroups that read W (prefetch into L2/MALL, values discarded)
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC mall_probe.hip -o mall_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int TAG>
__device__ __forceinline__ void stream_body(const uint4* __restrict__ w, long long n16, long long wave,
                                            long long nwaves, unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  unsigned acc = 0;
  // each wave takes contiguous 4 KB chunks (64 lanes x 16 B x 4 in flight), chunks strided by nwaves
  for (long long c = wave; c * 256 < n16; c += nwaves) {
    const uint4* p = w + c * 256 + lane;
    uint4 v0 = p[0], v1 = p[64], v2 = p[128], v3 = p[192];
    acc ^= v0.x ^ v1.y ^ v2.z ^ v3.w;
  }
  if (acc == 0x9e3779b9u + TAG) sink[TAG] = acc;  // keeps the loads live
}

__global__ __launch_bounds__(256) void flush_kernel(const uint4* w, long long n16, unsigned* sink) {
  const long long nw = (long long)gridDim.x * 4;
  stream_body<0>(w, n16, (long long)blockIdx.x * 4 + (threadIdx.x >> 6), nw, sink);
}

__global__ __launch_bounds__(256) void stream_kernel(const uint4* w, long long n16, unsigned* sink) {
  const long long nw = (long long)gridDim.x * 4;
  stream_body<1>(w, n16, (long long)blockIdx.x * 4 + (threadIdx.x >> 6), nw, sink);
}

__global__ __launch_bounds__(256) void spin_kernel(int busy, long long ticks, const uint4* w, long long n16,
                                                   unsigned* sink) {
  if ((int)blockIdx.x < busy) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(1);
    return;
  }
  const long long pf = (long long)(gridDim.x - busy) * 4;
  stream_body<2>(w, n16, (long long)(blockIdx.x - busy) * 4 + (threadIdx.x >> 6), pf, sink);
}

extern "C" int mp_flush(const void* w, long long bytes, int blocks, void* sink, hipStream_t s) {
  flush_kernel<<<blocks, 256, 0, s>>>((const uint4*)w, bytes / 16, (unsigned*)sink);
  return (int)hipGetLastError();
}

extern "C" int mp_stream(const void* w, long long bytes, int blocks, void* sink, hipStream_t s) {
  stream_kernel<<<blocks, 256, 0, s>>>((const uint4*)w, bytes / 16, (unsigned*)sink);
  return (int)hipGetLastError();
}

extern "C" int mp_spin(int busy, long long ticks, int pf_blocks, const void* w, long long bytes, void* sink,
                       hipStream_t s) {
  spin_kernel<<<busy + pf_blocks, 256, 0, s>>>(busy, ticks, (const uint4*)w, bytes / 16, (unsigned*)sink);
  return (int)hipGetLastError();
}
