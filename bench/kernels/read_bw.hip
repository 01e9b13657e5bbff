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

// Register loads with the non-temporal policy (aux nt): the same stream, once-read bytes
template <int U>
__global__ __launch_bounds__(256) void read_nt_kernel(const uint4* __restrict__ w, long long n16_per_wave,
                                                      unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const u32x4_t* p = reinterpret_cast<const u32x4_t*>(w) + wave * n16_per_wave + lane;
  unsigned acc = 0;
  for (long long i = 0; i < n16_per_wave; i += 64 * U) {
    u32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + i + 64 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// LDS-DMA stream: each wave keeps R 1-KB DMAs (global_load_lds, 16 B per lane) in flight through a private
// R-slot LDS ring and folds every landed slot (ds_read_b128); AUX 0 = default policy, 2 = non-temporal
template <int R, int AUX>
__global__ __launch_bounds__(256) void read_lds_kernel(const uint4* __restrict__ w, long long n16_per_wave,
                                                       unsigned* __restrict__ sink) {
  __shared__ __attribute__((aligned(1024))) uint4 ring[4][R][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long long wave = (long long)blockIdx.x * 4 + wid;
  const uint4* p = w + wave * n16_per_wave + lane;
  const long long nch = n16_per_wave / 64;  // 1 KB chunks of this wave
  auto dma = [&](long long c, int slot) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + c * 64),
                                     (__attribute__((address_space(3))) void*)&ring[wid][slot][0], 16, 0, AUX);
  };
#pragma unroll
  for (int r = 0; r < R; ++r) dma(r, r);
  unsigned acc = 0;
  for (long long c = 0; c < nch; ++c) {
    const int slot = (int)(c % R);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R - 1) : "memory");  // chunk c landed (R - 1 younger in flight)
    const uint4 v = ring[wid][slot][lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");              // slot read before it is refilled
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
    dma(c + R < nch ? c + R : c, slot);  // (past the end: a harmless re-read keeps the vmcnt arithmetic)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x12345678u) sink[0] = acc;
}

// Buffer loads (raw_buffer_load_b128) with an explicit cache-policy operand (gfx950 CPol bits: 1 = sc0,
// 2 = nt, 16 = sc1): which policy streams once-read weights fastest
template <int U, int AUX>
__global__ __launch_bounds__(256) void read_buf_kernel(const uint4* __restrict__ w, long long n16_per_wave,
                                                       unsigned* __restrict__ sink, long long bytes) {
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(w), (short)0,
                                                                       (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL),
                                                                       0x00020000);
  const long long base = (wave * n16_per_wave + lane) * 16;
  unsigned acc = 0;
  for (long long i = 0; i < n16_per_wave; i += 64 * U) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(base + (i + 64 * u) * 16), 0, AUX);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int run_read_buf(const void* w, long long bytes, int waves, int aux, void* sink, hipStream_t s) {
  const long long per_wave = bytes / 16 / waves;
  const int blocks = waves / 4;
  const uint4* wp = (const uint4*)w;
  switch (aux) {
    case 0: read_buf_kernel<8, 0><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink, bytes); break;
    case 1: read_buf_kernel<8, 1><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink, bytes); break;
    case 2: read_buf_kernel<8, 2><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink, bytes); break;
    case 3: read_buf_kernel<8, 3><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink, bytes); break;
    case 16: read_buf_kernel<8, 16><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink, bytes); break;
    case 17: read_buf_kernel<8, 17><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink, bytes); break;
    case 18: read_buf_kernel<8, 18><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink, bytes); break;
    default: read_buf_kernel<8, 19><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink, bytes); break;
  }
  return (int)hipGetLastError();
}

extern "C" int run_read_variant(const void* w, long long bytes, int waves, int variant, void* sink, hipStream_t s) {
  const long long per_wave = bytes / 16 / waves;
  const int blocks = waves / 4;
  const uint4* wp = (const uint4*)w;
  switch (variant) {
    case 0: read_kernel<8><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink); break;
    case 1: read_nt_kernel<8><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink); break;
    case 2: read_lds_kernel<8, 0><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink); break;
    case 3: read_lds_kernel<8, 2><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink); break;
    case 4: read_lds_kernel<16, 2><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink); break;
    case 5: read_lds_kernel<16, 0><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink); break;
    default: read_nt_kernel<16><<<blocks, 256, 0, s>>>(wp, per_wave, (unsigned*)sink); break;
  }
  return (int)hipGetLastError();
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
