// Shared device helpers for the symmetry_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64: all cross-lane reductions span 64 lanes (__shfl_xor over 32..1).
//   * bf16 storage is clang's native __bf16; f32 <-> bf16 conversion lowers to
//     v_cvt_pk_bf16_f32 on gfx950 (NaN preserving, RNE).
//   * memory-bound kernels move 16 B per lane per access (8 x bf16 / 4 x f32).
//   * MFMA operand/accumulator types for v_mfma_f32_16x16x32_bf16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define SYM_DEV __device__ __forceinline__

constexpr int kWave = 64;

// v_mfma_f32_16x16x32_bf16: C[16x16] += A[16x32] . B[32x16] (fragment layout: cdna_hip_programming.md §3)
SYM_DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

SYM_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

SYM_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `scratch` holds NT/64 floats.
template <int NT>
SYM_DEV float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += scratch[i];
  __syncthreads();
  return r;
}

// 16-byte vector of 8 bf16 <-> 8 floats.
union Pack8 {
  uint4 u;
  u32x4 w;
  bf16x8 v;
  bf16 h[8];
};

SYM_DEV void load8(const bf16* p, float* f) {
  Pack8 pk;
  pk.u = *reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)pk.h[i];
}

// Non-temporal 16-byte load (streamed-once weights: MI355X_MICROARCH.md row nt-weights).
SYM_DEV u32x4 ld_nt16(const bf16* p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)); }

SYM_DEV void store8(bf16* p, const float* f) {
  Pack8 pk;
#pragma unroll
  for (int i = 0; i < 8; ++i) pk.h[i] = (bf16)f[i];
  *reinterpret_cast<uint4*>(p) = pk.u;
}

SYM_DEV void load8f(const float* p, float* f) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

SYM_DEV void store8f(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}

// A "linear output" as produced by a projection: either a bf16 tensor [T][N]
// (library GEMM, prefill) or `nsplit` fp32 split-K partial slabs [S][T][N]
// produced by the skinny decode GEMM.  Consumers sum the slabs in their
// prologue (the launch-boundary reduce), so no separate reduce kernel runs.
struct LinOut {
  const void* ptr;
  int is_f32;          // 0: bf16 [T][N]; 1: fp32 [S][T][N]
  int nsplit;          // number of fp32 slabs (1 for bf16)
  long long split_stride;  // elements between slabs (T*N)
};

SYM_DEV void linout_load8(const LinOut& L, long long off, float* f) {
  if (L.is_f32) {
    const float* p = reinterpret_cast<const float*>(L.ptr) + off;
    load8f(p, f);
    for (int s = 1; s < L.nsplit; ++s) {
      float g[8];
      load8f(p + s * L.split_stride, g);
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] += g[i];
    }
  } else {
    load8(reinterpret_cast<const bf16*>(L.ptr) + off, f);
  }
}

SYM_DEV float linout_load1(const LinOut& L, long long off) {
  if (L.is_f32) {
    const float* p = reinterpret_cast<const float*>(L.ptr) + off;
    float r = p[0];
    for (int s = 1; s < L.nsplit; ++s) r += p[s * L.split_stride];
    return r;
  }
  return (float)reinterpret_cast<const bf16*>(L.ptr)[off];
}

SYM_DEV float silu(float x) { return x / (1.f + __expf(-x)); }

// Counter-based RNG (7 Philox-style multiply/xor rounds over a 64-bit key and
// a 64-bit counter), used by the sampler's Gumbel-max path so a decode step
// is graph-capturable: the step counter lives in device memory.  Bit-exact
// torch port: symmetry_amd/ops/reference.py::uniform01.
SYM_DEV float uniform01(uint64_t seed, uint64_t counter) {
  uint32_t x0 = (uint32_t)counter, x1 = (uint32_t)(counter >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    uint64_t p0 = (uint64_t)x0 * 0xD2511F53u;
    uint64_t p1 = (uint64_t)x1 * 0xCD9E8D57u;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ k0 ^ (uint32_t)p0;
    uint32_t n1 = (uint32_t)(p0 >> 32) ^ k1 ^ (uint32_t)p1;
    x0 = n0; x1 = n1;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  // 24 high-quality bits -> (0, 1)
  return ((x0 >> 8) + 0.5f) * (1.0f / 16777216.0f);
}
