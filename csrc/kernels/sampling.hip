// K6 (filtered): temperature + top-k + top-p (nucleus) sampling over full-vocabulary fp32 logits.
//
// The fused decode path samples greedy / plain-temperature rows inside the lm_head GEMM epilogue
// (decode_gemm.hip, DECODE_EPI_ARGMAX).  Rows that ask for top-k or top-p need the whole row, so the
// engine materialises their logits and this kernel resamples exactly those rows:
//
//   one 1024-thread workgroup per row (wave64 x 16), the row read from L2 a few times:
//   1. m = max(l), Z = sum exp((l - m) / t)                         (block reductions)
//   2. radix select, 4 passes x 8 bits over order-preserving uint32 keys of l, descending:
//        top-k: the key of the k-th largest logit;
//        top-p: the key at which the descending cumulative mass first reaches top_p * Z
//      per pass an LDS histogram of counts and of mass (exp((l - m) / t)) over the candidates that
//      share the prefix found so far; one lane scans the 256 bins from the top.
//   3. Gumbel-max over the kept set {key >= max(k_key, p_key)} with the same counter-based RNG
//      and counter (global vocab index) as the fused kernel, so a row is reproducible by seed.
// Rows with t == 0 (greedy: the argmax is always inside the kept set) or with neither filter are
// left untouched.  Graph-capturable: no host sync, no allocation.
#include "common.h"
#include "launchers.h"

namespace {

constexpr int NT = 1024;

SYM_DEV uint32_t okey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

SYM_DEV float block_max1024(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  return r;
}

SYM_DEV float block_sum1024(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  return r;
}

// Radix select of the threshold key.  mode 0: by count (target = k), mode 1: by mass (target = P).
SYM_DEV uint32_t radix_threshold(const float* __restrict__ row, int V, float m, float inv_t, int mode, float target,
                                 int* cnt, float* mass, uint32_t* s_prefix, float* s_target) {
  uint32_t prefix = 0, mask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += NT) {
      cnt[i] = 0;
      mass[i] = 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += NT) {
      const float l = row[i];
      const uint32_t k = okey(l);
      if ((k & mask) == prefix) {
        const int d = (k >> shift) & 255;
        if (mode == 0)
          atomicAdd(&cnt[d], 1);
        else
          atomicAdd(&mass[d], __expf((l - m) * inv_t));
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float acc = 0.f;
      int d = 255;
      for (; d > 0; --d) {
        const float b = mode == 0 ? (float)cnt[d] : mass[d];
        if (acc + b >= target) break;
        acc += b;
      }
      *s_prefix = prefix | ((uint32_t)d << shift);
      *s_target = target - acc;
    }
    __syncthreads();
    prefix = *s_prefix;
    target = *s_target;
    mask |= 255u << shift;
  }
  return prefix;
}

__global__ __launch_bounds__(NT) void sample_filtered_kernel(const float* __restrict__ logits, int V,
                                                             const float* __restrict__ temps,
                                                             const int* __restrict__ top_k,
                                                             const float* __restrict__ top_p,
                                                             const long long* __restrict__ seeds,
                                                             const long long* __restrict__ step,
                                                             int* __restrict__ out_ids) {
  const int r = blockIdx.x;
  const float t = temps[r];
  const int k = top_k[r];
  const float p = top_p[r];
  const bool use_k = k > 0 && k < V, use_p = p < 1.f;
  if (t <= 0.f || !(use_k || use_p)) return;  // uniform over the workgroup
  const float* row = logits + (long long)r * V;
  const float inv_t = 1.f / t;

  __shared__ float red[NT / 64];
  __shared__ int cnt[256];
  __shared__ float mass[256];
  __shared__ uint32_t s_prefix;
  __shared__ float s_target;
  __shared__ unsigned long long s_best[NT / 64];

  float lm = -INFINITY;
  for (int i = threadIdx.x; i < V; i += NT) lm = fmaxf(lm, row[i]);
  const float m = block_max1024(lm, red);

  uint32_t thr = 0;
  if (use_k) thr = radix_threshold(row, V, m, inv_t, 0, (float)k, cnt, mass, &s_prefix, &s_target);
  if (use_p) {
    float z = 0.f;
    for (int i = threadIdx.x; i < V; i += NT) z += __expf((row[i] - m) * inv_t);
    const float Z = block_sum1024(z, red);
    const uint32_t pk = radix_threshold(row, V, m, inv_t, 1, fmaxf(p, 0.f) * Z, cnt, mass, &s_prefix, &s_target);
    thr = thr > pk ? thr : pk;
  }

  // Gumbel-max over the kept set; same RNG stream as the fused lm_head epilogue.
  const unsigned long long seed = (unsigned long long)seeds[r] ^ ((unsigned long long)step[0] << 20);
  unsigned long long best = 0;
  for (int i = threadIdx.x; i < V; i += NT) {
    const float l = row[i];
    if (okey(l) < thr) continue;
    const float u = uniform01(seed, (unsigned long long)i);
    const float v = l * inv_t - __logf(-__logf(u));
    const unsigned long long key = ((unsigned long long)okey(v) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)i);
    best = key > best ? key : best;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long b = __shfl_xor(best, o, 64);
    best = b > best ? b : best;
  }
  if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = s_best[0];
    for (int i = 1; i < NT / 64; ++i) b = s_best[i] > b ? s_best[i] : b;
    out_ids[r] = (int)(0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull));
  }
}

// Greedy / plain-temperature sampling over materialised fp32 logits [B, V], for decode batches wider
// than the fused lm_head kernels take (> 64 rows; the logits come from one library GEMM).  Same packed
// key (order-preserving value bits, ~global vocab index: the smallest index wins a tie) and the same
// counter-based Gumbel noise, v / t - log(-log(u)), as the fused epilogue (skinny_gemm.hip), so a row
// samples the same token whichever path its batch took.  One workgroup per row, the row read once.
__global__ __launch_bounds__(NT) void logits_argmax_kernel(const float* __restrict__ logits, int V,
                                                           const float* __restrict__ temps,
                                                           const long long* __restrict__ seeds,
                                                           const long long* __restrict__ step, int n_offset,
                                                           unsigned long long* __restrict__ out_keys,
                                                           int* __restrict__ out_ids) {
  __shared__ unsigned long long s_best[NT / 64];
  const int r = blockIdx.x;
  const float t = temps[r];
  const float* row = logits + (long long)r * V;
  const unsigned long long seed = (unsigned long long)seeds[r] ^ ((unsigned long long)step[0] << 20);
  unsigned long long best = 0;
  for (int i = threadIdx.x; i < V; i += NT) {
    const uint32_t g = (uint32_t)(n_offset + i);
    float v = row[i];
    if (t > 0.f) v = v / t - __logf(-__logf(uniform01(seed, (unsigned long long)g)));
    const unsigned long long key = ((unsigned long long)okey(v) << 32) | (unsigned long long)(0xFFFFFFFFu - g);
    best = key > best ? key : best;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long b = __shfl_xor(best, o, 64);
    best = b > best ? b : best;
  }
  if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = s_best[0];
    for (int i = 1; i < NT / 64; ++i) b = s_best[i] > b ? s_best[i] : b;
    out_keys[r] = b;
    out_ids[r] = (int)(0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull));
  }
}

}  // namespace

void launch_logits_argmax(const float* logits, int B, int V, const float* temps, const long long* seeds,
                          const long long* step, int n_offset, unsigned long long* out_keys, int* out_ids,
                          hipStream_t s) {
  if (B == 0) return;
  logits_argmax_kernel<<<B, NT, 0, s>>>(logits, V, temps, seeds, step, n_offset, out_keys, out_ids);
}

void launch_sample_filtered(const float* logits, int B, int V, const float* temps, const int* top_k, const float* top_p,
                            const long long* seeds, const long long* step, int* out_ids, hipStream_t s) {
  if (B == 0) return;
  sample_filtered_kernel<<<B, NT, 0, s>>>(logits, V, temps, top_k, top_p, seeds, step, out_ids);
}
