// K9: skinny (decode) GEMM on MFMA, y = x . W^T with x [M][K] (M <= 64), W [N][K] bf16.
//
// Decode GEMMs are weight-streaming: every weight byte is read exactly once
// per step, so the kernel is built around the HBM stream.  The product is
// computed transposed, Y^T[n][m] = W[n][:] . x[m][:], with W as the MFMA A
// operand (v_mfma_f32_16x16x32_bf16: 16 weight rows x 16 batch columns per
// instruction).  A k permutation makes each lane read 32 contiguous bytes of
// its weight row per 64-deep k block (4 lanes cover one 128-B line), x is
// read with the same permutation from L2 (it is tiny and shared by all
// workgroups).  Batch columns >= M are clamped loads whose results are
// dropped.
//
// Decomposition: one 256-thread workgroup (4 waves) per 16-row tile and
// k split; the 4 waves split the workgroup's k range and are summed through
// LDS.  Across workgroups the k split S writes fp32 partial slabs
// y[S][M][N] that the consumer kernel (norm / rope / swiglu) sums in its
// prologue -- no extra reduce launch (cdna_hip_programming.md §5, "combine
// in the NEXT kernel's prologue").  S is chosen on the host so the grid has
// ~1024 workgroups (4 per CU) while keeping >= 2 k blocks per wave.
//
// Epilogue EPI_ARGMAX (lm_head, S == 1): instead of logits the kernel emits
// per-(row, tile) packed 64-bit keys (order-preserving float bits << 32 |
// ~index) of logit/temperature + Gumbel noise (temperature > 0) or the raw
// logit (greedy); argmax_reduce picks the max key per row.  Sampling is thus
// fused into the lm_head weight stream.  Vocab-parallel TP passes n_offset so
// keys carry global token ids and ranks combine with one MAX all-reduce.
#include "common.h"
#include "launchers.h"

namespace {

constexpr int NT = 256;

SYM_DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

SYM_DEV uint32_t ordered_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

SYM_DEV unsigned long long pack_key(float v, uint32_t idx) {
  return ((unsigned long long)ordered_bits(v) << 32) | (unsigned long long)(0xFFFFFFFFu - idx);
}

template <int MT, int U, int EPI>
__global__ __launch_bounds__(NT) void skinny_gemm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ W,
                                                         float* __restrict__ y, int M, int N, int K, int kchunk,
                                                         const float* __restrict__ temps,
                                                         const unsigned long long* __restrict__ seeds,
                                                         const long long* __restrict__ step_ctr,
                                                         unsigned long long* __restrict__ keys, int n_offset,
                                                         int ntiles) {
  const int tile = blockIdx.x, split = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int n0 = tile * 16;
  const int wk = kchunk / 4;  // k range of one wave
  const int kbeg = split * kchunk + wid * wk;
  const int nblk = wk / 64;

  const bf16* wrow = W + (long long)(n0 + r16) * K + kbeg + 16 * h;
  const bf16* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int mrow = min(16 * mt + r16, M - 1);
    xrow[mt] = x + (long long)mrow * K + kbeg + 16 * h;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  int b = 0;
  for (; b + U <= nblk; b += U) {
    Pack8 wa[U][2], xa[U][MT][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ko = (b + u) * 64;
      wa[u][0].w = ld_nt16(wrow + ko);
      wa[u][1].w = ld_nt16(wrow + ko + 8);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        xa[u][mt][0].u = *reinterpret_cast<const uint4*>(xrow[mt] + ko);
        xa[u][mt][1].u = *reinterpret_cast<const uint4*>(xrow[mt] + ko + 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[mt] = mfma16(wa[u][0].v, xa[u][mt][0].v, acc[mt]);
        acc[mt] = mfma16(wa[u][1].v, xa[u][mt][1].v, acc[mt]);
      }
  }
  for (; b < nblk; ++b) {
    const int ko = b * 64;
    Pack8 w0, w1;
    w0.w = ld_nt16(wrow + ko);
    w1.w = ld_nt16(wrow + ko + 8);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      Pack8 x0, x1;
      x0.u = *reinterpret_cast<const uint4*>(xrow[mt] + ko);
      x1.u = *reinterpret_cast<const uint4*>(xrow[mt] + ko + 8);
      acc[mt] = mfma16(w0.v, x0.v, acc[mt]);
      acc[mt] = mfma16(w1.v, x1.v, acc[mt]);
    }
  }

  // Sum the 4 waves' partial tiles through LDS.
  __shared__ f32x4 red[4][MT][64];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) red[wid][mt][lane] = acc[mt];
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt] = red[0][mt][lane] + red[1][mt][lane] + red[2][mt][lane] + red[3][mt][lane];
  }
  // lane (c = r16, h): rows n0 + 4h + i (i = 0..3), column m = 16 mt + c.
  if constexpr (EPI == 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + r16;
      if (m < M) {
        float* yp = y + ((long long)split * M + m) * N + n0 + 4 * h;
        *reinterpret_cast<float4*>(yp) = make_float4(acc[mt][0], acc[mt][1], acc[mt][2], acc[mt][3]);
      }
    }
  } else {
    const long long step = step_ctr ? *step_ctr : 0;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + r16;
      const bool mok = m < M;
      const int mm = mok ? m : 0;
      const float t = temps ? temps[mm] : 0.f;
      unsigned long long best = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int gidx = n_offset + n0 + 4 * h + i;
        float v = acc[mt][i];
        if (y && mok) y[(long long)m * N + n0 + 4 * h + i] = v;
        if (t > 0.f) {
          const unsigned long long seed = seeds ? seeds[mm] : 0ull;
          const float u = uniform01(seed ^ ((unsigned long long)step << 20), (unsigned long long)gidx);
          v = v / t - __logf(-__logf(u));
        }
        const unsigned long long kk = pack_key(v, (uint32_t)gidx);
        best = kk > best ? kk : best;
      }
      // reduce over the 4 lane groups (same column)
      unsigned long long o16 = __shfl_xor(best, 16, 64);
      best = o16 > best ? o16 : best;
      unsigned long long o32 = __shfl_xor(best, 32, 64);
      best = o32 > best ? o32 : best;
      if (h == 0 && mok) keys[(long long)m * ntiles + tile] = best;
    }
  }
}

__global__ __launch_bounds__(256) void argmax_reduce_kernel(const unsigned long long* __restrict__ keys, int ntiles,
                                                            unsigned long long* __restrict__ out_keys,
                                                            int* __restrict__ out_ids) {
  const int m = blockIdx.x;
  const unsigned long long* k = keys + (long long)m * ntiles;
  unsigned long long best = 0;
  for (int i = threadIdx.x; i < ntiles; i += 256) best = k[i] > best ? k[i] : best;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long v = __shfl_xor(best, o, 64);
    best = v > best ? v : best;
  }
  __shared__ unsigned long long sm[4];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) best = sm[i] > best ? sm[i] : best;
    if (out_keys) out_keys[m] = best;
    if (out_ids) out_ids[m] = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
  }
}

template <int MT, int EPI>
void launch_mt(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, const float* temps,
               const unsigned long long* seeds, const long long* step, unsigned long long* keys, int n_offset,
               hipStream_t s) {
  const int ntiles = N / 16;
  const int kchunk = K / S;
  dim3 grid(ntiles, S);
  constexpr int U = MT == 1 ? 4 : (MT == 2 ? 2 : 1);
  skinny_gemm_kernel<MT, U, EPI>
      <<<grid, NT, 0, s>>>(x, W, y, M, N, K, kchunk, temps, seeds, step, keys, n_offset, ntiles);
}

template <int EPI>
void launch_epi(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, const float* temps,
                const unsigned long long* seeds, const long long* step, unsigned long long* keys, int n_offset,
                hipStream_t s) {
  const int mt = (M + 15) / 16;
  switch (mt) {
    case 1: launch_mt<1, EPI>(x, W, y, M, N, K, S, temps, seeds, step, keys, n_offset, s); break;
    case 2: launch_mt<2, EPI>(x, W, y, M, N, K, S, temps, seeds, step, keys, n_offset, s); break;
    case 3: launch_mt<3, EPI>(x, W, y, M, N, K, S, temps, seeds, step, keys, n_offset, s); break;
    default: launch_mt<4, EPI>(x, W, y, M, N, K, S, temps, seeds, step, keys, n_offset, s); break;
  }
}

}  // namespace

void launch_skinny_gemm(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, hipStream_t s) {
  launch_epi<0>(x, W, y, M, N, K, S, nullptr, nullptr, nullptr, nullptr, 0, s);
}

void launch_skinny_gemm_argmax(const bf16* x, const bf16* W, float* logits_or_null, int M, int N, int K,
                               const float* temps, const unsigned long long* seeds, const long long* step,
                               unsigned long long* tile_keys, int n_offset, hipStream_t s) {
  launch_epi<1>(x, W, logits_or_null, M, N, K, 1, temps, seeds, step, tile_keys, n_offset, s);
}

void launch_argmax_reduce(const unsigned long long* tile_keys, int M, int ntiles, unsigned long long* out_keys,
                          int* out_ids, hipStream_t s) {
  argmax_reduce_kernel<<<M, 256, 0, s>>>(tile_keys, ntiles, out_keys, out_ids);
}
