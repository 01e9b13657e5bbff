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

// RT: 16-row weight tiles per wave (x fragments shared across them).
// NAT: natural k order (lane group h reads k 8h..8h+7 of each 32-deep MFMA step: 64 contiguous
//      bytes per row per instruction) vs the permuted order (32 contiguous bytes per lane).
// NTL: non-temporal weight loads.
template <int MT, int U, int EPI, int RT, bool NAT, bool NTL>
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
  const int n0 = tile * 16 * RT;
  const int wk = kchunk / 4;  // k range of one wave
  const int kbeg = split * kchunk + wid * wk;
  const int nblk = wk / 64;
  const int lo = NAT ? 8 * h : 16 * h;   // lane's offset inside a 64-deep k block, first MFMA
  const int hi = NAT ? 32 : 8;           // offset of the second MFMA's slice

  const bf16* wrow[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) wrow[rt] = W + (long long)(n0 + 16 * rt + r16) * K + kbeg + lo;
  const bf16* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int mrow = min(16 * mt + r16, M - 1);
    xrow[mt] = x + (long long)mrow * K + kbeg + lo;
  }
  f32x4 acc[RT][MT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto wload = [&](const bf16* p) -> u32x4 {
    if constexpr (NTL) return ld_nt16(p);
    else return *reinterpret_cast<const u32x4*>(p);
  };

  int b = 0;
  for (; b + U <= nblk; b += U) {
    Pack8 wa[U][RT][2], xa[U][MT][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ko = (b + u) * 64;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        wa[u][rt][0].w = wload(wrow[rt] + ko);
        wa[u][rt][1].w = wload(wrow[rt] + ko + hi);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        xa[u][mt][0].u = *reinterpret_cast<const uint4*>(xrow[mt] + ko);
        xa[u][mt][1].u = *reinterpret_cast<const uint4*>(xrow[mt] + ko + hi);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          acc[rt][mt] = mfma16(wa[u][rt][0].v, xa[u][mt][0].v, acc[rt][mt]);
          acc[rt][mt] = mfma16(wa[u][rt][1].v, xa[u][mt][1].v, acc[rt][mt]);
        }
  }
  for (; b < nblk; ++b) {
    const int ko = b * 64;
    Pack8 w0[RT], w1[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      w0[rt].w = wload(wrow[rt] + ko);
      w1[rt].w = wload(wrow[rt] + ko + hi);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      Pack8 x0, x1;
      x0.u = *reinterpret_cast<const uint4*>(xrow[mt] + ko);
      x1.u = *reinterpret_cast<const uint4*>(xrow[mt] + ko + hi);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        acc[rt][mt] = mfma16(w0[rt].v, x0.v, acc[rt][mt]);
        acc[rt][mt] = mfma16(w1[rt].v, x1.v, acc[rt][mt]);
      }
    }
  }

  // Sum the 4 waves' partial tiles through LDS.
  __shared__ f32x4 red[4][RT * MT][64];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wid][rt * MT + mt][lane] = acc[rt][mt];
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int i = rt * MT + mt;
      acc[rt][mt] = red[0][i][lane] + red[1][i][lane] + red[2][i][lane] + red[3][i][lane];
    }
  // lane (c = r16, h): rows n0 + 16 rt + 4h + i (i = 0..3), column m = 16 mt + c.
  if constexpr (EPI == 0) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + r16;
        if (m < M) {
          float* yp = y + ((long long)split * M + m) * N + n0 + 16 * rt + 4 * h;
          *reinterpret_cast<float4*>(yp) = make_float4(acc[rt][mt][0], acc[rt][mt][1], acc[rt][mt][2], acc[rt][mt][3]);
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
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int nl = n0 + 16 * rt + 4 * h + i;
          const int gidx = n_offset + nl;
          float v = acc[rt][mt][i];
          if (y && mok) y[(long long)m * N + nl] = v;
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

// One 1024-thread workgroup per row; each thread issues its (up to) 8 key loads of a 8K-key chunk before
// reducing them, so a Llama-3 vocabulary (8016 tile keys per row) costs one memory round trip instead of a
// chain of dependent ones (12.8 -> a few us per decode step at 10 rows).
constexpr int AR_NT = 1024, AR_U = 8;

__global__ __launch_bounds__(AR_NT) void argmax_reduce_kernel(const unsigned long long* __restrict__ keys, int ntiles,
                                                              unsigned long long* __restrict__ out_keys,
                                                              int* __restrict__ out_ids) {
  const int m = blockIdx.x;
  const unsigned long long* k = keys + (long long)m * ntiles;
  unsigned long long best = 0;
  for (int base = 0; base < ntiles; base += AR_NT * AR_U) {
    unsigned long long v[AR_U];
#pragma unroll
    for (int u = 0; u < AR_U; ++u) {
      const int i = base + u * AR_NT + threadIdx.x;
      v[u] = i < ntiles ? k[i] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < AR_U; ++u) best = v[u] > best ? v[u] : best;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long v = __shfl_xor(best, o, 64);
    best = v > best ? v : best;
  }
  __shared__ unsigned long long sm[AR_NT / 64];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < AR_NT / 64; ++i) best = sm[i] > best ? sm[i] : best;
    if (out_keys) out_keys[m] = best;
    if (out_ids) out_ids[m] = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
  }
}

template <int MT, int EPI, int RT, bool NAT, bool NTL>
void launch_mt(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, const float* temps,
               const unsigned long long* seeds, const long long* step, unsigned long long* keys, int n_offset,
               hipStream_t s) {
  const int ntiles = N / (16 * RT);
  const int kchunk = K / S;
  dim3 grid(ntiles, S);
  constexpr int U = MT == 1 ? (RT == 1 ? 4 : 2) : (MT == 2 ? 2 : 1);
  skinny_gemm_kernel<MT, U, EPI, RT, NAT, NTL>
      <<<grid, NT, 0, s>>>(x, W, y, M, N, K, kchunk, temps, seeds, step, keys, n_offset, ntiles);
}

template <int EPI, int RT, bool NAT, bool NTL>
void launch_epi(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, const float* temps,
                const unsigned long long* seeds, const long long* step, unsigned long long* keys, int n_offset,
                hipStream_t s) {
  const int mt = (M + 15) / 16;
  switch (mt) {
    case 1: launch_mt<1, EPI, RT, NAT, NTL>(x, W, y, M, N, K, S, temps, seeds, step, keys, n_offset, s); break;
    case 2: launch_mt<2, EPI, RT, NAT, NTL>(x, W, y, M, N, K, S, temps, seeds, step, keys, n_offset, s); break;
    case 3: launch_mt<3, EPI, RT, NAT, NTL>(x, W, y, M, N, K, S, temps, seeds, step, keys, n_offset, s); break;
    default: launch_mt<4, EPI, RT, NAT, NTL>(x, W, y, M, N, K, S, temps, seeds, step, keys, n_offset, s); break;
  }
}

}  // namespace

void launch_skinny_gemm(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, hipStream_t s,
                        int variant) {
  // variant 0 = auto: measured on MI355X (bench/kernels/bench_skinny.py, profiles/skinny_variants.md):
  // plain loads beat non-temporal ones for these 33-235 MB weight streams, and two row tiles per wave
  // (x fragments shared) win once M > 16.
  if (variant == 0) variant = (M > 16 && N % 32 == 0) ? 3 : 2;
  switch (variant) {
    case 1: launch_epi<0, 1, false, true>(x, W, y, M, N, K, S, nullptr, nullptr, nullptr, nullptr, 0, s); break;
    case 2: launch_epi<0, 1, true, false>(x, W, y, M, N, K, S, nullptr, nullptr, nullptr, nullptr, 0, s); break;
    case 3: launch_epi<0, 2, true, false>(x, W, y, M, N, K, S, nullptr, nullptr, nullptr, nullptr, 0, s); break;
    default: launch_epi<0, 1, true, true>(x, W, y, M, N, K, S, nullptr, nullptr, nullptr, nullptr, 0, s); break;
  }
}

void launch_skinny_gemm_argmax(const bf16* x, const bf16* W, float* logits_or_null, int M, int N, int K,
                               const float* temps, const unsigned long long* seeds, const long long* step,
                               unsigned long long* tile_keys, int n_offset, hipStream_t s) {
  launch_epi<1, 1, true, false>(x, W, logits_or_null, M, N, K, 1, temps, seeds, step, tile_keys, n_offset, s);
}

void launch_argmax_reduce(const unsigned long long* tile_keys, int M, int ntiles, unsigned long long* out_keys,
                          int* out_ids, hipStream_t s) {
  argmax_reduce_kernel<<<M, AR_NT, 0, s>>>(tile_keys, ntiles, out_keys, out_ids);
}
