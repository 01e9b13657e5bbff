// Fused decode projections: one weight-streaming MFMA GEMM per projection with the neighbouring
// elementwise / normalisation work folded into its prologue and epilogue.
//
// Per Llama layer the decode step becomes
//   QKV  (+ RMSNorm row scale, RoPE, paged K/V cache write, q out)
//   attention (+ split-KV reduce)
//   O    (+ residual add, next-norm prep)
//   gate_up (+ RMSNorm row scale, SwiGLU)
//   down (+ residual add, next-norm prep)
// instead of ten launches (profiles/r1_baseline: the small kernels cost ~1 ms per step).
//
// Deferred RMSNorm.  RMSNorm(r) * w = rsqrt(mean(r^2) + eps) * (r * w): the producer of the
// residual r (O / down epilogue, embed_prep, add_prep) stores xw = bf16(r * w) plus per-(row, tile)
// partial sums of r^2 (plain stores, fixed summation order: bitwise reproducible); the consumer GEMM
// sums the partials of its rows in the prologue and scales its accumulators by rsqrt(.) in the
// epilogue.  No norm kernel, no cross-workgroup synchronisation.
//
// Layout contracts (applied once at load by symmetry_amd.models.layout):
//   * q/k head rows are permuted so a 16-row tile j of a head holds dims 8j..8j+7 and
//     64+8j..64+8j+7: both halves of each rotate-half pair land in one MFMA tile, lanes l and
//     l^32 (one __shfl_xor) -- RoPE happens in registers;
//   * gate_up rows are interleaved per tile: rows 0-7 gate f = 8j.., rows 8-15 up f = 8j.. .
//
// Decomposition: one workgroup per 16-row weight tile, NW waves splitting K (no split-K across
// workgroups, so every epilogue sees final values), U 64-deep k blocks in flight per wave, partial
// accumulators summed through LDS.  MFMA v_mfma_f32_16x16x32_bf16, natural k order (each load
// instruction reads 16 rows x 64 contiguous bytes).
#include "attn_decode.h"
#include "common.h"
#include "decode_epi.h"
#include "launchers.h"
#include "xgmi_proto.h"

namespace {


// This lane's share of one row's sum-of-squares partials (deferred RMSNorm prologue): 16-B loads when the row
// holds a multiple of 4 (the d / 16 per-tile partials of the fused epilogues: 256 for d = 4096 = ONE load per
// lane instead of four dependent 4-B ones)
SYM_DEV float ss_row_share(const float* __restrict__ row, int n, int lane) {
  float s = 0.f;
  if ((n & 3) == 0) {
    for (int i = 4 * lane; i < n; i += 256) {
      const float4 q = *reinterpret_cast<const float4*>(row + i);
      s += (q.x + q.y) + (q.z + q.w);
    }
  } else {
    for (int i = lane; i < n; i += 64) s += row[i];
  }
  return s;
}

// One workgroup-tile of the decode GEMM (RT consecutive 16-row weight tiles starting at 16 * RT * blk).
// (The persistent MLP / attention-block launches that once reused this body with device-side phase waits
// measured slower than the launches and were removed: profiles/r3/mlp_xres_persistent.jsonl,
// profiles/r3/qkv_attn_fused.jsonl, profiles/decode_block_r1.jsonl.)
//
// KS > 1 (few output tiles, long K: the Llama-3-70B TP = 8 QKV shard has 80 tiles x K = 8192, i.e. 80 of 256 CUs
// streaming 262 KB each): workgroup blk computes tile blk / KS over the k range of split blk % KS, stores its
// reduced 16 x 16 fp32 partial write-through into the split-K workspace, drains, and bumps the tile's counter;
// the workgroup whose add completes the set sums the KS partials in split order (bitwise reproducible), applies
// the row scale and runs the epilogue, then re-arms the counter (graph-replay safe).  MI355X_MICROARCH.md
// hand-off: sc1 payload stores + agent-scope add, agent-scope (L2-bypassing) loads by the last arriver.
template <int MT, int NW, int U, int RT, int EPI, int KS = 1>
SYM_DEV void gemm_tile(const bf16* __restrict__ x, const bf16* __restrict__ W, int M, int N, int K,
                       const DecodeEpi& e, int blk) {
  static_assert(KS == 1 || (RT == 1 && EPI != DECODE_EPI_XAR && EPI != DECODE_EPI_ARGMAX), "split-K: one tile");
  const int split = KS > 1 ? blk % KS : 0;
  const int tile0 = (KS > 1 ? blk / KS : blk) * RT;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int wk = K / KS / NW;
  const int kbeg = split * (K / KS) + wid * wk;
  const int nblk = wk / 64;

  // weight stream: row-major (16 rows x 64 B per load) or preshuffled (1 KB contiguous per load)
  const bf16* wrow[RT];
  const int wmul = e.wshuf ? 16 : 1, wsec = e.wshuf ? 512 : 32;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
    wrow[rt] = e.wshuf ? W + ((long long)(tile0 + rt) * (K / 32) + kbeg / 32) * 512 + lane * 8
                       : W + (long long)(16 * (tile0 + rt) + r16) * K + kbeg + 8 * h;
  // x fragments of rows >= M are never fetched (masked lanes load nothing; MFMA sees zeros).
  const bf16* xrow[MT];
  bool xok[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    xok[mt] = 16 * mt + r16 < M;
    xrow[mt] = x + (long long)min(16 * mt + r16, M - 1) * K + kbeg + 8 * h;
  }
  auto ldx = [&](int mt, int ko) -> uint4 {
    return xok[mt] ? *reinterpret_cast<const uint4*>(xrow[mt] + ko) : make_uint4(0, 0, 0, 0);
  };

  __shared__ f32x4 red[NW][RT * MT][64];
  __shared__ float rn_s[64];
  unsigned xep = 0, xctr = 0;
  __shared__ unsigned s_xep;
  if constexpr (EPI == DECODE_EPI_XAR) {  // this tile's epoch counter (read now, used after the weight stream)
    static_assert(RT == 1, "XAR: one output tile per workgroup");
    if (threadIdx.x == 0) xctr = e.xar_ctr[tile0];
  }

  f32x4 acc[RT][MT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto row_scales = [&]() {
    // RMSNorm row scales of the input rows (deferred norm), overlapped with the weight loads in flight.
    // Four rows per batch: their loads are independent, so a wave with 16 rows (M = 64, 4 waves) pays 4 load
    // round trips instead of 16 (the 64-row lm_head: 295 -> ~230 us).
    if (e.ss_in) {
      for (int m0 = wid; m0 < M; m0 += 4 * NW) {
        float s[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = m0 + j * NW;
          s[j] = m < M ? ss_row_share(e.ss_in + (long long)m * e.ss_tiles, e.ss_tiles, lane) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = m0 + j * NW;
          const float t = wave_sum(s[j]);
          if (lane == 0 && m < M) rn_s[m] = rsqrtf(t * e.inv_d + e.eps);
        }
      }
    }
  };

  int b = 0;
  bool rn_done = false;
  for (; b + U <= nblk; b += U) {
    Pack8 wa[U][RT][2], xa[U][MT][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ko = (b + u) * 64;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        if (e.wnt) {
          wa[u][rt][0].w = ld_nt16(wrow[rt] + ko * wmul);
          wa[u][rt][1].w = ld_nt16(wrow[rt] + ko * wmul + wsec);
        } else {
          wa[u][rt][0].u = *reinterpret_cast<const uint4*>(wrow[rt] + ko * wmul);
          wa[u][rt][1].u = *reinterpret_cast<const uint4*>(wrow[rt] + ko * wmul + wsec);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ko = (b + u) * 64;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        xa[u][mt][0].u = ldx(mt, ko);
        xa[u][mt][1].u = ldx(mt, ko + 32);
      }
    }
    if (!rn_done) {
      rn_done = true;
      row_scales();
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
  // the remaining nblk % U k-blocks as ONE predicated batch (a per-block loop would pay one memory round
  // trip per block: Llama-3-8B down_proj at 16 waves has 14 = 3 x 4 + 2 blocks per wave)
  if (b < nblk) {
    const int rem = nblk - b;
    Pack8 wa[U][RT][2], xa[U][MT][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < rem) {
        const int ko = (b + u) * 64;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          wa[u][rt][0].u = *reinterpret_cast<const uint4*>(wrow[rt] + ko * wmul);
          wa[u][rt][1].u = *reinterpret_cast<const uint4*>(wrow[rt] + ko * wmul + wsec);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < rem) {
        const int ko = (b + u) * 64;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          xa[u][mt][0].u = ldx(mt, ko);
          xa[u][mt][1].u = ldx(mt, ko + 32);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < rem)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            acc[rt][mt] = mfma16(wa[u][rt][0].v, xa[u][mt][0].v, acc[rt][mt]);
            acc[rt][mt] = mfma16(wa[u][rt][1].v, xa[u][mt][1].v, acc[rt][mt]);
          }
  }
  if (!rn_done) row_scales();
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wid][rt * MT + mt][lane] = acc[rt][mt];
  __syncthreads();
  if constexpr (EPI == DECODE_EPI_XAR) {
    if (threadIdx.x == 0) {
      s_xep = xctr + 1u;
      e.xar_ctr[tile0] = xctr + 1u;
    }
    __syncthreads();
    xep = s_xep;
  }
  if constexpr (KS > 1) {  // publish this split's partial, the last arriver finishes the tile
    float* slot = e.ks_ws + ((long long)tile0 * KS + split) * (MT * 256);
    for (int job = wid; job < MT; job += NW) {
      f32x4 v = red[0][job][lane];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += red[w][job][lane];
      unsigned long long* q = reinterpret_cast<unsigned long long*>(slot + job * 256 + lane * 4);
      const float4 f4 = make_float4(v[0], v[1], v[2], v[3]);
      const unsigned long long* w64 = reinterpret_cast<const unsigned long long*>(&f4);
      __hip_atomic_store(q, w64[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(q + 1, w64[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int s_last;
    __syncthreads();
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(e.ks_cnt + tile0, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == KS - 1;
    __syncthreads();
    if (!s_last) return;
    const float* base = e.ks_ws + (long long)tile0 * KS * (MT * 256);
    for (int job = wid; job < MT; job += NW) {
      unsigned long long r[KS][2];
#pragma unroll
      for (int sp = 0; sp < KS; ++sp) {
        const unsigned long long* q =
            reinterpret_cast<const unsigned long long*>(base + sp * (MT * 256) + job * 256 + lane * 4);
        r[sp][0] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r[sp][1] = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < KS; ++sp) {  // split order
        const float* qq = reinterpret_cast<const float*>(r[sp]);
        v += f32x4{qq[0], qq[1], qq[2], qq[3]};
      }
      const int m = 16 * job + r16;
      const bool mok = m < M;
      const float sc = (e.ss_in && mok) ? rn_s[m] : 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] *= sc;
      epilogue<EPI>(e, v, tile0, m, mok, h, N, xep);
    }
    if (threadIdx.x == 0) __hip_atomic_store(e.ks_cnt + tile0, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // parallel epilogue: wave `wid` finishes accumulator tiles job = wid, wid + NW, ...
  for (int job = wid; job < RT * MT; job += NW) {
    const int rt = job / MT, mt = job % MT;
    f32x4 v = red[0][job][lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += red[w][job][lane];
    const int m = 16 * mt + r16;
    const bool mok = m < M;
    const float sc = (e.ss_in && mok) ? rn_s[m] : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= sc;
    epilogue<EPI>(e, v, tile0 + rt, m, mok, h, N, xep);
  }
}

template <int MT, int NW, int U, int RT, int EPI, int WPE = 1>
__global__ __launch_bounds__(NW * 64, WPE) void decode_gemm_kernel(const bf16* __restrict__ x,
                                                              const bf16* __restrict__ W, int M, int N, int K,
                                                              DecodeEpi e) {
  gemm_tile<MT, NW, U, RT, EPI>(x, W, M, N, K, e, blockIdx.x);
}

template <int MT, int NW, int U, int EPI, int KS>
__global__ __launch_bounds__(NW * 64) void decode_gemm_ks_kernel(const bf16* __restrict__ x,
                                                                const bf16* __restrict__ W, int M, int N, int K,
                                                                DecodeEpi e) {
  gemm_tile<MT, NW, U, 1, EPI, KS>(x, W, M, N, K, e, blockIdx.x);
}

// ---- residual producers without a GEMM ----------------------------------------------------------
// embed_prep: resid = table[tok]; xw = bf16(resid * w); ss[m][0] = sum(resid^2), where
//   tok = src[m] >= 0 ? prev[src[m]] : ids[m]  -- src/prev (optional) feed the previous step's sampled ids
//   straight from device memory (pipelined decode: the host has not seen them yet)
// add_prep:   resid += delta (LinOut); xw = bf16(resid * w); ss[m][0] = sum(resid^2)
template <int MODE>
__global__ __launch_bounds__(256) void prep_kernel(LinOut delta, const int* __restrict__ ids,
                                                   const int* __restrict__ src, const int* __restrict__ prev,
                                                   const bf16* __restrict__ table, float* __restrict__ resid,
                                                   const bf16* __restrict__ w, bf16* __restrict__ xw,
                                                   float* __restrict__ ss, int d) {
  // gridDim.y column parts per row (wide decode batches: 64 rows x 1 workgroup is latency-bound); part p
  // covers columns [p d / P, (p + 1) d / P) and writes its own partial ss[row][p]
  __shared__ float scratch[4];
  const int row = blockIdx.x, P = gridDim.y, dp = d / P;
  const long long rb = (long long)row * d + (long long)blockIdx.y * dp;
  float acc = 0.f;
  long long tok = 0;
  if constexpr (MODE == 0) {
    const int sr = src ? src[row] : -1;
    tok = sr >= 0 ? prev[sr] : ids[row];
  }
  const bf16* wp = w + (long long)blockIdx.y * dp;
  for (int vi = threadIdx.x; vi < dp / 8; vi += 256) {
    float r[8], g[8];
    if constexpr (MODE == 0) {
      load8(table + tok * d + (long long)blockIdx.y * dp + vi * 8, r);
    } else {
      float dd[8];
      load8f(resid + rb + vi * 8, r);
      linout_load8(delta, rb + vi * 8, dd);
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] += dd[i];
    }
    store8f(resid + rb + vi * 8, r);
    load8(wp + vi * 8, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc += r[i] * r[i];
      g[i] *= r[i];
    }
    store8(xw + rb + vi * 8, g);
  }
  acc = block_sum<256>(acc, scratch);
  if (threadIdx.x == 0) ss[row * P + blockIdx.y] = acc;
}

// Decomposition variants (A/B: bench/kernels/bench_decode_gemm.py; chosen by decode_gemm_variant()):
//   0  8 waves split K, 1 row tile, U = 4 / 2 / 1 k-blocks in flight for 1 / 2 / 3-4 column tiles
//   1  8 waves, 1 row tile, deeper: U = 8 / 4 / 2
//   2 16 waves (K % 1024 == 0), 1 row tile
//   3  8 waves, 2 row tiles per workgroup (x fragments shared by both)
//   4  4 waves, 1 row tile
//   5  8 waves, 4 row tiles (1 column tile only; else as 3)
//   6  4 waves, 2 row tiles
//   7  4 waves, 4 row tiles (1 column tile only; else as 6)
//   8  4 waves, 1 row tile, U <= 2 (70 VGPRs): 7 waves / SIMD resident
//  11  x-resident persistent: 16 waves per CU, x loaded once per workgroup, tiles walked with the next
//      tile's weights in flight (M <= 16, K in {1024, 2048, 4096}; else variant 0)
// ---------------------------------------------------------------------------------------------------
// x-resident persistent decode GEMM (M <= 16, K == 16 * 64 * U): one 16-wave workgroup per CU walks row tiles
// t = b, b + grid, ...; each wave loads ITS k-slice of the activations x ONCE (U k-blocks, 8U VGPRs) and keeps
// it for every tile, so the per-tile L1/TA traffic is the weight stream alone (with row-tile-per-workgroup
// kernels the x fragments cost as many load instructions as the weights at M = 16, and gate_up ran 41 us at
// M = 1 vs 53 us at M = 16).  The next tile's weights are issued right after this tile's MFMAs and are in
// flight while it is reduced (LDS, double-buffered) and finished by wave 0 (16 waves x 8 KB per CU in
// flight is above the ~50 KB Little's-law need); the grid gives every CU the same tile count.
// ---------------------------------------------------------------------------------------------------
// Remainder tiles split over K (KS > 1, chosen by go_xres when whole tiles leave CUs idle).  With ntiles =
// f * G + R (G workgroups), the first f * G tiles are walked whole as above and the R remainder tiles are cut
// into R * KS parts of K / KS, dealt out after them (part p: tile f G + p / KS, k-split p % KS, computed by the
// 16 / KS waves whose resident x slices cover that k range; the others add zeros).  Llama-3-8B QKV: 384 tiles
// = 2 per CU on 192 CUs whole -> 1 whole + 1 half per CU on all 256 (25 % fewer bytes on the busiest CU);
// TP = 8 shard: 48 tiles -> 192 quarter tiles.  Wave 0 stores each part's reduced 16 x 16 fp32 partial with
// write-through stores as it goes; after the last unit it drains them ONCE (vmcnt(0): the only point where it
// has no weight loads in flight), bumps the parts' tile counters (one lane per part), and for the tiles whose
// last split it delivered sums the KS partials in split order (bitwise reproducible whatever the arrival
// order), re-arms the counter and runs the epilogue.  No workgroup ever waits for another.  (A first version
// handed off after every part with agent fences: the fence writes back / invalidates the XCD's whole L2 and
// the drain stalls on the next unit's loads, +23 us per QKV launch.)
template <int U, int KS, int EPI>
SYM_DEV void xres_body(const bf16* __restrict__ x, const bf16* __restrict__ W, int M, int N, int K, const DecodeEpi& e,
                       int NF, int P, int b, int G) {
  constexpr int NW = 16;
  constexpr int WPS = NW / KS;  // waves per k-split
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int kbeg = wid * (K / NW);
  const int wmul = e.wshuf ? 16 : 1, wsec = e.wshuf ? 512 : 32;
  auto wptr = [&](int t) -> const bf16* {
    return e.wshuf ? W + ((long long)t * (K / 32) + kbeg / 32) * 512 + lane * 8
                   : W + (long long)(16 * t + r16) * K + kbeg + 8 * h;
  };
  // this workgroup's units: whole tiles b, b + G, ... < NF, then parts b, b + G, ... < P.  KS > 1: part p is
  // k-split p % KS of tile NF + p / KS; KS == 1 with P > 0: part p is row half p % 2 of tile NF + p / 2 -- rows
  // {0-3, 8-11} or {4-7, 12-15}, i.e. the A-operand lanes with ((lane >> 2) & 1) == half and the accumulator
  // lanes with (h & 1) == half: every RoPE / SwiGLU partner pair (rows r, r + 8) stays in one half, so a half
  // tile is final in one workgroup (no partial hand-off) and the weight loads of the other half's lanes are
  // masked off (half the bytes)
  constexpr int PDIV = KS > 1 ? KS : 2;
  const int nf = NF > b ? (NF - b + G - 1) / G : 0;
  const int np = P > b ? (P - b + G - 1) / G : 0;
  const int nu = nf + np;
  if (nu == 0) return;  // uniform over the workgroup
  // XAR: per-tile epoch counters of this workgroup's tiles (read now, bumped after the first barrier below)
  __shared__ unsigned s_xep[XAR_MAX_TILES];
  unsigned xctr = 0;
  if constexpr (EPI == DECODE_EPI_XAR)
    if (threadIdx.x < nf) xctr = e.xar_ctr[b + threadIdx.x * G];
  auto unit_tile = [&](int i) { return i < nf ? b + i * G : NF + (b + (i - nf) * G) / PDIV; };
  auto unit_active = [&](int i) { return KS == 1 || i < nf || wid / WPS == (b + (i - nf) * G) % KS; };
  auto unit_half = [&](int i) { return (KS > 1 || i < nf) ? -1 : (b + (i - nf) * G) % 2; };
  Pack8 wa[U][2];
  auto load_w = [&](int i) {
    if (!unit_active(i)) return;
    const bf16* wp = wptr(unit_tile(i));
    const int hf = unit_half(i);
    const bool on = hf < 0 || ((lane >> 2) & 1) == hf;
    if (e.wnt) {  // non-temporal: once-read weights (bench/kernels/read_bw_policy.py: 5.7 -> 6.1-6.4 TB/s)
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (on) {
          wa[j][0].w = ld_nt16(wp + j * 64 * wmul);
          wa[j][1].w = ld_nt16(wp + j * 64 * wmul + wsec);
        } else {
          wa[j][0].u = make_uint4(0, 0, 0, 0);
          wa[j][1].u = make_uint4(0, 0, 0, 0);
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      wa[j][0].u = on ? *reinterpret_cast<const uint4*>(wp + j * 64 * wmul) : make_uint4(0, 0, 0, 0);
      wa[j][1].u = on ? *reinterpret_cast<const uint4*>(wp + j * 64 * wmul + wsec) : make_uint4(0, 0, 0, 0);
    }
  };
  load_w(0);
  const bool xok = r16 < M;
  const bf16* xrow = x + (long long)min(r16, M - 1) * K + kbeg + 8 * h;
  Pack8 xa[U][2];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    xa[j][0].u = xok ? *reinterpret_cast<const uint4*>(xrow + j * 64) : make_uint4(0, 0, 0, 0);
    xa[j][1].u = xok ? *reinterpret_cast<const uint4*>(xrow + j * 64 + 32) : make_uint4(0, 0, 0, 0);
  }
  __shared__ float rn_s[16];
  if (e.ss_in) {  // deferred-RMSNorm row scales, once per workgroup
    for (int m = wid; m < M; m += NW) {
      const float sacc = wave_sum(ss_row_share(e.ss_in + (long long)m * e.ss_tiles, e.ss_tiles, lane));
      if (lane == 0) rn_s[m] = rsqrtf(sacc * e.inv_d + e.eps);
    }
  }
  __shared__ f32x4 red[2][NW][64];
  if constexpr (EPI == DECODE_EPI_XAR) {
    if (threadIdx.x < nf) {
      s_xep[threadIdx.x] = xctr + 1u;
      e.xar_ctr[b + threadIdx.x * G] = xctr + 1u;
    }
    __syncthreads();
  }
  const int m = r16;
  const bool mok = m < M;
  auto finish = [&](f32x4 v, int t, int hf = -1) {  // wave 0: row scale + epilogue of a final tile (or half)
    const float sc = (e.ss_in && mok) ? rn_s[m] : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= sc;
    unsigned xep = 0;
    if constexpr (EPI == DECODE_EPI_XAR) xep = s_xep[(t - b) / G];  // XAR: whole tiles only (t = b + i G)
    epilogue<EPI>(e, v, t, m, mok && (hf < 0 || (h & 1) == hf), h, N, xep);
  };
  int buf = 0;
  for (int i = 0; i < nu; ++i) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (unit_active(i)) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        acc = mfma16(wa[j][0].v, xa[j][0].v, acc);
        acc = mfma16(wa[j][1].v, xa[j][1].v, acc);
      }
    }
    // keep the next loads behind this tile's MFMAs: they reuse wa's registers (no renamed second copy)
    __builtin_amdgcn_sched_barrier(0);
    if (i + 1 < nu) load_w(i + 1);  // next unit's weight stream in flight during this unit's reduction/epilogue
    red[buf][wid][lane] = acc;
    __syncthreads();
    if (wid == 0) {
      f32x4 v = red[buf][0][lane];
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        v += red[buf][w][lane];
        if ((w & 3) == 3) asm volatile("" : "+v"(v)::"memory");  // <= 4 partials in registers at a time
      }
      if (i < nf) {
        finish(v, unit_tile(i));
      } else if constexpr (KS == 1) {  // row half of a remainder tile
        finish(v, unit_tile(i), unit_half(i));
      } else {  // part: publish the partial (write-through), no wait here
        unsigned long long* slot =
            reinterpret_cast<unsigned long long*>(e.ks_ws + (long long)(b + (i - nf) * G) * 256 + lane * 4);
        const float4 f4 = make_float4(v[0], v[1], v[2], v[3]);
        const unsigned long long* w64 = reinterpret_cast<const unsigned long long*>(&f4);
        __hip_atomic_store(slot, w64[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(slot + 1, w64[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    buf ^= 1;
  }
  if constexpr (KS > 1) {
    if (wid != 0 || np == 0) return;
    // MI355X_MICROARCH.md hand-off: write-through payload, vmcnt drain, relaxed agent add; the last split's
    // wave reads the payloads with agent-scope (L2-bypassing) loads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane < np) {
      const int tl = (b + lane * G) / KS;
      last = __hip_atomic_fetch_add(e.ks_cnt + tl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == KS - 1;
      if (last) __hip_atomic_store(e.ks_cnt + tl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long lastmask = __ballot(last);
    for (int j = 0; j < np; ++j) {
      if (!((lastmask >> j) & 1)) continue;
      const int tl = (b + j * G) / KS;
      const unsigned long long* base =
          reinterpret_cast<const unsigned long long*>(e.ks_ws + (long long)tl * KS * 256 + lane * 4);
      unsigned long long r[KS][2];
#pragma unroll
      for (int sp = 0; sp < KS; ++sp) {
        r[sp][0] = __hip_atomic_load(base + sp * 128, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r[sp][1] = __hip_atomic_load(base + sp * 128 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < KS; ++sp) {  // split order
        const float* q = reinterpret_cast<const float*>(r[sp]);
        v += f32x4{q[0], q[1], q[2], q[3]};
      }
      finish(v, NF + tl);
    }
  }
}

template <int U, int KS, int EPI>
__global__ __launch_bounds__(1024) void decode_gemm_xres_kernel(const bf16* __restrict__ x, const bf16* __restrict__ W,
                                                                int M, int N, int K, DecodeEpi e, int NF, int P) {
  xres_body<U, KS, EPI>(x, W, M, N, K, e, NF, P, blockIdx.x, gridDim.x);
}

int g_num_cus = 0;

// Remainder split: OFF by default.  Measured (profiles/r3/ksplit_ab.jsonl, alternating runs): 8B 10 clients
// 3.308 vs 3.230 ms per step, TP = 8 shard 1.576 vs 1.538, TP = 4 1.965 vs 1.817 -- at these sizes the launch
// is bound by latency (ramp, first loads, the tail), not by the busiest CU's bytes, and the hand-off adds a
// drain + atomic + L2-bypassing read round trip to the tail.  SYMMETRY_DG_KSPLIT=1 / set_decode_ksplit(1).
static bool g_dg_ksplit = [] {
  const char* knob = getenv("SYMMETRY_DG_KSPLIT");
  return knob && knob[0] == '1';
}();

// Split K of few-tile long-K launches across whole gemm_tile workgroups (launch_mt, variants 21..24): ON by
// default (a different regime from the remainder split above: there most CUs would otherwise sit idle).
// SYMMETRY_DG_TILE_KSPLIT=0 reverts.
static bool g_dg_tile_ksplit = [] {
  const char* knob = getenv("SYMMETRY_DG_TILE_KSPLIT");
  return !(knob && knob[0] == '0');
}();

// Remainder tiles as row halves: OFF by default.  Measured (profiles/r3/xres_row_halves_ab.jsonl, alternating
// runs): 8B 10 clients 3.316 vs 3.261 ms per step, TP = 4 / 8 shards unchanged.  A half tile issues as many
// load instructions as a whole one (half the lanes masked), and at M <= 16 the launch is bound by the load
// pipeline's latency per CU, not by its bytes -- the same finding as the k split above.
// SYMMETRY_DG_HALVES=1 / set_decode_halves(1).
static bool g_dg_halves = [] {
  const char* knob = getenv("SYMMETRY_DG_HALVES");
  return knob && knob[0] == '1';
}();

template <int U, int KS, int EPI>
void go_xres_ks(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e, int grid, int NF, int P,
                hipStream_t s) {
  decode_gemm_xres_kernel<U, KS, EPI><<<grid, 1024, 0, s>>>(x, W, M, N, K, e, NF, P);
}

template <int EPI>
bool go_xres(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e, hipStream_t s) {
  if (M > 16 || K % 1024 || K > 4096) return false;
  if (!g_num_cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
    g_num_cus = std::max(1, g_num_cus);
  }
  const int C = g_num_cus;
  const int ntiles = N / 16;
  const int per = (ntiles + C - 1) / C;  // whole tiles: equal tile count per workgroup
  // XAR keeps one epoch slot per walked tile in LDS: the real tiles-per-workgroup count (a partitioned GPU has
  // fewer CUs) must fit, else the caller falls back to the gemm_tile variant
  if (EPI == DECODE_EPI_XAR && per > XAR_MAX_TILES) return false;
  int grid = (ntiles + per - 1) / per, NF = ntiles, P = 0, KS = 1;
  // remainder split: weight bytes on the busiest CU, f K + q K / KS, must drop >= 10 % (<= 4 parts per
  // workgroup, >= 4 waves per part)
  const int f = ntiles / C, R = ntiles - f * C;
  if (g_dg_ksplit && R > 0 && e.ks_ws && e.ks_cnt && e.ks_ncnt >= R && EPI != DECODE_EPI_ARGMAX &&
      EPI != DECODE_EPI_XAR) {
    long long best = (long long)per * K * 9 / 10;
    for (int ks = 2; ks <= 4; ks *= 2) {
      const int parts = R * ks, g = f > 0 ? C : std::min(C, parts), q = (parts + g - 1) / g;
      const long long cost = (long long)f * K + (long long)q * (K / ks);
      if (q > 4 || (long long)parts * 256 > e.ks_cap || cost > best) continue;
      if (cost < best || KS == 1) {
        best = cost;
        KS = ks;
        grid = g;
        NF = f * C;
        P = parts;
      }
    }
  }
  // remainder tiles as row halves (xres_body): epilogues whose partner rows pair r with r + 8 and that reduce
  // nothing across a tile's rows -- when it lowers the busiest CU's weight bytes (Llama-3-8B QKV: 384 tiles =
  // 2 per CU on 192 CUs -> 1 whole + 1 half on all 256; TP = 8 QKV: 48 tiles -> 96 halves)
  constexpr bool kHalvable = EPI == DECODE_EPI_QKV || EPI == DECODE_EPI_SWIGLU || EPI == DECODE_EPI_F32;
  if (kHalvable && KS == 1 && g_dg_halves && R > 0) {
    const int parts = 2 * R, g = f > 0 ? C : std::min(C, parts), q = (parts + g - 1) / g;
    if (2 * f + q < 2 * per) {
      grid = g;
      NF = f * C;
      P = parts;
    }
  }
  switch (KS * 8 + K / 1024) {
    case 8 + 1: go_xres_ks<1, 1, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    case 8 + 2: go_xres_ks<2, 1, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    case 8 + 4: go_xres_ks<4, 1, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    case 16 + 1: go_xres_ks<1, 2, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    case 16 + 2: go_xres_ks<2, 2, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    case 16 + 4: go_xres_ks<4, 2, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    case 32 + 1: go_xres_ks<1, 4, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    case 32 + 2: go_xres_ks<2, 4, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    case 32 + 4: go_xres_ks<4, 4, EPI>(x, W, M, N, K, e, grid, NF, P, s); return true;
    default: return false;
  }
}

int g_variant = -1;
// Non-temporal weight loads (aux nt) in the decode GEMMs: ON by default.  Once-read weights stream faster
// without allocating in the caches (bench/kernels/read_bw_policy.py: 235 MB at 5.73 -> 6.08 TB/s); decode GEMMs
// at 10 rows (profiles/r3/nt_weights_xres_kernels.jsonl): gate_up 43.1 -> 39.1 us, qkv 14.6 -> 13.6, o 11.7 ->
// 10.6; 10-client step 3.281 -> 3.181 ms (profiles/r3/nt_weights_xres_ab.jsonl, 3 alternating runs).  (The round-2
// A/B that found no gain never reached the x-resident kernels, which ignored the knob.)  SYMMETRY_DG_NT=0 reverts.
const int g_wnt_default = [] {
  const char* knob = getenv("SYMMETRY_DG_NT");
  return knob && knob[0] == '0' ? 0 : 1;
}();
int g_wnt = g_wnt_default;

template <int MT, int NW, int U, int RT, int EPI, int WPE = 1>
void go(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e0, hipStream_t s) {
  DecodeEpi e = e0;
  e.wnt = g_wnt;
  decode_gemm_kernel<MT, NW, U, RT, EPI, WPE><<<N / (16 * RT), NW * 64, 0, s>>>(x, W, M, N, K, e);
}

template <int MT, int NW, int U, int EPI, int KS>
void go_ks(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e0, hipStream_t s) {
  DecodeEpi e = e0;
  e.wnt = g_wnt;
  decode_gemm_ks_kernel<MT, NW, U, EPI, KS><<<(N / 16) * KS, NW * 64, 0, s>>>(x, W, M, N, K, e);
}

// split-K of gemm_tile (variants 21..24): usable when every (tile, split) partial fits the workspace and each
// wave's k range is whole 64-blocks
template <int MT, int EPI>
bool ks_fits(int N, int K, int ks, int nw, const DecodeEpi& e) {
  if constexpr (EPI == DECODE_EPI_ARGMAX || EPI == DECODE_EPI_XAR) return false;
  const long long tiles = N / 16;
  return e.ks_ws && e.ks_cnt && tiles <= e.ks_ncnt && tiles * ks * MT * 256 <= e.ks_cap && K % (ks * nw * 64) == 0;
}

template <int MT, int EPI>
void launch_mt(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e, hipStream_t s) {
  constexpr int U0 = MT == 1 ? 4 : (MT == 2 ? 2 : 1);
  constexpr int U1 = MT == 1 ? 8 : (MT == 2 ? 4 : 2);
  int v = g_variant;
  if (v < 0 && g_dg_tile_ksplit && M <= 16 && K > 4096) {
    // few 16-row tiles over a long K, past the x-resident walk's K <= 4096 (Llama-3-70B TP = 8 QKV: 80 tiles x
    // K = 8192): whole-tile workgroups would leave 176 of 256 CUs idle, so split K in two across 8-wave
    // workgroups (profiles/r4/dg_tile_ksplit.jsonl: 12.93 -> 9.31 us at M = 1, 13.45 -> 9.88 at 4, 14.11 -> 11.39
    // at 10; 4 splits or 4 waves lose to it)
    if (g_num_cus == 0) {
      int dev = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
      g_num_cus = std::max(1, g_num_cus);
    }
    const int tiles = N / 16;
    if (2 * tiles <= g_num_cus) v = ks_fits<MT, EPI>(N, K, 2, 8, e) ? 23 : (ks_fits<MT, EPI>(N, K, 2, 4, e) ? 21 : v);
  }
  if ((v == 21 || v == 23) && !ks_fits<MT, EPI>(N, K, 2, v == 21 ? 4 : 8, e)) v = -2;
  if ((v == 22 || v == 24) && !ks_fits<MT, EPI>(N, K, 4, v == 22 ? 4 : 8, e)) v = -2;
  if constexpr (EPI != DECODE_EPI_ARGMAX && EPI != DECODE_EPI_XAR) {
    switch (v) {
      case 21: go_ks<MT, 4, U0, EPI, 2>(x, W, M, N, K, e, s); return;
      case 22: go_ks<MT, 4, U0, EPI, 4>(x, W, M, N, K, e, s); return;
      case 23: go_ks<MT, 8, U0, EPI, 2>(x, W, M, N, K, e, s); return;
      case 24: go_ks<MT, 8, U0, EPI, 4>(x, W, M, N, K, e, s); return;
      default: break;
    }
  }
  if (v == -2 || v >= 21) v = -1;  // split-K does not fit: the whole-tile heuristic
  if (v < 0) {
    // Measured on MI355X (profiles/decode_gemm_variants_r1.jsonl): the x fragments (re-read from L2 by
    // every workgroup) dominate the L1/TA traffic once M > 4, so wide-N projections share them over
    // 4 (2 for M > 16) row tiles per workgroup; the 4096-wide ones keep 256 workgroups and split K
    // over 4 waves; small TP shards keep the 8-wave split.
    if (e.wshuf) {
      // preshuffled stream (profiles/decode_gemm_preshuffle_r1.jsonl): 1 KB loads make the x-fragment
      // sharing of multi-tile workgroups unnecessary; wide N prefers 4 waves per tile
      // x-resident persistent tiles (profiles/decode_gemm_xres_r1.jsonl, M = 10: gate_up 49.1 -> 40.9 us,
      // qkv 15.6 -> 13.4, lm_head 205.9 -> 190.5; = variant 2 on the one-tile-per-CU O projection), except
      // the vocabulary projection at <= 2 rows where the 8-wave split stays ahead (lm_head 171 vs 177-183 us;
      // at 4 rows the walk wins, 179 vs 186: profiles/r4/dg_lm_head_small_m.jsonl)
      if (M <= 16 && K % 1024 == 0 && K <= 4096 && !(N >= 65536 && M <= 2)) v = 11;
      // wide N at 2..16 rows otherwise (Llama-3-70B at TP <= 4: gate_up, lm_head; K = 8192): 4 waves per tile.
      // (The round-1 pick, 7 resident 4-wave workgroups per CU -- variant 8, launch bounds (256, 7) -- now spills
      // 32 VGPRs to scratch with the grown epilogues: 70B gate_up 293-317 vs 165-204 us at 8-16 rows,
      // profiles/r4/dg_v8_spills.jsonl.)
      // above 16 rows (profiles/decode_gemm_bigm_r1.jsonl, M = 64): wide N shares each x fragment over
      // four row tiles (gate_up 93.6 -> 76.7 us, lm_head 367 -> 307), qkv over two (43.7 -> 33.3)
      // (eight row tiles from 25 rows: gate_up 77.0 -> 69.1 us at M = 64, profiles/decode_gemm_rt8_r1.jsonl)
      else if (N >= 12288) v = M > 16 ? (M > 24 ? 14 : 3) : (M <= 2 ? 0 : 4);
      else if (M > 16 && N > 4096) v = 3;
      else if (N <= 4096 && K % 1024 == 0) v = K > 4096 ? (M <= 4 ? 0 : 4) : 2;  // few row tiles: split K
        // (down_proj: 4 waves, 24.2 vs 25.7 us at M = 10; at <= 4 rows 8 waves: 24.2 vs 26.0 at 1 row,
        // profiles/r4/dg_sweep_8b.jsonl)
      // Llama-3-70B TP = 8 gate_up (7168 x 8192) and down (8192 x 3584) at 2..16 rows: 4 waves per tile
      // (profiles/r4/dg_tile_ksplit.jsonl, variant 4 vs -1: 27.6 vs 29.4 us and 15.2 vs 16.5 at M = 10)
      else if (M > 1 && N <= 8192 && K >= 3072 && K % 256 == 0) v = 4;
      else v = 0;
    } else if (M <= 4) {
      // row-major (models too large for a preshuffled copy: Llama-3-70B on one GPU) at <= 4 rows: two row tiles
      // per 8-wave workgroup when that grid is a whole number of rounds over the CUs, else 4 waves per tile
      // (profiles/r4/dg_70b_row.jsonl, 4 rows: gate_up 179.4 -> 163.4 us, down 92.6 -> 85.7, o 31.1 -> 29.8,
      // qkv 41.2 -> 40.1)
      if (g_num_cus == 0) {
        int dev = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
        g_num_cus = std::max(1, g_num_cus);
      }
      v = (N % 32 == 0 && (N / 32) % g_num_cus == 0) ? 3 : (K >= 4096 && K % 256 == 0 ? 4 : 0);
    } else if (N >= 12288) {
      // row-major wide N above 16 rows (the lm_head, whose weights are never preshuffled): 4 row tiles per
      // workgroup, lm_head 268 -> 224 us at M = 24, 421 -> 335 at M = 64 (profiles/decode_gemm_bigm_row_r1.jsonl)
      v = M > 16 ? (M > 24 ? 14 : 12) : 7;  // eight row tiles from 25 rows: 335 -> 311 us at M = 64
    } else if (N >= 6144 && K >= 4096) {
      v = 3;
    } else if (N <= 4096 && K >= 4096) {
      v = 4;
    } else {
      v = 0;
    }
  }
  if (v == 2 && K % 1024) v = 0;
  if ((v == 5 || v == 7) && (MT > 1 || N % 64)) v = v == 5 ? 3 : 6;
  if ((v == 3 || v == 6) && N % 32) v = 0;
  if ((v == 12 || v == 13 || v == 16) && N % 64) v = 0;
  if ((v == 14 || v == 15) && (N % 128 || MT == 1)) v = 0;
  if (K % 512) v = (v == 6 || v == 7) ? 6 : 4;  // e.g. Llama-3-8B down_proj under TP=8: K = 1792
  if (v == 6 && N % 32) v = 4;
  constexpr int UH = U0 > 1 ? U0 / 2 : 1;
  if (v == 11) {
    if constexpr (MT == 1) {
      DecodeEpi ex = e;
      ex.wnt = g_wnt;
      if (go_xres<EPI>(x, W, M, N, K, ex, s)) return;
    }
    v = 0;
  }
  switch (v) {
    case 1: go<MT, 8, U1, 1, EPI>(x, W, M, N, K, e, s); break;
    case 2: go<MT, 16, U0, 1, EPI>(x, W, M, N, K, e, s); break;
    case 3: go<MT, 8, UH, 2, EPI>(x, W, M, N, K, e, s); break;
    case 4: go<MT, 4, U0, 1, EPI>(x, W, M, N, K, e, s); break;
    case 5: if constexpr (MT == 1) go<1, 8, 1, 4, EPI>(x, W, M, N, K, e, s); break;
    case 6: go<MT, 4, UH, 2, EPI>(x, W, M, N, K, e, s); break;
    case 7: if constexpr (MT == 1) go<1, 4, 2, 4, EPI>(x, W, M, N, K, e, s); break;
    // occupancy-bounded: 7 waves / SIMD = 7 four-wave workgroups per CU, so Llama-3-8B gate_up's 1792
    // row tiles are all resident at once (one round, no second-round tail)
    case 8:  // one column tile only (the 7-waves-per-SIMD register budget)
      if constexpr (MT == 1) go<1, 4, 2, 1, EPI, 7>(x, W, M, N, K, e, s);
      else go<MT, 4, U0, 1, EPI>(x, W, M, N, K, e, s);
      break;

    // 17..64 rows: the x fragments every workgroup re-reads from L2 scale with MT, so four 16-row weight
    // tiles share each fragment (x traffic = weight traffic at M = 64); one k-block in flight per wave
    case 12: go<MT, 4, 1, 4, EPI>(x, W, M, N, K, e, s); break;
    case 13: go<MT, 8, 1, 4, EPI>(x, W, M, N, K, e, s); break;
    case 14: go<MT, 4, 1, 8, EPI>(x, W, M, N, K, e, s); break;
    case 15: go<MT, 2, 1, 8, EPI>(x, W, M, N, K, e, s); break;
    case 16: go<MT, 2, 1, 4, EPI>(x, W, M, N, K, e, s); break;

    default: go<MT, 8, U0, 1, EPI>(x, W, M, N, K, e, s); break;
  }
}

template <int EPI>
void launch_epi(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e, hipStream_t s) {
  switch ((M + 15) / 16) {
    case 1: launch_mt<1, EPI>(x, W, M, N, K, e, s); break;
    case 2: launch_mt<2, EPI>(x, W, M, N, K, e, s); break;
    case 3: launch_mt<3, EPI>(x, W, M, N, K, e, s); break;
    default: launch_mt<4, EPI>(x, W, M, N, K, e, s); break;
  }
}

}  // namespace


// ---- DECODE_EPI_XAR: row-parallel projection + xGMI all-reduce + residual epilogue in ONE launch ----------
// Every workgroup pushes its tiles to every rank, then WAITS for the other ranks' copies of the same tiles: the
// whole grid must be resident at once (a waiting workgroup holds its CU), so only one-tile-per-workgroup
// decompositions whose grid fits the occupancy are used -- the x-resident walk (one workgroup per CU) or
// gemm_tile with 8 / 4 waves -- and the caller falls back to GEMM + add_prep launches otherwise.
template <typename Kern>
bool xar_resident(Kern kern, int threads, long long grid) {
  int dev = 0, cus = 0, per_cu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0);
  return per_cu > 0 && grid <= (long long)cus * per_cu;
}

template <int MT>
bool xar_mt(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e0, hipStream_t s) {
  constexpr int U0 = MT == 1 ? 4 : (MT == 2 ? 2 : 1);
  DecodeEpi e = e0;
  e.wnt = g_wnt;
  if constexpr (MT == 1) {
    if (e.wshuf && K % 1024 == 0 && K <= 4096 && go_xres<DECODE_EPI_XAR>(x, W, M, N, K, e, s)) return true;
  }
  // 8 waves per tile where the plain launch would use them (else, or when 8-wave workgroups do not all fit at
  // once -- e.g. Llama-3-70B down at TP = 8: 512 tiles -- 4 waves)
  const int grid = N / 16;
  if (K % 512 == 0 && !(N <= 4096 && K >= 4096) &&
      xar_resident(decode_gemm_kernel<MT, 8, U0, 1, DECODE_EPI_XAR>, 512, grid)) {
    decode_gemm_kernel<MT, 8, U0, 1, DECODE_EPI_XAR><<<grid, 512, 0, s>>>(x, W, M, N, K, e);
    return true;
  }
  if (K % 256 || !xar_resident(decode_gemm_kernel<MT, 4, U0, 1, DECODE_EPI_XAR>, 256, grid)) return false;
  decode_gemm_kernel<MT, 4, U0, 1, DECODE_EPI_XAR><<<grid, 256, 0, s>>>(x, W, M, N, K, e);
  return true;
}

template <int MT, int NW, int U>
__global__ __launch_bounds__(NW * 64) void decode_gemm_xar_multi_kernel(XarMulti m, const bf16* __restrict__ W,
                                                                       int M, int N, int K) {
  const int r = blockIdx.z;
  if (r == m.delay_rank) xg_delay(m.delay_ticks);
  gemm_tile<MT, NW, U, 1, DECODE_EPI_XAR>(m.x[r], W, M, N, K, m.e[r], blockIdx.x);
}

template <int U>
__global__ __launch_bounds__(1024) void decode_gemm_xar_multi_xres_kernel(XarMulti m, const bf16* __restrict__ W,
                                                                          int M, int N, int K) {
  const int r = blockIdx.z;
  if (r == m.delay_rank) xg_delay(m.delay_ticks);
  xres_body<U, 1, DECODE_EPI_XAR>(m.x[r], W, M, N, K, m.e[r], N / 16, 0, blockIdx.x, gridDim.x);
}

void launch_decode_gemm(int epi, const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e,
                        hipStream_t s) {
  switch (epi) {
    case DECODE_EPI_F32: launch_epi<DECODE_EPI_F32>(x, W, M, N, K, e, s); break;
    case DECODE_EPI_QKV: launch_epi<DECODE_EPI_QKV>(x, W, M, N, K, e, s); break;
    case DECODE_EPI_RESID: launch_epi<DECODE_EPI_RESID>(x, W, M, N, K, e, s); break;
    case DECODE_EPI_SWIGLU: launch_epi<DECODE_EPI_SWIGLU>(x, W, M, N, K, e, s); break;
    default: launch_epi<DECODE_EPI_ARGMAX>(x, W, M, N, K, e, s); break;
  }
}


bool launch_decode_gemm_xar(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e, hipStream_t s) {
  if (M < 1 || M > 64 || N % 16 || N / 16 >= XG_KEYS_WG) return false;
  switch ((M + 15) / 16) {
    case 1: return xar_mt<1>(x, W, M, N, K, e, s);
    case 2: return xar_mt<2>(x, W, M, N, K, e, s);
    case 3: return xar_mt<3>(x, W, M, N, K, e, s);
    default: return xar_mt<4>(x, W, M, N, K, e, s);
  }
}

static_assert(sizeof(XarMulti) <= 4000, "XarMulti must fit the kernel argument space");

bool launch_decode_gemm_xar_multi(const XarMulti& m, int world, const bf16* W, int M, int N, int K, int xres,
                                  hipStream_t s) {
  if (M < 1 || M > 16 || N % 16 || world < 1 || world > XAR_MULTI_MAX) return false;
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (xres) {  // x-resident walk, ~cus / world workgroups per rank (one per CU, all ranks resident)
    if (K % 1024 || K > 4096 || !m.e[0].wshuf) return false;
    const int G = std::max(1, std::min(N / 16, cus / world));
    if ((N / 16 + G - 1) / G > XAR_MAX_TILES) return false;
    const dim3 grid(G, 1, world);
    switch (K / 1024) {
      case 1:
        if (!xar_resident(decode_gemm_xar_multi_xres_kernel<1>, 1024, (long long)G * world)) return false;
        decode_gemm_xar_multi_xres_kernel<1><<<grid, 1024, 0, s>>>(m, W, M, N, K);
        return true;
      case 2:
        if (!xar_resident(decode_gemm_xar_multi_xres_kernel<2>, 1024, (long long)G * world)) return false;
        decode_gemm_xar_multi_xres_kernel<2><<<grid, 1024, 0, s>>>(m, W, M, N, K);
        return true;
      case 4:
        if (!xar_resident(decode_gemm_xar_multi_xres_kernel<4>, 1024, (long long)G * world)) return false;
        decode_gemm_xar_multi_xres_kernel<4><<<grid, 1024, 0, s>>>(m, W, M, N, K);
        return true;
      default: return false;
    }
  }
  if (K % 256) return false;
  const dim3 grid(N / 16, 1, world);
  if (K % 512 == 0) {
    if (!xar_resident(decode_gemm_xar_multi_kernel<1, 8, 4>, 512, (long long)(N / 16) * world)) return false;
    decode_gemm_xar_multi_kernel<1, 8, 4><<<grid, 512, 0, s>>>(m, W, M, N, K);
  } else {
    if (!xar_resident(decode_gemm_xar_multi_kernel<1, 4, 4>, 256, (long long)(N / 16) * world)) return false;
    decode_gemm_xar_multi_kernel<1, 4, 4><<<grid, 256, 0, s>>>(m, W, M, N, K);
  }
  return true;
}

void set_decode_ksplit(int on) { g_dg_ksplit = on != 0; }
void set_decode_halves(int on) { g_dg_halves = on != 0; }

void set_decode_gemm_variant(int v) {
  // v >= 100: variant v - 100 with non-temporal weight loads, 0..99: with default-policy loads (A/B knob of
  // bench_decode_gemm.py); -1: the default heuristic and the default policy
  g_wnt = v >= 100 ? 1 : (v == -1 ? g_wnt_default : 0);
  g_variant = v >= 100 ? v - 100 : v;
}

void set_decode_gemm_nt(int on) { g_wnt = on ? 1 : 0; }

void launch_embed_prep(const int* ids, const int* src, const int* prev, const bf16* table, float* resid, const bf16* w,
                       bf16* xw, float* ss, int T, int d, int parts, hipStream_t s) {
  if (T == 0) return;
  LinOut none{nullptr, 0, 1, 0};
  prep_kernel<0><<<dim3(T, parts), 256, 0, s>>>(none, ids, src, prev, table, resid, w, xw, ss, d);
}

void launch_add_prep(LinOut delta, float* resid, const bf16* w, bf16* xw, float* ss, int T, int d, int parts,
                     hipStream_t s) {
  if (T == 0) return;
  prep_kernel<1><<<dim3(T, parts), 256, 0, s>>>(delta, nullptr, nullptr, nullptr, nullptr, resid, w, xw, ss, d);
}
