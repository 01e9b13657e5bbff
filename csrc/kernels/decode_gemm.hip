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

namespace {


struct NoWait {
  SYM_DEV void operator()() const {}
};

// One workgroup-tile of the decode GEMM (RT consecutive 16-row weight tiles starting at 16 * RT * blk).
// `wait` runs after the first batch of weight loads has been issued and before any activation is read:
// in the persistent MLP kernel it blocks until the producing phase has published the activations, so
// the weight stream of this tile overlaps the dependency wait.
template <int MT, int NW, int U, int RT, int EPI, typename WaitFn>
SYM_DEV void gemm_tile(const bf16* __restrict__ x, const bf16* __restrict__ W, int M, int N, int K,
                       const DecodeEpi& e, int blk, WaitFn wait) {
  const int tile0 = blk * RT;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int wk = K / NW;
  const int kbeg = wid * wk;
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
  unsigned xep = 0;
  if constexpr (EPI == DECODE_EPI_XPUSH) xep = xp_epoch(e.xp);

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
          s[j] = 0.f;
          if (m < M)
            for (int i = lane; i < e.ss_tiles; i += 64) s[j] += e.ss_in[(long long)m * e.ss_tiles + i];
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
  bool rn_done = false, waited = false;
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
    if (!waited) {
      waited = true;
      wait();
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
    if (!waited) {
      waited = true;
      wait();
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
  if (!waited) wait();
  if (!rn_done) row_scales();
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wid][rt * MT + mt][lane] = acc[rt][mt];
  __syncthreads();
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
  if constexpr (EPI == DECODE_EPI_XPUSH) {  // every wave's slot stores acknowledged, then the tile flags
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int tid = threadIdx.x;
    if (tid < RT * e.xp.world) xp_flag(e.xp, tid % e.xp.world, tile0 + tid / e.xp.world, xep);
  }
}

template <int MT, int NW, int U, int RT, int EPI, int WPE = 1>
__global__ __launch_bounds__(NW * 64, WPE) void decode_gemm_kernel(const bf16* __restrict__ x,
                                                              const bf16* __restrict__ W, int M, int N, int K,
                                                              DecodeEpi e) {
  gemm_tile<MT, NW, U, RT, EPI>(x, W, M, N, K, e, blockIdx.x, NoWait{});
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

// ---------------------------------------------------------------------------------------------------
// Persistent decode MLP block: O-proj -> gate_up -> down of one layer in ONE launch (M <= 16 rows).
//
// Tiles of the three GEMMs are numbered in phase order (d/16 O tiles, 2F/16 gate_up tiles, d/16 down
// tiles); resident workgroup b takes tiles b, b + grid, b + 2 grid, ...  A gate_up / down
// tile first issues its weight loads, THEN waits for the previous phase's completion counter, then
// reads the activations: the weight stream of the next phase overlaps the phase boundary that used
// to be a kernel launch (launch gap + first-load latency + tail).  Deadlock-free by construction:
// a workgroup runs its tiles in increasing order and the grid never exceeds the resident capacity, so
// every awaited tile belongs to a running workgroup that reaches it before waiting on anything later.
// Hand-off (MI355X_MICROARCH.md table): producers store resid / xw / ss / act write-through (sc1),
// drain vmcnt, then bump an agent-scope counter; consumers first touch those lines after the counter
// (caches were invalidated at kernel start, so plain loads see the written bytes).  Spins are bounded
// (error flag instead of a hang); the last workgroup re-arms the control words for the next launch.
// ---------------------------------------------------------------------------------------------------
// Completion counters are spread over 64 cache lines per phase (tile i of a phase bumps line i % 64):
// agent-scope atomics cross the XCDs to memory, so ~2k increments and ~1k pollers on ONE address
// serialise; 64 lines cut the per-address traffic 64x, and a waiting wave polls all 64 with one load
// per lane.  Layout (ints): [O lines | gate_up lines | done | err], 32-int (128 B) line stride.
constexpr int MLP_LINES = 64, MLP_STRIDE = 32;
constexpr int MLP_CNT_O = 0, MLP_CNT_GU = MLP_LINES * MLP_STRIDE, MLP_DONE = 2 * MLP_LINES * MLP_STRIDE,
              MLP_ERR = MLP_DONE + MLP_STRIDE;
static_assert(MLP_ERR + 1 <= DECODE_MLP_CTL_INTS, "ctl block too small");

struct WaitFor {
  const int* cnt;  // first line of the awaited phase
  int n;           // tiles in that phase
  int* err;
  SYM_DEV void operator()() const {
    if (threadIdx.x < 64) {
      const int l = threadIdx.x;
      const int target = n / MLP_LINES + (l < n % MLP_LINES ? 1 : 0);
      const int* c = cnt + l * MLP_STRIDE;
      int it = 0;
      while (!__all(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target)) {
        __builtin_amdgcn_s_sleep(2);
        if (++it > (1 << 22)) {  // ~0.2 s: never hang the GPU on a bug, flag it
          if (l == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // no activation load is hoisted above the wait
  }
};

SYM_DEV void publish(int* cnt, int tile) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores have landed
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(cnt + (tile % MLP_LINES) * MLP_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NW, int U, int WPE>
__global__ __launch_bounds__(NW * 64, WPE) void decode_mlp_kernel(DecodeMlpArgs a) {
  const int nO = a.d / 16, nG = 2 * a.F / 16, nD = a.d / 16;
  const int total = nO + nG + nD;
  int* ctl = a.ctl;
  DecodeEpi eo, eg, ed;
  eo.wshuf = eg.wshuf = ed.wshuf = a.wshuf;
  eo.resid = ed.resid = a.resid;
  eo.w_next = a.ln2;
  eo.xw_out = ed.xw_out = a.xw;
  eo.ss_out = ed.ss_out = a.ss;
  eo.sc1 = 1;
  eg.ss_in = a.ss;
  eg.ss_tiles = a.d / 16;
  eg.inv_d = 1.f / (float)a.d;
  eg.eps = a.eps;
  eg.act = a.act;
  eg.sc1 = 1;
  ed.w_next = a.w_next;
  ed.resid_sc1 = 1;
  // static striding (no queue atomics on the critical path): round r of workgroup b is tile b + r * grid,
  // so every O tile is in round 0 and phases are still dequeued in order
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    if (t < nO) {
      gemm_tile<1, NW, U, 1, DECODE_EPI_RESID>(a.attn, a.Wo, a.M, a.d, a.dq, eo, t, NoWait{});
      publish(ctl + MLP_CNT_O, t);
    } else if (t < nO + nG) {
      gemm_tile<1, NW, U, 1, DECODE_EPI_SWIGLU>(a.xw, a.Wgu, a.M, 2 * a.F, a.d, eg, t - nO,
                                                WaitFor{ctl + MLP_CNT_O, nO, ctl + MLP_ERR});
      publish(ctl + MLP_CNT_GU, t - nO);
    } else {
      gemm_tile<1, NW, U, 1, DECODE_EPI_RESID>(a.act, a.Wd, a.M, a.d, a.F, ed, t - nO - nG,
                                               WaitFor{ctl + MLP_CNT_GU, nG, ctl + MLP_ERR});
    }
    __syncthreads();  // LDS reduction buffers are reused by the next tile
  }
  __shared__ int s_last;
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(ctl + MLP_DONE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  __syncthreads();
  if (s_last) {  // last workgroup out (every other one is past its waits): re-arm for the next launch
    for (int i = threadIdx.x; i < 2 * MLP_LINES; i += blockDim.x)
      __hip_atomic_store(ctl + i * MLP_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(ctl + MLP_DONE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------------------------------
// Persistent decode MLP on x-resident bodies: O -> gate_up -> down of one layer in ONE launch, one 16-wave
// workgroup per CU (M <= 16, dq = d = 1024 U, F % 1024 == 0).
//
// decode_mlp_kernel above ran every phase on 8-wave gemm_tile bodies (10-38 spilled VGPRs) and lost to the
// three launches.  Here O and gate_up run the decode_gemm_xres_kernel body (each wave loads its k-slice of x
// once per phase, the next tile's weights are in flight during a tile's reduction and epilogue) and down runs
// 16 waves splitting K = F in rounds of U k-blocks.
//
// Where the launches lose time is where HBM idles: the latency-bound O projection (33.5 MB in ~10 us, half
// the chip's rate), the launch boundaries and every launch's ramp and tail.  So the weights of the NEXT
// phase's first round are staged into LDS by LDS-DMA early, with nothing waiting on them: gate_up tile 0
// (128 KB per CU at U = 4, 32 MB chip-wide) from the first instruction of the launch, behind the O loads;
// the down tile's first U k-blocks of every wave from gate_up tile 1 on (the LDS slice is free once tile
// 0's fragments are in registers).  A phase then starts on bytes that are already on chip.  Measured
// variants: profiles/r3/mlp_xres_*.jsonl (bench/kernels/bench_decode_mlp.py --xcfgs, --stamps).
//
// Hand-offs (MI355X_MICROARCH.md hand-off table, first row): wave 0 runs every epilogue of its workgroup and
// stores write-through (sc1); after the workgroup's last tile of a phase it drains vmcnt and ONE lane adds
// to the workgroup's counter line (b % 64); wave 0 keeps no weight loads of its own in flight across a
// publish or a poll (its slice of a next round is issued after them), so neither waits on the stream.  The
// consumer's wave 0 polls the 64 lines with sc1 loads, a workgroup barrier follows, then every read of
// handed-off bytes (xw, the ss partials, act, the residual) is an sc1 (L1-bypassing) load -- 16-B buffer
// loads (aux 16): the 8-B atomic form doubled the request count and cost 9 us per layer at M = 10.  No acquire
// fence: its buffer_inv + vmcnt(0) would wait for the weight stream in flight.  Write-after-read is safe by
// the edges: xw / ss are rewritten by the down epilogue only after every workgroup has published its
// gate_up phase, i.e. finished reading them.
// Deadlock freedom: grid = #CUs with one resident workgroup per CU (checked at the first launch).  Spins are
// bounded (error word); the last workgroup out re-arms the counter lines (graph-replay safe).
// O and gate_up are bitwise equal to the x-resident launches; down sums K in a different order than the
// 4-wave standalone kernel (fp32-close).
// ---------------------------------------------------------------------------------------------------
// 16 B from a buffer resource; aux 16 = sc1 (L1-bypassing: bytes written by another CU in this launch)
SYM_DEV uint4 ldbuf16_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

SYM_DEV __amdgpu_buffer_rsrc_t mk_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

int g_mlp_xcfg = 0;  // A/B knobs of decode_mlp_xres_kernel (set_decode_gemm_variant(2000 + bits)):
                     // 8 = no down-tile LDS staging, 16 = no gate_up-tile LDS staging

template <int U>
__global__ __launch_bounds__(1024) void decode_mlp_xres_kernel(DecodeMlpArgs a) {
  constexpr int NW = 16;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int b = blockIdx.x, G = gridDim.x;
  const int M = a.M, d = a.d, F = a.F;
  const int nO = d / 16, nG = 2 * F / 16, nD = d / 16;
  const int tO = nO > b ? (nO - b + G - 1) / G : 0;  // this workgroup's tiles per phase: b, b + G, ...
  const int tG = nG > b ? (nG - b + G - 1) / G : 0;
  const int tD = nD > b ? (nD - b + G - 1) / G : 0;
  const int nb = F / 1024;  // down k-blocks per wave
  const bool stage_g = !(a.xcfg & 16) && tG > 0, stage_d = !(a.xcfg & 8) && tD > 0 && tG > 1;
  int* ctl = a.ctl;
  const int wmul = a.wshuf ? 16 : 1, wsec = a.wshuf ? 512 : 32;
  const int m = r16;
  const bool mok = m < M;
  const int mr = min(r16, M - 1);
  auto wptr = [&](const bf16* W, int K, int t) -> const bf16* {  // this wave's k-slice of 16-row tile t
    const int kbeg = wid * (K / NW);
    return a.wshuf ? W + ((long long)t * (K / 32) + kbeg / 32) * 512 + lane * 8
                   : W + (long long)(16 * t + r16) * K + kbeg + 8 * h;
  };
  Pack8 wa[U][2];
  auto load_w = [&](const bf16* wp, int j0, int n) {  // k-blocks j0 .. j0 + U - 1 (< n) of a slice
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (j0 + j < n) {
        wa[j][0].u = *reinterpret_cast<const uint4*>(wp + (j0 + j) * 64 * wmul);
        wa[j][1].u = *reinterpret_cast<const uint4*>(wp + (j0 + j) * 64 * wmul + wsec);
      }
  };
  // per-wave LDS staging slice (U k-blocks x 2 halves x 1 KB) filled by LDS-DMA: lane l's 16 B land at l * 16
  __shared__ __attribute__((aligned(1024))) char pf[NW][U][2][1024];
  __shared__ f32x4 red[2][NW - 1][64];  // waves 1..15's partials (wave 0 keeps its own in registers)
  auto stage = [&](const bf16* wp, int n) {  // the first min(U, n) k-blocks of a slice -> this wave's pf
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (j < n) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(wp + j * 64 * wmul + hf * wsec),
              (__attribute__((address_space(3))) void*)&pf[wid][j][hf][0], 16, 0, 0);
      }
  };
  auto unstage = [&](int n) {  // staged k-blocks -> wa (the wave's own DMAs: vmcnt covers them)
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (j < n) {
        wa[j][0].u = *reinterpret_cast<const uint4*>(&pf[wid][j][0][lane * 16]);
        wa[j][1].u = *reinterpret_cast<const uint4*>(&pf[wid][j][1][lane * 16]);
      }
  };
  DecodeEpi eo, eg, ed;
  eo.resid = ed.resid = a.resid;
  eo.w_next = a.ln2;
  eo.xw_out = ed.xw_out = a.xw;
  eo.ss_out = ed.ss_out = a.ss;
  eo.sc1 = 1;  // resid / xw / ss read by other CUs of this launch
  eg.act = a.act;
  eg.sc1 = 1;
  ed.w_next = a.w_next;
  ed.resid_sc1 = 1;  // the residual was rewritten by the O phase of this launch
  int buf = 0;
  long long* st = a.stamps ? a.stamps + 8 * b : nullptr;  // phase stamps (timing only)
  auto stamp = [&](int k) {
    if (st && threadIdx.x == 0) st[k] = (long long)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // wave 0 reduces a tile's 16 partials (same order as decode_gemm_xres_kernel: bitwise-equal results)
  auto reduce = [&](f32x4 acc) -> f32x4 {
    if (wid != 0) red[buf][wid - 1][lane] = acc;
    __syncthreads();
    f32x4 v = acc;
    if (wid == 0) {
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        v += red[buf][w - 1][lane];
        if ((w & 3) == 3) asm volatile("" : "+v"(v)::"memory");
      }
    }
    buf ^= 1;
    return v;
  };
  auto publish = [&](int* lines) {  // wave 0 only: its write-through stores acknowledged, then one add
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_fetch_add(lines + (b % MLP_LINES) * MLP_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto mma = [&](const Pack8 (&xa)[U][2], int n) -> f32x4 {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (j < n) {
        acc = mfma16(wa[j][0].v, xa[j][0].v, acc);
        acc = mfma16(wa[j][1].v, xa[j][1].v, acc);
      }
    return acc;
  };

  // ---- phase O: attn [M, d] (previous launch's output: plain loads) x Wo -> resid, xw, ss (sc1) ----
  if (tO > 0) load_w(wptr(a.Wo, d, b), 0, U);
  {
    Pack8 xa[U][2];
    const bf16* xrow = a.attn + (long long)mr * d + wid * (d / NW) + 8 * h;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      xa[j][0].u = mok ? *reinterpret_cast<const uint4*>(xrow + j * 64) : make_uint4(0, 0, 0, 0);
      xa[j][1].u = mok ? *reinterpret_cast<const uint4*>(xrow + j * 64 + 32) : make_uint4(0, 0, 0, 0);
    }
    if (stage_g) stage(wptr(a.Wgu, d, b), U);  // gate_up tile 0 streams in behind the O loads
    for (int i = 0; i < tO; ++i) {
      const int t = b + i * G;
      const f32x4 acc = mma(xa, U);
      __builtin_amdgcn_sched_barrier(0);
      if (i + 1 < tO) load_w(wptr(a.Wo, d, t + G), 0, U);
      const f32x4 v = reduce(acc);
      if (wid == 0) epilogue<DECODE_EPI_RESID>(eo, v, t, m, mok, h, d);
    }
  }
  stamp(1);
  if (wid == 0) publish(ctl + MLP_CNT_O);

  // ---- phase gate_up: xw (sc1) x Wgu, RMSNorm row scale from the ss partials (sc1) -> act (sc1) ----
  if (wid != 0 && !stage_g && tG > 0) load_w(wptr(a.Wgu, d, b), 0, U);
  WaitFor{ctl + MLP_CNT_O, G, ctl + MLP_ERR}();
  stamp(2);
  {
    Pack8 xa[U][2];
    const __amdgpu_buffer_rsrc_t xr = mk_rsrc(a.xw, (long long)M * d * 2);
    const int xo = (mr * d + wid * (d / NW) + 8 * h) * 2;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      xa[j][0].u = mok ? ldbuf16_sc1(xr, xo + j * 128) : make_uint4(0, 0, 0, 0);
      xa[j][1].u = mok ? ldbuf16_sc1(xr, xo + j * 128 + 64) : make_uint4(0, 0, 0, 0);
    }
    if (wid == 0 && !stage_g && tG > 0) load_w(wptr(a.Wgu, d, b), 0, U);
    float rn = 1.f;  // wave 0: the deferred-RMSNorm scale of row r16 (lanes h = 0..3 sum a quarter each)
    if (wid == 0) {
      const __amdgpu_buffer_rsrc_t sr = mk_rsrc(a.ss, (long long)M * (d / 16) * 4);
      float s = 0.f;
      if (mok)
        for (int i = 4 * h; i < d / 16; i += 16) {  // 16-B chunks h, h + 4, ... of row r16's partials
          const uint4 q = ldbuf16_sc1(sr, (mr * (d / 16) + i) * 4);
          s += __uint_as_float(q.x) + __uint_as_float(q.y) + __uint_as_float(q.z) + __uint_as_float(q.w);
        }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      rn = rsqrtf(s / (float)d + a.eps);
    }
    for (int i = 0; i < tG; ++i) {
      const int t = b + i * G;
      if (i == 0 && stage_g) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA landed (and x, needed next anyway)
        unstage(U);
      }
      const f32x4 acc = mma(xa, U);
      __builtin_amdgcn_sched_barrier(0);
      if (i + 1 < tG) load_w(wptr(a.Wgu, d, t + G), 0, U);
      if (i == 0 && stage_d) {  // the down tile's first round streams in for the rest of this phase
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's pf reads are done
        stage(wptr(a.Wd, F, b), nb);
      }
      f32x4 v = reduce(acc);
      if (wid == 0) {
        const float sc = mok ? rn : 1.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] *= sc;
        epilogue<DECODE_EPI_SWIGLU>(eg, v, t, m, mok, h, 2 * F);
      }
    }
  }
  stamp(3);
  if (wid == 0) publish(ctl + MLP_CNT_GU);

  // ---- phase down: act (sc1) x Wd, 16 waves splitting K = F -> resid (sc1 reads), xw, ss for the next launch ----
  const int j1 = stage_d ? U : 0;  // first k-block not staged
  if (wid != 0 && tD > 0 && j1 < nb) load_w(wptr(a.Wd, F, b), j1, nb);  // the round after the staged one
  WaitFor{ctl + MLP_CNT_GU, G, ctl + MLP_ERR}();
  stamp(4);
  const __amdgpu_buffer_rsrc_t ar = mk_rsrc(a.act, (long long)M * F * 2);
  for (int i = 0; i < tD; ++i) {
    const int t = b + i * G;
    const bf16* wp = wptr(a.Wd, F, t);
    const int xo = (mr * F + wid * (F / NW) + 8 * h) * 2;
    auto ldx = [&](Pack8 (&xa)[U][2], int j0) {
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (j0 + j < nb) {
          xa[j][0].u = mok ? ldbuf16_sc1(ar, xo + (j0 + j) * 128) : make_uint4(0, 0, 0, 0);
          xa[j][1].u = mok ? ldbuf16_sc1(ar, xo + (j0 + j) * 128 + 64) : make_uint4(0, 0, 0, 0);
        }
    };
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int j0 = 0;
    if (i == 0 && stage_d) {  // round 0 from LDS; wave != 0 already has round 1 in flight in wa
      Pack8 xs[U][2];
      ldx(xs, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA landed (x is the youngest load anyway)
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (j < nb) {  // one k-block of staged weights in registers at a time (wa holds the next round)
          Pack8 w0, w1;
          w0.u = *reinterpret_cast<const uint4*>(&pf[wid][j][0][lane * 16]);
          w1.u = *reinterpret_cast<const uint4*>(&pf[wid][j][1][lane * 16]);
          acc = mfma16(w0.v, xs[j][0].v, acc);
          acc = mfma16(w1.v, xs[j][1].v, acc);
          __builtin_amdgcn_sched_barrier(0);
        }
      j0 = U;
    }
    for (; j0 < nb; j0 += U) {
      if (!(i == 0 && j0 == j1 && wid != 0)) load_w(wp, j0, nb);  // (wave != 0: round j1 is in flight)
      Pack8 xa[U][2];
      ldx(xa, j0);
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (j0 + j < nb) {
          acc = mfma16(wa[j][0].v, xa[j][0].v, acc);
          acc = mfma16(wa[j][1].v, xa[j][1].v, acc);
        }
    }
    const f32x4 v = reduce(acc);
    if (wid == 0) epilogue<DECODE_EPI_RESID>(ed, v, t, m, mok, h, d);
  }
  if (st && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(5);
  }

  // last workgroup out (every other one is past both waits): re-arm the counter lines for the next launch
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(ctl + MLP_DONE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
  __syncthreads();
  if (s_last) {
    for (int i = threadIdx.x; i < 2 * MLP_LINES; i += blockDim.x)
      __hip_atomic_store(ctl + i * MLP_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(ctl + MLP_DONE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// ---------------------------------------------------------------------------------------------------
// Fused decode attention block: QKV projection (+ RoPE, paged K/V write) -> split-KV attention ->
// O-projection (+ residual, ln2 prep) of one layer in ONE launch (M <= 16 rows, TP = 1).
//
// Grid = [QKV tiles | attention units (seq, kv head, partition) | O tiles], 512 threads each.
//   * QKV tile: the decode GEMM tile of the 5-launch path with write-through (sc1) q / K / V stores,
//     then one add to its kv group's counter (8 (G + 2) tiles per group).
//   * attention unit: loads its context length and block-table entries, polls its group's counter,
//     acquires, then runs the standalone kernel's arithmetic (attn_decode.h) and stores its output rows
//     write-through; the workgroup that produced final rows adds to a done line.
//   * O tile: issues its whole weight slice (8 k-blocks per wave) FIRST, then polls the done lines,
//     acquires and reads the attention output: the O weight stream overlaps the attention phase,
//     which moves few bytes, and the two launch boundaries of the 5-launch path disappear.
// Hand-offs follow MI355X_MICROARCH.md's valid forms: sc1 payload stores, every storing wave drains
// vmcnt, a barrier, ONE lane adds to the counter; the consumer polls relaxed, ONE agent acquire, vmcnt,
// barrier, then plain loads.  Deadlock freedom: consumers sit after every producer in the grid, and
// workgroups are dispatched in grid order, so a waiting workgroup only waits for workgroups that are
// already running; every spin is bounded (error word instead of a hang).  The last workgroup out
// re-arms the control words for the next launch (graph-replay safe, no memset node).
// Results are bitwise equal to dg_qkv + attn_decode + dg_resid with decode_gemm variant 0.
// ---------------------------------------------------------------------------------------------------
constexpr int DB_STRIDE = 32, DB_DONE_LINES = 8;

SYM_DEV void db_publish(int* word) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores have landed
  __syncthreads();                                   // ... and every other wave's
  if (threadIdx.x == 0) __hip_atomic_fetch_add(word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0 polls `nlines` counter lines (line l must reach base + (l < rem)), then acquires for the CU.
struct BlockWait {
  const int* cnt;
  int nlines, base, rem;
  int* err;
  long long* stamp;  // diagnostics: s_memrealtime when the wait completed (nullptr: off)
  int no_acquire;    // A/B timing knob only
  SYM_DEV void operator()() const {
    if (threadIdx.x < 64) {
      const int l = threadIdx.x;
      const bool mine = l < nlines;
      const int target = base + (l < rem ? 1 : 0);
      const int* c = cnt + (mine ? l : 0) * DB_STRIDE;
      int it = 0;
      while (!__all(!mine || __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target)) {
        __builtin_amdgcn_s_sleep(2);
        if (++it > (1 << 22)) {  // ~0.2 s: never hang the GPU on a bug, flag it
          if (l == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      if (!no_acquire) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drop this CU's stale L1 lines
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (stamp && threadIdx.x == 0) *stamp = (long long)__builtin_amdgcn_s_memrealtime();
  }
};

// O-projection tile of the fused block (16 output columns n0.., M <= 16 rows, 8 waves splitting K = Hq * 128).
// Before `wait` (the poll for the attention output): the first OPF k-blocks of every wave's weight slice
// (all of them at Llama-3-8B sizes), and, on the epilogue wave, the residual and next-norm weight it will
// read; after it: the attention rows (x) four k-blocks at a time, the LDS reduction and the residual
// epilogue.  Same arithmetic as gemm_tile<1, 8, *, 1, RESID>.
template <int OPF, typename WaitFn>
SYM_DEV void o_tile_fused(const DecodeBlockArgs& a, int tile, WaitFn wait) {
  const int K = a.Hq * 128, M = a.M, N = a.d;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int wk = K / 8, kbeg = wid * wk, nblk = wk / 64;
  const int wmul = a.wshuf ? 16 : 1, wsec = a.wshuf ? 512 : 32;
  const bf16* wrow = a.wshuf ? a.Wo + ((long long)tile * (K / 32) + kbeg / 32) * 512 + lane * 8
                             : a.Wo + (long long)(16 * tile + r16) * K + kbeg + 8 * h;
  const bool xok = r16 < M;
  const bf16* xrow = a.attn + (long long)min(r16, M - 1) * K + kbeg + 8 * h;
  Pack8 w[OPF][2];
#pragma unroll
  for (int u = 0; u < OPF; ++u) {
    if (u < nblk) {
      w[u][0].u = *reinterpret_cast<const uint4*>(wrow + u * 64 * wmul);
      w[u][1].u = *reinterpret_cast<const uint4*>(wrow + u * 64 * wmul + wsec);
    }
  }
  const int n0 = tile * 16;
  const int m = r16;
  float4 rpre = make_float4(0.f, 0.f, 0.f, 0.f);
  uint2 wnpre = make_uint2(0, 0);
  if (wid == 0 && xok) {  // bytes nobody writes in this launch: safe to read before the hand-off
    rpre = *reinterpret_cast<const float4*>(a.resid + (long long)m * N + n0 + 4 * h);
    wnpre = *reinterpret_cast<const uint2*>(a.ln2 + n0 + 4 * h);
  }
  wait();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  auto ldx = [&](int ko) -> uint4 {
    return xok ? *reinterpret_cast<const uint4*>(xrow + ko) : make_uint4(0, 0, 0, 0);
  };
#pragma unroll
  for (int u = 0; u < OPF; u += 4) {  // x of 4 k-blocks per round trip (32 VGPRs next to the 64 of W)
    Pack8 xa[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (u + j < nblk) {
        xa[j][0].u = ldx((u + j) * 64);
        xa[j][1].u = ldx((u + j) * 64 + 32);
      }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (u + j < nblk) {
        acc = mfma16(w[u + j][0].v, xa[j][0].v, acc);
        acc = mfma16(w[u + j][1].v, xa[j][1].v, acc);
      }
  }
  for (int b = OPF; b < nblk; ++b) {  // K > 8 * 64 * OPF (e.g. 70B at TP = 1): streamed after the wait
    Pack8 w0, w1, x0, x1;
    w0.u = *reinterpret_cast<const uint4*>(wrow + b * 64 * wmul);
    w1.u = *reinterpret_cast<const uint4*>(wrow + b * 64 * wmul + wsec);
    x0.u = ldx(b * 64);
    x1.u = ldx(b * 64 + 32);
    acc = mfma16(w0.v, x0.v, acc);
    acc = mfma16(w1.v, x1.v, acc);
  }
  __shared__ f32x4 ored[8][64];
  ored[wid][lane] = acc;
  __syncthreads();
  if (wid != 0) return;
  f32x4 v = ored[0][lane];
#pragma unroll
  for (int ww = 1; ww < 8; ++ww) v += ored[ww][lane];
  // residual epilogue (epilogue<DECODE_EPI_RESID> with the operands loaded before the wait)
  float sq = 0.f;
  if (xok) {
    const float rr[4] = {rpre.x + v[0], rpre.y + v[1], rpre.z + v[2], rpre.w + v[3]};
    Pack8 wp;
    wp.u = make_uint4(wnpre.x, wnpre.y, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) sq += rr[i] * rr[i];
    *reinterpret_cast<float4*>(a.resid + (long long)m * N + n0 + 4 * h) = make_float4(rr[0], rr[1], rr[2], rr[3]);
    store4bf(a.xw_out + (long long)m * N + n0 + 4 * h, rr[0] * (float)wp.h[0], rr[1] * (float)wp.h[1],
             rr[2] * (float)wp.h[2], rr[3] * (float)wp.h[3]);
  }
  sq += __shfl_xor(sq, 16, 64);
  sq += __shfl_xor(sq, 32, 64);
  if (xok && h == 0) a.ss_out[(long long)m * (N / 16) + tile] = sq;
}

__global__ __launch_bounds__(512, 4) void decode_block_kernel(DecodeBlockArgs a) {
  const int Hq = a.Hq, Hkv = a.Hkv, G = Hq / Hkv;
  const int nQ = (Hq + 2 * Hkv) * 8, nA = a.M * Hkv * a.max_parts, nO = a.d / 16;
  int* ctl = a.ctl;
  int* done = ctl + Hkv * DB_STRIDE;
  int* exit_word = done + DB_DONE_LINES * DB_STRIDE;
  int* err = exit_word + DB_STRIDE;
  const int b = blockIdx.x;
  long long* st = a.stamps ? a.stamps + 4 * b : nullptr;
  if (st && threadIdx.x == 0) {
    st[0] = (long long)__builtin_amdgcn_s_memrealtime();
    st[3] = b < nQ ? 0 : (b < nQ + nA ? 1 : 2);
  }
  if (b < nQ) {
    DecodeEpi e;
    e.wshuf = a.wshuf;
    e.sc1 = 1;
    e.ss_in = a.ss_in;
    e.ss_tiles = a.ss_tiles;
    e.inv_d = a.inv_d;
    e.eps = a.eps;
    e.positions = a.positions;
    e.slots = a.slots;
    e.cos_sin = a.cos_sin;
    e.q_out = a.q;
    e.k_cache = a.k_cache;
    e.v_cache = a.v_cache;
    e.Hq = Hq;
    e.Hkv = Hkv;
    e.BS = a.BS;
    gemm_tile<1, 8, 4, 1, DECODE_EPI_QKV>(a.xw, a.Wqkv, a.M, nQ * 16, a.d, e, b, NoWait{});
    const int head = b / 8;
    const int grp = head < Hq ? head / G : (head < Hq + Hkv ? head - Hq : head - Hq - Hkv);
    db_publish(ctl + grp * DB_STRIDE);
  } else if (b < nQ + nA) {
    const int u = b - nQ, per_part = a.M * Hkv;
    const int part = u / per_part, seq = (u % per_part) / Hkv, kvh = u % Hkv;
    const bool fin = attn_fused_unit<8>(a.q, a.k_cache, a.v_cache, a.block_tables, a.ctx_lens, a.attn, a.tmp_o,
                                        a.tmp_ml, a.part_counters, Hq, Hkv, a.BS, a.max_blocks, a.max_parts,
                                        a.scale_log2, seq, kvh, part,
                                        BlockWait{ctl + kvh * DB_STRIDE, 1, 8 * (G + 2), 0, err,
                                                  st ? st + 1 : nullptr, a.cfg & 2});
    if (fin) db_publish(done + ((seq * Hkv + kvh) % DB_DONE_LINES) * DB_STRIDE);
  } else {
    const int units = a.M * Hkv;
    o_tile_fused<8>(a, b - nQ - nA,
                 BlockWait{done, DB_DONE_LINES, units / DB_DONE_LINES, units % DB_DONE_LINES, err,
                           st ? st + 1 : nullptr, a.cfg & 2});
  }
  if (st && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st[2] = (long long)__builtin_amdgcn_s_memrealtime();
  }
  // last workgroup out (every other one is past its waits): re-arm the counters for the next launch
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(exit_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  __syncthreads();
  if (s_last) {
    for (int i = threadIdx.x; i < Hkv + DB_DONE_LINES; i += blockDim.x)
      __hip_atomic_store(ctl + i * DB_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(exit_word, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
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
      float sacc = 0.f;
      for (int i = lane; i < e.ss_tiles; i += 64) sacc += e.ss_in[(long long)m * e.ss_tiles + i];
      sacc = wave_sum(sacc);
      if (lane == 0) rn_s[m] = rsqrtf(sacc * e.inv_d + e.eps);
    }
  }
  __shared__ f32x4 red[2][NW][64];
  unsigned xep = 0;
  if constexpr (EPI == DECODE_EPI_XPUSH) xep = xp_epoch(e.xp);
  const int m = r16;
  const bool mok = m < M;
  auto finish = [&](f32x4 v, int t, int hf = -1) {  // wave 0: row scale + epilogue of a final tile (or half)
    const float sc = (e.ss_in && mok) ? rn_s[m] : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= sc;
    epilogue<EPI>(e, v, t, m, mok && (hf < 0 || (h & 1) == hf), h, N, xep);
    if constexpr (EPI == DECODE_EPI_XPUSH) {  // wave 0 stored the whole tile: acknowledged, then flag it
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane < e.xp.world) xp_flag(e.xp, lane, t, xep);
    }
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
  int grid = (ntiles + per - 1) / per, NF = ntiles, P = 0, KS = 1;
  // remainder split: weight bytes on the busiest CU, f K + q K / KS, must drop >= 10 % (<= 4 parts per
  // workgroup, >= 4 waves per part)
  const int f = ntiles / C, R = ntiles - f * C;
  if (g_dg_ksplit && R > 0 && e.ks_ws && e.ks_cnt && e.ks_ncnt >= R && EPI != DECODE_EPI_ARGMAX) {
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

// ---------------------------------------------------------------------------------------------------
// Fused QKV + decode attention launch (M <= 16, K = 1024 U, G = Hq / Hkv <= 8).
//
// The x-resident QKV GEMM walks its 16-row tiles on ceil(ntiles / per) workgroups -- Llama-3-8B: 384 tiles,
// two per workgroup on 192 of the 256 CUs -- and the decode attention then runs as its own launch: a launch
// boundary plus a dependent load chain (~6.5 us at 10 sequences) on a chip whose HBM sits idle.  Here the
// attention units ride in the same launch as extra 16-wave workgroups (two 8-wave units each, attn_decode.h
// attn_pair_units) after the QKV workgroups, i.e. on the CUs the QKV grid leaves idle: they read their
// context length, block-table entry and every K/V group not written this step while the QKV tiles stream,
// then wait for all QKV workgroups, and only the query and the newest token's group remain to be read.
// Hand-off (MI355X_MICROARCH.md hand-off table, first row): the QKV epilogue (wave 0) stores q / K / V
// write-through (sc1), drains vmcnt after the workgroup's last tile and ONE lane adds to the workgroup's
// counter line (b % 64); the attention workgroup's wave 0 polls the 64 lines, a barrier follows, and every
// load of those bytes is an sc1 load.  Deadlock freedom: the attention workgroups come after every QKV
// workgroup in the grid (dispatched in order), spins are bounded (error word), and the last workgroup out
// re-arms the lines (graph-replay safe).  Results equal dg_qkv + attn_decode (same arithmetic, same order).
// ctl: QKV_ATTN_CTL_INTS ints [64 lines x 32 | exit | error], zero-initialised once.
// ---------------------------------------------------------------------------------------------------
constexpr int QA_EXIT = MLP_LINES * MLP_STRIDE, QA_ERR = QA_EXIT + MLP_STRIDE;
static_assert(QA_ERR + 1 <= QKV_ATTN_CTL_INTS, "qkv_attn ctl block too small");

template <int U, int GMAX>
__global__ __launch_bounds__(1024) void decode_qkv_attn_kernel(const bf16* __restrict__ x, const bf16* __restrict__ W,
                                                               int M, int N, int K, DecodeEpi e, int Gq,
                                                               QkvAttnArgs aa) {
  int* ctl = aa.ctl;
  const int b = blockIdx.x;
  long long* st = aa.stamps ? aa.stamps + 4 * b : nullptr;  // timing only: start, mid, end, role
  if (st && threadIdx.x == 0) {
    st[0] = (long long)__builtin_amdgcn_s_memrealtime();
    st[3] = b < Gq ? 0 : 1;
  }
  if (b < Gq) {
    xres_body<U, 1, DECODE_EPI_QKV>(x, W, M, N, K, e, N / 16, 0, b, Gq);
    if (threadIdx.x < 64) {  // wave 0 ran every epilogue of this workgroup: its stores acknowledged, one add
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (threadIdx.x == 0)
        __hip_atomic_fetch_add(ctl + (b % MLP_LINES) * MLP_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (st && threadIdx.x == 0) st[1] = (long long)__builtin_amdgcn_s_memrealtime();
    }
  } else {
    WaitFor wf{ctl, Gq, ctl + QA_ERR};
    attn_pair_units<GMAX>(e.q_out, e.k_cache, e.v_cache, aa.block_tables, aa.ctx_lens, aa.out, aa.tmp_o, aa.tmp_ml,
                          aa.counters, e.Hq, e.Hkv, e.BS, aa.max_blocks, aa.max_parts, aa.scale_log2, M, b - Gq,
                          [&]() {
                            wf();
                            if (st && threadIdx.x == 0) st[1] = (long long)__builtin_amdgcn_s_memrealtime();
                          });
  }
  if (st && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st[2] = (long long)__builtin_amdgcn_s_memrealtime();
  }
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(ctl + QA_EXIT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  __syncthreads();
  if (s_last) {  // every other workgroup is past its wait: re-arm for the next launch
    for (int i = threadIdx.x; i < MLP_LINES; i += blockDim.x)
      __hip_atomic_store(ctl + i * MLP_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(ctl + QA_EXIT, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

template <int MT, int EPI>
void launch_mt(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e, hipStream_t s) {
  constexpr int U0 = MT == 1 ? 4 : (MT == 2 ? 2 : 1);
  constexpr int U1 = MT == 1 ? 8 : (MT == 2 ? 4 : 2);
  int v = g_variant;
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
      // the vocabulary projection at <= 4 rows where the 8-wave split stays ahead
      if (M <= 16 && K % 1024 == 0 && K <= 4096 && !(N >= 65536 && M <= 4)) v = 11;
      // wide N at 5..16 rows otherwise: 7 resident 4-wave workgroups per CU (gate_up's 1792 tiles in one
      // round): 45.3 vs 46.9 us (profiles/decode_gemm_occupancy_r1.jsonl)
      // above 16 rows (profiles/decode_gemm_bigm_r1.jsonl, M = 64): wide N shares each x fragment over
      // four row tiles (gate_up 93.6 -> 76.7 us, lm_head 367 -> 307), qkv over two (43.7 -> 33.3)
      // (eight row tiles from 25 rows: gate_up 77.0 -> 69.1 us at M = 64, profiles/decode_gemm_rt8_r1.jsonl)
      else if (N >= 12288) v = M > 16 ? (M > 24 ? 14 : 3) : (M <= 4 ? 0 : 8);
      else if (M > 16 && N > 4096) v = 3;
      else if (N <= 4096 && K % 1024 == 0) v = K > 4096 ? 4 : 2;  // few row tiles: split K (down_proj: 4 waves,
                                                                  // 24.2 vs 25.7 us at M = 10)
      else v = 0;
    } else if (M <= 4) {
      v = 0;
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

long long* g_qa_stamps = nullptr;
void set_qkv_attn_stamps(long long* p) { g_qa_stamps = p; }

bool launch_qkv_attn(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e0, const QkvAttnArgs& aa,
                     hipStream_t s) {
  const int G = e0.Hq / e0.Hkv;
  if (M > 16 || K % 1024 || K > 4096 || G > 8 || !e0.wshuf || (e0.BS & (e0.BS - 1)) ||
      !attn_decode_uses_grid(M, e0.Hkv, e0.BS, aa.max_blocks, G))
    return false;
  if (!g_num_cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
    g_num_cus = std::max(1, g_num_cus);
  }
  const int ntiles = N / 16, per = (ntiles + g_num_cus - 1) / g_num_cus;
  const int Gq = (ntiles + per - 1) / per;
  const int Ga = (M * e0.Hkv * aa.max_parts + 1) / 2;
  DecodeEpi e = e0;
  e.sc1 = 1;  // q / K / V read by the attention workgroups of this launch
  e.wnt = g_wnt;
  QkvAttnArgs a2 = aa;
  a2.stamps = g_qa_stamps;
  auto go = [&](auto kern) { kern<<<Gq + Ga, 1024, 0, s>>>(x, W, M, N, K, e, Gq, a2); };
  switch (K / 1024 * 16 + (G <= 4 ? 4 : 8)) {
    case 16 + 4: go(decode_qkv_attn_kernel<1, 4>); return true;
    case 16 + 8: go(decode_qkv_attn_kernel<1, 8>); return true;
    case 32 + 4: go(decode_qkv_attn_kernel<2, 4>); return true;
    case 32 + 8: go(decode_qkv_attn_kernel<2, 8>); return true;
    case 64 + 4: go(decode_qkv_attn_kernel<4, 4>); return true;
    case 64 + 8: go(decode_qkv_attn_kernel<4, 8>); return true;
    default: return false;
  }
}

void launch_decode_gemm(int epi, const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e,
                        hipStream_t s) {
  switch (epi) {
    case DECODE_EPI_F32: launch_epi<DECODE_EPI_F32>(x, W, M, N, K, e, s); break;
    case DECODE_EPI_QKV: launch_epi<DECODE_EPI_QKV>(x, W, M, N, K, e, s); break;
    case DECODE_EPI_RESID: launch_epi<DECODE_EPI_RESID>(x, W, M, N, K, e, s); break;
    case DECODE_EPI_SWIGLU: launch_epi<DECODE_EPI_SWIGLU>(x, W, M, N, K, e, s); break;
    case DECODE_EPI_XPUSH: launch_epi<DECODE_EPI_XPUSH>(x, W, M, N, K, e, s); break;
    default: launch_epi<DECODE_EPI_ARGMAX>(x, W, M, N, K, e, s); break;
  }
}

int g_mlp_cfg = -1;

template <int NW, int U, int WPE>
void go_mlp(const DecodeMlpArgs& a, hipStream_t s) {
  static int resident = 0;
  if (!resident) {  // one persistent workgroup per resident slot
    int dev = 0, cus = 0, per_cu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_mlp_kernel<NW, U, WPE>, NW * 64, 0);
    resident = std::max(1, cus) * std::max(1, per_cu);
  }
  const int total = a.d / 16 + 2 * a.F / 16 + a.d / 16;
  decode_mlp_kernel<NW, U, WPE><<<std::min(total, resident), NW * 64, 0, s>>>(a);
}

// x-resident persistent MLP: one 16-wave workgroup per CU; false when the shapes or the residency do not fit
long long* g_mlp_stamps = nullptr;

bool go_mlp_xres(const DecodeMlpArgs& a0, hipStream_t s) {
  DecodeMlpArgs a = a0;
  a.stamps = g_mlp_stamps;
  a.xcfg = g_mlp_xcfg;
  if (a.M > 16 || a.dq != a.d || a.d % 1024 || a.d > 4096 || a.F % 1024) return false;
  static int grid = -1;
  if (grid < 0) {  // every workgroup must be resident at once (they wait on each other)
    int dev = 0, cus = 0, per_cu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_mlp_xres_kernel<4>, 1024, 0);
    grid = per_cu >= 1 ? std::max(1, cus) : 0;
  }
  if (grid == 0) return false;
  switch (a.d / 1024) {
    case 1: decode_mlp_xres_kernel<1><<<grid, 1024, 0, s>>>(a); return true;
    case 2: decode_mlp_xres_kernel<2><<<grid, 1024, 0, s>>>(a); return true;
    case 4: decode_mlp_xres_kernel<4><<<grid, 1024, 0, s>>>(a); return true;
    default: return false;
  }
}

void launch_decode_mlp(const DecodeMlpArgs& a, hipStream_t s) {
  // default: the x-resident persistent kernel where it applies; configurations 0-6 select the gemm_tile
  // kernel's (waves per tile, k-blocks in flight per wave, waves per SIMD): A/B by bench/kernels/bench_decode_mlp.py
  if (g_mlp_cfg < 0 && go_mlp_xres(a, s)) return;
  switch (g_mlp_cfg < 0 ? 0 : g_mlp_cfg) {
    case 1: go_mlp<8, 4, 2>(a, s); break;   // 1 WG / CU, deeper
    case 2: go_mlp<4, 2, 4>(a, s); break;   // 4 WGs / CU
    case 3: go_mlp<4, 4, 3>(a, s); break;
    case 4: go_mlp<16, 1, 4>(a, s); break;  // 1 WG / CU, 16 waves
    case 5: go_mlp<8, 1, 4>(a, s); break;
    case 6: go_mlp<4, 1, 6>(a, s); break;   // 6 WGs / CU
    default: go_mlp<8, 2, 4>(a, s); break;  // 2 WGs / CU
  }
}

void set_decode_mlp_stamps(long long* stamps) { g_mlp_stamps = stamps; }

void set_decode_ksplit(int on) { g_dg_ksplit = on != 0; }
void set_decode_halves(int on) { g_dg_halves = on != 0; }

void set_decode_gemm_variant(int v) {
  // v >= 2000: A/B knob bits of the x-resident persistent MLP (decode_mlp_xres_kernel)
  if (v >= 2000) {
    g_mlp_xcfg = v - 2000;
    return;
  }
  // v >= 1000: persistent decode MLP configuration v - 1000 (launch_decode_mlp)
  if (v >= 1000 || v == -1) {
    g_mlp_cfg = v >= 1000 ? v - 1000 : -1;
    if (v >= 1000) return;
  }
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

void launch_decode_block(const DecodeBlockArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  const int grid = (a.Hq + 2 * a.Hkv) * 8 + a.M * a.Hkv * a.max_parts + a.d / 16;  // max_parts: 256-token
  decode_block_kernel<<<grid, 512, 0, s>>>(a);
}
