// The decode-step engine for tensor-parallel shards: ONE persistent launch runs every layer of a decode step
//
//   QKV (split-K slabs) -> attention (+ RMSNorm scale, RoPE, paged K/V write) -> O (+ xGMI all-reduce,
//   residual, ln2 prep) -> gate_up (+ RMSNorm scale, SwiGLU) -> down (+ xGMI all-reduce, residual, next-ln1 prep)
//
// Why (What's missing #2): at TP = 4 / 8 a rank's share of a layer is small (Llama-3-8B TP = 8:
// 54.5 MB, ~213 KB per CU) and each of the five launches per layer sits at its ~5-9 us floor -- launch boundary,
// the first weight loads' latency, the tail (profiles/r4/prof_tp8_shard_xar.csv: 36.3 us per layer against an
// 8.7 us weight floor).  Weights never depend on activations, so here every workgroup issues the weight loads of
// its NEXT phase's first unit into registers right after it signalled the current phase, and they stream while
// it waits on the edge: at TP = 8 a unit is a whole phase's share (QKV 32 KB, O 16 KB, gate_up 128 KB, down 56 KB
// per CU), so after an edge only the activations' round trip, the MFMAs and the epilogue remain.
//
// Geometry: one workgroup per CU (G of them, all co-resident: the edges wait on every workgroup), 8 waves (two per
// SIMD: 256 VGPRs each, so a unit's weights AND activations fit in registers):
//   * every wave streams: it owns the 32-deep k pieces w, w + 8, w + 16, ... of every GEMM unit (a 16-row weight
//     tile x a k range; one 16 B load per lane per piece, MFMA-preshuffled weights: 1 KB contiguous per wave
//     load), holds them AND the unit's activation fragments in registers, accumulates one
//     v_mfma_f32_16x16x32_bf16 chain and hands its 16 x 16 partial to LDS; in the attention phase the 8 waves are
//     the attention waves (one 32-token group each per pass);
//   * wave 7 doubles as the control wave: it sums the 8 partials, runs the epilogue (every hand-off store is
//     write-through: sc1), the xGMI all-reduce of O / down (push to every peer, collect in rank order,
//     decode_epi.h xar_push / xar_collect), the row scales and the edges.  Next-phase weight loads are issued only
//     after the phase's signal, so the drain before a signal waits for this phase's stores alone.
// Edges (MI355X_MICROARCH.md Valid forms, row 1): every storing wave drains (s_waitcnt vmcnt(0)), the workgroup
// barriers, ONE lane adds to an agent-scope counter (sharded 8 ways by blockIdx & 7); the consumer's control wave
// polls every shard with sc1 loads, the workgroup barriers, and every load of handed-off bytes is an sc1 (L1-
// bypassing) load.  Counters are zeroed by the launcher's memset node before every launch; every spin is bounded
// (a sticky fault word ends every later wait at once; the host discards such a step).
// The residual stream stays with its tile's workgroup: O and down deal the same d / 16 tiles to the same
// workgroups, so resid is never handed off (sc1 loads / stores anyway: it is rewritten in the launch).
#include "attn_decode.h"
#include "common.h"
#include "decode_epi.h"
#include "launchers.h"
#include "xgmi_proto.h"

namespace {

constexpr int DL_SW = 8;                 // streamer / attention waves
constexpr int DL_NT = DL_SW * 64;        // wave DL_CTL doubles as the control wave
constexpr int DL_CTL = DL_SW - 1;
constexpr int DL_MAXP = 16;              // pieces per streamer wave per unit: unit K <= 8 x 32 x 16 = 4096
constexpr int DL_GMAX = 8;               // query heads per kv head
constexpr int DL_MAXT = 64;              // O / down tiles per workgroup (epoch slots)
constexpr int DL_MAXKS = 4;              // QKV k-slabs
constexpr unsigned long long DL_WAIT_TICKS = 200000000ull;  // 2 s (100 MHz): an edge that never completes
enum { DL_QKV = 0, DL_ATTN = 1, DL_O = 2, DL_GU = 3, DL_DOWN = 4, DL_PH = 5 };
enum { EP_SLAB = 0, EP_RES = 1, EP_SWI = 2 };

typedef __amdgpu_buffer_rsrc_t rsrc_t;

SYM_DEV rsrc_t dl_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}
// 16 B L1-bypassing (sc1) load / write-through (sc1) store of hand-off data (aux 16 = sc1 on gfx950)
SYM_DEV u32x4 ld_sc1(rsrc_t r, int off) { return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16); }
SYM_DEV void st_sc1(rsrc_t r, int off, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16); }
SYM_DEV float ldf_sc1(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
SYM_DEV void stf_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
SYM_DEV void stbf_sc1(bf16* p, float v) {
  const bf16 b = (bf16)v;
  __hip_atomic_store(reinterpret_cast<unsigned short*>(p), __builtin_bit_cast(unsigned short, b), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// ---- edges --------------------------------------------------------------------------------------------------
SYM_DEV bool dl_faulted(const DLArgs& a) {
  return __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
         (a.xp.err != nullptr && __hip_atomic_load(a.xp.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0);
}

// diagnostics: wall clock (100 MHz) of this workgroup at event `which` (0: the edge in front of phase ev passed,
// 1: phase ev signalled), one lane, plain stores into a buffer nothing else reads
SYM_DEV void dl_stamp(const DLArgs& a, int ev, int b, int which) {
  if (a.stamps != nullptr && threadIdx.x == 0)
    a.stamps[((long long)b * a.L * DL_PH + ev) * 8 + which] = wall_clock64();
}
// sub-phase stamps of the first unit (which = 2..7), by the control wave's lane 0
SYM_DEV void dl_stamp_ctl(const DLArgs& a, int ev, int b, int which) {
  if (a.stamps != nullptr && threadIdx.x == DL_CTL * 64)
    a.stamps[((long long)b * a.L * DL_PH + ev) * 8 + which] = wall_clock64();
}

// Edge forms (DLArgs.edge_mode; the launcher zeroes the words before every launch):
//   0  arrival counters, one per (event, shard), 8 shards by blockIdx & 7, each on its own 128 B line: ONE lane
//      per workgroup adds (agent scope); the control wave's lanes 0..7 poll one shard each;
//   1  a flag board: one u32 per workgroup holding the last event it signalled + 1 (a write-through store, no
//      read-modify-write, no serialisation on a shared address); the control wave sweeps every workgroup's flag
//      (16 B sc1 loads, 4 workgroups per lane) until all reached the event.
constexpr int DL_SHARD_STRIDE = 32;  // u32 words between counter shards (128 B)

// every thread: this workgroup's hand-off stores are drained, then ONE lane signals
SYM_DEV void dl_signal(const DLArgs& a, int ev, int b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.edge_mode == 1)
      __hip_atomic_store(a.edge + b, (unsigned)(ev + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      __hip_atomic_fetch_add(a.edge + (ev * 8 + (b & 7)) * DL_SHARD_STRIDE, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
  dl_stamp(a, ev, b, 1);
}

// every thread: returns once every workgroup signalled `ev`
SYM_DEV void dl_wait(const DLArgs& a, int ev) {
  if ((threadIdx.x >> 6) == DL_CTL) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = wall_clock64();
    const rsrc_t rf = dl_rsrc(a.edge, (long long)((a.G + 255) / 256) * 1024);
    for (int it = 0;; ++it) {
      bool ok = true;
      if (a.edge_mode == 1) {
        for (int w0 = 4 * lane; w0 < a.G; w0 += 256) {
          Pack8 f;
          f.w = ld_sc1(rf, w0 * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) ok = ok && (w0 + e >= a.G || f.w[e] >= (unsigned)(ev + 1));
        }
      } else if (lane < 8) {
        const unsigned want = (unsigned)((a.G - lane + 7) / 8);
        ok = __hip_atomic_load(a.edge + (ev * 8 + lane) * DL_SHARD_STRIDE, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) >= want;
      }
      if (__all(ok)) break;
      if ((it & 63) == 63 && (dl_faulted(a) || wall_clock64() - t0 > DL_WAIT_TICKS)) {
        if (lane == 0) {
          __hip_atomic_store(a.fault, 1 + ev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // under TP the host polls the communicator's (host-mapped) error word after every step
          if (a.xp.err != nullptr && __hip_atomic_load(a.xp.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0)
            __hip_atomic_store(a.xp.err, 0x100 + ev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// ---- GEMM units ---------------------------------------------------------------------------------------------
// A unit = 16 weight rows (tile) x k range [k0, k0 + 256 CNT): streamer wave w owns pieces w + 8 i, i < CNT.
template <int CNT>
SYM_DEV void dl_load_w(Pack8 (&wa)[DL_MAXP], const bf16* __restrict__ W, int K, int tile, int k0, int wnt, int rot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bf16* p = W + ((long long)tile * (K / 32) + k0 / 32 + w) * 512 + lane * 8;
  if (wnt) {
#pragma unroll
    for (int j = 0; j < CNT; ++j) {
      const int i = CNT > 1 ? (j + rot) % CNT : 0;
      wa[j].w = ld_nt16(p + (long long)i * DL_SW * 512);
    }
  } else {
#pragma unroll
    for (int j = 0; j < CNT; ++j) {
      const int i = CNT > 1 ? (j + rot) % CNT : 0;
      wa[j].u = *reinterpret_cast<const uint4*>(p + (long long)i * DL_SW * 512);
    }
  }
}

// activations x [M][K] (hand-off data: sc1).  Lanes of rows >= M address past the buffer's range: the load
// returns zeros without touching memory (at M = 10 that is 6 of every 16 rows of fragment traffic).  Piece order
// rotated by `rot` (the workgroup index): every workgroup of an XCD reads the same activation lines, and in lockstep
// order they all queue on the same L2 channel at once.
template <int CNT>
SYM_DEV void dl_load_x(Pack8 (&xa)[DL_MAXP], rsrc_t rx, int K, int k0, int M, int rot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int off = r16 < M ? ((r16 * K) + k0 + w * 32 + 8 * h) * 2 : 0x7fff0000;
#pragma unroll
  for (int j = 0; j < CNT; ++j) {
    const int i = CNT > 1 ? (j + rot) % CNT : 0;
    xa[j].w = ld_sc1(rx, off + i * DL_SW * 64);
  }
}

template <int CNT>
SYM_DEV f32x4 dl_mma(const Pack8 (&wa)[DL_MAXP], const Pack8 (&xa)[DL_MAXP]) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < CNT; ++i) acc = mfma16(wa[i].v, xa[i].v, acc);
  return acc;
}

struct DLPhase {  // one GEMM phase of one layer
  const bf16* W;
  int K;        // weight row length (the projection's full K)
  int kunit;    // k range of one unit (K for whole-K units, K / KSq for the QKV slabs)
  int nunits;   // units dealt round-robin over the G workgroups (u = b, b + G, ...)
  int ksplit;   // QKV: units per tile (u -> tile u / ksplit, split u % ksplit)
  const bf16* x;  // activations [M][K]
};

SYM_DEV void dl_unit_of(const DLPhase& ph, int u, int& tile, int& k0) {
  tile = u / ph.ksplit;
  k0 = (u % ph.ksplit) * ph.kunit;
}

// (unconditional definitions of wa[0 .. CNT): a workgroup without a unit in the phase zeroes them, so no older
// value of the array stays live across the phases in between -- across attention that cost ~50 VGPRs)
// The control wave does not prefetch: its first vector load after the signal is the edge poll, which would
// otherwise wait behind its weight loads (vmcnt retires in order; a 128 KB gate_up share took ~5 us to land); it
// loads its pieces of the first unit with the activations, after the edge.
template <int CNT>
SYM_DEV void dl_prefetch(Pack8 (&wa)[DL_MAXP], const DLPhase& ph, int b, int wnt, int ctl_prefetch) {
  if (b >= ph.nunits || (!ctl_prefetch && (threadIdx.x >> 6) == DL_CTL)) {
#pragma unroll
    for (int i = 0; i < CNT; ++i) wa[i].u = make_uint4(0, 0, 0, 0);
    return;
  }
  int tile, k0;
  dl_unit_of(ph, b, tile, k0);
  dl_load_w<CNT>(wa, ph.W, ph.K, tile, k0, wnt, b);
}

// The control wave's view of a layer for the epilogues
struct DLEpi {
  int kind;             // EP_*
  float* slab;          // EP_SLAB: qkv_ws [KSq][M][Nq]
  int Nq;
  const bf16* w_next;   // EP_RES
  bf16* act;            // EP_SWI: [M][N / 2]
  int N;                // output features of the projection
};

// Residual epilogue of one O / down tile on the control wave: resid += all_reduce(v); xw = bf16(resid * w_next);
// ss[m][tile] = sum over the tile's 16 columns of resid^2.  All rows of resid / xw / ss of this tile belong to
// this workgroup in both phases; xw / ss are handed to the next phase (sc1).
SYM_DEV void dl_epi_res(const DLArgs& a, f32x4 v, int tile, const bf16* __restrict__ w_next, unsigned ep) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, h = lane >> 4;
  const int m = r16, d = a.d, n = tile * 16 + 4 * h;
  const bool mok = m < a.M;
  const rsrc_t rr = dl_rsrc(a.resid, (long long)a.M * d * 4);
  f32x4 r = {0.f, 0.f, 0.f, 0.f};
  uint2 wraw = make_uint2(0, 0);
  const long long goff = xar_goff(m, d, n);
  const bool xar = a.xp.world > 1;
  if (mok) {
    Pack8 t;
    t.w = ld_sc1(rr, (m * d + n) * 4);
    r = f32x4{__uint_as_float(t.w[0]), __uint_as_float(t.w[1]), __uint_as_float(t.w[2]), __uint_as_float(t.w[3])};
    wraw = *reinterpret_cast<const uint2*>(w_next + n);
    if (xar) xar_push(a.xp, v, goff, ep);
  }
  f32x4 s = v;
  if (xar) s = mok ? xar_collect(a.xp, v, goff, ep) : f32x4{0.f, 0.f, 0.f, 0.f};
  float sq = 0.f;
  if (mok) {
    const float q[4] = {r[0] + s[0], r[1] + s[1], r[2] + s[2], r[3] + s[3]};
    Pack8 wp;
    wp.u = make_uint4(wraw.x, wraw.y, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) sq += q[i] * q[i];
    st_sc1(rr, (m * d + n) * 4, u32x4{__float_as_uint(q[0]), __float_as_uint(q[1]), __float_as_uint(q[2]),
                                      __float_as_uint(q[3])});
    store4bf_sc1(a.xw + (long long)m * d + n, q[0] * (float)wp.h[0], q[1] * (float)wp.h[1], q[2] * (float)wp.h[2],
                 q[3] * (float)wp.h[3]);
  }
  sq += __shfl_xor(sq, 16, 64);
  sq += __shfl_xor(sq, 32, 64);
  if (mok && h == 0) stf_sc1(a.ss + (long long)m * (d / 16) + tile, sq);
}

// row scales rsqrt(mean(x^2) + eps) of the M input rows from their sum-of-squares partials: every wave two rows
// (wave w: rows w and w + 8), 16 B sc1 loads issued together; the caller's next barrier publishes rn_s
SYM_DEV void dl_row_scales(const DLArgs& a, const float* __restrict__ ss, int tiles, float* rn_s) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float inv_d = 1.f / (float)a.d;
  const rsrc_t rs = dl_rsrc(ss, (long long)a.M * tiles * 4);
  float s[2] = {0.f, 0.f};
  if ((tiles & 3) == 0) {
    Pack8 q[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = min(w + DL_SW * j, a.M - 1);
#pragma unroll
      for (int c = 0; c < 2; ++c) {  // up to 512 partials per row (d <= 8192)
        const int i = 4 * lane + 256 * c;
        q[j][c].w = i < tiles ? ld_sc1(rs, (m * tiles + i) * 4) : u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[j] += __uint_as_float(q[j][c].w[e]);
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = min(w + DL_SW * j, a.M - 1);
      for (int i = lane; i < tiles; i += 64) s[j] += ldf_sc1(ss + (long long)m * tiles + i);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = w + DL_SW * j;
    const float t = wave_sum(s[j]);
    if (lane == 0 && m < a.M) rn_s[m] = rsqrtf(t * inv_d + a.eps);
  }
}

// One GEMM phase: the workgroup's units b, b + G, ... (the first unit's weights already in flight in wa)
template <int CNT, int EPI>
SYM_DEV void dl_gemm_phase(const DLArgs& a, const DLPhase& ph, const DLEpi& ep, Pack8 (&wa)[DL_MAXP],
                           Pack8 (&xa)[DL_MAXP], int b, f32x4 (*red)[DL_SW][64], const float* rn_s,
                           unsigned* xep_s, int ev) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool ctl = wid == DL_CTL;
  const rsrc_t rx = dl_rsrc(ph.x, (long long)a.M * ph.K * 2);
  int buf = 0, i = 0;
  for (int u = b; u < ph.nunits; u += a.G, ++i) {
    int tile, k0;
    dl_unit_of(ph, u, tile, k0);
    {
      if (ctl && i == 0 && !a.ctl_prefetch) dl_load_w<CNT>(wa, ph.W, ph.K, tile, k0, a.wnt, b);
      dl_load_x<CNT>(xa, rx, ph.K, k0, a.M, b);
      const f32x4 acc = dl_mma<CNT>(wa, xa);
      if (i == 0 && a.stamps != nullptr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        dl_stamp_ctl(a, ev, b, 2);
      }
      // the next unit's weights behind this unit's MFMAs (same registers: no renamed second copy)
      __builtin_amdgcn_sched_barrier(0);
      if (u + a.G < ph.nunits) {
        int t2, k2;
        dl_unit_of(ph, u + a.G, t2, k2);
        dl_load_w<CNT>(wa, ph.W, ph.K, t2, k2, a.wnt, b);
      }
      red[buf][wid][lane] = acc;
    }
    __syncthreads();
    if (i == 0) dl_stamp_ctl(a, ev, b, 3);
    if (ctl) {
      f32x4 v = red[buf][0][lane];
#pragma unroll
      for (int w = 1; w < DL_SW; ++w) v += red[buf][w][lane];
      const int r16 = lane & 15, h = lane >> 4;
      const int m = r16;
      const bool mok = m < a.M;
      if constexpr (EPI == EP_SLAB) {
        if (mok) {
          const rsrc_t rs = dl_rsrc(ep.slab, (long long)ph.ksplit * a.M * ep.Nq * 4);
          const int off = (((u % ph.ksplit) * a.M + m) * ep.Nq + tile * 16 + 4 * h) * 4;
          st_sc1(rs, off, u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                __float_as_uint(v[3])});
        }
      } else if constexpr (EPI == EP_RES) {
        const unsigned e = ++xep_s[i];
        dl_epi_res(a, v, tile, ep.w_next, e);
      } else {  // EP_SWI: rows 0-7 gate, 8-15 up (interleaved per tile), row scale of the deferred norm
        const float sc = mok ? rn_s[m] : 1.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] *= sc;
        float up[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) up[q] = __shfl_xor(v[q], 32, 64);
        if (mok && h < 2) {
          const int f = 8 * tile + 4 * h;
          store4bf_sc1(ep.act + (long long)m * (ep.N / 2) + f, silu(v[0]) * up[0], silu(v[1]) * up[1],
                       silu(v[2]) * up[2], silu(v[3]) * up[3]);
        }
      }
    }
    if (i == 0) dl_stamp_ctl(a, ev, b, 4);
    buf ^= 1;
  }
}

// ---- attention ----------------------------------------------------------------------------------------------
// The newest token's K / V come out of this step's QKV slabs; every OLDER token is in the paged cache since an
// earlier launch.  So the old K / V do not wait for the QKV edge beyond one round trip: the block-table entries are
// read before the edge and the K / V loads issue together with the slab loads right after it; the newest token
// joins in the merge (its score and value from the rebuilt rows in LDS) and goes to the cache with plain stores for
// the NEXT step (no drain, no read-back).  (Holding the whole first pass in registers across the edge spilled.)
struct DLAttnLds {
  float qkv[(DL_GMAX + 2) * 128];  // the unit's q / k / v rows (slab sums, not yet row-scaled; permuted order)
  bf16 q[DL_GMAX][128];            // roped q, natural dim order
  bf16 knew[128], vnew[128];       // the newest token's roped k and its v (bf16, as the cache holds them)
  float cs[128];                   // RoPE cos (0..63) / sin (64..127) of the unit's position
  float m[DL_SW][DL_GMAX], l[DL_SW][DL_GMAX];
  float o[DL_SW][DL_GMAX][D + 4];
};

// What a unit needs that does not depend on this step's QKV, read BEFORE the QKV edge: the sequence's context
// length / cache slot / position, the block of wave w's first 32-token group of old tokens [0, ctx - 1) (-1: none),
// and the position's RoPE cos / sin row (into LDS) -- so after the edge the unit's first loads (old K / V, the
// slabs, the row scale's partials) all issue at once and nothing else waits on a round trip.
struct DLAttnMeta {
  int ctx, slot, pos, bk0;
};

SYM_DEV DLAttnMeta dl_attn_meta(const DLArgs& a, int s, float* cs_lds) {
  DLAttnMeta mt;
  mt.ctx = a.ctx_lens[s];
  mt.slot = a.slots[s];
  mt.pos = a.positions[s];
  const int tok0 = (threadIdx.x >> 6) * 32;
  mt.bk0 = tok0 < mt.ctx - 1 ? a.block_tables[(long long)s * a.max_blocks + (tok0 >> __builtin_ctz(a.BS))] : -1;
  if (threadIdx.x < 32)
    *reinterpret_cast<float4*>(cs_lds + 4 * threadIdx.x) =
        *reinterpret_cast<const float4*>(a.cos_sin + (long long)mt.pos * 128 + 4 * threadIdx.x);
  return mt;
}

// One (sequence, kv head) unit on the 8 waves: rebuild its q / k / v rows from the QKV slabs (x the row scale,
// RoPE), store the newest K / V for the next step, flash-decode over the old tokens (first pass from `pre` when
// `use_pre`; wave w: 32-token groups w, w + 8, ...), merge the waves and the newest token through LDS, store the
// head outputs (sc1: handed to O).
SYM_DEV void dl_attn_unit(const DLArgs& a, const DLLayer& ly, int s, int g, const float* __restrict__ ss_in,
                          int ss_tiles, DLAttnLds& L, DLAttnMeta mt, int stamp_ev) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int Hq = a.Hq, Hkv = a.Hkv, G = Hq / Hkv;
  const int Nq = (Hq + 2 * Hkv) * 128;
  const int nval = (G + 2) * 128;
  const int ctx = mt.ctx;
  const int ctx_old = ctx - 1;
  const int slot = mt.slot;
  const int c = lane & 15, h = lane >> 4;
  // the first pass of old K / V (block known from before the edge: bk0), the slab rows (4 consecutive values per
  // thread, every slab's 16 B at once) and, in every wave, the row scale from the residual's sum-of-squares
  // partials (one 16 B load per lane for d / 16 partials) -- all issued together
  const int bsh = __builtin_ctz(a.BS);
  const int* bt = a.block_tables + (long long)s * a.max_blocks;
  KVFrag f;
  int tok0 = wid * 32;
  if (tok0 < ctx_old) {
    const int bk = mt.bk0 >= 0 ? mt.bk0 : bt[tok0 >> bsh];
    const int boff = tok0 & (a.BS - 1);
    load_group(ly.k_cache + (((long long)bk * Hkv + g) * a.BS + boff) * D,
               ly.v_cache + ((long long)bk * Hkv + g) * (long long)D * a.BS + boff, a.BS, f);
  }
  Pack8 q[DL_MAXKS];
  const int t4 = threadIdx.x * 4;
  const int row = t4 < G * 128 ? g * G * 128 + t4
                               : (t4 < (G + 1) * 128 ? Hq * 128 + g * 128 + (t4 - G * 128)
                                                     : (Hq + Hkv) * 128 + g * 128 + (t4 - (G + 1) * 128));
  if (t4 < nval) {
    const rsrc_t rq = dl_rsrc(a.qkv_ws, (long long)a.KSq * a.M * Nq * 4);
#pragma unroll
    for (int sp = 0; sp < DL_MAXKS; ++sp)
      if (sp < a.KSq) q[sp].w = ld_sc1(rq, ((sp * a.M + s) * Nq + row) * 4);
  }
  float ssum = 0.f;
  {
    const rsrc_t rs = dl_rsrc(ss_in, (long long)a.M * ss_tiles * 4);
    if ((ss_tiles & 3) == 0) {
      Pack8 sq[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int i = 4 * lane + 256 * c;
        sq[c].w = i < ss_tiles ? ld_sc1(rs, (s * ss_tiles + i) * 4) : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) ssum += __uint_as_float(sq[c].w[e]);
    } else {
      for (int i = lane; i < ss_tiles; i += 64) ssum += ldf_sc1(ss_in + (long long)s * ss_tiles + i);
    }
  }
  const float rn = rsqrtf(wave_sum(ssum) * (1.f / (float)a.d) + a.eps);
  if (stamp_ev >= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dl_stamp_ctl(a, stamp_ev, blockIdx.x, 2);
  }
  if (t4 < nval) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sp = 0; sp < DL_MAXKS; ++sp)
      if (sp < a.KSq)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += __uint_as_float(q[sp].w[e]);
#pragma unroll
    for (int e = 0; e < 4; ++e) L.qkv[t4 + e] = v[e] * rn;
  }
  __syncthreads();
  {
    const float* cs = L.cs;  // the position's cos / sin row (staged before the edge)
    const long long blk = slot >= 0 ? slot / a.BS : 0, off = slot >= 0 ? slot % a.BS : 0;
    // q heads and the k head: RoPE over the permuted rows (partner row = r ^ 8); thread -> 8 consecutive dims of
    // one head (natural order)
    const int nqk = (G + 1) * 16;
    if ((int)threadIdx.x < nqk) {
      const int head = threadIdx.x >> 4, c8 = threadIdx.x & 15;  // dims 8 c8 .. 8 c8 + 7
      const bool lo = c8 < 8;
      Pack8 pk;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int dim = 8 * c8 + e, dh = dim & 63, j = dh >> 3, c = (dh & 7) + (lo ? 0 : 8);
        const int r = 16 * j + c;  // permuted row of this dim within the head
        const float x = L.qkv[head * 128 + r], p = L.qkv[head * 128 + (r ^ 8)];
        const float co = cs[dh], si = cs[64 + dh];
        pk.h[e] = (bf16)(lo ? x * co - p * si : x * co + p * si);
      }
      if (head < G) {
        *reinterpret_cast<uint4*>(&L.q[head][8 * c8]) = pk.u;
      } else {
        *reinterpret_cast<uint4*>(&L.knew[8 * c8]) = pk.u;
        if (slot >= 0)  // for the next step (kernel boundary: plain stores)
          *reinterpret_cast<uint4*>(ly.k_cache + ((blk * Hkv + g) * a.BS + off) * 128 + 8 * c8) = pk.u;
      }
    } else if ((int)threadIdx.x < nqk + 128) {  // v: natural order; dim-major cache (one bf16 per line)
      const int dim = threadIdx.x - nqk;
      const bf16 bv = (bf16)L.qkv[(G + 1) * 128 + dim];
      L.vnew[dim] = bv;
      if (slot >= 0) ly.v_cache[((blk * Hkv + g) * 128 + dim) * (long long)a.BS + off] = bv;
    }
  }
  __syncthreads();
  if (stamp_ev >= 0) dl_stamp_ctl(a, stamp_ev, blockIdx.x, 3);
  // old tokens [0, ctx - 1)
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  {
    bf16x8 qf[4];
    if (c < G) {
#pragma unroll
      for (int i = 0; i < 4; ++i) qf[i] = *reinterpret_cast<const bf16x8*>(&L.q[c][32 * h + 8 * i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) qf[i] = zero8();
    }
    if (tok0 < ctx_old)
      compute_group(f, qf, a.scale_log2, [&](int aa, int r) { return tok0 + 8 * h + 4 * aa + r < ctx_old; }, o, m,
                    lsum);
    tok0 += DL_SW * 32;
#pragma unroll 1
    for (; tok0 < ctx_old; tok0 += DL_SW * 32) {
      const int bk = bt[tok0 >> bsh];
      const int boff = tok0 & (a.BS - 1);
      load_group(ly.k_cache + (((long long)bk * Hkv + g) * a.BS + boff) * D,
                 ly.v_cache + ((long long)bk * Hkv + g) * (long long)D * a.BS + boff, a.BS, f);
      compute_group(f, qf, a.scale_log2, [&](int aa, int r) { return tok0 + 8 * h + 4 * aa + r < ctx_old; }, o, m,
                    lsum);
    }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    if (c < DL_GMAX) {
      if (h == 0) {
        L.m[wid][c] = m;
        L.l[wid][c] = lsum;
      }
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) L.o[wid][c][16 * dt + 4 * h + r] = o[dt][r];
    }
  }
  __syncthreads();
  if (stamp_ev >= 0) dl_stamp_ctl(a, stamp_ev, blockIdx.x, 4);
  {  // thread (qq, d0): 8 dims of query head qq; the 16 threads of a head are 16 consecutive lanes
    const int qq = threadIdx.x >> 4, d0 = (threadIdx.x & 15) * 8;
    float sn = 0.f;  // the newest token's score: q . k_new over this thread's 8 dims, then over the 16 threads
    if (qq < G) {
#pragma unroll
      for (int j = 0; j < 8; ++j) sn += (float)L.q[qq][d0 + j] * (float)L.knew[d0 + j];
    }
#pragma unroll
    for (int o2 = 8; o2 > 0; o2 >>= 1) sn += __shfl_xor(sn, o2, 64);
    if (qq < G) {
      sn *= a.scale_log2;
      const bool has_new = ctx >= 1;
      float M_ = has_new ? sn : -INFINITY, Lsum = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < DL_SW; ++w) M_ = fmaxf(M_, L.m[w][qq]);
#pragma unroll
      for (int w = 0; w < DL_SW; ++w) {
        const float mw = L.m[w][qq];
        const float f = (mw == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(mw - M_);
        Lsum += L.l[w][qq] * f;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += L.o[w][qq][d0 + j] * f;
      }
      if (has_new) {
        const float f = __builtin_amdgcn_exp2f(sn - M_);
        Lsum += f;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f * (float)L.vnew[d0 + j];
      }
      const float inv = Lsum > 0.f ? 1.f / Lsum : 0.f;  // ctx == 0 (padding row): zeros
      Pack8 pk;
#pragma unroll
      for (int j = 0; j < 8; ++j) pk.h[j] = (bf16)(acc[j] * inv);
      const rsrc_t ro = dl_rsrc(a.attn, (long long)a.M * Hq * 128 * 2);
      st_sc1(ro, ((s * Hq + g * G + qq) * 128 + d0) * 2, pk.w);
    }
  }
  __syncthreads();  // the LDS staging is reused by the next unit
}

// ---- the step ---------------------------------------------------------------------------------------------
// Specialised per shape class: the k pieces per streamer wave of the QKV, O, gate_up and down units are template
// parameters, so every register array has its exact size (a runtime-dispatched form inlined every instantiation
// into one body and spilled).
template <int CQ, int CO, int CG, int CD>
SYM_DEV void dl_body(const DLArgs& a, int b) {
  __shared__ f32x4 red[2][DL_SW][64];
  __shared__ float rn_s[16];
  __shared__ unsigned xep_s[DL_MAXT];
  __shared__ DLAttnLds lds_attn;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool ctl = wid == DL_CTL;
  const int d = a.d, Nq = (a.Hq + 2 * a.Hkv) * 128;
  const int ntile_d = d / 16;
  // this workgroup's O / down tiles (b, b + G, ...): their all-reduce epochs, read once, bumped by every O and
  // every down phase, written back at exit (the per-tile counters of the fused launches, decode_gemm.hip)
  const int nmine = b < ntile_d ? (ntile_d - b + a.G - 1) / a.G : 0;
  if (ctl && a.xp.world > 1)
    for (int i = lane; i < nmine; i += 64) xep_s[i] = a.xar_ctr[b + i * a.G];
  __syncthreads();

  // weight registers: wa = QKV / O units, wb = gate_up (prefetched at the attention signal, across O), wc = down
  // (prefetched at the O signal, across gate_up): each phase's stream starts as early as its registers allow
  Pack8 wa[DL_MAXP], wb[DL_MAXP], wc[DL_MAXP], xa[DL_MAXP];
  auto phase_of = [&](int l, int p) -> DLPhase {
    const DLLayer& ly = a.layers[l];
    if (p == DL_QKV) return DLPhase{ly.wqkv, d, d / a.KSq, (Nq / 16) * a.KSq, a.KSq, a.xw};
    if (p == DL_O) return DLPhase{ly.wo, a.Hq * 128, a.Hq * 128, ntile_d, 1, a.attn};
    if (p == DL_GU) return DLPhase{ly.wgu, d, d, (2 * a.Fl) / 16, 1, a.xw};
    return DLPhase{ly.wdown, a.Fl, a.Fl, ntile_d, 1, a.act};
  };
  dl_prefetch<CQ>(wa, phase_of(0, DL_QKV), b, a.wnt, a.ctl_prefetch);
  for (int l = 0; l < a.L; ++l) {
    const DLLayer& ly = a.layers[l];
    const int ev0 = l * DL_PH;
    // ---- QKV: split-K slabs (the row scale waits for the attention phase)
    if (l > 0) dl_wait(a, ev0 - DL_PH + DL_DOWN);
    dl_stamp(a, ev0 + DL_QKV, b, 0);
    dl_gemm_phase<CQ, EP_SLAB>(a, phase_of(l, DL_QKV), DLEpi{EP_SLAB, a.qkv_ws, Nq, nullptr, nullptr, Nq}, wa, xa, b,
                               red, rn_s, xep_s, ev0 + DL_QKV);
    dl_signal(a, ev0 + DL_QKV, b);
    // ---- attention: the first unit's old K / V stream in before the edge
    {
      const bool have = b < a.M * a.Hkv;
      DLAttnMeta mt{0, -1, 0, -1};
      if (have) mt = dl_attn_meta(a, b / a.Hkv, lds_attn.cs);
      dl_wait(a, ev0 + DL_QKV);  // (its barrier publishes the staged cos / sin row)
      dl_stamp(a, ev0 + DL_ATTN, b, 0);
      const float* ss_in = l == 0 ? a.ss0 : a.ss;
      const int ss_tiles = l == 0 ? a.ss0_tiles : ntile_d;
      for (int u = b; u < a.M * a.Hkv; u += a.G) {
        if (u != b) {  // a later unit of this workgroup: its own pre-stage (after the previous unit's last barrier)
          mt = dl_attn_meta(a, u / a.Hkv, lds_attn.cs);
          __syncthreads();
        }
        dl_attn_unit(a, ly, u / a.Hkv, u % a.Hkv, ss_in, ss_tiles, lds_attn, mt, u == b ? ev0 + DL_ATTN : -1);
      }
    }
    dl_signal(a, ev0 + DL_ATTN, b);
    dl_prefetch<CO>(wa, phase_of(l, DL_O), b, a.wnt, a.ctl_prefetch);
    dl_prefetch<CG>(wb, phase_of(l, DL_GU), b, a.wnt, a.ctl_prefetch);
    // ---- O (+ all-reduce, residual, ln2 prep)
    dl_wait(a, ev0 + DL_ATTN);
    dl_stamp(a, ev0 + DL_O, b, 0);
    dl_gemm_phase<CO, EP_RES>(a, phase_of(l, DL_O), DLEpi{EP_RES, nullptr, 0, ly.ln2, nullptr, d}, wa, xa, b, red,
                              rn_s, xep_s, ev0 + DL_O);
    dl_signal(a, ev0 + DL_O, b);
    dl_prefetch<CD>(wc, phase_of(l, DL_DOWN), b, a.wnt, a.ctl_prefetch);
    // ---- gate_up (+ row scale, SwiGLU)
    dl_wait(a, ev0 + DL_O);
    dl_stamp(a, ev0 + DL_GU, b, 0);
    dl_row_scales(a, a.ss, ntile_d, rn_s);  // published by the first unit's barrier, before any epilogue reads it
    dl_gemm_phase<CG, EP_SWI>(a, phase_of(l, DL_GU), DLEpi{EP_SWI, nullptr, 0, nullptr, a.act, 2 * a.Fl}, wb, xa, b,
                              red, rn_s, xep_s, ev0 + DL_GU);
    dl_signal(a, ev0 + DL_GU, b);
    // ---- down (+ all-reduce, residual, next-norm prep)
    dl_wait(a, ev0 + DL_GU);
    dl_stamp(a, ev0 + DL_DOWN, b, 0);
    dl_gemm_phase<CD, EP_RES>(a, phase_of(l, DL_DOWN), DLEpi{EP_RES, nullptr, 0, ly.lnn, nullptr, d}, wc, xa, b, red,
                              rn_s, xep_s, ev0 + DL_DOWN);
    dl_signal(a, ev0 + DL_DOWN, b);
    if (l + 1 < a.L) dl_prefetch<CQ>(wa, phase_of(l + 1, DL_QKV), b, a.wnt, a.ctl_prefetch);
  }
  if (ctl && a.xp.world > 1)
    for (int i = lane; i < nmine; i += 64) a.xar_ctr[b + i * a.G] = xep_s[i];
}

template <int CQ, int CO, int CG, int CD>
__global__ __launch_bounds__(DL_NT) void decode_layers_kernel(DLArgs a) {
  dl_body<CQ, CO, CG, CD>(a, blockIdx.x);
}

struct DLMulti {
  DLArgs a[DL_MULTI_MAX];
};
template <int CQ, int CO, int CG, int CD>
__global__ __launch_bounds__(DL_NT) void decode_layers_multi_kernel(DLMulti m) {
  dl_body<CQ, CO, CG, CD>(m.a[blockIdx.z], blockIdx.x);
}

// The shape classes built (pieces per streamer wave = unit K / 256 for QKV (K = d / KSq), O (K = Hq x 128 / tp),
// gate_up (K = d), down (K = F / tp)):
//   Llama-3-8B TP = 8: QKV 1024 (KSq 4), O 512, gate_up 4096, down 1792   -> (4, 2, 16, 7)
//   Llama-3-8B TP = 4: QKV 2048 (KSq 2), O 1024, gate_up 4096, down 3584  -> (8, 4, 16, 14)
//   Llama-3-8B TP = 2: QKV 2048 (KSq 2), O 2048, gate_up 4096, down 7168  -> (not built: down K > 4096)
//   small-llama TP = 1 / 2 (tests): QKV 512 (KSq 2) / 256 (KSq 4), O 1024 / 512, gate_up 1024, down 3584 / 1792;
//   its TP = 2 one-GPU rehearsal (128 workgroups per rank): QKV 512 (KSq 2)
#define DL_SHAPES(X) X(4, 2, 16, 7) X(8, 4, 16, 14) X(2, 4, 4, 14) X(1, 2, 4, 7) X(2, 2, 4, 7)

bool dl_check(const DLArgs& a) {
  return a.M >= 1 && a.M <= 16 && a.L >= 1 && a.Hkv >= 1 && a.Hq % a.Hkv == 0 && a.Hq / a.Hkv <= DL_GMAX &&
         a.d % 256 == 0 && a.Fl % 256 == 0 && a.BS >= 32 && (a.BS & (a.BS - 1)) == 0 && a.G >= 1 &&
         (a.d / 16 + a.G - 1) / a.G <= DL_MAXT && a.KSq >= 1 && a.KSq <= DL_MAXKS && a.d % (a.KSq * 256) == 0;
}

// bytes of edge words one launch uses (zeroed before it)
size_t dl_edge_bytes(const DLArgs& a) {
  return a.edge_mode == 1 ? (size_t)(a.G + 255) / 256 * 1024 : (size_t)a.L * DL_PH * 8 * DL_SHARD_STRIDE * 4;
}

int g_dl_resident[16];  // per shape: workgroups per CU the kernel admits (occupancy query, once; 0 = unknown)

template <typename Kern>
int dl_per_cu(Kern k, int& cache) {
  if (cache <= 0) {
    int n = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, DL_NT, 0);
    cache = n > 0 ? n : -1;
  }
  return cache;
}

int dl_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  return cus;
}

}  // namespace

int decode_layers_pieces_ok(int cq, int co, int cg, int cd) {
#define DL_MATCH(A, B, C, D_) \
  if (cq == A && co == B && cg == C && cd == D_) return 1;
  DL_SHAPES(DL_MATCH)
#undef DL_MATCH
  return 0;
}

bool launch_decode_layers(const DLArgs& a, hipStream_t s) {
  if (!dl_check(a)) return false;
  int idx = 0;
#define DL_LAUNCH(A, B, C, D_)                                                                          \
  if (a.cq == A && a.co == B && a.cg == C && a.cd == D_) {                                               \
    auto k = decode_layers_kernel<A, B, C, D_>;                                                          \
    if (a.G > dl_cus() * dl_per_cu(k, g_dl_resident[idx])) return false; /* every workgroup resident */ \
    (void)hipMemsetAsync(a.edge, 0, dl_edge_bytes(a), s);                                               \
    k<<<a.G, DL_NT, 0, s>>>(a);                                                                          \
    return true;                                                                                         \
  }                                                                                                      \
  ++idx;
  DL_SHAPES(DL_LAUNCH)
#undef DL_LAUNCH
  return false;
}

bool launch_decode_layers_multi(const DLArgs* a, int world, hipStream_t s) {
  if (world < 1 || world > DL_MULTI_MAX) return false;
  DLMulti m{};
  for (int r = 0; r < world; ++r) {
    if (!dl_check(a[r]) || a[r].G != a[0].G || a[r].cq != a[0].cq || a[r].co != a[0].co || a[r].cg != a[0].cg ||
        a[r].cd != a[0].cd)
      return false;
    m.a[r] = a[r];
  }
#define DL_LAUNCH(A, B, C, D_)                                                                      \
  if (a[0].cq == A && a[0].co == B && a[0].cg == C && a[0].cd == D_) {                               \
    auto k = decode_layers_multi_kernel<A, B, C, D_>;                                                \
    int per_cu = 0;                                                                                  \
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, DL_NT, 0);                              \
    if (per_cu < 1 || (long long)a[0].G * world > (long long)dl_cus() * per_cu) return false;        \
    for (int r = 0; r < world; ++r)                                                                  \
      (void)hipMemsetAsync(a[r].edge, 0, dl_edge_bytes(a[r]), s);                                   \
    k<<<dim3(a[0].G, 1, world), DL_NT, 0, s>>>(m);                                                   \
    return true;                                                                                     \
  }
  DL_SHAPES(DL_LAUNCH)
#undef DL_LAUNCH
  return false;
}
