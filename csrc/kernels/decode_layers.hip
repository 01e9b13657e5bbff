// The decode-step engine for tensor-parallel shards: ONE persistent launch runs every layer of a decode step
//
//   QKV (split-K slabs) -> attention (+ RMSNorm scale, RoPE, paged K/V write) -> O (+ xGMI all-reduce,
//   residual, ln2 prep) -> gate_up (+ RMSNorm scale, SwiGLU) -> down (+ xGMI all-reduce, residual, next-ln1 prep)
//
// Why (What's missing #2): at TP = 4 / 8 a rank's share of a layer is small (Llama-3-8B TP = 8:
// 54.5 MB, ~213 KB per CU) and each of the five launches per layer sits at its ~5-9 us floor -- launch boundary,
// the first weight loads' latency, the tail (profiles/r4/prof_tp8_shard_xar.csv: 36.3 us per layer against an
// 8.7 us weight floor).  Weights never depend on activations, so here every workgroup issues the weight loads of
// its NEXT phase's first unit into registers while it runs the current phase, and they stream across the edge:
// at TP = 8 a unit is a whole phase's share (QKV 32 KB, O 16 KB, gate_up 128 KB, down 56 KB per CU), so after an
// edge only the activations' round trip, the MFMAs and the epilogue remain.
//
// Geometry: one workgroup per CU (G of them, all co-resident: the edges wait on every workgroup), 8 waves (two per
// SIMD: 256 VGPRs each, so a unit's weights AND activations fit in registers):
//   * every wave streams: it owns the 32-deep k pieces w, w + 8, w + 16, ... of every GEMM unit (a 16-row weight
//     tile x a k range; one 16 B buffer load per lane per piece, MFMA-preshuffled weights: 1 KB contiguous per
//     wave load), holds them AND the unit's activation fragments in registers, accumulates one
//     v_mfma_f32_16x16x32_bf16 chain and hands its 16 x 16 partial to LDS;
//   * wave 7 doubles as the control wave: it sums the 8 partials, runs the epilogue (every hand-off store is
//     write-through: sc1), the xGMI all-reduce of O / down (push to every peer, collect in rank order,
//     decode_epi.h xar_push / xar_collect), the row scales and the edges;
//   * attention is wave-level split-KV (dl_attn_wave): (sequence, kv head, context partition) units, one per wave,
//     dealt over the workgroups first, the partitions merged by the last arriver.
// Weight streaming: a wave's loads and stores retire in issue order (MI355X_MICROARCH.md, vmcnt), so the next
// phase's weights are issued right AFTER this phase's activation loads (`after_x`), never before them, and the
// streamer waves do not drain at a signal (they store nothing in a GEMM phase): the stream stays in flight across
// the edge.  The control wave -- which polls and stores -- loads its own pieces after the edge instead.  Every load
// is a buffer load with the per-piece offset in an SGPR and no branch between an MFMA's operands and the next
// phase's loads, so the compiler's waits count exactly the operands (flat loads, or path-dependent load counts,
// made it wait for everything).
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

#include <type_traits>

namespace {

constexpr int DL_SW = 8;                 // streamer / attention waves
constexpr int DL_NT = DL_SW * 64;        // wave DL_CTL doubles as the control wave
constexpr int DL_CTL = DL_SW - 1;
constexpr int DL_MAXP = 16;              // pieces per streamer wave per unit: unit K <= 8 x 32 x 16 = 4096
constexpr int DL_GMAX = 8;               // query heads per kv head
constexpr int DL_MAXT = 64;              // O / down tiles per workgroup (epoch slots)
constexpr int DL_MAXKS = 4;              // QKV k-slabs
constexpr int DL_MAXL = 128;             // layers
constexpr unsigned long long DL_WAIT_TICKS = 200000000ull;  // 2 s (100 MHz): an edge that never completes
enum { DL_QKV = 0, DL_ATTN = 1, DL_O = 2, DL_GU = 3, DL_DOWN = 4, DL_PH = 5 };
enum { EP_SLAB = 0, EP_RES = 1, EP_SWI = 2 };

typedef __amdgpu_buffer_rsrc_t rsrc_t;

// a pointer the wave holds in every lane (read from LDS): into SGPRs, so buffer descriptors built from it need
// no waterfall loop
template <typename T>
SYM_DEV T* dl_uni(T* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}

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
  return __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
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

// Edge counters, one per (event, shard), 8 shards by blockIdx & 7, each on its own 128 B line: ONE lane per
// workgroup adds (agent scope); the control wave's lanes 0..7 poll one shard each.  The counters are never
// cleared: launch E (the E-th launch on this buffer) waits for (E + 1) x the shard's workgroups.  E comes from the
// LAST event's shard-0 counter read at kernel start (every earlier launch completed, no workgroup of this one has
// reached that event yet).  (The first form zeroed them with a memset node in front of every launch: once another
// hipGraph was captured, the replayed memset of an earlier decode graph no longer cleared them -- its waits then
// passed at once and the step computed garbage.)
constexpr int DL_SHARD_STRIDE = 32;  // u32 words between counter shards (128 B)

SYM_DEV unsigned dl_epoch(const DLArgs& a) {
  const unsigned c = __hip_atomic_load(a.edge + ((a.L * DL_PH - 1) * 8) * DL_SHARD_STRIDE, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return c / (unsigned)((a.G + 7) / 8);
}

// every thread: this workgroup's hand-off stores are drained, then ONE lane signals.  `drain`: this wave stored
// hand-off data in the phase.  In a GEMM phase only the control wave stores (the epilogue); the streamer waves skip
// the drain, so the next phase's weight loads they issued during this phase stay in flight across the signal (a
// wave's loads and stores retire in order: draining would wait for that whole stream).
SYM_DEV void dl_signal(const DLArgs& a, int ev, int b, bool drain = true) {
  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(a.edge + (ev * 8 + (b & 7)) * DL_SHARD_STRIDE, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  dl_stamp(a, ev, b, 1);
}

// every thread: returns once every workgroup signalled `ev` (epoch: dl_epoch, read by the control wave at start)
SYM_DEV void dl_wait(const DLArgs& a, int ev, unsigned epoch) {
  if ((threadIdx.x >> 6) == DL_CTL) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = wall_clock64();
    for (int it = 0;; ++it) {
      bool ok = true;
      if (lane < 8) {
        const unsigned want = (epoch + 1u) * (unsigned)((a.G - lane + 7) / 8);
        ok = __hip_atomic_load(a.edge + (ev * 8 + lane) * DL_SHARD_STRIDE, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) >= want;
      }
      if (__all(ok)) break;
      if ((it & 63) == 63 && (dl_faulted(a) || wall_clock64() - t0 > DL_WAIT_TICKS)) {
        if (lane == 0) {
          __hip_atomic_store(a.fault, 1 + ev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
SYM_DEV void dl_load_w(Pack8 (&wa)[DL_MAXP], const bf16* __restrict__ W, int K, int tile, int k0, int rot,
                       bool on = true) {
  // buffer loads, nt (aux 2), no branches: the compiler's wait before an MFMA counts the loads issued after its
  // operands, which needs the same instruction sequence on every path (loads through the generic pointers of the
  // argument table were flat loads, after which it can only wait for everything -- the next phase's whole prefetch
  // included).  !on: a zero-length descriptor -- every load returns 0 without touching memory.
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const rsrc_t rw = dl_rsrc(dl_uni(W) + ((long long)tile * (K / 32) + k0 / 32) * 512, on ? 0x7fffffffLL : 0LL);
  const int off = (w * 512 + lane * 8) * 2;  // the lane's part in a VGPR, the piece's in an SGPR (soffset)
#pragma unroll
  for (int j = 0; j < CNT; ++j) {
    const int i = CNT > 1 ? (j + rot) % CNT : 0;
    wa[j].w = __builtin_amdgcn_raw_buffer_load_b128(rw, off, __builtin_amdgcn_readfirstlane(i * DL_SW * 1024), 2);
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
    xa[j].w = __builtin_amdgcn_raw_buffer_load_b128(rx, off, __builtin_amdgcn_readfirstlane(i * DL_SW * 64), 16);
  }
}

template <int CNT>
SYM_DEV f32x4 dl_mma(const Pack8 (&wa)[DL_MAXP], const Pack8 (&xa)[DL_MAXP]) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < CNT; ++i) acc = mfma16(wa[i].v, xa[i].v, acc);
  return acc;
}

// One unit's MFMA chain with the NEXT unit's weights rolled in behind it: piece j's register is reloaded with the
// next unit's piece j right after its MFMA read it, so a workgroup walking several units keeps about a unit of
// pieces in flight instead of draining the pipe at every unit boundary.  Only with the activations resident
// (loaded once per phase): a per-unit reload queued behind the rolled weights would wait for all of them (that
// form measured slower).  No next unit: a zero-length descriptor (the same instructions, no traffic).
template <int CNT>
SYM_DEV f32x4 dl_mma_roll(Pack8 (&wa)[DL_MAXP], const Pack8 (&xa)[DL_MAXP], const bf16* W_next, int rot, bool roll) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const rsrc_t rw = dl_rsrc(dl_uni(W_next), roll ? 0x7fffffffLL : 0LL);
  const int off = (w * 512 + lane * 8) * 2;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < CNT; ++j) {
    acc = mfma16(wa[j].v, xa[j].v, acc);
    const int i = CNT > 1 ? (j + rot) % CNT : 0;
    wa[j].w = __builtin_amdgcn_raw_buffer_load_b128(rw, off, __builtin_amdgcn_readfirstlane(i * DL_SW * 1024), 2);
  }
  return acc;
}

// Activations resident in LDS for a rolled phase: rows m < M of x[:, k0 : k0 + kunit], row stride kunit + 8
// bf16 (16 B of padding: the 16 rows of a fragment read fall on different banks).  DL_XS: 16 rows x 4104.
constexpr int DL_XPAD = 8;
constexpr int DL_XS = 16 * (4096 + DL_XPAD);

// stage x[:M, k0 : k0 + kunit] into LDS by LDS-DMA (sc1: hand-off data), no registers: 1 KB per wave instruction
// (64 lanes x 16 B of one row), instructions dealt over the waves; kunit % 512 == 0.  The caller waits
// (vmcnt(0)) and barriers before the rows are read.
typedef __attribute__((address_space(3))) void dl_lds_t;
SYM_DEV void dl_xs_dma(const DLArgs& a, const bf16* x, int K, int k0, int kunit, bf16* xs) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ipr = kunit / 512;  // instructions per row
  const rsrc_t rx = dl_rsrc(x, (long long)a.M * K * 2);
  for (int q = w; q < a.M * ipr; q += DL_SW) {  // wave-uniform
    const int row = q / ipr, part = q - row * ipr;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (dl_lds_t*)(xs + row * (kunit + DL_XPAD) + part * 512), 16,
                                             ((row * K + k0) * 2 + part * 1024) + lane * 16, 0, 0, 16);
  }
}
// the wave's fragments of one unit from LDS (piece order as dl_load_x)
template <int CNT>
SYM_DEV void dl_xs_frags(Pack8 (&xa)[DL_MAXP], const bf16* xs, int kunit, int rot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const bf16* p = xs + r16 * (kunit + DL_XPAD) + w * 32 + 8 * h;
#pragma unroll
  for (int j = 0; j < CNT; ++j) {
    const int i = CNT > 1 ? (j + rot) % CNT : 0;
    xa[j].u = *reinterpret_cast<const uint4*>(p + i * DL_SW * 32);
  }
}

struct DLPhase {  // one GEMM phase of one layer
  const bf16* W;
  int K;          // weight row length (the projection's full K)
  int kunit;      // k range of one unit (K / ksplit)
  int ntiles;     // 16-row output tiles
  int ksplit;     // units per tile
  int tile_major; // 0: the ntiles x ksplit units dealt round-robin (QKV slabs: each split its own fp32 slab);
                  // 1: the TILES dealt round-robin, a tile's splits consecutive on one workgroup, summed by its control
                  //    wave (gate_up at K = 8192: two 4096-deep units per tile)
  const bf16* x;  // activations [M][K]
};

SYM_DEV int dl_units(const DLPhase& ph, int b, int G) {  // units of workgroup b
  if (ph.tile_major) return b < ph.ntiles ? ph.ksplit * ((ph.ntiles - b + G - 1) / G) : 0;
  const int n = ph.ntiles * ph.ksplit;
  return b < n ? (n - b + G - 1) / G : 0;
}

SYM_DEV void dl_unit_at(const DLPhase& ph, int b, int i, int G, int& tile, int& split) {
  if (ph.tile_major) {
    tile = b + (i / ph.ksplit) * G;
    split = i % ph.ksplit;
  } else {
    const int u = b + i * G;
    tile = u / ph.ksplit;
    split = u % ph.ksplit;
  }
}

// (every path issues the same loads -- zero-length descriptors where the workgroup has no unit -- so no older value
// of the array stays live and the compiler's waits stay exact).  `with_ctl`: the control wave loads its pieces too.
// It does at a signal (its poll then waits for its few pieces, issued before any later stream), not inside a
// phase: there its epilogue drain would wait for the next phase's whole stream; it loads those pieces with the
// activations after the edge instead (dl_gemm_phase `ctl_late`).
template <int CNT, bool LOAD = true>
SYM_DEV void dl_prefetch(Pack8 (&wa)[DL_MAXP], const DLPhase& ph, int b, bool with_ctl, bool any = true) {
  if constexpr (!LOAD) {  // the control wave's instance inside a phase: defined, nothing issued
#pragma unroll
    for (int i = 0; i < CNT; ++i) wa[i].u = make_uint4(0, 0, 0, 0);
    return;
  }
  const bool have = dl_units(ph, b, gridDim.x) > 0;
  const bool on = any && have && (with_ctl || (threadIdx.x >> 6) != DL_CTL);
  int tile = 0, split = 0;
  if (have) dl_unit_at(ph, b, 0, gridDim.x, tile, split);
  dl_load_w<CNT>(wa, ph.W, ph.K, tile, split * ph.kunit, b, on);
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
struct DLResIn {  // the residual epilogue's loads, issued with the unit's activations (before any prefetch)
  f32x4 r;
  uint2 w;
};
SYM_DEV DLResIn dl_epi_res_load(const DLArgs& a, int tile, const bf16* __restrict__ w_next) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, h = lane >> 4;
  const int m = r16, d = a.d, n = tile * 16 + 4 * h;
  const rsrc_t rr = dl_rsrc(a.resid, m < a.M ? (long long)a.M * d * 4 : 0LL);  // rows >= M: zeros, no traffic
  const rsrc_t rw = dl_rsrc(dl_uni(w_next), (long long)d * 2);
  DLResIn in;
  Pack8 t;
  t.w = ld_sc1(rr, (m * d + n) * 4);
  in.r = f32x4{__uint_as_float(t.w[0]), __uint_as_float(t.w[1]), __uint_as_float(t.w[2]), __uint_as_float(t.w[3])};
  const unsigned long long wv = __builtin_bit_cast(unsigned long long,
                                                   __builtin_amdgcn_raw_buffer_load_b64(rw, n * 2, 0, 0));
  in.w = make_uint2((unsigned)wv, (unsigned)(wv >> 32));
  return in;
}

SYM_DEV void dl_epi_res(const DLArgs& a, f32x4 v, int tile, DLResIn in, unsigned ep) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, h = lane >> 4;
  const int m = r16, d = a.d, n = tile * 16 + 4 * h;
  const bool mok = m < a.M;
  const rsrc_t rr = dl_rsrc(a.resid, (long long)a.M * d * 4);
  const f32x4 r = in.r;
  const uint2 wraw = in.w;
  const long long goff = xar_goff(m, d, n);
  const bool xar = a.xp.world > 1;
  if (mok && xar) xar_push(a.xp, v, goff, ep);
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

struct DLNoHook {
  SYM_DEV void operator()() const {}
};

// One GEMM phase: the workgroup's units b, b + G, ... (the first unit's weights already in flight in wa).
// `after_x` runs right after the first unit's activation loads are issued: the NEXT phase's weight prefetch goes
// there, behind this phase's operands (a wave's loads retire in order: weights issued before the activations --
// at the previous signal -- made this phase's first MFMA wait for the next phase's whole stream).
// `tail` runs after the LAST unit's MFMAs instead of a next unit's weight loads: a next phase whose weights do not
// fit beside this phase's registers streams from there, into this phase's own (then free) registers.
template <int CNT, int EPI, bool ROLL = false, typename AfterX, typename Tail>
SYM_DEV void dl_gemm_phase(const DLArgs& a, const DLPhase& ph, const DLEpi& ep, Pack8 (&wa)[DL_MAXP],
                           Pack8 (&xa)[DL_MAXP], int b, f32x4 (*red)[DL_SW][64], const float* rn_s,
                           unsigned* xep_s, int ev, bool ctl_late, AfterX after_x, Tail tail, bf16* xs = nullptr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool ctl = wid == DL_CTL;
  const rsrc_t rx = dl_rsrc(ph.x, (long long)a.M * ph.K * 2);
  int buf = 0;
  // (the first unit peeled: `after_x` defines the prefetch registers on every path, so no older value of them
  // stays live through the phase -- a conditional definition inside the loop kept both and spilled)
  const int nu = dl_units(ph, b, a.G);
  f32x4 gacc = {0.f, 0.f, 0.f, 0.f};  // tile-major: the control wave's running sum over a tile's splits
  auto unit = [&](int i, auto hook) {
    int tile, split;
    dl_unit_at(ph, b, i, a.G, tile, split);
    const int k0 = split * ph.kunit;
    DLResIn res_in{};
    {
      if (ctl && i == 0 && ctl_late) dl_load_w<CNT>(wa, ph.W, ph.K, tile, k0, b);
      // ROLL (round-robin phases: every unit of the workgroup has the same k range): the activations are staged
      // into LDS once, by the first unit, and every unit reads its fragments there
      constexpr bool first = !std::is_same_v<decltype(hook), DLNoHook>;
      if constexpr (ROLL) {
        if constexpr (first) dl_xs_dma(a, ph.x, ph.K, k0, ph.kunit, xs);
      } else {
        dl_load_x<CNT>(xa, rx, ph.K, k0, a.M, b);
      }
      if constexpr (EPI == EP_RES)
        if (ctl) res_in = dl_epi_res_load(a, tile, ep.w_next);
      if constexpr (first) {
        // every wave's operand loads (the control wave's late weight pieces too) are queued before any wave's
        // prefetch: a CU's vector memory path returns in issue order, so a load queued behind the next phase's
        // stream waited for all of it (the control wave's -- whose partial every unit's epilogue needs -- ~3 us).
        // A bare s_barrier: __syncthreads' fence would wait for the loads themselves.  Staged activations: every
        // wave's DMA landed, then the barrier publishes the rows (MI355X_MICROARCH.md, LDS-DMA).
        if constexpr (ROLL) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
        } else {
          __builtin_amdgcn_s_barrier();
        }
        hook();
      }
      if constexpr (ROLL) dl_xs_frags<CNT>(xa, xs, ph.kunit, b);
      // every activation load issued before the first MFMA waits (left to itself the scheduler interleaved them
      // with the MFMAs to save registers, one memory round trip per piece)
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc;
      if constexpr (ROLL) {
        int t2 = 0, s2 = 0;
        if (i + 1 < nu) dl_unit_at(ph, b, i + 1, a.G, t2, s2);
        acc = dl_mma_roll<CNT>(wa, xa, ph.W + ((long long)t2 * (ph.K / 32) + s2 * ph.kunit / 32) * 512, b, i + 1 < nu);
      } else {
        acc = dl_mma<CNT>(wa, xa);
      }
      // the next unit's weights behind this unit's MFMAs (same registers: no renamed second copy)
      __builtin_amdgcn_sched_barrier(0);
      if (ROLL && i + 1 < nu) {
      } else if (i + 1 < nu) {
        int t2, s2;
        dl_unit_at(ph, b, i + 1, a.G, t2, s2);
        dl_load_w<CNT>(wa, ph.W, ph.K, t2, s2 * ph.kunit, b);
      } else if (ctl) {
        tail(std::false_type{});
      } else {
        tail(std::true_type{});
      }
      red[buf][wid][lane] = acc;
      if (i == 0 && ctl && a.stamps != nullptr) {  // operands landed: the store above needed the MFMA result (no
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // vmcnt wait: it would also wait for the prefetch)
        dl_stamp_ctl(a, ev, b, 2);
      }
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
      bool last = true;
      if (ph.tile_major && ph.ksplit > 1) {
        v += gacc;
        last = split == ph.ksplit - 1;
        gacc = last ? f32x4{0.f, 0.f, 0.f, 0.f} : v;
      }
      if constexpr (EPI == EP_SLAB) {
        if (mok) {
          const rsrc_t rs = dl_rsrc(ep.slab, (long long)ph.ksplit * a.M * ep.Nq * 4);
          const int off = ((split * a.M + m) * ep.Nq + tile * 16 + 4 * h) * 4;
          st_sc1(rs, off, u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                __float_as_uint(v[3])});
        }
      } else if constexpr (EPI == EP_RES) {
        if (last) {
          const unsigned e = ++xep_s[ph.tile_major ? i / ph.ksplit : i];
          dl_epi_res(a, v, tile, res_in, e);
        }
      } else if (last) {  // EP_SWI: rows 0-7 gate, 8-15 up (interleaved per tile), row scale of the deferred norm
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
  };
  // the control wave runs an instance whose hook issues nothing: its epilogue loads and its drain must not queue
  // behind the next phase's stream (the streamers' instance issues it)
  const auto hook_load = [&] { after_x(std::true_type{}); };
  const auto hook_none = [&] { after_x(std::false_type{}); };
  if (nu > 0) {
    if (ctl)
      unit(0, hook_none);
    else
      unit(0, hook_load);
  } else {
    if (ctl) {
      hook_none();
      tail(std::false_type{});
    } else {
      hook_load();
      tail(std::true_type{});
    }
  }
  for (int i = 1; i < nu; ++i) unit(i, DLNoHook{});
}

// ---- attention ----------------------------------------------------------------------------------------------
// Wave-level split-KV: a (sequence, kv head) is DL_APARTS units, one per wave (partition p: the 32-token groups p,
// p + DL_APARTS, ... of the old tokens), dealt over the workgroups first (at TP = 8, 10 sequences: 80 workgroups with
// one attention wave each), so the old K / V stream in over 80 CUs' load paths instead of 10 (a 128 KB per-CU share
// took ~8 us).  Every unit rebuilds the (small) q / k / v rows of its (sequence, kv head) from the QKV slabs (x the
// row scale, RoPE through a lane shuffle: the partner row r ^ 8 sits two lanes away), publishes its partial
// softmax state (sc1), drains, and bumps the (sequence, kv head) counter; the last arriver merges the partials with
// the newest token (its score and value from its own rebuilt rows) and stores the head outputs (sc1: handed to O).
// The newest token's K / V come out of this step's slabs; every OLDER token is in the paged cache since an earlier
// launch, so the first group's block-table entry is read before the edge and its K / V loads issue together with
// the slab loads right after it.  Partition 0 stores the newest K / V for the next step (kernel boundary: plain).
struct DLWaveLds {  // per wave: the roped q rows and the newest token's k / v (bf16, natural dim order)
  bf16 q[DL_GMAX][128];
  bf16 knew[128], vnew[128];
};

struct DLAttnMeta {
  int ctx, slot, pos, bk0;
};

SYM_DEV DLAttnMeta dl_attn_meta(const DLArgs& a, int s, int p) {
  DLAttnMeta mt;
  mt.ctx = a.ctx_lens[s];
  mt.slot = a.slots[s];
  mt.pos = a.positions[s];
  const int tok0 = 32 * p;
  mt.bk0 = tok0 < mt.ctx - 1 ? a.block_tables[(long long)s * a.max_blocks + (tok0 >> __builtin_ctz(a.BS))] : -1;
  return mt;
}

// One 32-token group's K / V fragments (attn_decode.h load_group's layout) by buffer loads off the group's block
SYM_DEV void dl_load_kv(const DLLayer& ly, int Hkv, int BS, int bk, int g, int tok0, KVFrag& f) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, h = lane >> 4;
  const int boff = tok0 & (BS - 1);
  const rsrc_t rk = dl_rsrc(dl_uni(ly.k_cache) + (((long long)bk * Hkv + g) * BS + boff) * D, 0x7fffffffLL);
  const rsrc_t rv = dl_rsrc(dl_uni(ly.v_cache) + ((long long)bk * Hkv + g) * (long long)D * BS + boff, 0x7fffffffLL);
#pragma unroll
  for (int aa = 0; aa < 2; ++aa) {
    const int trow = (r16 >> 2) * 8 + 4 * aa + (r16 & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Pack8 t;
      t.w = __builtin_amdgcn_raw_buffer_load_b128(rk, (trow * D + 32 * h + 8 * i) * 2, 0, 0);
      f.k[aa][i] = t.v;
    }
  }
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    Pack8 t;
    t.w = __builtin_amdgcn_raw_buffer_load_b128(rv, ((16 * dt + r16) * BS + 8 * h) * 2, 0, 0);
    f.v[dt] = t.v;
  }
}

// KS: QKV k-slabs, GH: query heads per kv head (4 or 8) -- template parameters of the shape class, so every
// register array below has its exact size
// What a unit loads that does not depend on this step's QKV -- the row scale (the layer input's sum-of-squares
// partials: published before the QKV phase began) and the RoPE cos / sin -- issued right after the QKV signal.
struct DLAttnPre {
  float4 co, si;
  float rn;
};

SYM_DEV void dl_attn_pre(const DLArgs& a, int sg, const float* __restrict__ ss_in,
                         int ss_tiles, DLAttnMeta mt, DLAttnPre& pre) {
  const int lane = threadIdx.x & 63;
  const int s = sg / a.Hkv;
  const int r4 = (4 * lane) & 127;  // the lane's rows within a head (permuted order)
  const int dh0 = 8 * (r4 >> 4) + (r4 & 7);
  const rsrc_t rc = dl_rsrc(a.cos_sin + (long long)mt.pos * 128, 512);
  Pack8 c, t;
  c.w = __builtin_amdgcn_raw_buffer_load_b128(rc, dh0 * 4, 0, 0);
  t.w = __builtin_amdgcn_raw_buffer_load_b128(rc, (64 + dh0) * 4, 0, 0);
  float ssum = 0.f;
  const rsrc_t rs = dl_rsrc(ss_in, (long long)a.M * ss_tiles * 4);
  if ((ss_tiles & 3) == 0) {
    Pack8 sq[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = 4 * lane + 256 * k;
      sq[k].w = i < ss_tiles ? ld_sc1(rs, (s * ss_tiles + i) * 4) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) ssum += __uint_as_float(sq[k].w[e]);
  } else {
    for (int i = lane; i < ss_tiles; i += 64) ssum += ldf_sc1(ss_in + (long long)s * ss_tiles + i);
  }
  pre.co = make_float4(__uint_as_float(c.w[0]), __uint_as_float(c.w[1]), __uint_as_float(c.w[2]),
                       __uint_as_float(c.w[3]));
  pre.si = make_float4(__uint_as_float(t.w[0]), __uint_as_float(t.w[1]), __uint_as_float(t.w[2]),
                       __uint_as_float(t.w[3]));
  pre.rn = rsqrtf(wave_sum(ssum) * (1.f / (float)a.d) + a.eps);
}

template <int KS, int GH>
SYM_DEV void dl_attn_wave(const DLArgs& a, const DLLayer& ly, int sg, int p, DLWaveLds& W, DLAttnMeta mt,
                          const DLAttnPre& pre, int stamp_ev) {
  const int lane = threadIdx.x & 63;
  constexpr int Gh = GH, R = (GH + 2) / 2;  // R: 256-value rounds of the unit's q / k / v rows
  const int Hq = a.Hq, Hkv = a.Hkv;
  const int s = sg / Hkv, g = sg % Hkv;
  const int Nq = (Hq + 2 * Hkv) * 128;
  const int ctx = mt.ctx, ctx_old = ctx - 1, slot = mt.slot;
  const int c = lane & 15, h = lane >> 4;
  const int bsh = __builtin_ctz(a.BS);
  const int* bt = a.block_tables + (long long)s * a.max_blocks;
  // ---- after the edge: the first group's old K / V and the slab rows (4 consecutive values per lane per round),
  // all at once (the old K / V held across the edge instead spilled)
  KVFrag f;
  int tok0 = 32 * p;
  if (tok0 < ctx_old) dl_load_kv(ly, Hkv, a.BS, mt.bk0, g, tok0, f);
  Pack8 q[R][KS];
  {
    const rsrc_t rq = dl_rsrc(a.qkv_ws, (long long)KS * a.M * Nq * 4);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int t4 = 4 * lane + 256 * j;
      const int row = t4 < Gh * 128 ? g * Gh * 128 + t4
                                    : (t4 < (Gh + 1) * 128 ? Hq * 128 + g * 128 + (t4 - Gh * 128)
                                                           : (Hq + Hkv) * 128 + g * 128 + (t4 - (Gh + 1) * 128));
#pragma unroll
      for (int sp = 0; sp < KS; ++sp) q[j][sp].w = ld_sc1(rq, ((sp * a.M + s) * Nq + row) * 4);
    }
  }
  const int r4 = (4 * lane) & 127;
  const bool lo = (r4 & 15) < 8;
  const int dh0 = 8 * (r4 >> 4) + (r4 & 7);
  const float4 co = pre.co, si = pre.si;
  const float rn = pre.rn;
  if (stamp_ev >= 0 && a.stamps != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) a.stamps[((long long)blockIdx.x * a.L * DL_PH + stamp_ev) * 8 + 2] = wall_clock64();
  }
  // ---- rebuild the rows (slab sum x row scale), RoPE on q / k, into the wave's LDS; partition 0 writes the cache
  {
    const long long blk = slot >= 0 ? slot / a.BS : 0, off = slot >= 0 ? slot % a.BS : 0;
    const float cof[4] = {co.x, co.y, co.z, co.w}, sif[4] = {si.x, si.y, si.z, si.w};
#pragma unroll
    for (int j = 0; j < R; ++j) {
      float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < KS; ++sp)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += __uint_as_float(q[j][sp].w[e]);
      float pv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] *= rn;
        pv[e] = __shfl_xor(v[e], 2, 64);
      }
      const int t4 = 4 * lane + 256 * j;
      const int dim0 = dh0 + (lo ? 0 : 64);
      Pack8 pk;
      if (t4 < (Gh + 1) * 128) {
#pragma unroll
        for (int e = 0; e < 4; ++e) pk.h[e] = (bf16)(lo ? v[e] * cof[e] - pv[e] * sif[e] : v[e] * cof[e] + pv[e] * sif[e]);
        const uint2 u = make_uint2(pk.w[0], pk.w[1]);
        if (t4 < Gh * 128) {
          *reinterpret_cast<uint2*>(&W.q[t4 >> 7][dim0]) = u;
        } else {
          *reinterpret_cast<uint2*>(&W.knew[dim0]) = u;
          if (p == 0 && slot >= 0)
            *reinterpret_cast<uint2*>(ly.k_cache + ((blk * Hkv + g) * a.BS + off) * 128 + dim0) = u;
        }
      } else {  // v: natural order; dim-major cache (one bf16 per line)
        const int dim = t4 - (Gh + 1) * 128;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16 bv = (bf16)v[e];
          W.vnew[dim + e] = bv;
          if (p == 0 && slot >= 0) ly.v_cache[((blk * Hkv + g) * 128 + dim + e) * (long long)a.BS + off] = bv;
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS rows, read back across lanes
  // ---- old tokens of this partition
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  bf16x8 qf[4];
  if (c < Gh) {
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = *reinterpret_cast<const bf16x8*>(&W.q[c][32 * h + 8 * i]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = zero8();
  }
  if (tok0 < ctx_old)
    compute_group(f, qf, a.scale_log2, [&](int aa, int r) { return tok0 + 8 * h + 4 * aa + r < ctx_old; }, o, m, lsum);
  tok0 += DL_APARTS * 32;
#pragma unroll 1
  for (; tok0 < ctx_old; tok0 += DL_APARTS * 32) {
    dl_load_kv(ly, Hkv, a.BS, __builtin_amdgcn_readfirstlane(bt[tok0 >> bsh]), g, tok0, f);
    compute_group(f, qf, a.scale_log2, [&](int aa, int r) { return tok0 + 8 * h + 4 * aa + r < ctx_old; }, o, m,
                  lsum);
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  // ---- publish the partial, count in; the last arriver merges
  const int nused = ctx_old > 0 ? min(DL_APARTS, (ctx_old + 31) / 32) : 0;
  const long long sync_w = dl_edge_sync_words(a.L, a.M, Hkv);
  unsigned* cnt = a.edge + (long long)a.L * DL_PH * 8 * DL_SHARD_STRIDE + sg * 32;
  float* po = reinterpret_cast<float*>(a.edge + sync_w);
  float* pml = po + (long long)a.M * Hkv * DL_APARTS * Gh * 128;
  const rsrc_t rpo = dl_rsrc(po, (long long)a.M * Hkv * DL_APARTS * Gh * 128 * 4);
  const rsrc_t rpm = dl_rsrc(pml, (long long)a.M * Hkv * Gh * DL_APARTS * 2 * 4);
  if (p < nused && c < Gh) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      st_sc1(rpo, ((((sg * DL_APARTS + p) * Gh + c) * 128) + 16 * dt + 4 * h) * 4,
             u32x4{__float_as_uint(o[dt][0]), __float_as_uint(o[dt][1]), __float_as_uint(o[dt][2]),
                   __float_as_uint(o[dt][3])});
    if (h == 0) {
      stf_sc1(pml + ((sg * Gh + c) * DL_APARTS + p) * 2, m);
      stf_sc1(pml + ((sg * Gh + c) * DL_APARTS + p) * 2 + 1, lsum);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  if (old != DL_APARTS - 1) return;
  if (lane == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next layer's
  if (stamp_ev >= 0 && a.stamps != nullptr && lane == 0)
    a.stamps[((long long)blockIdx.x * a.L * DL_PH + stamp_ev) * 8 + 3] = wall_clock64();
  // ---- merge: lane -> head qq, 2 Gh consecutive dims
  constexpr int LPH = 64 / Gh, DPL = 2 * Gh, CH = Gh / 2;
  const int qq = lane / LPH, d0 = (lane % LPH) * DPL;
  Pack8 mlv[DL_APARTS / 2];
#pragma unroll
  for (int i = 0; i < DL_APARTS / 2; ++i) mlv[i].w = ld_sc1(rpm, (((sg * Gh + qq) * DL_APARTS) * 2 + 4 * i) * 4);
  Pack8 ov[DL_APARTS][CH];
#pragma unroll
  for (int pp = 0; pp < DL_APARTS; ++pp)
#pragma unroll
    for (int k = 0; k < CH; ++k)
      ov[pp][k].w = pp < nused
                        ? ld_sc1(rpo, ((((sg * DL_APARTS + pp) * Gh + qq) * 128) + d0 + 4 * k) * 4)
                        : u32x4{0u, 0u, 0u, 0u};
  float sn = 0.f;  // the newest token's score over the lane's dims, then over the head's lanes
#pragma unroll
  for (int j = 0; j < DPL; ++j) sn += (float)W.q[qq][d0 + j] * (float)W.knew[d0 + j];
#pragma unroll
  for (int x = LPH / 2; x > 0; x >>= 1) sn += __shfl_xor(sn, x, 64);
  sn *= a.scale_log2;
  const bool has_new = ctx >= 1;
  float Mx = has_new ? sn : -INFINITY;
#pragma unroll
  for (int pp = 0; pp < DL_APARTS; ++pp)
    if (pp < nused) Mx = fmaxf(Mx, __uint_as_float(mlv[pp / 2].w[(pp & 1) * 2]));
  float Ls = 0.f, acc[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
#pragma unroll
  for (int pp = 0; pp < DL_APARTS; ++pp) {
    const float mp = __uint_as_float(mlv[pp / 2].w[(pp & 1) * 2]), lp = __uint_as_float(mlv[pp / 2].w[(pp & 1) * 2 + 1]);
    const float fct = pp < nused ? __builtin_amdgcn_exp2f(mp - Mx) : 0.f;
    Ls += pp < nused ? lp * fct : 0.f;
#pragma unroll
    for (int k = 0; k < CH; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4 * k + e] += __uint_as_float(ov[pp][k].w[e]) * fct;
  }
  if (has_new) {
    const float fct = __builtin_amdgcn_exp2f(sn - Mx);
    Ls += fct;
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[j] += fct * (float)W.vnew[d0 + j];
  }
  const float inv = Ls > 0.f ? 1.f / Ls : 0.f;  // ctx == 0 (padding row): zeros
  const rsrc_t ro = dl_rsrc(a.attn, (long long)a.M * Hq * 128 * 2);
#pragma unroll
  for (int k = 0; k < DPL / 8; ++k) {
    Pack8 pk;
#pragma unroll
    for (int j = 0; j < 8; ++j) pk.h[j] = (bf16)(acc[8 * k + j] * inv);
    st_sc1(ro, ((s * Hq + g * Gh + qq) * 128 + d0 + 8 * k) * 2, pk.w);
  }
}

// ---- the step ---------------------------------------------------------------------------------------------
// Specialised per shape class: the k pieces per streamer wave of the QKV, O, gate_up and down units are template
// parameters, so every register array has its exact size (a runtime-dispatched form inlined every instantiation
// into one body and spilled).
template <int CQ, int CO, int CG, int CD, int KS, int GH>
SYM_DEV void dl_body(const DLArgs& a, int b) {
  __shared__ f32x4 red[2][DL_SW][64];
  __shared__ float rn_s[16];
  __shared__ unsigned xep_s[DL_MAXT];
  // the attention phase's per-wave rows and a rolled GEMM phase's resident activations share the space
  __shared__ __attribute__((aligned(16))) char lds_u[DL_XS * 2 > (int)sizeof(DLWaveLds) * DL_SW ? DL_XS * 2
                                                                                               : sizeof(DLWaveLds) * DL_SW];
  DLWaveLds* lds_wave = reinterpret_cast<DLWaveLds*>(lds_u);
  bf16* xs = reinterpret_cast<bf16*>(lds_u);
  __shared__ DLLayer lay_s[DL_MAXL];  // the layer table (LDS reads: no vector-memory wait behind streaming loads)
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool ctl = wid == DL_CTL;
  const int d = a.d, Nq = (a.Hq + 2 * a.Hkv) * 128;
  const int ntile_d = d / 16;
  // this workgroup's O / down tiles (b, b + G, ...): their all-reduce epochs, read once, bumped by every O and
  // every down phase, written back at exit (the per-tile counters of the fused launches, decode_gemm.hip)
  const int nmine = b < ntile_d ? (ntile_d - b + a.G - 1) / a.G : 0;
  const unsigned epoch = ctl ? dl_epoch(a) : 0u;  // (read before this workgroup's first signal)
  {
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(a.layers);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(lay_s);
    for (int i = threadIdx.x; i < a.L * (int)(sizeof(DLLayer) / 8); i += DL_NT) dst[i] = src[i];
  }
  if (ctl && a.xp.world > 1)
    for (int i = lane; i < nmine; i += 64) xep_s[i] = a.xar_ctr[b + i * a.G];
  __syncthreads();

  // Weight registers.  A phase's weights stream as early as the registers allow: "early" into a register set of
  // their own during the previous phase (right behind its first unit's activations: TP = 8, whose units are a whole
  // phase's share), otherwise from the previous phase's last MFMAs on, into that phase's (then free) set ("tail").
  //   O: wa (from the attention signal); gate_up: wb early / wa; down: wc early / gate_up's; the next layer's QKV:
  //   wa early / down's.
  Pack8 wa[DL_MAXP], wb[DL_MAXP], wc[DL_MAXP], xa[DL_MAXP];
  constexpr bool kEarlyGu = CO + CG <= 24;    // TP = 8 / 4: O 2-4 pieces beside gate_up's 16
  constexpr bool kEarlyDown = CG + CD <= 24;  // TP = 8: 16 + 7 (TP = 4's 16 + 14 spilled ~190 VGPRs)
  constexpr bool kEarlyQkv = CD + CQ <= 16 && (kEarlyDown || kEarlyGu);  // (down's set must not be wa)
  // Phases whose workgroups walk several units of one k range run with their activations resident in LDS and the
  // next unit's weights rolled in behind the MFMAs (dl_mma_roll): 8B TP = 1 QKV (3 units) and gate_up (7), 8B
  // TP = 4 gate_up (2), 70B TP = 8 O and down (2 each).  Not 70B gate_up, whose tile-major units change k range;
  // not single-unit phases (the LDS staging step would only add latency there).
  constexpr bool kTp1 = CO == 16 && GH == 4, kTp4 = CO == 4 && GH == 4, k70 = GH == 8;
  constexpr bool kRollQkv = kTp1, kRollO = k70, kRollGu = kTp1 || kTp4, kRollDown = k70;
  Pack8(&w_gu)[DL_MAXP] = kEarlyGu ? wb : wa;
  Pack8(&w_dn)[DL_MAXP] = kEarlyDown ? wc : w_gu;
  Pack8(&w_qkv)[DL_MAXP] = kEarlyQkv ? wa : w_dn;
  auto phase_of = [&](int l, int p) -> DLPhase {
    const DLLayer& ly = lay_s[l];
    if (p == DL_QKV) return DLPhase{ly.wqkv, d, d / a.KSq, Nq / 16, a.KSq, 0, a.xw};
    if (p == DL_O) return DLPhase{ly.wo, a.Hq * 128, a.Hq * 128, ntile_d, 1, 0, a.attn};
    if (p == DL_GU) return DLPhase{ly.wgu, d, d / a.KSg, (2 * a.Fl) / 16, a.KSg, 1, a.xw};
    return DLPhase{ly.wdown, a.Fl, a.Fl / a.KSd, ntile_d, a.KSd, 1, a.act};
  };
  const auto none = [](auto) {};
  dl_prefetch<CQ>(w_qkv, phase_of(0, DL_QKV), b, true);
  for (int l = 0; l < a.L; ++l) {
    const DLLayer& ly = lay_s[l];
    const int ev0 = l * DL_PH;
    // ---- QKV: split-K slabs (the row scale waits for the attention phase)
    if (l > 0) dl_wait(a, ev0 - DL_PH + DL_DOWN, epoch);
    dl_stamp(a, ev0 + DL_QKV, b, 0);
    dl_gemm_phase<CQ, EP_SLAB, kRollQkv>(a, phase_of(l, DL_QKV), DLEpi{EP_SLAB, a.qkv_ws, Nq, nullptr, nullptr, Nq},
                                         w_qkv, xa, b, red, rn_s, xep_s, ev0 + DL_QKV, l > 0, none, none, xs);
    dl_signal(a, ev0 + DL_QKV, b, ctl);
    // ---- attention: wave-level units (sequence x kv head x partition), dealt over the workgroups first; the first
    // unit's metadata read before the edge
    {
      const int nv = a.M * a.Hkv * DL_APARTS;
      const int v0 = b + a.G * wid;
      const float* ss_in = l == 0 ? a.ss0 : a.ss;
      const int ss_tiles = l == 0 ? a.ss0_tiles : ntile_d;
      DLAttnMeta mt{0, -1, 0, -1};
      DLAttnPre pre;
      if (v0 < nv) {
        mt = dl_attn_meta(a, v0 / DL_APARTS / a.Hkv, v0 % DL_APARTS);
        dl_attn_pre(a, v0 / DL_APARTS, ss_in, ss_tiles, mt, pre);
      }
      dl_wait(a, ev0 + DL_QKV, epoch);
      dl_stamp(a, ev0 + DL_ATTN, b, 0);
      for (int v = v0; v < nv; v += a.G * DL_SW) {
        if (v != v0) {
          mt = dl_attn_meta(a, v / DL_APARTS / a.Hkv, v % DL_APARTS);
          dl_attn_pre(a, v / DL_APARTS, ss_in, ss_tiles, mt, pre);
        }
        dl_attn_wave<KS, GH>(a, ly, v / DL_APARTS, v % DL_APARTS, lds_wave[wid], mt, pre, v == b ? ev0 + DL_ATTN : -1);
      }
    }
    dl_signal(a, ev0 + DL_ATTN, b);
    dl_prefetch<CO>(wa, phase_of(l, DL_O), b, true);  // before any later stream
    // ---- O (+ all-reduce, residual, ln2 prep)
    dl_wait(a, ev0 + DL_ATTN, epoch);
    dl_stamp(a, ev0 + DL_O, b, 0);
    dl_gemm_phase<CO, EP_RES, kRollO>(
        a, phase_of(l, DL_O), DLEpi{EP_RES, nullptr, 0, ly.ln2, nullptr, d}, wa, xa, b, red, rn_s, xep_s, ev0 + DL_O,
        false, [&](auto load) { if constexpr (kEarlyGu) dl_prefetch<CG, load>(wb, phase_of(l, DL_GU), b, false); },
        [&](auto load) { if constexpr (!kEarlyGu) dl_prefetch<CG, load>(wa, phase_of(l, DL_GU), b, false); }, xs);
    dl_signal(a, ev0 + DL_O, b, ctl);
    // ---- gate_up (+ row scale, SwiGLU)
    dl_wait(a, ev0 + DL_O, epoch);
    dl_stamp(a, ev0 + DL_GU, b, 0);
    dl_row_scales(a, a.ss, ntile_d, rn_s);  // published by the first unit's barrier, before any epilogue reads it
    dl_gemm_phase<CG, EP_SWI, kRollGu>(
        a, phase_of(l, DL_GU), DLEpi{EP_SWI, nullptr, 0, nullptr, a.act, 2 * a.Fl}, w_gu, xa, b, red, rn_s, xep_s,
        ev0 + DL_GU, true,
        [&](auto load) { if constexpr (kEarlyDown) dl_prefetch<CD, load>(wc, phase_of(l, DL_DOWN), b, false); },
        [&](auto load) { if constexpr (!kEarlyDown) dl_prefetch<CD, load>(w_gu, phase_of(l, DL_DOWN), b, false); },
        xs);
    dl_signal(a, ev0 + DL_GU, b, ctl);
    // ---- down (+ all-reduce, residual, next-norm prep)
    dl_wait(a, ev0 + DL_GU, epoch);
    dl_stamp(a, ev0 + DL_DOWN, b, 0);
    const int ln = l + 1 < a.L ? l + 1 : l;  // (the last layer issues zero-length loads: the same instructions)
    dl_gemm_phase<CD, EP_RES, kRollDown>(
        a, phase_of(l, DL_DOWN), DLEpi{EP_RES, nullptr, 0, ly.lnn, nullptr, d}, w_dn, xa, b, red, rn_s, xep_s,
        ev0 + DL_DOWN, true,
        [&](auto load) {
          if constexpr (kEarlyQkv) dl_prefetch<CQ, load>(wa, phase_of(ln, DL_QKV), b, false, ln != l);
        },
        [&](auto load) {
          if constexpr (!kEarlyQkv) dl_prefetch<CQ, load>(w_dn, phase_of(ln, DL_QKV), b, false, ln != l);
        },
        xs);
    dl_signal(a, ev0 + DL_DOWN, b, ctl);
  }
  if (ctl && a.xp.world > 1)
    for (int i = lane; i < nmine; i += 64) a.xar_ctr[b + i * a.G] = xep_s[i];
}

// (the arguments indexed by blockIdx.z, always 0 here: a dynamically indexed kernel argument is read from the
// kernarg segment where used -- passed plainly, every field was hoisted into SGPRs at entry and ~300 of them
// spilled, through VGPR lanes into scratch)
struct DLOne {
  DLArgs a[1];
};
template <int CQ, int CO, int CG, int CD, int KS, int GH>
__global__ __launch_bounds__(DL_NT) void decode_layers_kernel(DLOne m) {
  dl_body<CQ, CO, CG, CD, KS, GH>(m.a[blockIdx.z], blockIdx.x);
}

// The shape classes built (pieces per streamer wave = unit K / 256 for QKV (K = d / KSq), O (K = Hq x 128 / tp),
// gate_up (K = d), down (K = F / tp)):
//   Llama-3-8B TP = 8: QKV 1024 (KSq 4), O 512, gate_up 4096, down 1792   -> (4, 2, 16, 7)
//   Llama-3-8B TP = 4: QKV 2048 (KSq 2), O 1024, gate_up 4096, down 3584  -> (8, 4, 16, 14)
//   small-llama TP = 1 / 2 (tests): QKV 512 (KSq 2) / 256 (KSq 4), O 1024 / 512, gate_up 1024, down 3584 / 1792;
//   its TP = 2 one-GPU rehearsal (128 workgroups per rank): QKV 512 (KSq 2)
// (+ the QKV k-slabs and the query heads per kv head: 4 for both models)
//   Llama-3-70B TP = 8: QKV 4096 (KSq 2), O 1024, gate_up 2 x 4096 (KSg 2, tile-major), down 3584 -> (16, 4, 16, 14)
//   Llama-3-8B TP = 1: QKV 2048 (KSq 2), O 4096, gate_up 4096, down 4 x 3584 (KSd 4, tile-major) -> (8, 16, 16, 14)
//   Llama-3-8B TP = 2: QKV 1024 (KSq 4), O 2048, gate_up 4096, down 2 x 3584 (KSd 2)              -> (4, 8, 16, 14)
#define DL_SHAPES(X)                                                                                        \
  X(4, 2, 16, 7, 4, 4) X(8, 4, 16, 14, 2, 4) X(2, 4, 4, 14, 2, 4) X(1, 2, 4, 7, 4, 4) X(2, 2, 4, 7, 2, 4) \
  X(16, 4, 16, 14, 2, 8) X(8, 16, 16, 14, 2, 4) X(4, 8, 16, 14, 4, 4)

bool dl_check(const DLArgs& a) {
  return a.M >= 1 && a.M <= 16 && a.L >= 1 && a.Hkv >= 1 && a.Hq % a.Hkv == 0 && (a.Hq / a.Hkv == 4 || a.Hq / a.Hkv == 8) &&
         a.d % 256 == 0 && a.Fl % 256 == 0 && a.BS >= 32 && (a.BS & (a.BS - 1)) == 0 && a.G >= 1 &&
         (a.d / 16 + a.G - 1) / a.G <= DL_MAXT && a.L <= DL_MAXL && a.KSq >= 1 && a.KSq <= DL_MAXKS &&
         a.d % (a.KSq * 256) == 0 && a.KSg >= 1 && a.d % (a.KSg * 256) == 0 && a.KSd >= 1 &&
         a.Fl % (a.KSd * 256) == 0;
}


int g_dl_resident[16];  // per shape: workgroups per CU the kernel admits (occupancy query, once; 0 = unknown)

template <typename Kern>
int dl_per_cu(Kern k, int& cache) {
  if (cache <= 0) {
    int n = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, DL_NT, 0);
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

int decode_layers_pieces_ok(int cq, int co, int cg, int cd, int ks, int gh) {
#define DL_MATCH(A, B, C, D_, KS, GH) \
  if (cq == A && co == B && cg == C && cd == D_ && ks == KS && gh == GH) return 1;
  DL_SHAPES(DL_MATCH)
#undef DL_MATCH
  return 0;
}

bool launch_decode_layers(const DLArgs& a, hipStream_t s) {
  if (!dl_check(a)) return false;
  int idx = 0;
#define DL_LAUNCH(A, B, C, D_, KS, GH)                                                                  \
  if (a.cq == A && a.co == B && a.cg == C && a.cd == D_ && a.KSq == KS && a.Hq / a.Hkv == GH) {          \
    auto k = decode_layers_kernel<A, B, C, D_, KS, GH>;                                                  \
    if (a.G > dl_cus() * dl_per_cu(k, g_dl_resident[idx])) return false; /* every workgroup resident */ \
    k<<<a.G, DL_NT, 0, s>>>(DLOne{{a}});                                                                 \
    return true;                                                                                         \
  }                                                                                                      \
  ++idx;
  DL_SHAPES(DL_LAUNCH)
#undef DL_LAUNCH
  return false;
}
