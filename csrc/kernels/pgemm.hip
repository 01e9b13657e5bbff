// Prefill projection GEMM (hundreds to a few thousand rows): the compute-bound regime of a dense layer.
//   y[m][n] = rs[m] * sum_k x[m][k] * W[n][k],   x [M][K] bf16 row-major, W [N][K] bf16 MFMA-preshuffled
//   (models/layout.py::preshuffle -- the SAME copy the decode GEMMs stream, so no row-major weight copy is
//   needed for the library), rs the deferred-RMSNorm row scale (optional).
//
// Why not hipBLASLt: config 3's first prefill step (6 x 128 = 768 tokens) spent 76 % of its time in four
// library GEMMs at 0.78-1.16 PF (profiles/r4/prof_prefill768.csv), gate_up at 768 x 28672 runs 336 of the
// library's 256x256 tiles = 1.31 waves on 256 CUs, and every consumer (RMSNorm, RoPE + cache write, SwiGLU,
// residual add) re-read the library's output in its own launch.  Here:
//
//   * block tile BM x BN = (4 m-waves x WM 16-token tiles) x (2 n-waves x WN 16-feature tiles), 8 waves,
//     the whole K (or a K slice) per block, tile sizes chosen per shape on the host so the grid is one
//     (or a whole number of) waves of 256 CUs -- e.g. gate_up at 768 rows: 384 x 224 tiles, 2 x 128 = 256;
//   * orientation Y^T = W . x^T on v_mfma_f32_16x16x32_bf16: a preshuffled weight block (16 rows x 32 k)
//     is 1 KB in A-fragment order, so its LDS-DMA and its ds_read_b128 are lane-linear (conflict-free);
//     x rows are the B operand, staged as 64-B rows per slot with the 16-B chunk XOR-swizzled by (row >> 1) & 3
//     on the DMA source and on the read (conflict-free ds_read_b128, cdna_hip_programming.md T2 / rule 21);
//   * both operands by LDS-DMA (buffer_load ... lds) into a ring of 32-deep k slots (4-6 slots, up to 155 KB of
//     the 160 KB LDS): D = slots - 1 steps are in flight, one counted vmcnt per step (every wave issues the
//     same number of DMAs per slot -- a surplus instruction fills a dummy region), one barrier per step, the
//     refill of the slot freed by that barrier issued before the step's MFMAs (cdna_hip_programming.md
//     "Pipelining across barriers": raw s_barrier, never vmcnt(0) in the loop); x rows past M read as zeros;
//   * XCD-aware tile order (cdna_hip_programming.md T1, the bijective form): consecutive tiles -- the
//     m-tiles of one weight column block -- run on one XCD, so each weight block is fetched from HBM once
//     per XCD and the x slices stay L2-resident;
//   * epilogues from the accumulators (decode_epi.h's 16x16 tile layout: lane (r16, h) holds features
//     n0 + 4h .. + 3 of token row m): fp32 / bf16 out, QKV (RoPE + paged K/V write), SWIGLU (interleaved
//     gate/up tiles), RESID (residual add + next-norm prep with ONE sum-of-squares partial per row and
//     block column, so the consumer's row-scale prologue reads N / BN partials instead of N / 16);
//   * optional split-K over grid.y: fp32 slabs (write-through stores) + a per-tile arrival counter; the
//     last of the S blocks of a tile sums the slabs in a fixed order and runs the epilogue (the in-launch
//     reduction of mgemm.hip).
#include "common.h"
#include "decode_epi.h"
#include "launchers.h"

namespace {

constexpr int PG_THR = 512;
#ifndef PG_ABLATE
#define PG_ABLATE 0
#endif
#ifndef PG_SPLIT_ISSUE  // 1: a wave's weight DMAs go out between its MFMAs (compute phase), 0: right after them
#define PG_SPLIT_ISSUE 1
#endif
#ifndef PG_MAX_SLOTS
#define PG_MAX_SLOTS 4
#endif

typedef __attribute__((address_space(3))) void lds_t;

SYM_DEV __amdgpu_buffer_rsrc_t pg_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}

SYM_DEV void pg_dma(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t*)lds, 16, voff, soff, 0, 0);
}

template <int WM, int WN>
struct PgCfg {
  static constexpr int BM = 64 * WM;        // tokens per block
  static constexpr int BN = 32 * WN;        // output features per block
  static constexpr int XS = BM * 64;        // x bytes of one 32-deep slot ([BM rows][64 B], swizzled)
  static constexpr int SLOT = XS + BN * 64;  // + weight blocks (BN / 16 tiles x one 1 KB k-block)
  static constexpr int NX = BM / 16;        // x DMA instructions per slot (16 rows x 64 B each)
  static constexpr int NW = BN / 16;        // weight DMA instructions per slot
  static constexpr int NXU = (NX + 7) / 8;  // ... per wave (every wave issues the same count: the surplus of the
  static constexpr int NWU = (NW + 7) / 8;  //     last round is a dummy fill, so one vmcnt immediate fits all)
  static constexpr int PW = NXU + NWU;      // DMA instructions per wave per slot
  static constexpr int EXTRA = BM * 4 + 1024 + 16;  // row scales, dummy-fill target, split-K "last" flag
  static constexpr int SLOTS_FIT = (160 * 1024 - EXTRA) / SLOT;
  static constexpr int SLOTS = SLOTS_FIT > PG_MAX_SLOTS ? PG_MAX_SLOTS : SLOTS_FIT;
  static constexpr int KEEP = (SLOTS - 2) * PW;  // this wave's younger DMAs left in flight at a step's wait (A)
  static constexpr int KEEP_B = (SLOTS - 3) * PW + NXU;  // ... at group B's wait (see the main loop)
  static constexpr int RS_OFF = SLOTS * SLOT;
  static constexpr int DUMMY_OFF = RS_OFF + BM * 4;
  static constexpr int LAST_OFF = DUMMY_OFF + 1024;
  static constexpr int LDS = LAST_OFF + 16;
  static_assert(SLOTS >= 3 && KEEP <= 63 && LDS <= 160 * 1024, "pgemm tile config");
};

SYM_DEV void store4bf16(bf16* p, const f32x4& v) {
  bf16x4 o;
  o[0] = (bf16)v[0];
  o[1] = (bf16)v[1];
  o[2] = (bf16)v[2];
  o[3] = (bf16)v[3];
  *reinterpret_cast<bf16x4*>(p) = o;
}

// Block tile of M-rows [m0, m0 + BM) x features [n0, n0 + BN); K slice [k0, k0 + kslice).
// GRP: grouped experts (launch_pgemm_grouped): m-tile slot -> (expert, tile of its segment) from the device offsets.
template <int WM, int WN, int EPI, bool GRP>
__global__ __launch_bounds__(PG_THR, 1) void pgemm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ W,
                                                           int M, int N, int K, int kslice, int mtiles, DecodeEpi e,
                                                           float* __restrict__ slab, int* __restrict__ counters,
                                                           PgGroup g) {
  using C = PgCfg<WM, WN>;
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
  // (no AGPR clobber: with none used the whole 256-register budget of 2 waves / SIMD goes to VGPRs)

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably wave-uniform (scalar branches)
  const int wm = wid & 3, wn = wid >> 2;

  // ---- XCD-aware tile order: blocks b, b + 8, ... share an XCD; each XCD gets a contiguous run of tiles
  const int nwg = gridDim.x, b = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  int mt = t % mtiles;
  const int nt = t / mtiles;
  const int n0 = nt * C::BN;
  // block rows [m0, Mend) (Mend: the end of the block's segment -- M, or its expert's last row); rows past Mend
  // are zero-filled by the x buffer range and never stored
  int m0, Mend;
  const bf16* wb = W;
  if constexpr (GRP) {
    int ex = 0, s0 = 0, s1 = 0;
    for (; ex < g.E; ++ex) {  // <= 64 scalar loads (segment bounds in device memory: graph-capturable)
      s0 = g.offsets[g.e_lo + ex];
      s1 = g.offsets[g.e_lo + ex + 1];
      const int nmt = (s1 - s0 + C::BM - 1) / C::BM;
      if (mt < nmt) break;
      mt -= nmt;
    }
    if (ex == g.E) return;  // a surplus slot of the grid (the whole block, before any barrier)
    m0 = s0 + mt * C::BM;
    Mend = s1;
    wb = W + ex * g.wstride;
  } else {
    m0 = mt * C::BM;
    Mend = M;
  }
  const int split = blockIdx.y;
  const int k0 = split * kslice;

  // ---- DMA sources (one 32-deep k slot per issue).  x: instruction g covers block rows 16g .. 16g + 15;
  // lane -> (row lane >> 2, LDS chunk slot lane & 3), loading source chunk slot ^ ((row >> 1) & 3) (the read
  // side's XOR: conflict-free ds_read_b128 over 64-B rows).  Rows >= M read as zeros.  Weights: instruction j
  // is tile n0 / 16 + j's 1 KB block of the slot, lane-linear.  Every wave issues NXU + NWU instructions per
  // slot (one vmcnt immediate fits all): a surplus instruction of a last round re-reads a valid 1 KB into the
  // dummy region.  (One pooled x + weight list with a per-instruction kind branch measured 10-20 % slower.)
  const __amdgpu_buffer_rsrc_t rx = pg_rsrc(x + (long long)m0 * K, (long long)(Mend - m0) * K * 2);
  const __amdgpu_buffer_rsrc_t rw = pg_rsrc(wb, (long long)N * K * 2);
  int vx[C::NXU], vw[C::NWU], dx[C::NXU], dw[C::NWU];
#pragma unroll
  for (int u = 0; u < C::NXU; ++u) {
    const int g = u * 8 + wid;
    const int row = 16 * g + (lane >> 2);
    const bool real = g < C::NX;
    vx[u] = real ? row * K * 2 + 2 * k0 + 16 * ((lane & 3) ^ ((row >> 1) & 3)) : 0;
    dx[u] = real ? g * 1024 : -1;
  }
#pragma unroll
  for (int u = 0; u < C::NWU; ++u) {
    const int j = u * 8 + wid;
    const bool real = j < C::NW;
    // SWIGLU_SPLIT: local tiles alternate gate (even) and up (odd) rows of the same 16 features (W = [gate; up])
    const int jt = real ? j : 0;
    const int tile = EPI == DECODE_EPI_SWIGLU_SPLIT ? (jt & 1 ? N / 32 : 0) + nt * (C::NW / 2) + jt / 2 : n0 / 16 + jt;
    vw[u] = (tile * (K / 32) + k0 / 32) * 1024 + lane * 16;
    dw[u] = real ? C::XS + j * 1024 : -1;
  }

  auto issue_x = [&](int c, int slot) {
    char* const sb = smem + slot * C::SLOT;
#pragma unroll
    for (int u = 0; u < C::NXU; ++u) {
      if ((C::NX % 8) == 0 || u + 1 < C::NXU || dx[u] >= 0) pg_dma(rx, vx[u], c * 64, sb + dx[u]);
      else pg_dma(rw, vw[0], 0, smem + C::DUMMY_OFF);
    }
  };
  auto issue_w = [&](int c, int slot) {
    char* const sb = smem + slot * C::SLOT;
#pragma unroll
    for (int u = 0; u < C::NWU; ++u) {
      if ((C::NW % 8) == 0 || u + 1 < C::NWU || dw[u] >= 0) pg_dma(rw, vw[u], c * 1024, sb + dw[u]);
      else pg_dma(rw, vw[u], 0, smem + C::DUMMY_OFF);
    }
  };
  auto issue = [&](int c, int slot) {
    issue_x(c, slot);
    issue_w(c, slot);
  };

  // ---- fragment addresses: x lane reads token row (lane & 15) of its 16-row tile, k 8 (lane >> 4) .. + 8 of the
  // slot (swizzled chunk); weight reads lane-linear
  const int fr = lane & 15;
  const int xo = (wm * WM * 16 + fr) * 64 + 16 * ((lane >> 4) ^ ((fr >> 1) & 3));
  const int wo = C::XS + wn * WN * 1024 + lane * 16;

  f32x4 acc[WN][WM];
#pragma unroll
  for (int j = 0; j < WN; ++j)
#pragma unroll
    for (int i = 0; i < WM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 wf[WN], xf[WM];
  auto read_frags = [&](int slot) {
    const char* const sb = smem + slot * C::SLOT;
#pragma unroll
    for (int j = 0; j < WN; ++j) wf[j] = *(const bf16x8*)(sb + wo + j * 1024);
#pragma unroll
    for (int i = 0; i < WM; ++i) xf[i] = *(const bf16x8*)(sb + xo + i * 1024);
  };
  // the compute phase: the MFMAs of the fragments in registers, with this wave's weight DMAs of step ci (into
  // slot si) issued after the first two rows (DMA issue spread over both phases of every wave)
  auto mfmas = [&](int ci, int si) {
#if PG_ABLATE == 1  // probe builds only (bench/kernels/pgemm_probe.py): no MFMAs, fragments kept live
#pragma unroll
    for (int j = 0; j < WN; ++j) asm volatile("" ::"v"(wf[j]));
#pragma unroll
    for (int i = 0; i < WM; ++i) asm volatile("" ::"v"(xf[i]));
    if (ci >= 0) issue_w(ci, si);
#else
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < WN; ++j) {
#pragma unroll
      for (int i = 0; i < WM; ++i) acc[j][i] = mfma16(wf[j], xf[i], acc[j][i]);
      if (PG_SPLIT_ISSUE && (j == 1 || (WN == 1 && j == 0))) {
        __builtin_amdgcn_sched_barrier(0);
        if (ci >= 0) issue_w(ci, si);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (!PG_SPLIT_ISSUE && ci >= 0) issue_w(ci, si);
#endif
  };

  float* const rs = reinterpret_cast<float*>(smem + C::RS_OFF);
  const bool has_rs = e.ss_in != nullptr;

  const int nch = kslice / 32;
#pragma unroll
  for (int c = 0; c < C::SLOTS - 1; ++c)
    if (c < nch) issue(c, c);


  // Ping-pong over two wave groups (one wave of each per SIMD): group A (waves 0-3) reads step c's fragments in
  // phase 2c and runs its MFMAs in phase 2c + 1; group B (waves 4-7) reads in 2c + 1 and computes in 2c + 2 -- in
  // every phase one wave of each SIMD feeds the matrix pipe while its partner reads LDS and issues DMAs
  // (MI355X_MICROARCH.md "Two waves per SIMD").  Step c lives in slot c % SLOTS; a wave's read phase of step c
  // also issues its share of step c + SLOTS - 1 into the slot of step c - 1 (read by both groups before).  Before
  // the barrier that opens phase 2c every wave has waited for its own DMAs of step c (vmcnt, the SLOTS - 2
  // younger steps stay in flight), so the barrier publishes the whole slot.
  // A wave issues step c + SLOTS - 1 in two parts: its x DMAs in its read phase of step c, its weight DMAs in its
  // compute phase of step c.  Waits: A (top of step c) has issued every DMA of steps <= c + SLOTS - 2, so it keeps
  // (SLOTS - 2) PW younger ones; B waits for step c + 1 inside its read phase of step c, after the x part of step
  // c + SLOTS - 1: (SLOTS - 3) PW + NXU younger ones.  At the tail both wait for everything.
  const int grp = wid >> 2;
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto read_phase = [&](int c, int slot) {
#if PG_ABLATE != 2  // probe builds: 2 = no DMAs after the prologue (MFMAs on stale slots)
    if (c + C::SLOTS - 1 < nch) issue_x(c + C::SLOTS - 1, slot == 0 ? C::SLOTS - 1 : slot - 1);
#endif
    read_frags(slot);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto wnext = [&](int c, int slot) {  // (step, slot) of the weight DMAs of this compute phase, or (-1, 0)
#if PG_ABLATE == 2
    return -1;
#endif
    return c + C::SLOTS - 1 < nch ? c + C::SLOTS - 1 : -1;
  };
  int slot = 0;
  if (grp == 0) {
    for (int c = 0; c < nch; ++c) {
      if (c + C::SLOTS - 2 < nch) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::KEEP) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      read_phase(c, slot);
      bar();
      mfmas(wnext(c, slot), slot == 0 ? C::SLOTS - 1 : slot - 1);
      slot = slot == C::SLOTS - 1 ? 0 : slot + 1;
    }
    bar();  // B's last compute phase
  } else {
    if (C::SLOTS - 2 < nch) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::KEEP) : "memory");  // prologue: step 0
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();  // phase 0: A reads step 0
    for (int c = 0; c < nch; ++c) {
      bar();
      read_phase(c, slot);
      if (c + C::SLOTS - 1 < nch) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::KEEP_B) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      mfmas(wnext(c, slot), slot == 0 ? C::SLOTS - 1 : slot - 1);
      slot = slot == C::SLOTS - 1 ? 0 : slot + 1;
    }
  }

  // ---- deferred-RMSNorm row scales of the block's rows (after the main loop: the fragment registers are free
  // then; computed in the prologue they pushed the big tiles' register count into scratch): TPR threads per row
  // sum the producer's partials with independent 16-B loads
  if (has_rs) {
    constexpr int TPR = (PG_THR / C::BM) >= 8 ? 8 : (PG_THR / C::BM) >= 4 ? 4 : (PG_THR / C::BM) >= 2 ? 2 : 1;
    float rpart = 0.f;
    for (int rrow = threadIdx.x / TPR; rrow < C::BM; rrow += PG_THR / TPR) {
      const int rsub = threadIdx.x % TPR;
      rpart = 0.f;
      if (m0 + rrow < Mend) {
        const float* sp = e.ss_in + (long long)(m0 + rrow) * e.ss_tiles;
        if ((e.ss_tiles & 3) == 0) {
          const float4* s4 = reinterpret_cast<const float4*>(sp);
          float4 a[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int i = rsub + u * TPR;
            a[u] = i < e.ss_tiles / 4 ? s4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) rpart += (a[u].x + a[u].y) + (a[u].z + a[u].w);
          for (int i = rsub + 4 * TPR; i < e.ss_tiles / 4; i += TPR) {
            const float4 b4 = s4[i];
            rpart += (b4.x + b4.y) + (b4.z + b4.w);
          }
        } else {
          for (int i = rsub; i < e.ss_tiles; i += TPR) rpart += sp[i];
        }
      }
#pragma unroll
      for (int o = 1; o < TPR; o *= 2) rpart += __shfl_xor(rpart, o, 64);
      if (rsub == 0) rs[rrow] = rsqrtf(rpart * e.inv_d + e.eps);
    }
    __syncthreads();
  }

  // ---- epilogue
  const int h = lane >> 4;
  const int S = gridDim.y;
  // split-K without counters (F32 only): every split stores its own fp32 slab [S][M][N] through the plain F32
  // epilogue below; the consumer kernel sums the slabs (LinOut).  (A separate early-return store loop here pushed
  // the big tiles' register allocation into scratch.)
  if constexpr (EPI == DECODE_EPI_F32) {
    if (S > 1 && counters == nullptr) e.y = slab + (long long)split * M * N;
  }
  if (S > 1 && counters != nullptr) {
    // split-K: write-through slab stores, then the last arriving split of this tile reduces
    float* ys = slab + (long long)split * M * N;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = n0 + (wn * WN + j) * 16 + 4 * h;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int m = m0 + (wm * WM + i) * 16 + fr;
        if (m >= Mend) continue;
        const float4 f4 = make_float4(acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]);
        unsigned long long* qd = reinterpret_cast<unsigned long long*>(ys + (long long)m * N + n);
        const unsigned long long* w64 = reinterpret_cast<const unsigned long long*>(&f4);
        __hip_atomic_store(qd, w64[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(qd + 1, w64[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem + C::LAST_OFF);
    if (threadIdx.x == 0) {
      const int got = __hip_atomic_fetch_add(counters + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = got == S - 1;
      if (is_last) __hip_atomic_store(counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last = is_last;
    }
    __syncthreads();
    if (!*last) return;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = n0 + (wn * WN + j) * 16 + 4 * h;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int m = m0 + (wm * WM + i) * 16 + fr;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (m < Mend)
          for (int sp = 0; sp < S; ++sp) {  // fixed split order: bitwise reproducible
            const unsigned long long* qs =
                reinterpret_cast<const unsigned long long*>(slab + ((long long)sp * M + m) * N + n);
            unsigned long long rr[2];
            rr[0] = __hip_atomic_load(qs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            rr[1] = __hip_atomic_load(qs + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float* p = reinterpret_cast<const float*>(rr);
            v += f32x4{p[0], p[1], p[2], p[3]};
          }
        acc[j][i] = v;
      }
    }
  }

  if constexpr (EPI == DECODE_EPI_RESID) {
    // residual add + next-norm prep through an fp32 LDS image of the accumulators (NP passes of whole m-waves when
    // the image is bigger than the ring): then TW threads per row walk the row's BN columns in 16-B steps --
    // coalesced resid read-modify-write, 8-B xw stores back to back, and ONE sum-of-squares partial per (row, block
    // column) reduced across the row's lanes (ss_out [M][N / BN])
    constexpr int RBF = C::BN * 4 + 16;
    constexpr int NP = C::BM * RBF <= C::RS_OFF ? 1 : (C::BM / 2) * RBF <= C::RS_OFF ? 2 : 4;
    constexpr int PR = C::BM / NP;
    static_assert(PR * RBF <= C::RS_OFF, "pgemm: resid image exceeds the ring");
    constexpr int TW = C::BN / 4 <= 32 ? 32 : 64;  // threads per row (lanes past BN / 4 idle)
    constexpr int RPI = PG_THR / TW;               // rows per iteration
    char* const img = smem;
    const int P = N / C::BN;
    const int tc = threadIdx.x % TW, tr = threadIdx.x / TW;
    Pack8 wp;
    if (4 * tc < C::BN) {
      const uint2 raw = *reinterpret_cast<const uint2*>(e.w_next + n0 + 4 * tc);
      wp.u = make_uint4(raw.x, raw.y, 0, 0);
    }
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
      __syncthreads();  // every wave is past its last fragment read / the previous pass's rows
      if (NP == 1 || (wm / (4 / NP)) == pass) {
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
          for (int i = 0; i < WM; ++i) {
            const int r = (wm * WM + i) * 16 + fr - pass * PR;
            *reinterpret_cast<f32x4*>(img + r * RBF + (16 * (wn * WN + j) + 4 * h) * 4) = acc[j][i];
          }
      }
      __syncthreads();
      for (int r = tr; r < PR; r += RPI) {
        const int m = m0 + pass * PR + r;
        float sq = 0.f;
        if (m < Mend && 4 * tc < C::BN) {
          const f32x4 y = *reinterpret_cast<const f32x4*>(img + r * RBF + tc * 16);
          float* rp = e.resid + (long long)m * N + n0 + 4 * tc;
          const float4 q = *reinterpret_cast<const float4*>(rp);
          const float rr[4] = {q.x + y[0], q.y + y[1], q.z + y[2], q.w + y[3]};
          *reinterpret_cast<float4*>(rp) = make_float4(rr[0], rr[1], rr[2], rr[3]);
          store4bf(e.xw_out + (long long)m * N + n0 + 4 * tc, rr[0] * (float)wp.h[0], rr[1] * (float)wp.h[1],
                   rr[2] * (float)wp.h[2], rr[3] * (float)wp.h[3]);
          sq = rr[0] * rr[0] + rr[1] * rr[1] + rr[2] * rr[2] + rr[3] * rr[3];
        }
#pragma unroll
        for (int o = 1; o < TW; o *= 2) sq += __shfl_xor(sq, o, 64);
        if (m < Mend && tc == 0) e.ss_out[(long long)m * P + nt] = sq;
      }
    }
  } else if constexpr (EPI == DECODE_EPI_QKV && C::BN % 128 == 0) {
    // QKV: the row scale and RoPE in registers (a rotate-half pair sits in lanes l and l ^ 32 of one accumulator,
    // models/layout.py), the roped heads as a bf16 LDS image [rows][BN] in natural dim order, then whole 256-B head
    // rows out: q rows and paged K rows with 16-B stores; V (dim-major cache blocks) as 16-B runs of 8 tokens where
    // the 8 rows' slots are consecutive and aligned in one cache block (a prefill sequence's tokens), else per token
    constexpr int D = 128;
    constexpr int RB = C::BN * 2 + 16;
    constexpr int NP = C::BM * RB <= C::RS_OFF ? 1 : 2;
    constexpr int PR = C::BM / NP;
    static_assert(PR * RB <= C::RS_OFF, "pgemm: qkv image exceeds the ring");
    constexpr int HB = C::BN / D;  // heads per block
    char* const img = smem;
    const int head0 = n0 / D;
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
      __syncthreads();
      if (NP == 1 || (wm >> 1) == pass) {
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          const int tl = wn * WN + j;
          const int hl = tl / 8, jj = tl % 8;  // head within the block, 16-row tile within the head
#pragma unroll
          for (int i = 0; i < WM; ++i) {
            const int mloc = (wm * WM + i) * 16 + fr;
            const int m = m0 + mloc;
            f32x4 v = acc[j][i];
            if (has_rs) v *= rs[mloc];
            float pr[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) pr[q] = __shfl_xor(v[q], 32, 64);
            f32x4 o = v;
            int d;
            if (head0 + hl < e.Hq + e.Hkv) {  // q / k head: RoPE
              const bool lo = h < 2;
              const int dh = 8 * jj + 4 * (h & 1);
              const float* cs = e.cos_sin + (long long)(m < Mend ? e.positions[m] : 0) * D;
              const float4 c4 = *reinterpret_cast<const float4*>(cs + dh);
              const float4 s4 = *reinterpret_cast<const float4*>(cs + 64 + dh);
              const float cc[4] = {c4.x, c4.y, c4.z, c4.w}, ss4[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
              for (int q = 0; q < 4; ++q) o[q] = lo ? (v[q] * cc[q] - pr[q] * ss4[q]) : (v[q] * cc[q] + pr[q] * ss4[q]);
              d = (lo ? 0 : 64) + dh;
            } else {
              d = 16 * jj + 4 * h;
            }
            store4bf16(reinterpret_cast<bf16*>(img + (mloc - pass * PR) * RB + (hl * D + d) * 2), o);
          }
        }
      }
      __syncthreads();
      // q / k rows: (row, head, 16-B chunk) per thread
      for (int q = threadIdx.x; q < PR * HB * 16; q += PG_THR) {
        const int r = q / (HB * 16), hl = (q / 16) % HB, ch = q % 16;
        const int m = m0 + pass * PR + r, head = head0 + hl;
        if (m >= Mend || head >= e.Hq + e.Hkv) continue;
        bf16* dst;
        if (head < e.Hq) {
          dst = e.q_out + ((long long)m * e.Hq + head) * D;
        } else {
          const int slot = e.slots[m];
          if (slot < 0) continue;
          dst = e.k_cache + (((long long)(slot / e.BS) * e.Hkv + (head - e.Hq)) * e.BS + slot % e.BS) * D;
        }
        *reinterpret_cast<uint4*>(dst + ch * 8) = *reinterpret_cast<const uint4*>(img + r * RB + hl * D * 2 + ch * 16);
      }
      // V heads: (8-row group, head, dim) per thread
      if (head0 + HB > e.Hq + e.Hkv) {
        for (int q = threadIdx.x; q < (PR / 8) * HB * D; q += PG_THR) {
          const int g8 = q / (HB * D), hl = (q / D) % HB, dd = q % D;
          const int head = head0 + hl;
          if (head < e.Hq + e.Hkv) continue;
          const int vh = head - e.Hq - e.Hkv;
          const int r0 = 8 * g8, mb = m0 + pass * PR + r0;
          bf16 vals[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            vals[k] = *reinterpret_cast<const bf16*>(img + (r0 + k) * RB + (hl * D + dd) * 2);
          const int s0 = mb < Mend ? e.slots[mb] : -1;
          bool run = s0 >= 0 && (s0 % 8) == 0 && (s0 % e.BS) + 8 <= e.BS && mb + 8 <= Mend;
          if (run) {
#pragma unroll
            for (int k = 1; k < 8; ++k) run = run && e.slots[mb + k] == s0 + k;
          }
          if (run) {
            Pack8 pk;
#pragma unroll
            for (int k = 0; k < 8; ++k) pk.h[k] = vals[k];
            *reinterpret_cast<uint4*>(e.v_cache + (((long long)(s0 / e.BS) * e.Hkv + vh) * D + dd) * e.BS + s0 % e.BS) =
                pk.u;
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const int m = mb + k;
              const int sl = m < Mend ? e.slots[m] : -1;
              if (sl >= 0) e.v_cache[(((long long)(sl / e.BS) * e.Hkv + vh) * D + dd) * e.BS + sl % e.BS] = vals[k];
            }
          }
        }
      }
    }
  } else if constexpr (EPI == DECODE_EPI_BF16 || EPI == DECODE_EPI_SWIGLU || EPI == DECODE_EPI_SWIGLU_SPLIT) {
    // bf16 outputs through an LDS image of the block's output tile [BM][OW] (OW = BN, or BN / 2 after SwiGLU),
    // then coalesced 16-B row stores: an accumulator tile alone would store 8 B per lane into 16 rows
    constexpr bool SW = EPI == DECODE_EPI_SWIGLU || EPI == DECODE_EPI_SWIGLU_SPLIT;
    static_assert(EPI != DECODE_EPI_SWIGLU_SPLIT || WN % 2 == 0, "pgemm: split SwiGLU pairs a wave's tiles");
    constexpr int OW = SW ? C::BN / 2 : C::BN;
    constexpr int RB = OW * 2 + 16;  // row bytes in LDS (+16: rows of a lane group land on distinct banks)
    constexpr int NP = C::BM * RB <= C::RS_OFF ? 1 : 2;  // passes (half the m-waves each when the image is big)
    constexpr int PR = C::BM / NP;                       // rows per pass
    static_assert(PR * RB <= C::RS_OFF, "pgemm: output image exceeds the ring");
    char* const img = smem;
    bf16* const out = SW ? e.act : e.out_bf;
    const int ldo = SW ? N / 2 : N;
    const int c0 = SW ? n0 / 2 : n0;
    constexpr int CPR = OW * 2 / 16;  // 16-B chunks per row
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
      __syncthreads();  // every wave is past its last fragment read / the previous pass's copy-out
      if (NP == 1 || (wm >> 1) == pass) {
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          const int tl = wn * WN + j;  // tile within the block
#pragma unroll
          for (int i = 0; i < WM; ++i) {
            const int mloc = (wm * WM + i) * 16 + fr;
            const int r = mloc - pass * PR;
            f32x4 v = acc[j][i];
            if (has_rs) v *= rs[mloc];
            if constexpr (EPI == DECODE_EPI_SWIGLU_SPLIT) {
              if (j % 2 == 0) {  // (gate, up) = tiles (j, j + 1) of this wave, features 16 (tl / 2) + 4h ..
                f32x4 u = acc[j + 1][i];
                if (has_rs) u *= rs[mloc];
                f32x4 a;
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = silu(v[q]) * u[q];
                store4bf16(reinterpret_cast<bf16*>(img + r * RB + (16 * (tl / 2) + 4 * h) * 2), a);
              }
            } else if constexpr (EPI == DECODE_EPI_SWIGLU) {
              f32x4 u;
#pragma unroll
              for (int q = 0; q < 4; ++q) u[q] = __shfl_xor(v[q], 32, 64);
              if (h < 2) {
                f32x4 a;
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = silu(v[q]) * u[q];
                store4bf16(reinterpret_cast<bf16*>(img + r * RB + (8 * tl + 4 * h) * 2), a);
              }
            } else {
              store4bf16(reinterpret_cast<bf16*>(img + r * RB + (16 * tl + 4 * h) * 2), v);
            }
          }
        }
      }
      __syncthreads();
      for (int q = threadIdx.x; q < PR * CPR; q += PG_THR) {
        const int r = q / CPR, ch = q % CPR;
        const int m = m0 + pass * PR + r;
        if (m < Mend)
          *reinterpret_cast<uint4*>(out + (long long)m * ldo + c0 + ch * 8) =
              *reinterpret_cast<const uint4*>(img + r * RB + ch * 16);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int tile = n0 / 16 + wn * WN + j;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int mloc = (wm * WM + i) * 16 + fr;
        const int m = m0 + mloc;
        const bool mok = m < Mend;
        f32x4 v = acc[j][i];
        if (has_rs) {
          const float sc = rs[mloc];
          v *= sc;
        }
        epilogue<EPI>(e, v, tile, m, mok, h, N);
      }
    }
  }
}

template <int WM, int WN, int EPI>
void launch_cfg(const bf16* x, const bf16* W, int M, int N, int K, int S, const DecodeEpi& e, float* slab,
                int* counters, hipStream_t s) {
  using C = PgCfg<WM, WN>;
  const int mtiles = (M + C::BM - 1) / C::BM;
  const int ntiles = N / C::BN;
  pgemm_kernel<WM, WN, EPI, false><<<dim3(mtiles * ntiles, S), dim3(PG_THR), 0, s>>>(x, W, M, N, K, K / S, mtiles, e,
                                                                                     slab, counters, PgGroup{});
}

template <int WM, int WN, int EPI>
void launch_cfg_grouped(const bf16* x, const bf16* W, int R, int N, int K, int S, const PgGroup& g,
                        const DecodeEpi& e, float* slab, hipStream_t s) {
  using C = PgCfg<WM, WN>;
  const int mslots = (R + C::BM - 1) / C::BM + g.E;  // >= sum over experts of ceil(rows / BM)
  const int ntiles = N / C::BN;
  pgemm_kernel<WM, WN, EPI, true><<<dim3(mslots * ntiles, S), dim3(PG_THR), 0, s>>>(x, W, R, N, K, K / S, mslots, e,
                                                                                    slab, nullptr, g);
}

// the instantiated tile shapes (index = PG_CFG id, kept in sync with pgemm_cfg_shape below)
#define PG_CFGS(X) \
  X(0, 6, 7)       \
  X(1, 4, 8)       \
  X(2, 3, 6)       \
  X(3, 3, 4)       \
  X(4, 4, 4)       \
  X(5, 2, 4)       \
  X(6, 5, 7)       \
  X(7, 4, 7)       \
  X(8, 3, 7)       \
  X(9, 3, 8)       \
  X(10, 2, 8)

template <int EPI>
void launch_epi(int cfg, const bf16* x, const bf16* W, int M, int N, int K, int S, const DecodeEpi& e, float* slab,
                int* counters, hipStream_t s) {
  switch (cfg) {
#define PG_CASE(id, wm, wn) \
  case id: launch_cfg<wm, wn, EPI>(x, W, M, N, K, S, e, slab, counters, s); break;
    PG_CFGS(PG_CASE)
#undef PG_CASE
    default: break;
  }
}

// grouped experts: the shapes the MoE layers use (WN even for the split SwiGLU)
#define PG_GRP_CFGS(X) \
  X(1, 4, 8)           \
  X(4, 4, 4)           \
  X(5, 2, 4)           \
  X(9, 3, 8)           \
  X(10, 2, 8)

template <int EPI>
bool launch_grp_epi(int cfg, const bf16* x, const bf16* W, int R, int N, int K, int S, const PgGroup& g,
                    const DecodeEpi& e, float* slab, hipStream_t s) {
  switch (cfg) {
#define PG_GCASE(id, wm, wn) \
  case id: launch_cfg_grouped<wm, wn, EPI>(x, W, R, N, K, S, g, e, slab, s); return true;
    PG_GRP_CFGS(PG_GCASE)
#undef PG_GCASE
    default: return false;
  }
}

}  // namespace

int pgemm_cfg_shape(int cfg, int* bm, int* bn) {
  switch (cfg) {
#define PG_SHAPE(id, wm, wn) \
  case id: *bm = 64 * wm; *bn = 32 * wn; return 1;
    PG_CFGS(PG_SHAPE)
#undef PG_SHAPE
    default: return 0;
  }
}

void launch_pgemm(int epi, int cfg, const bf16* x, const bf16* Wshuf, int M, int N, int K, int S, const DecodeEpi& e,
                  float* slab, int* counters, hipStream_t s) {
  switch (epi) {
    case DECODE_EPI_QKV: launch_epi<DECODE_EPI_QKV>(cfg, x, Wshuf, M, N, K, S, e, slab, counters, s); break;
    case DECODE_EPI_RESID: launch_epi<DECODE_EPI_RESID>(cfg, x, Wshuf, M, N, K, S, e, slab, counters, s); break;
    case DECODE_EPI_SWIGLU: launch_epi<DECODE_EPI_SWIGLU>(cfg, x, Wshuf, M, N, K, S, e, slab, counters, s); break;
    case DECODE_EPI_BF16: launch_epi<DECODE_EPI_BF16>(cfg, x, Wshuf, M, N, K, S, e, slab, counters, s); break;
    default: launch_epi<DECODE_EPI_F32>(cfg, x, Wshuf, M, N, K, S, e, slab, counters, s); break;
  }
}

void launch_pgemm_grouped(int epi, int cfg, const bf16* x, const bf16* Wshuf, int R, int N, int K, int S,
                          const PgGroup& g, const DecodeEpi& e, float* slab, hipStream_t s) {
  switch (epi) {
    case DECODE_EPI_SWIGLU_SPLIT: launch_grp_epi<DECODE_EPI_SWIGLU_SPLIT>(cfg, x, Wshuf, R, N, K, 1, g, e, slab, s); break;
    case DECODE_EPI_BF16: launch_grp_epi<DECODE_EPI_BF16>(cfg, x, Wshuf, R, N, K, 1, g, e, slab, s); break;
    default: launch_grp_epi<DECODE_EPI_F32>(cfg, x, Wshuf, R, N, K, S, g, e, slab, s); break;
  }
}

#ifdef PG_PROBE
// standalone probe entry (bench/kernels/pgemm_probe.py builds this file with -DPG_PROBE and PG_ABLATE / PG_MAX_SLOTS
// variants into its own .so): bf16 y [M][N] = x @ W^T
// S > 1: y is the fp32 slab array [S][M][N] (no in-launch reduction)
extern "C" int pg_probe(int cfg, const void* x, const void* w, void* y, int M, int N, int K, int S, void* stream) {
  int bm = 0, bn = 0;
  if (!pgemm_cfg_shape(cfg, &bm, &bn) || N % bn || K % (64 * S)) return -1;
  DecodeEpi e;
  e.wshuf = 1;
  e.out_bf = reinterpret_cast<bf16*>(y);
  launch_pgemm(S > 1 ? DECODE_EPI_F32 : DECODE_EPI_BF16, cfg, reinterpret_cast<const bf16*>(x),
               reinterpret_cast<const bf16*>(w), M, N, K, S, e, reinterpret_cast<float*>(y), nullptr,
               reinterpret_cast<hipStream_t>(stream));
  return 0;
}

// grouped probe: experts [0, E) of W [E][N][K] over the rows of offsets[0..E] (device int32), bf16 y [R][N]
extern "C" int pg_probe_grouped(int cfg, const void* x, const void* w, const void* offsets, int E, void* y, int R, int N,
                                int K, void* stream) {
  int bm = 0, bn = 0;
  if (!pgemm_cfg_shape(cfg, &bm, &bn) || N % bn || K % 64) return -1;
  DecodeEpi e;
  e.wshuf = 1;
  e.out_bf = reinterpret_cast<bf16*>(y);
  PgGroup g;
  g.offsets = reinterpret_cast<const int*>(offsets);
  g.E = E;
  g.wstride = (long long)N * K;
  launch_pgemm_grouped(DECODE_EPI_BF16, cfg, reinterpret_cast<const bf16*>(x), reinterpret_cast<const bf16*>(w), R, N,
                       K, 1, g, e, nullptr, reinterpret_cast<hipStream_t>(stream));
  return 0;
}
#endif
