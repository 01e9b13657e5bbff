// Prefill GEMM on gfx950 MFMA: Y[M, N] = X[M, K] . W[N, K]^T, bf16 in, fp32 accumulate.
//
// Built for the prefill projections of the engine (M = prompt tokens of a step, 64 .. 8192+; N, K the
// model's projection shapes, both operands K-contiguous), replacing the library GEMM of the general
// forward path.  Structure (cdna_hip_programming.md §5, "Pipelining across barriers"):
//
//   * 256 x 256 output tile per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 per wave,
//     4 x 2 accumulators of v_mfma_f32_32x32x16_bf16), one workgroup per CU.
//   * K is consumed in 32-deep sub-tiles through a 5-slot LDS ring (5 x 32 KB = the whole LDS).  Every
//     sub-tile is staged by LDS-DMA (global_load_lds_dwordx4, 4 per wave) four sub-tiles ahead; the
//     wait before each barrier is a COUNTED vmcnt that leaves the two newest sub-tiles' DMA in flight
//     across the barrier (raw s_barrier, never __syncthreads: its fence would drain the DMA).  With
//     fewer slots the loop is bound by the DMA latency (4 slots: ~0.78 us per 32-deep step).
//   * The fragments of the next 16-deep k step are read from LDS into a second register set while the
//     MFMAs of the current one run (24 VGPRs per set), so neither a k step nor the barrier restart
//     waits for LDS.
//   * LDS image: 64-B rows (32 bf16 of K), lane-linear as the DMA writes it; the 16-B chunk index is
//     XOR-swizzled with a bijection of the row's 4-row group (source-side permutation + the same XOR on
//     the read, rule 21), which makes every ds_read_b128 lane group hit 16 distinct bank slots.
//   * Tile order is XCD-aware (bijective remap, T1): the tiles one XCD runs share X row panels and
//     W column panels in that XCD's L2.
//
// Epilogues (PgemmEpi) are fused where the unfused path would run an elementwise kernel over the
// output: see the enum in launchers.h.
#include "common.h"
#include "pgemm.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 32, SLOTS = 5, NTHR = 512;
constexpr int OPB = BM * BK * 2;     // 16 KB: one operand of one ring slot
constexpr int SLOTB = 2 * OPB;       // 32 KB
constexpr int LDSB = SLOTS * SLOTB;  // 160 KB: the whole LDS of the CU

typedef __attribute__((address_space(3))) void lds_t;
typedef const __attribute__((address_space(1))) void gbl_t;

// 16-B chunk XOR of a row, from its row index mod 16: {0, 2, 3, 1} over the four 4-row groups.
SYM_DEV int chunk_swz(int r16) { return (0x1320 >> (4 * ((r16 >> 2) & 3))) & 3; }

// LDS byte address of a __shared__ pointer (for inline-asm ds_read)
SYM_DEV unsigned lds_addr(const char* p) {
  return (unsigned)(unsigned long long)(const __attribute__((address_space(3))) char*)p;
}

// ds_read_b128 with an immediate offset, invisible to the compiler's waitcnt insertion: the k loop
// counts its LDS reads itself (lgkmcnt(6) leaves the next k step's six reads in flight).
template <int OFF>
SYM_DEV void ds_read16(bf16x8& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}

// Buffer resource over [base, base + bytes): raw loads past the end return zeros (rows >= M / N).
SYM_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}

// LDS-DMA of 16 B per lane (buffer_load_dwordx4 ... lds): lane l's bytes land at lds + 16 l.
SYM_DEV void bdma16(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t*)lds, 16, voff, soff, 0, 0);
}

template <int EPI, int DIAG = 0>
__global__ __launch_bounds__(NTHR, 1) void pgemm_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                         PgemmEpi e, int M, int N, int K, int tiles_m) {
  __shared__ __attribute__((aligned(1024))) char smem[LDSB];
  asm volatile("" ::: "a0");  // lets the register allocator keep the accumulators in AGPRs
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;

  // XCD-aware tile order: consecutive logical tiles run on one XCD (bijective for any grid size)
  const int nwg = gridDim.x, b = blockIdx.x;
  const int q = nwg >> 3, rem = nwg & 7, xcd = b & 7;
  const int t = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int m0 = (t % tiles_m) * BM, n0 = (t / tiles_m) * BN;

  // ---- LDS-DMA sources: wave w fills rows (2w + i) * 16 .. + 16 of both operands of a slot; lane ->
  // (row lane >> 2, chunk lane & 3) with the chunk XOR swizzle applied on the source.  Row offsets are
  // per-lane byte offsets into buffer resources (rows past M / N read as zeros), the k offset is scalar.
  const int lr = lane >> 2;
  const int sch = ((lane & 3) ^ chunk_swz(lr)) * 16;
  const __amdgpu_buffer_rsrc_t rX = make_rsrc(X, (long long)M * K * 2);
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, (long long)N * K * 2);
  const int va0 = (m0 + (2 * wid) * 16 + lr) * K * 2 + sch;
  const int va1 = va0 + 16 * K * 2;
  const int vb0 = (n0 + (2 * wid) * 16 + lr) * K * 2 + sch;
  const int vb1 = vb0 + 16 * K * 2;
  char* const dA = smem + (2 * wid) * 1024;
  char* const dB = smem + OPB + (2 * wid) * 1024;

  const int nk = K / BK;
  auto issue = [&](int kt, int so) {
    if constexpr (DIAG == 2) return;  // diagnostic build: no DMA
    const int ko = kt * BK * 2;
    bdma16(rX, va0, ko, dA + so);
    bdma16(rX, va1, ko, dA + so + 1024);
    bdma16(rW, vb0, ko, dB + so);
    bdma16(rW, vb1, ko, dB + so + 1024);
  };

  // ---- fragment reads (32x32x16: lane holds row lane & 31, k 8 * (lane >> 5) .. + 8 of a 16-deep k step;
  // k step s of a 32-deep sub-tile is 16-B chunk 2s + (lane >> 5) of the 64-B LDS row)
  const int fr = lane & 31, fh = lane >> 5;
  const int fo0 = fr * 64 + 16 * ((fh) ^ chunk_swz(fr));
  const int fo1 = fr * 64 + 16 * ((2 + fh) ^ chunk_swz(fr));
  const char* const rA = smem + wr * 128 * 64;
  const char* const rB = smem + OPB + wc * 64 * 64;

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  bf16x8 fa0[4], fb0[2], fa1[4], fb1[2];
  const unsigned lA0 = lds_addr(rA) + fo0, lA1 = lds_addr(rA) + fo1;
  const unsigned lB0 = lds_addr(rB) + fo0, lB1 = lds_addr(rB) + fo1;
  // fragments of one k step of the sub-tile in ring slot offset SO_: 2 B tiles of 32 columns, 4 A tiles of 32 rows (6 reads)
#define PG_READ(A_, B_, SO_, LA_, LB_)                              \
  {                                                                 \
    const unsigned so_ = (SO_);                                     \
    ds_read16<0>(B_[0], LB_ + so_);                                 \
    ds_read16<2048>(B_[1], LB_ + so_);                              \
    ds_read16<0>(A_[0], LA_ + so_);                                 \
    ds_read16<2048>(A_[1], LA_ + so_);                              \
    ds_read16<4096>(A_[2], LA_ + so_);                              \
    ds_read16<6144>(A_[3], LA_ + so_);                              \
  }
  // wait for all but the newest six LDS reads, then 8 MFMAs (sched_barrier keeps them behind the
  // inline wait: cdna_hip_programming.md §5.4 rule 18)
#define PG_MFMA(A_, B_)                                                                               \
  {                                                                                                   \
    asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");                                                \
    __builtin_amdgcn_sched_barrier(0);                                                                \
    __builtin_amdgcn_s_setprio(1);                                                                    \
    if constexpr (DIAG != 1) {                                                                        \
      _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j)     \
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A_[i], B_[j], acc[i][j], 0, 0, 0);        \
    } else {                                                                                          \
      _Pragma("unroll") for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(A_[i]));                    \
      _Pragma("unroll") for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(B_[j]));                    \
    }                                                                                                 \
    __builtin_amdgcn_s_setprio(0);                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                                \
  }

  // prologue: sub-tiles 0..3 in flight; 0 and 1 landed before the first barrier
  issue(0, 0);
  if (nk > 1) issue(1, SLOTB);
  if (nk > 2) issue(2, 2 * SLOTB);
  if (nk > 3) {
    issue(3, 3 * SLOTB);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  PG_READ(fa0, fb0, 0, lA0, lB0);

  // sub-tile kt (ring slot kt % 5): refill the slot of kt - 1 (its fragments were consumed before the
  // previous barrier) with kt + 4; two 16-deep k steps, each reading the next step's fragments into the
  // other register set while its MFMAs run (the second reads sub-tile kt + 1, visible since the previous
  // barrier; past the last sub-tile it reads a stale slot that is never used); then wait for this wave's
  // DMA of kt + 2 and barrier, leaving kt + 3 and kt + 4 in flight across it (three steps of DMA latency
  // hidden per sub-tile)
  int kt = 0, s_cur = 0;
  auto nxt = [](int so) { return so + SLOTB == LDSB ? 0 : so + SLOTB; };
  for (; kt + 4 < nk; ++kt) {
    const int s_nx = nxt(s_cur);
    issue(kt + 4, s_cur == 0 ? LDSB - SLOTB : s_cur - SLOTB);
    PG_READ(fa1, fb1, s_cur, lA1, lB1);
    PG_MFMA(fa0, fb0);
    PG_READ(fa0, fb0, s_nx, lA0, lB0);
    PG_MFMA(fa1, fb1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    s_cur = s_nx;
  }
  for (; kt < nk; ++kt) {
    const int s_nx = nxt(s_cur);
    PG_READ(fa1, fb1, s_cur, lA1, lB1);
    PG_MFMA(fa0, fb0);
    PG_READ(fa0, fb0, s_nx, lA0, lB0);
    PG_MFMA(fa1, fb1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    s_cur = s_nx;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the stale trailing reads
#undef PG_READ
#undef PG_MFMA

  // ---- epilogue straight from the accumulators (32x32 C layout: column lane & 31,
  // row (r & 3) + 8 (r >> 2) + 4 (lane >> 5) for register r)
  const int col0 = n0 + wc * 64 + (lane & 31);
  const int row0 = m0 + wr * 128 + 4 * (lane >> 5);
  if constexpr (EPI == PGEMM_EPI_BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + i * 32 + (r & 3) + 8 * (r >> 2);
        if (row < M) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            if (col0 + j * 32 < N) e.y[(long long)row * e.ldy + col0 + j * 32] = (bf16)acc[i][j][r];
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------------
// Variant 1: 4 waves x (128 x 128) per 256 x 256 tile, one wave per SIMD (256 accumulator AGPRs), 64-deep
// K-tiles double-buffered in LDS with 128-B rows (the DMA moves whole 128-B row pieces: half the L2
// requests of the 64-B rows above).  Chunk swizzle for 128-B rows: chunk ^ ((row >> 1) & 7).
constexpr int V1_THR = 256, V1_BK = 64;
constexpr int V1_OPB = 256 * V1_BK * 2;  // 32 KB
constexpr int V1_BUFB = 2 * V1_OPB;      // 64 KB
constexpr int V1_LDSB = 2 * V1_BUFB;     // 128 KB

template <int EPI>
__global__ __launch_bounds__(V1_THR, 1) void pgemm4_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                            PgemmEpi e, int M, int N, int K, int tiles_m) {
  __shared__ __attribute__((aligned(1024))) char smem[V1_LDSB];
  asm volatile("" ::: "a0");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int q = nwg >> 3, rem = nwg & 7, xcd = b & 7;
  const int t = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int m0 = (t % tiles_m) * BM, n0 = (t / tiles_m) * BN;

  // DMA: wave w fills rows (8w + i) * 8 .. + 8, i = 0..7, of both operands (1 KB per instruction);
  // lane -> (row lane >> 3, chunk lane & 7), source chunk swizzled by the row's (row >> 1) & 7
  const __amdgpu_buffer_rsrc_t rX = make_rsrc(X, (long long)M * K * 2);
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, (long long)N * K * 2);
  const int lrow = lane >> 3;
  // (row >> 1) & 7 for row = 8 g + lrow: (4 (g & 1) + (lrow >> 1)) & 7
  const int sw_e = ((lane & 7) ^ ((lrow >> 1) & 7)) * 16;
  const int sw_o = ((lane & 7) ^ ((4 + (lrow >> 1)) & 7)) * 16;
  int va[8], vb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int g = 8 * wid + i;
    const int sw = (g & 1) ? sw_o : sw_e;
    va[i] = (m0 + 8 * g + lrow) * K * 2 + sw;
    vb[i] = (n0 + 8 * g + lrow) * K * 2 + sw;
  }
  char* const dBase = smem + (8 * wid) * 1024;
  const int nk = K / V1_BK;

  // fragment offsets: lane (r = lane & 31, h = lane >> 5), k step s -> chunk 2 s + h of row r
  const int fr = lane & 31, fh = lane >> 5;
  const unsigned lbase = lds_addr(smem) + fr * 128;
  unsigned fo[4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) fo[s4] = lbase + 16 * ((2 * s4 + fh) ^ ((fr >> 1) & 7));
  const unsigned aoff = wr * 128 * 128, boff = V1_OPB + wc * 128 * 128;

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  bf16x8 fa0[4], fb0[4], fa1[4], fb1[4];
#define V1_READ(A_, B_, BUF_, S_)                                      \
  {                                                                    \
    const unsigned ba_ = fo[S_] + (BUF_) + aoff, bb_ = fo[S_] + (BUF_) + boff; \
    ds_read16<0>(A_[0], ba_);                                          \
    ds_read16<4096>(A_[1], ba_);                                       \
    ds_read16<8192>(A_[2], ba_);                                       \
    ds_read16<12288>(A_[3], ba_);                                      \
    ds_read16<0>(B_[0], bb_);                                          \
    ds_read16<4096>(B_[1], bb_);                                       \
    ds_read16<8192>(B_[2], bb_);                                       \
    ds_read16<12288>(B_[3], bb_);                                      \
  }
#define V1_MFMA(A_, B_, WAIT_)                                                                        \
  {                                                                                                   \
    asm volatile(WAIT_ ::: "memory");                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                                \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 4; ++j)       \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A_[i], B_[j], acc[i][j], 0, 0, 0);          \
    __builtin_amdgcn_sched_barrier(0);                                                                \
  }
  auto dma = [&](int kt, int buf) {
    const int ko = kt * V1_BK * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) bdma16(rX, va[i], ko, dBase + buf + i * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) bdma16(rW, vb[i], ko, dBase + buf + V1_OPB + i * 1024);
  };

  dma(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  V1_READ(fa0, fb0, 0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned buf = (kt & 1) * V1_BUFB, nbuf = V1_BUFB - buf;
    // next K-tile's DMA first: four k steps (64 MFMAs) of latency before its wait
    if (kt + 1 < nk) dma(kt + 1, nbuf);
    __builtin_amdgcn_sched_barrier(0);
    V1_READ(fa1, fb1, buf, 1);
    V1_MFMA(fa0, fb0, "s_waitcnt lgkmcnt(8)");
    V1_READ(fa0, fb0, buf, 2);
    V1_MFMA(fa1, fb1, "s_waitcnt lgkmcnt(8)");
    V1_READ(fa1, fb1, buf, 3);
    V1_MFMA(fa0, fb0, "s_waitcnt lgkmcnt(8)");
    V1_MFMA(fa1, fb1, "s_waitcnt lgkmcnt(0)");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) V1_READ(fa0, fb0, nbuf, 0);
  }
#undef V1_READ
#undef V1_MFMA

  const int col0 = n0 + wc * 128 + (lane & 31);
  const int row0 = m0 + wr * 128 + 4 * (lane >> 5);
  if constexpr (EPI == PGEMM_EPI_BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + i * 32 + (r & 3) + 8 * (r >> 2);
        if (row < M) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (col0 + j * 32 < N) e.y[(long long)row * e.ldy + col0 + j * 32] = (bf16)acc[i][j][r];
        }
      }
  }
}

int g_pgemm_variant = 0;

}  // namespace

void set_pgemm_variant(int v) { g_pgemm_variant = v; }

void launch_pgemm(int epi, const bf16* X, const bf16* W, int M, int N, int K, const PgemmEpi& e, hipStream_t s) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  const dim3 grid(tm * tn), block(NTHR);
  if (g_pgemm_variant == 10) {  // diagnostics: DMA + LDS reads only / MFMA + LDS reads only
    pgemm_kernel<PGEMM_EPI_BF16, 1><<<grid, block, 0, s>>>(X, W, e, M, N, K, tm);
    return;
  }
  if (g_pgemm_variant == 11) {
    pgemm_kernel<PGEMM_EPI_BF16, 2><<<grid, block, 0, s>>>(X, W, e, M, N, K, tm);
    return;
  }
  if (g_pgemm_variant == 1) {
    pgemm4_kernel<PGEMM_EPI_BF16><<<grid, dim3(V1_THR), 0, s>>>(X, W, e, M, N, K, tm);
    return;
  }
  switch (epi) {
    default:
      pgemm_kernel<PGEMM_EPI_BF16><<<grid, block, 0, s>>>(X, W, e, M, N, K, tm);
      break;
  }
}
