// Medium-M projection GEMM (17..256 rows: prefill chunks, wide decode batches): fp32 split-K slabs
//   y[s][m][n] = sum_{k in slice s} x[m][k] * W[n][k],   x [M][K], W [N][K] bf16, M <= 256.
//
// Why a separate kernel: at these M a projection is still weight-streaming (Llama-3-8B: 128 tokens x
// 436 MB of weights per layer), but the library GEMM picks tiles that leave most CUs idle or stream the
// weights at 1.3-2.7 TB/s (profiles/prefill_gemm_hipblaslt_r1.jsonl), and the decode kernels re-read
// x once per 16-row weight tile (built for M <= 64).  Here every CU streams its own weight rows once,
// while the activation slice it needs is shared by its 4 waves through LDS:
//
//   * orientation Y^T = W . x^T on v_mfma_f32_16x16x32_bf16: the weight tile is the A operand and comes
//     from the MFMA-preshuffled weight copy (models/layout.py::preshuffle, the decode layout), so every
//     weight DMA instruction reads 1 KB contiguous; x fragments are the B operand;
//   * workgroup = 4 waves x RW 16-row weight tiles (64 RW output features) x all M tokens x one k slice;
//     the k split S is chosen on the host so the grid fills the 256 CUs; partial sums go to fp32 slabs
//     that the consumer (rope_cache / add_rms_norm / swiglu, LinOut) sums in its prologue, as the skinny
//     decode GEMM's do;
//   * x AND the weight blocks stream through an LDS ring of 64-deep chunks by LDS-DMA (buffer loads: x
//     rows past M read as zeros), up to 7 chunks ahead (as many as 160 KB of LDS holds), so one counted
//     vmcnt per chunk covers both operands (an ordinary weight load beside LDS-DMA makes hipcc drain
//     vmcnt to 0 at its first use: cdna_hip_programming.md §5 item 4(b)); a preshuffled weight block is
//     1 KB in fragment order, so its DMA and its ds_read_b128 are both lane-linear; the 16-B chunk index
//     of each 128-B x row is XOR-swizzled with (row >> 1) & 7 on the DMA source and on the read, which
//     makes the x fragment reads bank-conflict free;
//   * the 16x16 accumulator of (weight tile, token tile) holds 4 consecutive features of one token per
//     lane: one float4 store per accumulator into the slab.
#include "common.h"
#include "decode_epi.h"
#include "launchers.h"

namespace {

constexpr int MG_THR = 256;
constexpr int MG_LDS = 160 * 1024;

typedef __attribute__((address_space(3))) void lds_t;

SYM_DEV __amdgpu_buffer_rsrc_t mg_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}

SYM_DEV void mg_dma(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t*)lds, 16, voff, soff, 0, 0);
}

// non-temporal (aux = 2) LDS-DMA for the once-read weight stream (MI355X_MICROARCH.md row nt-weights)
SYM_DEV void mg_dma_nt(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t*)lds, 16, voff, soff, 0, 2);
}

template <int MT, int RW>
struct MgCfg {
  static constexpr int XB = 16 * MT * 128;                   // x bytes of one 64-deep chunk
  static constexpr int WB = 4 * RW * 2 * 1024;               // weight bytes of one chunk (2 blocks per tile)
  static constexpr int SLOT = XB + WB;
  static constexpr int SLOTS = MG_LDS / SLOT > 8 ? 8 : MG_LDS / SLOT;
  static constexpr int D = SLOTS - 1;                        // chunks in flight ahead of the computed one
  static constexpr int NX = 16 * MT / 32;                    // x DMA instructions per wave per chunk (MT >= 2)
  static constexpr int NDMA = NX + 2 * RW;                   // DMA instructions per wave per chunk
  static constexpr int VM_KEEP = (D - 1) * NDMA;             // younger DMAs left in flight at the wait
  static_assert(D >= 1 && VM_KEEP <= 63, "mgemm config");
};

// MT: 16-token tiles (M <= 16 MT); RW: 16-row weight tiles per wave.  Weights MFMA-preshuffled
// (models/layout.py::preshuffle): block (t, kb) = 16 rows x 32 k, 1 KB in fragment order.
// EPI < 0: the k split's fp32 slab is the output (the consumer kernel sums the slabs).  EPI >= 0: a fused
// consumer (decode_epi.h): with one split the accumulators go straight to epilogue<EPI>; with S splits every
// workgroup stores its slab, and the LAST of the S workgroups of a column group (agent-scope release /
// acquire around a per-group counter, cdna_hip_programming.md §5 "In-launch split-K reduction") sums the S
// slabs of its columns in the accumulator layout, applies the deferred-RMSNorm row scale (e.ss_in) and runs
// the epilogue -- the separate rope_cache / add+RMSNorm / SwiGLU launches of the slab path disappear.
// `counters` [N / (64 RW)] start at zero and are re-armed by the last arriver (graph-replay safe).
template <int MT, int RW, bool WNT, int EPI>
__global__ __launch_bounds__(MG_THR, 1) void mgemm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ W,
                                                           float* __restrict__ y, int M, int N, int K, int kslice,
                                                           DecodeEpi e, int* __restrict__ counters) {
  using C = MgCfg<MT, RW>;
  __shared__ __attribute__((aligned(1024))) char smem[C::SLOTS * C::SLOT];
  asm volatile("" ::: "a0");  // accumulators may live in AGPRs

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int split = blockIdx.y;
  const int k0 = split * kslice;
  const int nch = kslice / 64;
  const int tile0 = (blockIdx.x * 4 + wid) * RW;  // first 16-row weight tile of this wave

  // ---- x DMA: wave w fills rows (NX w + i) * 8 .. + 8 of each chunk; lane -> (row lane >> 3, 16-B chunk
  // lane & 7), source chunk swizzled by (row >> 1) & 7.  Rows >= M read as zeros (buffer range).
  const __amdgpu_buffer_rsrc_t rx = mg_rsrc(x, (long long)M * K * 2);
  int vx[C::NX];
#pragma unroll
  for (int i = 0; i < C::NX; ++i) {
    const int row = (C::NX * wid + i) * 8 + (lane >> 3);
    vx[i] = row * K * 2 + 16 * ((lane & 7) ^ ((row >> 1) & 7)) + k0 * 2;
  }
  // ---- weight DMA: the wave's own tiles, block (tile, 2c + s) -> its 1 KB LDS block, lane-linear
  const __amdgpu_buffer_rsrc_t rw = mg_rsrc(W, (long long)N * K * 2);
  const int vw = (tile0 * (K / 32) + k0 / 32) * 1024 + lane * 16;
  const int wstride = (K / 32) * 1024;  // bytes between consecutive weight tiles
  char* const dx = smem + (C::NX * wid) * 1024;
  char* const dw = smem + C::XB + wid * RW * 2 * 1024;

  auto issue = [&](int c, int slot) {
    const int xo = c * 128, wo = c * 2048;
#pragma unroll
    for (int i = 0; i < C::NX; ++i) mg_dma(rx, vx[i], xo, dx + slot * C::SLOT + i * 1024);
#pragma unroll
    for (int rt = 0; rt < RW; ++rt) {
      if constexpr (WNT) {
        mg_dma_nt(rw, vw + rt * wstride, wo, dw + slot * C::SLOT + (2 * rt) * 1024);
        mg_dma_nt(rw, vw + rt * wstride, wo + 1024, dw + slot * C::SLOT + (2 * rt + 1) * 1024);
      } else {
        mg_dma(rw, vw + rt * wstride, wo, dw + slot * C::SLOT + (2 * rt) * 1024);
        mg_dma(rw, vw + rt * wstride, wo + 1024, dw + slot * C::SLOT + (2 * rt + 1) * 1024);
      }
    }
  };

  // ---- fragment reads: x lane holds token (16 mt + (lane & 15)), k 8 (lane >> 4) .. + 8 of step s
  // (swizzled chunk 4 s + (lane >> 4)); weight block reads are lane-linear (fragment order)
  const int fr = lane & 15;
  const int xo0 = fr * 128 + 16 * ((lane >> 4) ^ ((fr >> 1) & 7));
  const int xo1 = fr * 128 + 16 * ((4 + (lane >> 4)) ^ ((fr >> 1) & 7));
  const int wo_l = C::XB + wid * RW * 2 * 1024 + lane * 16;

  f32x4 acc[RW][MT];
#pragma unroll
  for (int rt = 0; rt < RW; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int slot) {
    const char* const sb = smem + slot * C::SLOT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 wf[RW], xf[MT];
#pragma unroll
      for (int rt = 0; rt < RW; ++rt) wf[rt] = *(const bf16x8*)(sb + wo_l + (2 * rt + s) * 1024);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xf[mt] = *(const bf16x8*)(sb + (s ? xo1 : xo0) + mt * 2048);
#pragma unroll
      for (int rt = 0; rt < RW; ++rt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = mfma16(wf[rt], xf[mt], acc[rt][mt]);
    }
  };

  // deferred-RMSNorm row scales (EPI >= 0 with e.ss_in): tpr threads per row sum the producer's partials.
  // Loads issued before the DMA prologue, summed after it (the DMAs stay in flight); the scale lives in one
  // register until the epilogue.  (Computed in the epilogue with one wave-serial loop per row, it cost
  // ~13 us per launch at 64 rows: 16 dependent load round trips per wave.)
  float rn_reg = 1.f;
  int rn_row = -1;
  float rn_part = 0.f;
  int tpr = 1;
  if constexpr (EPI >= 0) {
    if (e.ss_in) {
      while (tpr < 64 && tpr * 2 * M <= MG_THR) tpr *= 2;
      const int row = threadIdx.x / tpr, sub = threadIdx.x % tpr;
      if (row < M) {
        rn_row = row;
        const float* sp = e.ss_in + (long long)row * e.ss_tiles;
        if (e.ss_tiles % (4 * tpr) == 0) {
          const float4* s4 = reinterpret_cast<const float4*>(sp);
#pragma unroll 8
          for (int i = sub; i < e.ss_tiles / 4; i += tpr) {
            const float4 q = s4[i];
            rn_part += (q.x + q.y) + (q.z + q.w);
          }
        } else {
#pragma unroll 8
          for (int i = sub; i < e.ss_tiles; i += tpr) rn_part += sp[i];
        }
      }
    }
  }

  // prologue: chunks 0 .. D-1 in flight
#pragma unroll
  for (int c = 0; c < C::D; ++c)
    if (c < nch) issue(c, c);

  if constexpr (EPI >= 0) {
    if (e.ss_in) {  // tpr consecutive lanes of one wave (tpr divides 64)
      for (int o = 1; o < tpr; o *= 2) rn_part += __shfl_xor(rn_part, o, 64);
      rn_reg = rsqrtf(rn_part * e.inv_d + e.eps);
    }
  }

  // chunk c lives in ring slot c % SLOTS.  Before computing it: wait until this wave's DMAs of chunk c
  // have landed (the D - 1 younger chunks stay in flight), barrier (every wave's x rows of the chunk are
  // visible), then refill the slot of chunk c - 1 (all its reads happened before this barrier) with c + D.
  int slot = 0;
  for (int c = 0; c < nch; ++c) {
    if (c + C::D - 1 < nch) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::VM_KEEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (c + C::D < nch) issue(c + C::D, slot == 0 ? C::SLOTS - 1 : slot - 1);
    compute(slot);
    slot = slot == C::SLOTS - 1 ? 0 : slot + 1;
  }

  // ---- epilogue: lane holds features 16 t + 4 (lane >> 4) .. + 3 of token 16 mt + (lane & 15)
  const int S = gridDim.y;
  float* ys = y + (long long)split * M * N;
  if (EPI < 0 || S > 1) {
#pragma unroll
    for (int rt = 0; rt < RW; ++rt) {
      const int n = 16 * (tile0 + rt) + 4 * (lane >> 4);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + (lane & 15);
        if (m >= M) continue;
        const float4 f4 = make_float4(acc[rt][mt][0], acc[rt][mt][1], acc[rt][mt][2], acc[rt][mt][3]);
        if constexpr (EPI >= 0) {  // read back in this launch by the last split: write-through (see below)
          unsigned long long* q = reinterpret_cast<unsigned long long*>(ys + (long long)m * N + n);
          const unsigned long long* w64 = reinterpret_cast<const unsigned long long*>(&f4);
          __hip_atomic_store(q, w64[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(q + 1, w64[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          *reinterpret_cast<float4*>(ys + (long long)m * N + n) = f4;
        }
      }
    }
  }
  if constexpr (EPI >= 0) {
    // LDS ring is free once every wave is past its last compute: row scales + the "last arriver" word
    __syncthreads();
    float* rn = reinterpret_cast<float*>(smem);
    int* last = reinterpret_cast<int*>(smem + 1024 * 4);
    if (S > 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores are out
      __syncthreads();
      // hand-off without L2 maintenance (MI355X_MICROARCH.md): write-through slab stores drained above,
      // relaxed agent add, the last split reads the slabs with agent-scope (L2-bypassing) loads.  Agent
      // fences here wrote back / invalidated the XCD's whole L2 once per workgroup: the fused general path
      // ran 6.22 vs 4.43 ms per 64-client step (profiles/r3/mg_fused_ab.jsonl).
      if (threadIdx.x == 0) {
        const int got = __hip_atomic_fetch_add(counters + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int is_last = got == S - 1;
        if (is_last) __hip_atomic_store(counters + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *last = is_last;
      }
      __syncthreads();
      if (!*last) return;
    }
    // deferred-RMSNorm row scales of the input rows (summed before the main loop)
    if (e.ss_in) {
      if (rn_row >= 0 && threadIdx.x % tpr == 0) rn[rn_row] = rn_reg;
      __syncthreads();
    }
#pragma unroll
    for (int rt = 0; rt < RW; ++rt) {
      const int n = 16 * (tile0 + rt) + 4 * (lane >> 4);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + (lane & 15);
        const bool mok = m < M;
        f32x4 v = acc[rt][mt];
        if (S > 1) {
          v = f32x4{0.f, 0.f, 0.f, 0.f};
          if (mok)
            for (int sp = 0; sp < S; ++sp) {  // fixed split order: bitwise reproducible
              const unsigned long long* q =
                  reinterpret_cast<const unsigned long long*>(y + ((long long)sp * M + m) * N + n);
              unsigned long long r[2];
              r[0] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              r[1] = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const float* p = reinterpret_cast<const float*>(r);
              v[0] += p[0];
              v[1] += p[1];
              v[2] += p[2];
              v[3] += p[3];
            }
        }
        const float sc = (e.ss_in && mok) ? rn[m] : 1.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] *= sc;
        epilogue<EPI>(e, v, tile0 + rt, m, mok, lane >> 4, N);
      }
    }
  }
}

int g_mgemm_nt = 0;

template <int MT, int RW, int EPI>
void launch_mt_rw(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, const DecodeEpi& e,
                  int* counters, hipStream_t s) {
  if (g_mgemm_nt && EPI < 0)
    mgemm_kernel<MT, RW, true, EPI><<<dim3(N / (64 * RW), S), dim3(MG_THR), 0, s>>>(x, W, y, M, N, K, K / S, e,
                                                                                   counters);
  else
    mgemm_kernel<MT, RW, false, EPI><<<dim3(N / (64 * RW), S), dim3(MG_THR), 0, s>>>(x, W, y, M, N, K, K / S, e,
                                                                                    counters);
}

template <int MT, int EPI>
void launch_mt(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, int rw, const DecodeEpi& e,
               int* counters, hipStream_t s) {
  if constexpr (MT > 8) {  // 256 rows: at most 2 weight tiles per wave (accumulators + LDS ring)
    if (rw == 1) launch_mt_rw<MT, 1, EPI>(x, W, y, M, N, K, S, e, counters, s);
    else launch_mt_rw<MT, 2, EPI>(x, W, y, M, N, K, S, e, counters, s);
    return;
  }
  switch (rw) {
    case 1: launch_mt_rw<MT, 1, EPI>(x, W, y, M, N, K, S, e, counters, s); break;
    case 3: launch_mt_rw<MT, 3, EPI>(x, W, y, M, N, K, S, e, counters, s); break;
    case 4: launch_mt_rw<MT, 4, EPI>(x, W, y, M, N, K, S, e, counters, s); break;
    default: launch_mt_rw<MT, 2, EPI>(x, W, y, M, N, K, S, e, counters, s); break;
  }
}

template <int EPI>
void launch_epi_m(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, int rw, const DecodeEpi& e,
                  int* counters, hipStream_t s) {
  if (M <= 32)
    launch_mt<2, EPI>(x, W, y, M, N, K, S, rw, e, counters, s);
  else if (M <= 64)
    launch_mt<4, EPI>(x, W, y, M, N, K, S, rw, e, counters, s);
  else if (M <= 128)
    launch_mt<8, EPI>(x, W, y, M, N, K, S, rw, e, counters, s);
  else
    launch_mt<16, EPI>(x, W, y, M, N, K, S, rw, e, counters, s);
}

}  // namespace

void set_mgemm_nt(int on) { g_mgemm_nt = on; }

void launch_mgemm(const bf16* x, const bf16* Wshuf, float* y, int M, int N, int K, int S, int rw, hipStream_t s) {
  launch_epi_m<-1>(x, Wshuf, y, M, N, K, S, rw, DecodeEpi{}, nullptr, s);
}

void launch_mgemm_epi(int epi, const bf16* x, const bf16* Wshuf, float* y, int M, int N, int K, int S, int rw,
                      const DecodeEpi& e, int* counters, hipStream_t s) {
  switch (epi) {
    case DECODE_EPI_QKV: launch_epi_m<DECODE_EPI_QKV>(x, Wshuf, y, M, N, K, S, rw, e, counters, s); break;
    case DECODE_EPI_RESID: launch_epi_m<DECODE_EPI_RESID>(x, Wshuf, y, M, N, K, S, rw, e, counters, s); break;
    case DECODE_EPI_SWIGLU: launch_epi_m<DECODE_EPI_SWIGLU>(x, Wshuf, y, M, N, K, S, rw, e, counters, s); break;
    default: launch_epi_m<DECODE_EPI_F32>(x, Wshuf, y, M, N, K, S, rw, e, counters, s); break;
  }
}
