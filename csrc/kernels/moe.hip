// K10-K12: Mixture-of-Experts routing, permutation, grouped GEMM and combine (Mixtral 8x7B).
//
//   moe_route     router logits (LinOut [T][E]) -> top-k ids + softmax-renormalised weights
//   moe_align     one workgroup: expert histogram + exclusive prefix sum -> segment offsets [E+1]
//   moe_scatter   copy each (token, slot) row of x into its expert segment; dst[t][j] = row
//   grouped_skinny  Y[rows of expert e] = Xs[rows of e] . W[e]^T on MFMA, one weight tile per
//                 workgroup, reading the segment bounds from device memory (graph-capturable,
//                 no host sync); fp32 split-K slabs like the dense skinny GEMM
//   grouped_gemm  the same for any number of routed rows (prefill): 128 x 128 MFMA tiles over the
//                 concatenated expert segments, the tile -> (expert, row block) map computed on the
//                 device from the segment offsets (no host sync, graph-capturable); optional fused
//                 SwiGLU epilogue (gate and up columns of one tile meet through LDS)
//   moe_combine   out[t] = sum_j w[t][j] * Y[dst[t][j]]  (fixed slot order -> deterministic)
//
// Rows inside an expert segment are placed by atomics (order varies run to run) but every row
// is computed independently and the combine sums in slot order, so results are bitwise stable.
#include "common.h"
#include "launchers.h"

namespace {


// Router logits of a prefill-sized step: fp32 [T][16] = x [T][d] . Wr[16][d]^T (Wr: the router rows padded to 16).
// One workgroup per 16 tokens, its NW waves splitting d (16 waves when d % 512 == 0: every wave's loads are in
// flight at once -- with 4 waves the 32-deep k loop was latency-bound, 14.2 us at 512 tokens); v_mfma_f32_16x16x32_bf16
// with the router rows as the A operand (a lane (token r16, h) ends with experts 4h .. 4h + 3 of its token), the
// partials summed through LDS.  Replaces a library GEMM of N = 16 (15.3 us per Mixtral layer at 512 tokens).
template <int NW>
__global__ __launch_bounds__(NW * 64) void moe_router_kernel(const bf16* __restrict__ x, const bf16* __restrict__ Wr,
                                                             float* __restrict__ logits, int T, int d) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int row = blockIdx.x * 16 + r16;
  const int kw = d / NW;  // this wave's k range (a multiple of 32)
  const bf16* xr = x + (long long)min(row, T - 1) * d + wid * kw + 8 * h;
  const bf16* wr = Wr + (long long)r16 * d + wid * kw + 8 * h;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int k0 = 0; k0 < kw; k0 += 32) {
    Pack8 a, b;
    a.u = *reinterpret_cast<const uint4*>(wr + k0);
    b.u = *reinterpret_cast<const uint4*>(xr + k0);
    acc = mfma16(a.v, b.v, acc);
  }
  __shared__ f32x4 red[NW][64];
  red[wid][lane] = acc;
  __syncthreads();
  if (wid == 0 && row < T) {
    f32x4 v = red[0][lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += red[w][lane];
    *reinterpret_cast<float4*>(logits + (long long)row * 16 + 4 * h) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// One wave per token.  E <= 64 experts (lane e holds logit e), k <= 8.
__global__ __launch_bounds__(256) void moe_route_kernel(LinOut logits, int ld, int T, int E, int k,
                                                        int* __restrict__ ids, float* __restrict__ w) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  float v = lane < E ? linout_load1(logits, (long long)t * ld + lane) : -INFINITY;
  if (v != v) v = -INFINITY;  // a NaN logit never wins (and never selects a lane >= E)
  // unrolled over the 8-slot maximum with guards: a runtime-indexed private array would live in scratch memory
  float sel[8];
  int seli[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sel[j] = 0.f;
    seli[j] = j;
    if (j < k) {
      float m = v;
      int mi = lane;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float om = __shfl_xor(m, o, 64);
        const int oi = __shfl_xor(mi, o, 64);
        if (om > m || (om == m && oi < mi)) {
          m = om;
          mi = oi;
        }
      }
      if (mi >= E) mi = j;  // degenerate rows (all -inf): fall back to experts 0..k-1
      sel[j] = m;
      seli[j] = mi;
      if (lane == mi) v = -INFINITY;
    }
  }
  if (lane == 0) {
    float mx = sel[0], s = 0.f;
    const bool deg = mx == -INFINITY;
    if (deg) mx = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (deg) sel[j] = 0.f;
      if (j < k) s += __expf(sel[j] - mx);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < k) {
        ids[t * k + j] = seli[j];
        w[t * k + j] = __expf(sel[j] - mx) / s;
      }
  }
}

// Single workgroup: histogram of the routed expert ids (LDS atomics), exclusive prefix sum ->
// offsets[E+1], counts[E], and the scatter cursor zeroed.  Doing the zeroing here (instead of a
// hipMemsetAsync node) keeps the whole MoE step a plain kernel chain under hipGraph replay.
// dst (optional): each assignment's row in its segment, placed here with LDS atomics, so the scatter needs no
// global atomics (1024 workgroups bumping 8 global cursors serialised a 4 x 128-token Mixtral scatter: 15.6 us).
__global__ __launch_bounds__(1024) void moe_align_kernel(const int* __restrict__ ids, int n, int E,
                                                         int* __restrict__ counts, int* __restrict__ offsets,
                                                         int* __restrict__ cursor, int* __restrict__ dst) {
  __shared__ int hist[64];
  __shared__ int base[64];
  if (threadIdx.x < 64) hist[threadIdx.x] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i];
    if (e >= 0 && e < E) atomicAdd(&hist[e], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      offsets[e] = acc;
      counts[e] = hist[e];
      cursor[e] = 0;
      base[e] = acc;
      acc += hist[e];
    }
    offsets[E] = acc;
  }
  if (dst == nullptr) return;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i];
    if (e >= 0 && e < E) dst[i] = atomicAdd(&base[e], 1);
  }
}

// one 256-thread block per (token, slot); cursor[E] zeroed by the op.  Assignments with an expert id
// outside [0, E) (empty slots of an expert-parallel receive buffer) are skipped.  cursor == nullptr: the rows
// were placed by moe_align (dst precomputed).
__global__ __launch_bounds__(256) void moe_scatter_kernel(const bf16* __restrict__ x, int d, int k, int R, int E,
                                                          const int* __restrict__ ids, const int* __restrict__ offsets,
                                                          int* __restrict__ cursor, bf16* __restrict__ xs,
                                                          int* __restrict__ dst, int* __restrict__ src_tok) {
  const int a = blockIdx.x;  // assignment t * k + j
  const int t = a / k;
  const int e = ids[a];
  if (e < 0 || e >= E) return;
  __shared__ int row;
  if (threadIdx.x == 0) {
    row = cursor != nullptr ? offsets[e] + atomicAdd(&cursor[e], 1) : dst[a];
    if (cursor != nullptr) dst[a] = row;
    if (src_tok) src_tok[row] = t;
  }
  __syncthreads();
  if (row < 0 || row >= R) return;
  const uint4* s = reinterpret_cast<const uint4*>(x + (long long)t * d);
  uint4* o = reinterpret_cast<uint4*>(xs + (long long)row * d);
  for (int i = threadIdx.x; i < d / 8; i += 256) o[i] = s[i];
}

// Grouped skinny GEMM: grid (N/16, E, S).  W [E][N][K] holds experts e0 .. e0+E-1 of the global
// numbering; rows of expert e: [off[e0+e], off[e0+e+1]) (absolute rows of xs / y).
// Up to 64 rows per expert (4 MFMA column tiles); the prefill path uses library GEMMs instead.
// wshuf: W MFMA-preshuffled per expert (models/layout.py): a lane's 16 B of k-block kb of its 16-row tile sit at
// lane * 16 B of that 1 KB block -- the same (row r16, k group h) fragment as the row-major read, one contiguous
// 1 KB per wave instruction (decode_weights="replace": the expert stacks exist only in this layout).
template <bool WSHUF>
__global__ __launch_bounds__(256) void grouped_skinny_kernel(const bf16* __restrict__ xs, const bf16* __restrict__ W,
                                                             const int* __restrict__ offsets, float* __restrict__ y,
                                                             int R, int N, int K, int kchunk, int e0) {
  const int tile = blockIdx.x, e = blockIdx.y, split = blockIdx.z;
  const int r0 = offsets[e + e0], r1 = min(offsets[e + e0 + 1], R);
  const int n_e = r1 - r0;
  if (n_e <= 0 || r0 < 0) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, h = lane >> 4;
  const int n0 = tile * 16;
  const int wk = kchunk / 4;
  const int kbeg = split * kchunk + wid * wk;
  const int nblk = wk / 64;
  const bf16* wrow = WSHUF ? W + (((long long)e * (N / 16) + tile) * (K / 32) + kbeg / 32) * 512 + lane * 8
                          : W + ((long long)e * N + n0 + r16) * K + kbeg + 8 * h;
  const int MT = min(4, (n_e + 15) / 16);
  const bf16* xrow[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int m = r0 + min(16 * mt + r16, n_e - 1);
    xrow[mt] = xs + (long long)m * K + kbeg + 8 * h;
  }
  f32x4 acc[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < nblk; ++b) {
    const int ko = b * 64;
    Pack8 w0, w1;
    if constexpr (WSHUF) {  // k-blocks (kbeg + ko) / 32 and the next one: 1 KB apart
      w0.u = *reinterpret_cast<const uint4*>(wrow + ko * 16);
      w1.u = *reinterpret_cast<const uint4*>(wrow + ko * 16 + 512);
    } else {
      w0.u = *reinterpret_cast<const uint4*>(wrow + ko);
      w1.u = *reinterpret_cast<const uint4*>(wrow + ko + 32);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      if (mt < MT) {
        Pack8 x0, x1;
        x0.u = *reinterpret_cast<const uint4*>(xrow[mt] + ko);
        x1.u = *reinterpret_cast<const uint4*>(xrow[mt] + ko + 32);
        acc[mt] = mfma16(w0.v, x0.v, acc[mt]);
        acc[mt] = mfma16(w1.v, x1.v, acc[mt]);
      }
    }
  }
  __shared__ f32x4 red[4][4][64];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) red[wid][mt][lane] = acc[mt];
  __syncthreads();
  if (wid != 0) return;
  for (int mt = 0; mt < MT; ++mt) {
    const f32x4 s = red[0][mt][lane] + red[1][mt][lane] + red[2][mt][lane] + red[3][mt][lane];
    const int m = 16 * mt + r16;
    if (m < n_e) {
      float* yp = y + ((long long)split * R + r0 + m) * N + n0 + 4 * h;
      *reinterpret_cast<float4*>(yp) = make_float4(s[0], s[1], s[2], s[3]);
    }
  }
}


// ---------------------------------------------------------------------------------------------------
// Grouped GEMM for prefill-sized routed batches (K12): Y[rows of expert e] = Xs[rows of e] . W[e]^T.
//
// Tiles of 128 routed rows x 128 weight rows, BK = 64, 256 threads = 4 waves in a 2 x 2 grid of 64 x 64
// wave tiles, v_mfma_f32_16x16x32_bf16 with the WEIGHT fragment as the A operand (a lane then holds four
// consecutive output columns of one row: 16-B fp32 / 8-B bf16 stores).  Both operand tiles are staged
// global -> LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per lane, double-buffered: the next k-tile's
// DMA overlaps this one's MFMAs); the LDS images are [128 rows][8 chunks of 16 B] with chunk
// c stored at c ^ ((row >> 1) & 7) (pre-swizzled on the per-lane GLOBAL address, the LDS side of a DMA
// being lane-linear), so the 16-row x 4-chunk fragment reads are bank-conflict free.
//
// Grid: x = weight-row tiles, y = an upper bound on the row tiles (ceil(R / 128) + experts); workgroup
// (x, y) walks the device-side segment offsets to find which expert's which row block y is (or exits).
// SWIGLU: weight rows are [gate (F) ; up (F)]; x-tile j covers output columns f = 64 j .. 64 j + 63 and
// stages gate rows 64 j.. as tile rows 0-63 and up rows F + 64 j.. as rows 64-127, so waves wn = 0 / 1
// hold gate / up of the same (row, f); the up waves hand theirs over through LDS and the gate waves store
// act = bf16(silu(gate) * up) -- the [R, 2F] intermediate never exists.
// OUT: 0 = bf16 Y, 1 = fp32 Y, 2 = SwiGLU act (bf16 [R][F]).
// ---------------------------------------------------------------------------------------------------
constexpr int GG_BM = 128, GG_BN = 128, GG_BK = 64, GG_THREADS = 256;
constexpr int GG_TILE_BYTES = GG_BM * GG_BK * 2;  // 16 KB per operand tile

SYM_DEV void gg_glds16(const bf16* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

SYM_DEV int gg_swz(int row) { return (row >> 1) & 7; }

template <int OUT>
__global__ __launch_bounds__(GG_THREADS, 2) void grouped_gemm_kernel(const bf16* __restrict__ xs,
                                                                     const bf16* __restrict__ W,
                                                                     const int* __restrict__ offsets,
                                                                     void* __restrict__ y, int R, int N, int K,
                                                                     int E, int e0) {
  extern __shared__ __attribute__((aligned(16))) char gg_smem[];
  // ---- which expert / row block is this workgroup (device-side segment walk, E <= 64)
  int e = -1, rb = 0, r0 = 0, n_e = 0;
  {
    int cum = 0;
    for (int i = 0; i < E; ++i) {
      const int a = offsets[e0 + i], b = min(offsets[e0 + i + 1], R);
      const int n = max(0, b - a);
      const int t = (n + GG_BM - 1) / GG_BM;
      if ((int)blockIdx.y < cum + t) {
        e = i;
        rb = blockIdx.y - cum;
        r0 = a + rb * GG_BM;
        n_e = min(GG_BM, b - r0);
        break;
      }
      cum += t;
    }
  }
  if (e < 0) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  // ---- DMA source addresses: wave w stages rows 8 (4 i + w) + lane / 8 of each 128-row tile, i = 0..3,
  // chunk (lane & 7) of the LDS row <- global chunk (lane & 7) ^ swz(row)
  const bf16* asrc[4];
  const bf16* bsrc[4];
  const long long Nw = OUT == 2 ? 2LL * N : N;  // weight rows per expert (SwiGLU: N = F output columns)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * i + wid) + (lane >> 3);
    const int ch = (lane & 7) ^ gg_swz(row);
    const int m = r0 + min(row, n_e - 1);  // rows past the segment re-read its last row (never stored)
    asrc[i] = xs + (long long)m * K + 8 * ch;
    long long wrow;
    if constexpr (OUT == 2) wrow = row < 64 ? 64LL * blockIdx.x + row : (long long)N + 64LL * blockIdx.x + (row - 64);
    else wrow = (long long)GG_BN * blockIdx.x + row;
    bsrc[i] = W + (long long)e * Nw * K + wrow * K + 8 * ch;  // W holds the local experts only
  }
  auto stage = [&](int kt, int buf) {
    char* base = gg_smem + buf * 2 * GG_TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      gg_glds16(asrc[i] + kt * GG_BK, base + (4 * i + wid) * 1024);
      gg_glds16(bsrc[i] + kt * GG_BK, base + GG_TILE_BYTES + (4 * i + wid) * 1024);
    }
  };
  f32x4 acc[4][4];  // [n subtile][m subtile]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, h = lane >> 4;
  const int nk = K / GG_BK;
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile kt landed for every wave; every wave finished reading buffer (kt + 1) & 1
    if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
    const char* A = gg_smem + (kt & 1) * 2 * GG_TILE_BYTES;  // routed rows
    const char* B = A + GG_TILE_BYTES;                        // weight rows
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = 4 * ks + h;  // 16-B chunk of the fragment (k = 32 ks + 8 h ..)
      Pack8 bf[4], af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 64 * wn + 16 * i + r16;
        bf[i].u = *reinterpret_cast<const uint4*>(B + row * 128 + 16 * (c ^ gg_swz(row)));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 64 * wm + 16 * j + r16;
        af[j].u = *reinterpret_cast<const uint4*>(A + row * 128 + 16 * (c ^ gg_swz(row)));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bf[i].v, af[j].v, acc[i][j]);
    }
  }
  // ---- epilogue: lane (r16, h) of acc[i][j] holds output row m = 64 wm + 16 j + r16, weight columns
  // 64 wn + 16 i + 4 h .. + 3 of the tile
  if constexpr (OUT == 2) {
    __syncthreads();  // staging buffers are free: the up waves hand over their accumulators
    f32x4* xch = reinterpret_cast<f32x4*>(gg_smem);
    if (wn == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) xch[((wm * 4 + i) * 4 + j) * 64 + lane] = acc[i][j];
    }
    __syncthreads();
    if (wn == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 64 * wm + 16 * j + r16;
        if (m >= n_e) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 u = xch[((wm * 4 + i) * 4 + j) * 64 + lane];
          const f32x4 g = acc[i][j];
          float o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = g[q] / (1.f + __expf(-g[q])) * u[q];
          bf16* yp = reinterpret_cast<bf16*>(y) + (long long)(r0 + m) * N + 64 * blockIdx.x + 16 * i + 4 * h;
          bf16x4 pk = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
          *reinterpret_cast<bf16x4*>(yp) = pk;
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 64 * wm + 16 * j + r16;
      if (m >= n_e) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long off = (long long)(r0 + m) * N + GG_BN * blockIdx.x + 64 * wn + 16 * i + 4 * h;
        const f32x4 v = acc[i][j];
        if constexpr (OUT == 1) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(y) + off) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          bf16x4 pk = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(y) + off) = pk;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Weight-streaming grouped GEMM for medium routed batches (K12, ~32-256 rows per expert: Mixtral prefill
// of a few prompts).  There the expert weights (Mixtral: 2.8 GB per layer) are read once and the routed
// rows are few, so the 128 x 128 tile kernel above -- every tile re-stages its activation rows and pays a
// prologue / epilogue per tile, 2 waves per CU -- streams the weights at ~3 TB/s
// (profiles/r5/prof_mixtral_prefill_4x128.csv).  This kernel is mgemm.hip's weight stream made grouped and
// persistent:
//
//   * a unit = (expert, block of up to 16 MT routed rows, n-block of 64 RW weight rows) over the whole K;
//     units are numbered n-block-major, so with one row block per expert and a grid that is a multiple of 8
//     every workgroup keeps ONE expert (blockIdx % 8 is the XCD: that expert's activation rows stay in its
//     L2) and walks the n-blocks; the unit -> (expert, rows) map is computed on the device from the
//     segment offsets (graph-capturable, no host sync);
//   * one workgroup per CU, 4 waves x RW 16-row weight tiles; activation rows and weight rows stream
//     through ONE LDS ring of 64-deep chunks by LDS-DMA (buffer loads: activation rows past the segment
//     read as zeros without memory traffic), the ring continuing across unit boundaries, so the next
//     unit's first chunks are in flight while this one's last chunks and its epilogue run;
//   * both LDS images are [rows][128 B] with the 16-B chunk c stored at c ^ ((row >> 1) & 7) (swizzled on
//     the DMA source), so fragment reads are conflict-free; the weight tile is the A operand of
//     v_mfma_f32_16x16x32_bf16 (a lane ends with 4 consecutive features of one routed row), MFMAs on
//     16-row token tiles past the segment are skipped (uniform branch);
//   * OUT 2 (SwiGLU, W = [gate; up] rows): a wave's tiles alternate gate / up of the same 16 features, so
//     act = silu(gate) * up is formed in registers -- the [R, 2F] intermediate never exists.
// ---------------------------------------------------------------------------------------------------
constexpr int GS_THR = 256, GS_EMAX = 8, GS_LDS = 160 * 1024;
typedef __attribute__((address_space(3))) void lds_t;

template <int MT, int RW, int D>
struct GsCfg {
  static constexpr int BM = 16 * MT;                         // routed rows per unit
  static constexpr int XB = BM * 128;                        // activation bytes of one 64-deep chunk (LDS slot)
  static constexpr int NX = MT / 2;                          // activation DMA instructions per wave per chunk
  static constexpr int NW = 2 * RW;                          // weight load instructions per wave per chunk
  // younger vector-memory ops when chunk g's activation DMA must have landed: W(g+1 .. g+D-1), X(g+1 .. g+D-2)
  static constexpr int VM_KEEP = (D - 1) * NW + (D - 2) * NX;
  static_assert(MT % 4 == 0 && D >= 3 && D * XB <= GS_LDS && VM_KEEP <= 63, "grouped stream config");
};

SYM_DEV __amdgpu_buffer_rsrc_t gs_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}

// (the LDS-DMA builtin behind a device function: called directly inside the kernel's lambda, it makes the host
// pass drop the kernel's launch stub)
SYM_DEV void gs_dma(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t*)lds, 16, voff, soff, 0, 0);
}

SYM_DEV void gs_dma_nt(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t*)lds, 16, voff, soff, 0, 2);
}

SYM_DEV bf16x8 gs_ldw(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 2);  // nt: weights are read once
  return __builtin_bit_cast(bf16x8, v);
}

struct GsUnit {
  int e, row0, rows, nb;
};

// unit u -> (expert, rows, n-block); a[] / nrb[] hold the segment starts and row-block counts (uniform)
SYM_DEV GsUnit gs_unit(int u, int ERB, const int (&a)[GS_EMAX], const int (&n)[GS_EMAX], const int (&nrb)[GS_EMAX],
                       int E, int BM) {
  GsUnit r{0, 0, 0, u / ERB};
  int j = u - r.nb * ERB;
  bool found = false;
#pragma unroll
  for (int i = 0; i < GS_EMAX; ++i) {
    if (i < E && !found) {
      if (j < nrb[i]) {
        found = true;
        r.e = i;
        r.row0 = a[i] + j * BM;
        r.rows = min(BM, n[i] - j * BM);
      } else {
        j -= nrb[i];
      }
    }
  }
  return r;
}

// Nw: weight rows per expert (SwiGLU: 2 Ny); Ny: output columns.  PRE: W MFMA-preshuffled per expert
// (models/layout.py::preshuffle: a wave's fragment load reads 1 KB contiguous instead of 16 rows x 64 B).
//
// Pipeline (one workgroup per CU): the weight fragments go straight into VGPRs (a register ring of D chunks
// per wave, no LDS), the activation rows through an LDS ring of D slots, so a CU keeps D x (16 RW KB of weights
// + 2 MT KB of activations) in flight -- the LDS alone (weights and activations both staged) held 96-128 KB,
// and the activation bytes queued in front of the weights capped the stream at ~3 TB/s from 128 rows.
// Per chunk g: wait for X(g) (W(g) is older), barrier, DMA X(g+D-1) into the slot chunk g-1 freed, MFMAs of
// chunk g, then load W(g+D) into the register slot chunk g freed.  A unit is a whole number of ring turns and
// loads past the last unit use a zero-range descriptor, so every iteration issues the same instructions and one
// constant vmcnt covers every wait.
//
// offsets == nullptr is ONE segment of R rows; S > 1 splits K over S units per n-block, each writing its fp32
// slab y[ks] (OUT 1).
template <int MT, int RW, int D, int OUT, bool PRE>
__global__ __launch_bounds__(GS_THR, 1) void grouped_stream_kernel(const bf16* __restrict__ xs,
                                                                   const bf16* __restrict__ W,
                                                                   const int* __restrict__ offsets,
                                                                   void* __restrict__ y, int R, int Nw, int Ny, int K,
                                                                   int E, int e0, int S) {
  using C = GsCfg<MT, RW, D>;
  __shared__ __attribute__((aligned(1024))) char smem[D * C::XB];
  asm volatile("" ::: "a0");  // accumulators may live in AGPRs
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

  // ---- segment table (uniform) and the unit count
  int a[GS_EMAX], n[GS_EMAX], nrb[GS_EMAX];
  int ERB = 0;
#pragma unroll
  for (int i = 0; i < GS_EMAX; ++i) {
    a[i] = 0;
    n[i] = 0;
    nrb[i] = 0;
    if (i < E) {
      a[i] = offsets ? offsets[e0 + i] : 0;
      n[i] = offsets ? max(0, min(offsets[e0 + i + 1], R) - a[i]) : R;
      nrb[i] = (n[i] + C::BM - 1) / C::BM;
      ERB += nrb[i];
    }
  }
  const int rows_nb = OUT == 2 ? 32 * RW : 64 * RW;  // expert-local weight rows per n-block (SwiGLU: gate rows)
  const int NB = (OUT == 2 ? Ny : Nw) / rows_nb;
  const int U = NB * ERB * S;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= U) return;  // uniform: the whole workgroup
  const int nch = K / 64 / S;  // chunks per unit (its k slice)
  const int T = ((U - 1 - (int)blockIdx.x) / G + 1) * nch;  // chunks this workgroup streams (nch % D == 0)

  // ---- per-lane offsets (unit-invariant: the unit lives in the descriptor bases)
  int vx[C::NX];
#pragma unroll
  for (int i = 0; i < C::NX; ++i) {
    const int row = (C::NX * wid + i) * 8 + (lane >> 3);
    vx[i] = row * K * 2 + 16 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  int vw[RW];  // k-step 0 of chunk 0; k-step 1 adds 64 B (row-major) / 1 KB (preshuffled)
#pragma unroll
  for (int rt = 0; rt < RW; ++rt) {
    const int row0 = OUT == 2 ? (rt & 1) * Ny + 16 * (wid * (RW / 2) + rt / 2) : 16 * (wid * RW + rt);
    if constexpr (PRE) vw[rt] = (row0 >> 4) * (K / 32) * 1024 + lane * 16;
    else vw[rt] = (row0 + (lane & 15)) * K * 2 + 16 * (lane >> 4);
  }
  char* const dx = smem + (C::NX * wid) * 1024;

  // ---- issue cursors: activations (unit xu, chunk xc) and weights (unit wu, chunk wc)
  int xu = blockIdx.x, xc = 0, wu = blockIdx.x, wc = 0, xk0 = 0, wk0 = 0;  // xk0 / wk0: the unit's first chunk
  const bf16* xb = xs;
  const bf16* wb = W;
  long long xbytes = 0, wbytes = 0;
  auto bind_x = [&](int u) {
    xbytes = 0;
    if (u < U) {
      const GsUnit un = gs_unit(u / S, ERB, a, n, nrb, E, C::BM);
      xb = xs + (long long)un.row0 * K;
      xbytes = (long long)un.rows * K * 2;
      xk0 = (u % S) * nch;
    }
  };
  auto bind_w = [&](int u) {
    wbytes = 0;
    if (u < U) {
      const GsUnit un = gs_unit(u / S, ERB, a, n, nrb, E, C::BM);
      wk0 = (u % S) * nch;
      const long long wrow = (long long)un.e * Nw + (long long)un.nb * rows_nb;
      wb = W + wrow * K;
      wbytes = ((long long)un.e * Nw + Nw - wrow) * K * 2;
    }
  };
  bind_x(xu);
  bind_w(wu);
  auto issue_x = [&](int slot) {
    const __amdgpu_buffer_rsrc_t rx = gs_rsrc(xb, xbytes);
#pragma unroll
    for (int i = 0; i < C::NX; ++i) gs_dma(rx, vx[i], (xk0 + xc) * 128, dx + slot * C::XB + i * 1024);
    if (++xc == nch) {
      xc = 0;
      xu += G;
      bind_x(xu);
    }
  };
  bf16x8 wr[D][RW][2];
  auto issue_w = [&](bf16x8 (&dst)[RW][2]) {
    const __amdgpu_buffer_rsrc_t rw = gs_rsrc(wb, wbytes);
    const int so = PRE ? (wk0 + wc) * 2048 : (wk0 + wc) * 128;
#pragma unroll
    for (int rt = 0; rt < RW; ++rt)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        dst[rt][s] = gs_ldw(rw, vw[rt] + (PRE ? s * 1024 : s * 64), so);
    if (++wc == nch) {
      wc = 0;
      wu += G;
      bind_w(wu);
    }
  };

  // ---- fragment offsets of the activation image: row fr of a 16-row tile, global chunk 4 s + (lane >> 4)
  const int fr = lane & 15;
  const int fo0 = fr * 128 + 16 * ((lane >> 4) ^ ((fr >> 1) & 7));
  const int fo1 = fr * 128 + 16 * ((4 + (lane >> 4)) ^ ((fr >> 1) & 7));

  f32x4 acc[RW][MT];
#pragma unroll
  for (int rt = 0; rt < RW; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  int cu = blockIdx.x, cc = 0;
  GsUnit cun = gs_unit(cu / S, ERB, a, n, nrb, E, C::BM);
  int mact = (cun.rows + 15) / 16;

  // prologue in the steady state's order: W(0), then X(c), W(c + 1) for c = 0 .. D-2
  issue_w(wr[0]);
#pragma unroll
  for (int c = 0; c < D - 1; ++c) {
    issue_x(c);
    issue_w(wr[c + 1]);
  }

  for (int g0 = 0; g0 < T; g0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::VM_KEEP) : "memory");
      __builtin_amdgcn_s_barrier();
      issue_x((j + D - 1) % D);  // X(g + D - 1) into the slot chunk g - 1 freed (every wave is past its reads)
      const char* const sb = smem + j * C::XB;
      // token tiles in groups of 4 under one uniform skip branch: a group's 4 fragment reads are issued together
      // (a read per tile under its own branch exposed the LDS latency once per tile: 1.3 us per chunk at 128 rows),
      // and a unit sized for the largest segment costs the LDS reads / MFMAs of its actual rows only
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int g4 = 0; g4 < MT / 4; ++g4) {
          if (4 * g4 < mact) {
            bf16x8 xf[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) xf[q] = *(const bf16x8*)(sb + (4 * g4 + q) * 2048 + (s ? fo1 : fo0));
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
              for (int rt = 0; rt < RW; ++rt) acc[rt][4 * g4 + q] = mfma16(wr[j][rt][s], xf[q], acc[rt][4 * g4 + q]);
          }
        }
      }
      issue_w(wr[j]);  // W(g + D) into the register slot chunk g freed
    }
    // a unit is a whole number of ring turns (host-checked nch % D == 0): its epilogue stays out of the unrolled
    // body (inside it the SwiGLU variant's code size stopped the unroll and the register ring went to scratch)
    cc += D;
    if (cc < nch || cu >= U) continue;
    // ---- unit done: epilogue, lane holds features 4 (lane >> 4) .. + 3 of routed row 16 mt + (lane & 15)
    cc = 0;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + (lane & 15);
      if (mt < mact && m < cun.rows) {
        const long long yrow = ((long long)(cu % S) * R + cun.row0 + m) * Ny;
        if constexpr (OUT == 2) {
#pragma unroll
          for (int p = 0; p < RW / 2; ++p) {
            const f32x4 gt = acc[2 * p][mt], up = acc[2 * p + 1][mt];
            const int f = cun.nb * rows_nb + 16 * (wid * (RW / 2) + p) + 4 * (lane >> 4);
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = gt[q] / (1.f + __expf(-gt[q])) * up[q];
            bf16x4 pk = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
            *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(y) + yrow + f) = pk;
          }
        } else {
#pragma unroll
          for (int rt = 0; rt < RW; ++rt) {
            const f32x4 v = acc[rt][mt];
            const int f = cun.nb * rows_nb + 16 * (wid * RW + rt) + 4 * (lane >> 4);
            if constexpr (OUT == 1) {
              *reinterpret_cast<float4*>(reinterpret_cast<float*>(y) + yrow + f) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
              bf16x4 pk = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
              *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(y) + yrow + f) = pk;
            }
          }
        }
      }
#pragma unroll
      for (int rt = 0; rt < RW; ++rt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    cu += G;
    if (cu < U) {
      cun = gs_unit(cu / S, ERB, a, n, nrb, E, C::BM);
      mact = (cun.rows + 15) / 16;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup's LDS is released
}

template <int MT, int RW, int D, int OUT>
void gs_launch(const bf16* xs, const bf16* W, const int* offsets, void* y, int R, int E, int e0, int Nw, int Ny, int K,
               int G, bool pre, hipStream_t s, int S = 1) {
  if (pre) grouped_stream_kernel<MT, RW, D, OUT, true><<<G, GS_THR, 0, s>>>(xs, W, offsets, y, R, Nw, Ny, K, E, e0, S);
  else grouped_stream_kernel<MT, RW, D, OUT, false><<<G, GS_THR, 0, s>>>(xs, W, offsets, y, R, Nw, Ny, K, E, e0, S);
}

template <int MT, int RW, int D>
void gs_launch_out(int out, const bf16* xs, const bf16* W, const int* offsets, void* y, int R, int E, int e0, int Nw,
                   int Ny, int K, int G, bool pre, hipStream_t s) {
  if (out == 2) gs_launch<MT, RW, D, 2>(xs, W, offsets, y, R, E, e0, Nw, Ny, K, G, pre, s);
  else if (out == 1) gs_launch<MT, RW, D, 1>(xs, W, offsets, y, R, E, e0, Nw, Ny, K, G, pre, s);
  else gs_launch<MT, RW, D, 0>(xs, W, offsets, y, R, E, e0, Nw, Ny, K, G, pre, s);
}

int g_gs_policy = 1;  // grouped_stream with row-major weights: 0 never, 1 where it measured faster, 2 always
int g_gs_rw = 0;      // weight tiles per wave: 0 = by the unit count, 2, 4
int g_gs_mt = 0;      // unit rows / 16: 0 = from the mean segment
int g_gs_cus = 0;

// E_all: experts of the global numbering (the routed rows R spread over them)
bool launch_grouped_stream(const bf16* xs, const bf16* W, const int* offsets, void* y, int R, int E, int E_all, int e0,
                           int N, int K, int out) {
  (void)y;
  if (g_gs_policy == 0 || E > GS_EMAX || K % 256 || K > (1 << 16)) return false;  // K % 256: whole ring turns
  const int RW = 2;
  const int Nw = out == 2 ? 2 * N : N;
  if ((out == 2 ? N % (32 * RW) : N % (64 * RW)) != 0) return false;
  if ((long long)Nw * K * 2 >= 0x7fffffffLL) return false;  // one expert's weights within one buffer descriptor
  const int avg = (R + E_all - 1) / std::max(1, E_all);
  // auto, row-major weights (bench/kernels/bench_grouped.py, profiles/r5/grouped_stream.jsonl): the stream beats
  // the tile kernel on w2-shaped launches up to ~80 rows per expert (fragment loads of 16 rows x 64 B), never
  // clearly on SwiGLU gate/up; preshuffled weights always take the stream (launch_grouped_gemm's `pre`)
  if (g_gs_policy == 1 && (out == 2 || avg > 80)) return false;
  return true;
}

// out[t] (fp32 [T][d]) = sum_j w[t][j] * y[dst[t][j]] over assignments whose expert is in
// [e_lo, e_hi) (the experts this rank computed); y is a LinOut over R rows
__global__ __launch_bounds__(256) void moe_combine_kernel(LinOut y, int R, const int* __restrict__ dst,
                                                          const int* __restrict__ ids, int e_lo, int e_hi,
                                                          const float* __restrict__ w, int k, int d,
                                                          float* __restrict__ out, int accumulate) {
  const int t = blockIdx.x;
  for (int i = threadIdx.x; i < d / 8; i += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int row = dst[t * k + j];
      const int ex = ids[t * k + j];
      if (row < 0 || row >= R || ex < e_lo || ex >= e_hi) continue;
      const float wj = w[t * k + j];
      float v[8];
      linout_load8(y, (long long)row * d + i * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wj * v[q];
    }
    float* o = out + (long long)t * d + i * 8;
    if (accumulate) {
      float prev[8];
      load8f(o, prev);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += prev[q];
    }
    store8f(o, acc);
  }
}

// ---------------------------------------------------------------------------------------------------
// Decode-sized MoE routing in ONE launch (T <= 16 token rows, E <= 64 experts, k <= 8; one 16-wave
// workgroup): RMSNorm of the fp32 residual rows, router logits, top-k + renormalised softmax, expert
// histogram / offsets, segment rows in token order, and the permuted normalised rows xs -- what rms_norm,
// the router GEMM, moe_route, moe_align and moe_scatter do as five launches on the general path (4.5-5.2 us
// each at 4 rows: launch-floor-sized, profiles/r4/prof_mixtral_4clients_decode.csv).  xs rows equal the
// rms_norm kernel's bf16 output (bf16(w * (x * rsqrt(mean(x^2) + eps)))); the router reads the same values.
// ---------------------------------------------------------------------------------------------------
constexpr int MDR_T = 8, MDR_K = 8, MDR_D = 4096, MDR_U = MDR_D / 512;  // rows, top-k, max d, 16-B loads per lane
constexpr int MDR_WR = 8 * 4096;  // router elements staged in LDS (E * d up to this; else read from global)
constexpr int MDR_NT = 512;       // 8 waves: 256 VGPRs per lane, so the staged router and a residual row fit

// Latency shape (one workgroup: every step is at most one dependent memory round trip): the router weights
// are loaded by all threads at entry and parked in LDS (they depend on nothing; parking them keeps registers
// free -- held in registers across the norm phase they spilled to scratch); wave t < T loads residual row t
// with the norm weights, reduces its sum of squares and writes the bf16 normalised row into LDS; the logits
// are LDS x LDS dot products; top-k per token; the segment bookkeeping in parallel; the permuted rows go out
// from LDS.
__global__ __launch_bounds__(MDR_NT) void moe_decode_route_kernel(const float* __restrict__ resid,
                                                                const bf16* __restrict__ lnw, float eps,
                                                                const bf16* __restrict__ Wr, int T, int d, int E, int k,
                                                                int* __restrict__ ids, float* __restrict__ w,
                                                                int* __restrict__ counts, int* __restrict__ offsets,
                                                                int* __restrict__ cursor, bf16* __restrict__ xs,
                                                                int* __restrict__ dst) {
  __shared__ uint4 s_xn[MDR_T * MDR_D / 8];  // bf16 normalised rows, 8 per uint4
  __shared__ uint4 s_wr[MDR_WR / 8];         // bf16 router rows
  __shared__ float s_lg[MDR_T][64];
  __shared__ int s_ids[MDR_T * MDR_K];
  __shared__ int s_dst[MDR_T * MDR_K];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nv = d / 8;  // 16-B vectors per row
  const bool wr_lds = E * d <= MDR_WR;
  uint4 wst[MDR_WR / 8 / MDR_NT];
  if (wr_lds) {
#pragma unroll
    for (int u = 0; u < MDR_WR / 8 / MDR_NT; ++u) {
      const int v = threadIdx.x + MDR_NT * u;
      wst[u] = v < E * nv ? reinterpret_cast<const uint4*>(Wr)[v] : make_uint4(0, 0, 0, 0);
    }
  }
  if (wid < T) {
    float rv[MDR_U][8];
    Pack8 gw[MDR_U];  // the norm weights, loaded with the row (one memory round trip)
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < MDR_U; ++u) {
      const int v = lane + 64 * u;
      if (v < nv) {
        load8f(resid + (long long)wid * d + 8 * v, rv[u]);
        gw[u].u = *reinterpret_cast<const uint4*>(lnw + 8 * v);
      }
    }
#pragma unroll
    for (int u = 0; u < MDR_U; ++u)
      if (lane + 64 * u < nv)
#pragma unroll
        for (int q = 0; q < 8; ++q) ss += rv[u][q] * rv[u][q];
    ss = wave_sum(ss);
    const float rn = rsqrtf(ss / (float)d + eps);
#pragma unroll
    for (int u = 0; u < MDR_U; ++u) {
      const int v = lane + 64 * u;
      if (v < nv) {
        Pack8 pk;
#pragma unroll
        for (int q = 0; q < 8; ++q) pk.h[q] = (bf16)((float)gw[u].h[q] * (rv[u][q] * rn));
        s_xn[wid * (MDR_D / 8) + v] = pk.u;
      }
    }
  }
  if (wr_lds) {
#pragma unroll
    for (int u = 0; u < MDR_WR / 8 / MDR_NT; ++u) s_wr[threadIdx.x + MDR_NT * u] = wst[u];
  }
  __syncthreads();
  // logits: wave e against every row
  for (int e = wid; e < E; e += MDR_NT / 64) {
    float acc[MDR_T];
#pragma unroll
    for (int t = 0; t < MDR_T; ++t) acc[t] = 0.f;
#pragma unroll
    for (int u = 0; u < MDR_U; ++u) {
      const int v = lane + 64 * u;
      if (v < nv) {
        Pack8 wv;
        wv.u = wr_lds ? s_wr[e * nv + v] : *reinterpret_cast<const uint4*>(Wr + (long long)e * d + 8 * v);
#pragma unroll
        for (int t = 0; t < MDR_T; ++t)
          if (t < T) {
            Pack8 xv;
            xv.u = s_xn[t * (MDR_D / 8) + v];
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[t] += (float)xv.h[q] * (float)wv.h[q];
          }
      }
    }
#pragma unroll
    for (int t = 0; t < MDR_T; ++t)
      if (t < T) {
        const float sum = wave_sum(acc[t]);
        if (lane == 0) s_lg[t][e] = sum;
      }
  }
  __syncthreads();
  // top-k per token (wave t): the moe_route_kernel selection, ties to the lower expert
  if (wid < T) {
    float v = lane < E ? s_lg[wid][lane] : -INFINITY;
    if (v != v) v = -INFINITY;
    // (fully unrolled over MDR_K with guards: a runtime-indexed private array would live in scratch memory,
    // one global round trip per access)
    float sel[MDR_K];
    int seli[MDR_K];
#pragma unroll
    for (int j = 0; j < MDR_K; ++j) {
      sel[j] = 0.f;
      seli[j] = j;
      if (j < k) {
        float m = v;
        int mi = lane;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const float om = __shfl_xor(m, o, 64);
          const int oi = __shfl_xor(mi, o, 64);
          if (om > m || (om == m && oi < mi)) {
            m = om;
            mi = oi;
          }
        }
        if (mi >= E) mi = j;
        sel[j] = m;
        seli[j] = mi;
        if (lane == mi) v = -INFINITY;
      }
    }
    if (lane == 0) {
      float mx = sel[0], sum = 0.f;
      const bool deg = mx == -INFINITY;
      if (deg) mx = 0.f;
#pragma unroll
      for (int j = 0; j < MDR_K; ++j) {
        if (deg) sel[j] = 0.f;
        if (j < k) sum += __expf(sel[j] - mx);
      }
#pragma unroll
      for (int j = 0; j < MDR_K; ++j)
        if (j < k) {
          ids[wid * k + j] = seli[j];
          s_ids[wid * k + j] = seli[j];
          w[wid * k + j] = __expf(sel[j] - mx) / sum;
        }
    }
  }
  __syncthreads();
  const int R = T * k;
  // histogram, offsets and segment rows in token order, in parallel (R <= 64, E <= 64): lane e of wave 0 counts
  // expert e, a wave scan gives the offsets, and thread a < R places assignment a after the earlier ones of
  // its expert
  __shared__ int s_off[65];
  if (wid == 0) {
    int c = 0;
    if (lane < E)
      for (int a = 0; a < R; ++a) c += s_ids[a] == lane;
    int incl = c;  // inclusive scan over the 64 lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane < E) {
      s_off[lane] = incl - c;
      counts[lane] = c;
      cursor[lane] = 0;
      offsets[lane] = incl - c;
    }
    if (lane == E - 1) {
      s_off[E] = incl;
      offsets[E] = incl;
    }
  }
  __syncthreads();
  if (threadIdx.x < R) {
    const int a = threadIdx.x, e = s_ids[a];
    int before = 0;
    for (int b = 0; b < a; ++b) before += s_ids[b] == e;
    s_dst[a] = s_off[e] + before;
    dst[a] = s_off[e] + before;
  }
  __syncthreads();
  // xs[dst[a]] = normalised row of token a / k, from LDS
  for (int a = 0; a < R; ++a) {
    const int t = a / k, row = s_dst[a];
    for (int v = threadIdx.x; v < nv; v += MDR_NT)
      reinterpret_cast<uint4*>(xs + (long long)row * d)[v] = s_xn[t * (MDR_D / 8) + v];
  }
}

// moe_combine + add_prep in one launch (decode, experts all local): resid[t] += sum_j w[t][j] Y[dst[t][j]];
// xw[t] = bf16(resid[t] * w_next); ss[t][p] = sum of resid[t]^2 over column part p (grid (T, P): one 8-column
// vector per thread, one load round trip per workgroup; the consumer's deferred norm sums the P partials)
__global__ __launch_bounds__(64) void moe_combine_prep_kernel(LinOut y, int R, const int* __restrict__ dst,
                                                              const int* __restrict__ ids, int E,
                                                              const float* __restrict__ w, int k, int d,
                                                              float* __restrict__ resid,
                                                              const bf16* __restrict__ w_next, bf16* __restrict__ xw,
                                                              float* __restrict__ ss) {
  const int t = blockIdx.x, P = gridDim.y, vp = d / 8 / P;
  float sq = 0.f;
  for (int i = blockIdx.y * vp + threadIdx.x; i < (blockIdx.y + 1) * vp; i += 64) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int row = dst[t * k + j];
      const int ex = ids[t * k + j];
      if (row < 0 || row >= R || ex < 0 || ex >= E) continue;
      const float wj = w[t * k + j];
      float v[8];
      linout_load8(y, (long long)row * d + i * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wj * v[q];
    }
    float* rp = resid + (long long)t * d + i * 8;
    float r[8], g[8];
    load8f(rp, r);
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] += acc[q];
    store8f(rp, r);
    load8(w_next + i * 8, g);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sq += r[q] * r[q];
      g[q] *= r[q];
    }
    store8(xw + (long long)t * d + i * 8, g);
  }
  sq = wave_sum(sq);
  if (threadIdx.x == 0) ss[t * P + blockIdx.y] = sq;
}

// ---------------------------------------------------------------------------------------------------
// Expert parallelism over REPLICATED tokens (attention is tensor-parallel, so every rank holds all T rows):
// every rank routes all T tokens, runs its own experts on its own routed rows, and then
//  (1) moe_owner_pack: for each token with >= 1 local expert, the weighted partial sum over its local experts
//      (fp32, j order) becomes ONE row pushed to the token's slice owner (owner = t / S), in owner-grouped
//      blocks of capacity S with the token's slice-local index beside it (the xGMI a2a kernel moves only the
//      counted rows);
//  (2) moe_owner_index: the owner turns the received side ints into pos[s][t] = row of source s's partial
//      for its token t (or -1);
//  (3) moe_owner_combine: out[t] = sum over sources in rank order (deterministic), written as bf16 straight
//      into the all-gather's send rows (rows past the slice's token count are zero).
// ---------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void moe_owner_pack_kernel(LinOut y, int R, const int* __restrict__ dst,
                                                             const int* __restrict__ ids, const float* __restrict__ w,
                                                             int e_lo, int e_hi, int k, int d, int S, int cap,
                                                             int* __restrict__ cursor, float* __restrict__ send,
                                                             int* __restrict__ side) {
  const int t = blockIdx.x;
  bool any = false;
  for (int j = 0; j < k; ++j) {
    const int ex = ids[t * k + j];
    any = any || (ex >= e_lo && ex < e_hi);
  }
  if (!any) return;  // uniform across the block
  const int owner = t / S;
  __shared__ int slot;
  if (threadIdx.x == 0) {
    slot = atomicAdd(&cursor[owner], 1);
    if (slot < cap) side[(long long)owner * cap + slot] = t - owner * S;
  }
  __syncthreads();
  if (slot >= cap) return;  // (cannot happen: a token sends at most one row)
  float* o = send + ((long long)owner * cap + slot) * d;
  for (int i = threadIdx.x; i < d / 8; i += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int row = dst[t * k + j];
      const int ex = ids[t * k + j];
      if (row < 0 || row >= R || ex < e_lo || ex >= e_hi) continue;
      const float wj = w[t * k + j];
      float v[8];
      linout_load8(y, (long long)row * d + i * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wj * v[q];
    }
    store8f(o + i * 8, acc);
  }
}

// pos [N][S] (-1 from the op's memset first): the row of source s's partial for slice token t; grid
// (N, ceil(cap / 256))
__global__ __launch_bounds__(256) void moe_owner_index_kernel(const int* __restrict__ side,
                                                              const int* __restrict__ rcnt, int cap, int S,
                                                              int* __restrict__ pos) {
  const int s = blockIdx.x;
  const int i = blockIdx.y * 256 + threadIdx.x;
  if (i >= min(rcnt[s], cap)) return;
  const int t = side[(long long)s * cap + i];
  if (t >= 0 && t < S) pos[(long long)s * S + t] = i;
}

// out bf16 [S][d]: row t = sum_s recv[s cap + pos[s][t]] (sources in rank order); t >= Tr: zeros
__global__ __launch_bounds__(256) void moe_owner_combine_kernel(const float* __restrict__ recv,
                                                                const int* __restrict__ pos, int N, int cap, int S,
                                                                int Tr, int d, bf16* __restrict__ out) {
  const int t = blockIdx.x;
  for (int i = threadIdx.x; i < d / 8; i += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (t < Tr) {
      for (int s = 0; s < N; ++s) {
        const int p = pos[(long long)s * S + t];
        if (p < 0 || p >= cap) continue;
        float v[8];
        load8f(recv + ((long long)s * cap + p) * d + i * 8, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += v[q];
      }
    }
    store8(out + (long long)t * d + i * 8, acc);
  }
}

}  // namespace

void launch_moe_decode_route(const float* resid, const bf16* lnw, float eps, const bf16* Wr, int T, int d, int E, int k,
                             int* ids, float* w, int* counts, int* offsets, int* cursor, bf16* xs, int* dst,
                             hipStream_t s) {
  if (T == 0) return;
  moe_decode_route_kernel<<<1, MDR_NT, 0, s>>>(resid, lnw, eps, Wr, T, d, E, k, ids, w, counts, offsets, cursor, xs,
                                             dst);
}

void launch_moe_combine_prep(LinOut y, int R, const int* dst, const int* ids, int E, const float* w, int T, int k, int d,
                             float* resid, const bf16* w_next, bf16* xw, float* ss, int parts, hipStream_t s) {
  if (T == 0) return;
  moe_combine_prep_kernel<<<dim3(T, parts), 64, 0, s>>>(y, R, dst, ids, E, w, k, d, resid, w_next, xw, ss);
}

void launch_moe_router(const bf16* x, const bf16* Wr, float* logits, int T, int d, hipStream_t s) {
  if (T == 0) return;
  if (d % 512 == 0) moe_router_kernel<16><<<(T + 15) / 16, 1024, 0, s>>>(x, Wr, logits, T, d);
  else moe_router_kernel<4><<<(T + 15) / 16, 256, 0, s>>>(x, Wr, logits, T, d);
}

void launch_moe_route(LinOut logits, int ld, int T, int E, int k, int* ids, float* w, hipStream_t s) {
  if (T == 0) return;
  moe_route_kernel<<<(T + 3) / 4, 256, 0, s>>>(logits, ld, T, E, k, ids, w);
}

void launch_moe_align(const int* ids, int n, int E, int* counts, int* offsets, int* cursor, hipStream_t s, int* dst) {
  moe_align_kernel<<<1, 1024, 0, s>>>(ids, n, E, counts, offsets, cursor, dst);
}

void launch_moe_scatter(const bf16* x, int T, int d, int k, int E, const int* ids, const int* offsets, int* cursor,
                        bf16* xs, int R, int* dst, int* src_tok, hipStream_t s) {
  if (T == 0) return;
  moe_scatter_kernel<<<T * k, 256, 0, s>>>(x, d, k, R, E, ids, offsets, cursor, xs, dst, src_tok);
}

void launch_grouped_skinny(const bf16* xs, const bf16* W, const int* offsets, float* y, int R, int E, int e0, int N,
                           int K, int S, hipStream_t s, bool wshuf) {
  if (R == 0) return;
  dim3 grid(N / 16, E, S);
  if (wshuf) grouped_skinny_kernel<true><<<grid, 256, 0, s>>>(xs, W, offsets, y, R, N, K, K / S, e0);
  else grouped_skinny_kernel<false><<<grid, 256, 0, s>>>(xs, W, offsets, y, R, N, K, K / S, e0);
}

void set_grouped_stream_policy(int p) {
  g_gs_policy = p % 10;
  g_gs_rw = p / 10 % 10;  // tens digit: weight tiles per wave (0 = auto)
  g_gs_mt = p / 100;      // hundreds: unit rows / 16 (8 / 12 / 16; 0 = from the mean segment)
}

void launch_grouped_gemm(const bf16* xs, const bf16* W, const int* offsets, void* y, int R, int E, int e0, int N,
                         int K, int out, hipStream_t s, int E_all, bool pre) {
  if (R == 0) return;
  if (pre || launch_grouped_stream(xs, W, offsets, y, R, E, E_all > 0 ? E_all : E, e0, N, K, out)) {
    if (!g_gs_cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&g_gs_cus, hipDeviceAttributeMultiprocessorCount, dev);
      g_gs_cus = std::max(8, g_gs_cus);
    }
    const int Nw = out == 2 ? 2 * N : N;
    const int avg = (R + std::max(1, E_all > 0 ? E_all : E) - 1) / std::max(1, E_all > 0 ? E_all : E);
    // unit rows: twice the mean segment (routing is uneven: a segment past the unit streams its weights again,
    // and extra units leave a partial last round), the compute skipping the unit's empty token tiles
    const int want = 2 * avg;
    // (SwiGLU gate/up: 128-row units always -- their 4-tile-per-wave variant outruns the larger units even when
    // longer segments take two units: Mixtral w13 at 128 rows per expert 606 -> 468 us, tile kernel 598-614;
    // profiles/r5/grouped_stream.jsonl)
    const int MT = g_gs_mt == 8 || g_gs_mt == 12 || g_gs_mt == 16 ? g_gs_mt
                   : (out == 2 || want <= 128) ? 8 : want <= 192 ? 12 : 16;
    // RW = 4 halves the activation LDS reads per weight byte, but its units (256 weight rows) must still
    // give every CU work: taken when there are >= 3 units per CU, at 128-row units (it spills at 192)
    const int rows4 = out == 2 ? 128 : 256;
    int RW = g_gs_rw;
    if (RW != 2 && RW != 4) RW = MT == 8 && (long long)((out == 2 ? N : Nw) / rows4) * E >= 3LL * g_gs_cus ? 4 : 2;
    if (MT != 8 || (out == 2 ? N : Nw) % rows4) RW = 2;
    const int NB = (out == 2 ? N : Nw) / (RW == 4 ? rows4 : rows4 / 2);
    const long long upper = (long long)NB * ((R + 16 * MT - 1) / (16 * MT) + E);
    const int G = (int)std::min<long long>(g_gs_cus, upper);
    if (RW == 4 && MT == 8) {
      gs_launch_out<8, 4, 4>(out, xs, W, offsets, y, R, E, e0, Nw, N, K, G, pre, s);
    } else {
      if (MT == 8 && (K / 64) % 8 == 0) gs_launch_out<8, 2, 8>(out, xs, W, offsets, y, R, E, e0, Nw, N, K, G, pre, s);
      else if (MT == 8) gs_launch_out<8, 2, 4>(out, xs, W, offsets, y, R, E, e0, Nw, N, K, G, pre, s);
      else if (MT == 12) gs_launch_out<12, 2, 4>(out, xs, W, offsets, y, R, E, e0, Nw, N, K, G, pre, s);
      else gs_launch_out<16, 2, 4>(out, xs, W, offsets, y, R, E, e0, Nw, N, K, G, pre, s);
    }
    return;
  }
  const int ntile = out == 2 ? N / 64 : N / GG_BN;
  const dim3 grid(ntile, (R + GG_BM - 1) / GG_BM + E);
  const size_t lds = 4 * GG_TILE_BYTES;
  if (out == 2)
    grouped_gemm_kernel<2><<<grid, GG_THREADS, lds, s>>>(xs, W, offsets, y, R, N, K, E, e0);
  else if (out == 1)
    grouped_gemm_kernel<1><<<grid, GG_THREADS, lds, s>>>(xs, W, offsets, y, R, N, K, E, e0);
  else
    grouped_gemm_kernel<0><<<grid, GG_THREADS, lds, s>>>(xs, W, offsets, y, R, N, K, E, e0);
}

void launch_moe_combine(LinOut y, int R, const int* dst, const int* ids, int e_lo, int e_hi, const float* w, int T, int k,
                        int d, float* out, int accumulate, hipStream_t s) {
  if (T == 0) return;
  moe_combine_kernel<<<T, 256, 0, s>>>(y, R, dst, ids, e_lo, e_hi, w, k, d, out, accumulate);
}

void launch_moe_owner_pack(LinOut y, int R, const int* dst, const int* ids, const float* w, int e_lo, int e_hi, int T,
                           int k, int d, int S, int cap, int* cursor, float* send, int* side, hipStream_t s) {
  if (T == 0) return;
  moe_owner_pack_kernel<<<T, 256, 0, s>>>(y, R, dst, ids, w, e_lo, e_hi, k, d, S, cap, cursor, send, side);
}

void launch_moe_owner_combine(const float* recv, const int* side, const int* rcnt, int N, int cap, int S, int Tr,
                              int d, int* pos, bf16* out, hipStream_t s) {
  (void)hipMemsetAsync(pos, 0xff, (size_t)N * S * sizeof(int), s);  // -1: no partial from that source
  moe_owner_index_kernel<<<dim3(N, (cap + 255) / 256), 256, 0, s>>>(side, rcnt, cap, S, pos);
  if (S > 0) moe_owner_combine_kernel<<<S, 256, 0, s>>>(recv, pos, N, cap, S, Tr, d, out);
}
