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
__global__ __launch_bounds__(1024) void moe_align_kernel(const int* __restrict__ ids, int n, int E,
                                                         int* __restrict__ counts, int* __restrict__ offsets,
                                                         int* __restrict__ cursor) {
  __shared__ int hist[64];
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
      acc += hist[e];
    }
    offsets[E] = acc;
  }
}

// one 256-thread block per (token, slot); cursor[E] zeroed by the op.  Assignments with an expert id
// outside [0, E) (empty slots of an expert-parallel receive buffer) are skipped.
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
    row = offsets[e] + atomicAdd(&cursor[e], 1);
    dst[a] = row;
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
  const bf16* wrow = W + ((long long)e * N + n0 + r16) * K + kbeg + 8 * h;
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
    w0.u = *reinterpret_cast<const uint4*>(wrow + ko);
    w1.u = *reinterpret_cast<const uint4*>(wrow + ko + 32);
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

void launch_moe_route(LinOut logits, int ld, int T, int E, int k, int* ids, float* w, hipStream_t s) {
  if (T == 0) return;
  moe_route_kernel<<<(T + 3) / 4, 256, 0, s>>>(logits, ld, T, E, k, ids, w);
}

void launch_moe_align(const int* ids, int n, int E, int* counts, int* offsets, int* cursor, hipStream_t s) {
  moe_align_kernel<<<1, 1024, 0, s>>>(ids, n, E, counts, offsets, cursor);
}

void launch_moe_scatter(const bf16* x, int T, int d, int k, int E, const int* ids, const int* offsets, int* cursor,
                        bf16* xs, int R, int* dst, int* src_tok, hipStream_t s) {
  if (T == 0) return;
  moe_scatter_kernel<<<T * k, 256, 0, s>>>(x, d, k, R, E, ids, offsets, cursor, xs, dst, src_tok);
}

void launch_grouped_skinny(const bf16* xs, const bf16* W, const int* offsets, float* y, int R, int E, int e0, int N,
                           int K, int S, hipStream_t s) {
  if (R == 0) return;
  dim3 grid(N / 16, E, S);
  grouped_skinny_kernel<<<grid, 256, 0, s>>>(xs, W, offsets, y, R, N, K, K / S, e0);
}

// out: 0 bf16 [R][N], 1 fp32 [R][N], 2 SwiGLU act bf16 [R][N] with W holding 2N rows per expert
void launch_grouped_gemm(const bf16* xs, const bf16* W, const int* offsets, void* y, int R, int E, int e0, int N,
                         int K, int out, hipStream_t s) {
  if (R == 0) return;
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
