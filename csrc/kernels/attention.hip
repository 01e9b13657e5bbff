// K4 / K5: paged attention on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), D = 128.
//
// Cache layout (written by rope_cache.hip):
//   k_cache [NB][Hkv][BS][D]   token-major
//   v_cache [NB][Hkv][D][BS]   dim-major
// Both kernels use the "swapped" products so that no operand needs an LDS
// transpose and every operand fragment is a contiguous 16-byte load:
//   S^T[tok][q] = K[tok][:] . Q[q][:]      A = K rows,   B = Q^T
//   O^T[d][q]  += V^T[d][tok] . P^T[tok][q] A = V^T rows, B = P^T
// The accumulator of S^T (lane: column q = lane&15, rows 4*(lane>>4)+r) is
// turned into the P^T B-operand in registers: a 32-token group is computed as
// two 16-token S^T tiles whose token lists interleave in 4s
// (tile a holds tokens 8*(row>>2) + 4a + (row&3)), so lane group h owns tokens
// 8h..8h+7 of the group = exactly the k-slice its B fragment needs.
// The contraction over D uses a k permutation (lane group h covers dims
// 32h..32h+31 across the 4 MFMAs), making each lane's K and Q reads 64
// contiguous bytes.  Softmax is online (running max / sum per query column),
// in base 2 with the 1/sqrt(D)*log2(e) scale folded into one multiply.
//
// Decode (K5): grid (seq, kv_head, partition); 8 waves x 64 tokens = 512
// tokens per partition; the G = Hq/Hkv query heads of a kv head are the MFMA
// columns (K/V are read once per kv head).  Multi-partition sequences write
// fp32 partials that the last-arriving partition combines (split-KV,
// flash-decoding, one launch).
// The grid is sized for the max context so the launch is hipGraph-capturable;
// partitions past a sequence's context exit at once.
//
// Prefill (K4): grid (q tile, kv_head * G); each wave owns 16 query rows of
// one head, causal + varlen + chunked prefill (queries are the LAST qlen
// positions of a context of length ctx), reading K/V from the paged cache.
#include "attn_decode.h"
#include "common.h"
#include "launchers.h"

namespace {

// ---------------------------------------------------------------------------------------------
// Decode (body: attn_decode.h, shared with the fused decode block launch)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(DWAVES * 64) void attn_decode_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ ctx_lens, bf16* __restrict__ out,
    float* __restrict__ tmp_o, float* __restrict__ tmp_ml, int* __restrict__ counters, int Hq, int Hkv, int BS,
    int max_blocks, int max_parts, float scale_log2) {
  attn_decode_unit<16>(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml, counters, Hq, Hkv, BS,
                       max_blocks, max_parts, scale_log2, blockIdx.x, blockIdx.y, blockIdx.z);
}

// ---------------------------------------------------------------------------------------------
// Prefill (varlen, causal, paged, chunked)
// ---------------------------------------------------------------------------------------------
// tiles[i] = {seq, first query row within the seq's new tokens}; a tile is 64 query rows
// (4 waves x 16 rows) of one query head.
__global__ __launch_bounds__(256) void attn_prefill_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ ctx_lens, const int* __restrict__ cu_q,
    const int* __restrict__ tiles, bf16* __restrict__ out, int Hq, int Hkv, int BS, int max_blocks,
    float scale_log2) {
  const int tile = blockIdx.x, head = blockIdx.y;
  const int seq = tiles[2 * tile], qrow0 = tiles[2 * tile + 1];
  const int G = Hq / Hkv, kvh = head / G;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 15, h = lane >> 4;
  const int qstart = cu_q[seq], qlen = cu_q[seq + 1] - qstart;
  const int ctx = ctx_lens[seq];
  const int pos0 = ctx - qlen;  // absolute position of query row 0
  const int row0 = qrow0 + 16 * wid;
  if (row0 >= qlen) return;
  const int myrow = row0 + c;
  const bool row_ok = myrow < qlen;
  const int mypos = pos0 + myrow;

  bf16x8 qf[4];
  if (row_ok) {
    const bf16* qp = q + ((long long)(qstart + myrow) * Hq + head) * D + 32 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = ld16(qp + 8 * i);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = zero8();
  }
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  const int* bt = block_tables + (long long)seq * max_blocks;
  // last key any row of this wave may see
  const int kend = min(ctx, pos0 + min(row0 + 16, qlen));
  // software pipeline: group g+1's K/V loads are in flight while group g is computed
  auto kv_ptrs = [&](int tbase, const bf16*& kb, const bf16*& vb) {
    const long long blk = bt[tbase / BS];
    const int boff = tbase % BS;
    kb = k_cache + ((blk * Hkv + kvh) * BS + boff) * D;
    vb = v_cache + (blk * Hkv + kvh) * (long long)D * BS + boff;
  };
  KVFrag cur, nxt;
  if (kend > 0) {
    const bf16 *kb, *vb;
    kv_ptrs(0, kb, vb);
    load_group(kb, vb, BS, cur);
  }
  for (int tbase = 0; tbase < kend; tbase += 32) {
    if (tbase + 32 < kend) {
      const bf16 *kb, *vb;
      kv_ptrs(tbase + 32, kb, vb);
      load_group(kb, vb, BS, nxt);
    }
    compute_group(cur, qf, scale_log2,
                  [&](int a, int r) {
                    const int t = tbase + 8 * h + 4 * a + r;
                    return row_ok && t <= mypos && t < ctx;
                  },
                  o, m, lsum);
    cur = nxt;
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (!row_ok) return;
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  bf16* op = out + ((long long)(qstart + myrow) * Hq + head) * D;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    bf16x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[dt][r] * inv);
    *reinterpret_cast<bf16x4*>(op + 16 * dt + 4 * h) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// Prefill, LDS-staged (K4): one workgroup per (64-query-row tile, kv head, head slice).
// The HPW query heads that share the kv head (GQA) are processed by the same workgroup, so every
// 64-token K/V tile is read from the paged cache ONCE per workgroup (cooperative 16-byte loads,
// double-buffered through LDS: the next tile's global loads are in flight while the current one is
// computed) and each wave reuses every K/V fragment it reads from LDS for its 2 query-column blocks
// (32 query rows).  Wave w: head = slice * HPW + w % HPW, rows 32 * (w / HPW) .. +31 of the tile.
// Math per 32-token group is compute_group (swapped products, in-register P^T).
// ---------------------------------------------------------------------------------------------
constexpr int KST = D + 8;   // LDS row stride of the K tile (elements): 272 B, 16-B aligned, skewed banks
constexpr int VST = 64 + 8;  // LDS row stride of the V^T tile (elements): 144 B

SYM_DEV void lds_group(const bf16* sk, const bf16* sv, int g, KVFrag& f) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, h = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int trow = 32 * g + (r16 >> 2) * 8 + 4 * a + (r16 & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) f.k[a][i] = *reinterpret_cast<const bf16x8*>(sk + trow * KST + 32 * h + 8 * i);
  }
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
    f.v[dt] = *reinterpret_cast<const bf16x8*>(sv + (16 * dt + r16) * VST + 32 * g + 8 * h);
}

template <int HPW>
__global__ __launch_bounds__(128 * HPW) void attn_prefill_lds_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ ctx_lens, const int* __restrict__ cu_q,
    const int* __restrict__ tiles, bf16* __restrict__ out, int Hq, int Hkv, int BS, int max_blocks,
    float scale_log2) {
  constexpr int NT = 128 * HPW;
  constexpr int CH = 1024 / NT;  // 16-byte chunks per thread, per K and per V tile
  __shared__ bf16 sK[2][64 * KST];
  __shared__ bf16 sV[2][D * VST];
  const int tile = blockIdx.x, kvh = blockIdx.y;
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 15, h = lane >> 4;
  const int head = kvh * G + blockIdx.z * HPW + wid % HPW;
  const int half = wid / HPW;
  const int seq = tiles[2 * tile], qrow0 = tiles[2 * tile + 1];
  const int qstart = cu_q[seq], qlen = cu_q[seq + 1] - qstart;
  const int ctx = ctx_lens[seq];
  const int pos0 = ctx - qlen;
  const int* bt = block_tables + (long long)seq * max_blocks;
  // keys visible to any row of the workgroup / of this wave
  const int kend_wg = min(ctx, pos0 + min(qrow0 + 64, qlen));
  const int row0 = qrow0 + 32 * half;
  const int kend_w = min(ctx, pos0 + min(row0 + 32, qlen));

  bf16x8 qf[2][4];
  int mypos[2];
  bool row_ok[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int myrow = row0 + 16 * cb + c;
    row_ok[cb] = myrow < qlen;
    mypos[cb] = pos0 + myrow;
    if (row_ok[cb]) {
      const bf16* qp = q + ((long long)(qstart + myrow) * Hq + head) * D + 32 * h;
#pragma unroll
      for (int i = 0; i < 4; ++i) qf[cb][i] = ld16(qp + 8 * i);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) qf[cb][i] = zero8();
    }
  }
  f32x4 o[2][8];
  float m[2] = {-INFINITY, -INFINITY}, lsum[2] = {0.f, 0.f};
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[cb][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // cooperative tile loads: chunk ci -> K (token ci >> 4, 16-B piece ci & 15), V (dim ci >> 3, tokens 8 (ci & 7)..)
  uint4 rk[CH], rv[CH];
  auto gload = [&](int t0) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int ci = threadIdx.x + j * NT;
      const int tk = t0 + (ci >> 4);
      const long long bk = tk < ctx ? bt[tk / BS] : 0;  // past the context: reserved block 0 (finite)
      rk[j] = *reinterpret_cast<const uint4*>(k_cache + ((bk * Hkv + kvh) * BS + tk % BS) * D + (ci & 15) * 8);
      const int tv = t0 + 8 * (ci & 7);
      const long long bv = tv < ctx ? bt[tv / BS] : 0;
      rv[j] = *reinterpret_cast<const uint4*>(v_cache + ((bv * Hkv + kvh) * D + (ci >> 3)) * (long long)BS + tv % BS);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int ci = threadIdx.x + j * NT;
      *reinterpret_cast<uint4*>(&sK[buf][(ci >> 4) * KST + (ci & 15) * 8]) = rk[j];
      *reinterpret_cast<uint4*>(&sV[buf][(ci >> 3) * VST + 8 * (ci & 7)]) = rv[j];
    }
  };

  const int ntiles = (kend_wg + 63) / 64;
  if (ntiles > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int it = 0; it < ntiles; ++it) {
    const int t0 = it * 64;
    if (it + 1 < ntiles) gload(t0 + 64);
    const bf16* sk = sK[it & 1];
    const bf16* sv = sV[it & 1];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int tbase = t0 + 32 * g;
      if (tbase < kend_w) {
        KVFrag f;
        lds_group(sk, sv, g, f);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          compute_group(f, qf[cb], scale_log2,
                        [&](int a, int r) {
                          const int t = tbase + 8 * h + 4 * a + r;
                          return row_ok[cb] && t <= mypos[cb] && t < ctx;
                        },
                        o[cb], m[cb], lsum[cb]);
      }
    }
    if (it + 1 < ntiles) lstore((it + 1) & 1);
    __syncthreads();
  }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    float l = lsum[cb];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (!row_ok[cb]) continue;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* op = out + ((long long)(qstart + row0 + 16 * cb + c) * Hq + head) * D;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[cb][dt][r] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * dt + 4 * h) = v;
    }
  }
}

}  // namespace

void launch_attn_decode(const bf16* q, const bf16* k_cache, const bf16* v_cache, const int* block_tables,
                        const int* ctx_lens, bf16* out, float* tmp_o, float* tmp_ml, int* counters, int num_seqs,
                        int Hq, int Hkv, int BS, int max_blocks, int max_parts, float scale, hipStream_t s) {
  if (num_seqs == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(num_seqs, Hkv, max_parts);
  attn_decode_kernel<<<grid, DWAVES * 64, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml, counters,
                                          Hq, Hkv, BS, max_blocks, max_parts, scale_log2);
}

void launch_attn_prefill(const bf16* q, const bf16* k_cache, const bf16* v_cache, const int* block_tables,
                         const int* ctx_lens, const int* cu_q, const int* tiles, int num_tiles, bf16* out, int Hq,
                         int Hkv, int BS, int max_blocks, float scale, hipStream_t s) {
  if (num_tiles == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  if (BS % 8 == 0 && (G == 1 || G == 2 || G % 4 == 0)) {
    // LDS-staged kernel: the kv head's query heads share every K/V tile (slices of <= 4 heads)
    const int hpw = G >= 4 ? 4 : G;
    const dim3 grid(num_tiles, Hkv, G / hpw);
    if (hpw == 4)
      attn_prefill_lds_kernel<4><<<grid, 512, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles, out,
                                                      Hq, Hkv, BS, max_blocks, scale_log2);
    else if (hpw == 2)
      attn_prefill_lds_kernel<2><<<grid, 256, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles, out,
                                                      Hq, Hkv, BS, max_blocks, scale_log2);
    else
      attn_prefill_lds_kernel<1><<<grid, 128, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles, out,
                                                      Hq, Hkv, BS, max_blocks, scale_log2);
    return;
  }
  attn_prefill_kernel<<<dim3(num_tiles, Hq), 256, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles,
                                                          out, Hq, Hkv, BS, max_blocks, scale_log2);
}
