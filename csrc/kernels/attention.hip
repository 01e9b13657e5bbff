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
// Decode (K5): grid (seq, kv_head, partition); 8 waves x 32 tokens = 256
// tokens per partition (two workgroups resident per CU); the G = Hq/Hkv query heads of a kv head are the MFMA
// columns (K/V are read once per kv head).  Multi-partition sequences write
// fp32 partials that the last-arriving partition combines (split-KV,
// flash-decoding, one launch).
// The grid is sized for the max context so the launch is hipGraph-capturable;
// partitions past a sequence's context exit at once.
//
// Prefill (K4): causal + varlen + chunked prefill (queries are the LAST qlen
// positions of a context of length ctx), reading K/V from the paged cache.
// Default: attn_prefill_m32p_kernel (32x32x16 MFMA, GQA heads share K/V tiles,
// see its comment); the 16x16 kernels remain for GQA groups of 1/2 heads.
#include <stdlib.h>
#include <string.h>

#include "attn_decode.h"
#include "common.h"
#include "launchers.h"

namespace {

// ---------------------------------------------------------------------------------------------
// Decode (body: attn_decode.h)
// ---------------------------------------------------------------------------------------------
// GMAX >= G query heads per kv head: the cross-wave merge stages GMAX columns in LDS (GMAX = 4 for
// Llama-3 GQA: 17 KB instead of 68 KB, so LDS no longer caps the resident workgroups per CU)
template <int GMAX>
__global__ __launch_bounds__(DWAVES * 64, 4) void attn_decode_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ ctx_lens, bf16* __restrict__ out,
    float* __restrict__ tmp_o, float* __restrict__ tmp_ml, int* __restrict__ counters, int Hq, int Hkv, int BS,
    int max_blocks, int max_parts, float scale_log2) {
  attn_decode_unit<GMAX>(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml, counters, Hq, Hkv, BS,
                       max_blocks, max_parts, scale_log2, blockIdx.x, blockIdx.y, blockIdx.z);
}

// ---------------------------------------------------------------------------------------------
// Decode, wide batches: one wave per (seq, kv head) walking its whole context
// ---------------------------------------------------------------------------------------------
// The grid kernel spends an 8-wave workgroup per (seq, kv head, 256-token partition): built for a few
// sequences, where spreading one context over 8 waves shortens the step.  At wide decode batches (128-256
// sequences of 0.5-4K tokens) the units outnumber the resident workgroups several times over and each
// unit's latency chain (metadata, K/V, cross-wave LDS merge, split-KV publish) is paid per round: K/V
// streams at 4.3-5.0 TB/s (grid / streaming kernels).  Here a unit is ONE wave that walks the 32-token
// groups of its context with the next group's K/V loads in flight (two register sets), keeps the online
// softmax in registers (compute_group, attn_decode.h) and writes its output rows itself: no LDS, no
// barrier, no partials.  The 2048 units of a 256-sequence Llama-3-8B step are resident at once (two
// waves per SIMD).  The block-table row (<= 64 entries) is read once, one entry per lane, and each
// group's block number is a lane read (v_readlane) instead of a dependent load: no load in the loop
// besides the K/V stream, so the compiler's counted waits keep the next group's loads in flight.
constexpr int WAVE_UNITS = 4;  // units (waves) per workgroup

__global__ __launch_bounds__(WAVE_UNITS * 64, 2) void attn_decode_wave_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ ctx_lens, bf16* __restrict__ out, int num_units,
    int Hq, int Hkv, int BS, int max_blocks, float scale_log2) {
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * WAVE_UNITS + (threadIdx.x >> 6);
  if (unit >= num_units) return;  // uniform over the wave
  const int seq = unit / Hkv, kvh = unit - seq * Hkv;
  const int G = Hq / Hkv;
  const int c = lane & 15, h = lane >> 4;
  const int bsh = __builtin_ctz(BS);
  const int* bt = block_tables + (long long)seq * max_blocks;
  const int btv = bt[min(lane, max_blocks - 1)];  // max_blocks <= 64 (launcher)
  bf16x8 qf[4];
  load_q(q, seq, Hq, kvh, G, qf);
  const int ctx = ctx_lens[seq];
  const int ngroups = (ctx + 31) >> 5;

  auto issue = [&](int g, KVFrag& f) {
    const int tok0 = g << 5;
    const int blk = __builtin_amdgcn_readlane(btv, tok0 >> bsh);
    const int boff = tok0 & (BS - 1);
    load_group(k_cache + (((long long)blk * Hkv + kvh) * BS + boff) * D,
               v_cache + ((long long)blk * Hkv + kvh) * (long long)D * BS + boff, BS, f);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the compute (no load sinking)
  };
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  auto compute = [&](const KVFrag& f, int g) {
    const int tok0 = g << 5;
    compute_group(f, qf, scale_log2, [&](int a, int r) { return tok0 + 8 * h + 4 * a + r < ctx; }, o, m, lsum);
  };
  // two register sets: group g computes while g + 1 loads.  The prefetch is unconditional (the last
  // group is re-read past the end): a conditional one makes the compiler's wait before the compute drain
  // the prefetched loads too (vmcnt(0) at the merge point), serialising the stream.
  const int last = max(ngroups - 1, 0);
  KVFrag f0, f1;
  issue(0, f0);
  for (int g = 0; g < ngroups; g += 2) {
    issue(min(g + 1, last), f1);
    compute(f0, g);
    if (g + 1 >= ngroups) break;
    issue(min(g + 2, last), f0);
    compute(f1, g + 1);
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (c < G) {
    // lane (c, h) holds dims 16 dt + 4 h .. + 3 of query column c
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16* op = out + ((long long)seq * Hq + kvh * G + c) * D + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      union {
        uint2 u;
        bf16 h[4];
      } pk;
#pragma unroll
      for (int r = 0; r < 4; ++r) pk.h[r] = (bf16)(o[dt][r] * inv);
      *reinterpret_cast<uint2*>(op + 16 * dt) = pk.u;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Decode, long contexts: one wave per (seq, kv head, 384-token partition) streaming its K/V groups
// through a private LDS ring by LDS-DMA
// ---------------------------------------------------------------------------------------------
// The grid kernel above gives every wave ONE 32-token group: at 2K+ contexts each unit is one load round
// trip followed by a cross-wave merge and a split-KV publish, so HBM idles through the finish phases
// (2.9 TB/s at 2K in a real decode step).  Here a single-wave workgroup walks SG groups of its partition
// with up to 3 groups' K/V in flight by LDS-DMA (16 KB per group, a 64 KB ring, two workgroups per CU:
// ~96 KB in flight per CU without spending registers), reuses the group math of attn_decode.h
// (compute_group) on fragments read from the ring, and publishes one partial per 384 tokens into the same
// split-KV combine.  LDS images are XOR-swizzled so every fragment read is bank-conflict free:
//   K: 32 token rows x 256 B, 16-B chunk ^ ((t & 3) | ((t >> 4) & 1) << 3);
//   V: 128 dim rows x 64 B (32 tokens), chunk ^ {0, 2, 3, 1}[(d >> 2) & 3].
// SG: 32-token groups per streamed partition; SNS: ring slots (16 KB each: K 8 KB + V 8 KB)

SYM_DEV int kswz(int t) { return (t & 3) | (((t >> 4) & 1) << 3); }
SYM_DEV int vswz(int d) { return (0x1320 >> (4 * ((d >> 2) & 3))) & 3; }

SYM_DEV unsigned sm_addr(const char* p) {
  return (unsigned)(unsigned long long)(const __attribute__((address_space(3))) char*)p;
}

SYM_DEV void glds16(const bf16* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
SYM_DEV void wait_vm_groups() {  // all but the N youngest groups' 16 DMAs each
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
}

template <int GMAX, int SG, int SNS>
__global__ __launch_bounds__(64) void attn_decode_stream_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ ctx_lens, bf16* __restrict__ out,
    float* __restrict__ tmp_o, float* __restrict__ tmp_ml, int* __restrict__ counters, int Hq, int Hkv, int BS,
    int max_blocks, int max_parts, float scale_log2) {
  static_assert((SNS & (SNS - 1)) == 0 && SNS >= 2 && SNS <= 4 + 1, "ring slots");
  constexpr int SPART = SG * 32;
  __shared__ __attribute__((aligned(1024))) char smem[SNS * 16384];
  const int seq = blockIdx.x, kvh = blockIdx.y, part = blockIdx.z;
  const int lane = threadIdx.x;
  const int r16 = lane & 15, h = lane >> 4;
  const int G = Hq / Hkv;
  const int bsh = __builtin_ctz(BS);
  const int* bt = block_tables + (long long)seq * max_blocks;
  const int t0 = part * SPART;
  // context, this lane's block-table entry (lane g: group g of the partition) and the query are
  // independent loads: one round trip before the stream starts
  const int myblk = bt[min((t0 + 32 * min(lane, SG - 1)) >> bsh, max_blocks - 1)];
  bf16x8 qf[4];
  load_q(q, seq, Hq, kvh, G, qf);
  const int ctx = ctx_lens[seq];
  if (t0 >= ctx) return;
  const int ng = min(SG, (ctx - t0 + 31) >> 5);

  // DMA of group g into ring slot so: K rows token-major (8 x 1 KB: 4 rows of 256 B each), V rows
  // dim-major (8 x 1 KB: 16 dims x 64 B each); the swizzle permutes the SOURCE chunks, the LDS image
  // is written lane-linear
  const int kt = lane >> 4, kc = lane & 15;   // K: row within a 4-row piece, chunk
  const int vd = lane >> 2, vc = lane & 3;    // V: dim within a 16-dim piece, chunk
  auto issue = [&](int g, int so) {
    const int blk = __shfl(myblk, g, 64);
    const int boff = (t0 + 32 * g) & (BS - 1);
    const bf16* kb = k_cache + (((long long)blk * Hkv + kvh) * BS + boff) * D;
    const bf16* vb = v_cache + ((long long)blk * Hkv + kvh) * (long long)D * BS + boff;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = 4 * j + kt;
      glds16(kb + t * D + 8 * (kc ^ kswz(t)), smem + so + j * 1024);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 16 * j + vd;
      glds16(vb + (long long)d * BS + 8 * (vc ^ vswz(d)), smem + so + 8192 + j * 1024);
    }
  };

  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;

  // fragment read offsets (load_group's layouts): K row trow(a), dims 32 h + 8 i = chunk 4 h + i;
  // V row 16 dt + r16, chunk h
  const unsigned base = sm_addr(smem);
  int koff[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int trow = (r16 >> 2) * 8 + 4 * a + (r16 & 3);
    koff[a] = trow * 256;
  }
#pragma unroll
  for (int g = 0; g < SNS - 1; ++g)
    if (g < ng) issue(g, g * 16384);
  for (int g = 0; g < ng; ++g) {
    // this group's 16 DMAs landed; the (up to SNS - 2) younger groups stay in flight
    const int younger = min(ng - 1 - g, SNS - 2);
    if (younger >= 3) wait_vm_groups<3>();
    else if (younger == 2) wait_vm_groups<2>();
    else if (younger == 1) wait_vm_groups<1>();
    else wait_vm_groups<0>();
    const int so = (g & (SNS - 1)) * 16384;
    if (g + SNS - 1 < ng) issue(g + SNS - 1, ((g + SNS - 1) & (SNS - 1)) * 16384);  // slot of g - 1, read before
    KVFrag f;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int trow = (r16 >> 2) * 8 + 4 * a + (r16 & 3);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        f.k[a][i] = *(const bf16x8*)(smem + so + koff[a] + 16 * ((4 * h + i) ^ kswz(trow)));
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int d = 16 * dt + r16;
      f.v[dt] = *(const bf16x8*)(smem + so + 8192 + d * 64 + 16 * (h ^ vswz(d)));
    }
    const int tg = t0 + 32 * g;
    compute_group(f, qf, scale_log2, [&](int a, int r) { return tg + 8 * h + 4 * a + r < ctx; }, o, m, lsum);
  }
  (void)base;

  // ---- finish: one wave holds the whole partition state.  Lane (c = r16, h) owns query column c,
  // dims 16 dt + 4 h + r.
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  const int nparts = (ctx + SPART - 1) / SPART;
  const bool col = r16 < G;
  const int head = kvh * G + r16;
  if (nparts == 1) {
    if (col) {
      const float inv = 1.f / lsum;
      bf16* op = out + ((long long)seq * Hq + head) * D + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[dt][r] * inv);
        *reinterpret_cast<bf16x4*>(op + 16 * dt) = v;
      }
    }
    return;
  }
  // split-KV publish (write-through partials, drained, then the arrival counter; the last partition
  // combines: the hand-off protocol of attn_finish in attn_decode.h)
  if (col) {
    const long long pb = (((long long)seq * Hq + head) * max_parts + part);
    float* po = tmp_o + pb * D + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __hip_atomic_store(po + 16 * dt + r, o[dt][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (h == 0) {
      __hip_atomic_store(tmp_ml + pb * 2, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(tmp_ml + pb * 2 + 1, lsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int* cnt = counters + (long long)seq * Hkv + kvh;
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  if (old != nparts - 1) return;
  // combine: lane (qq = lane >> 4 within a batch of 4 query columns, 8 dims d0 = (lane & 15) * 8)
  const int d0 = (lane & 15) * 8;
  for (int c0 = 0; c0 < G; c0 += 4) {
    const int qq = c0 + (lane >> 4);
    if (qq < G) {
      const long long bb = ((long long)seq * Hq + kvh * G + qq) * max_parts;
      float M = -INFINITY, L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int p0 = 0; p0 < nparts; p0 += 4) {
        float mp[4], lp[4], vp[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int p = min(p0 + i, nparts - 1);
          mp[i] = __hip_atomic_load(tmp_ml + (bb + p) * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          lp[i] = __hip_atomic_load(tmp_ml + (bb + p) * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const float* po = tmp_o + (bb + p) * D + d0;
#pragma unroll
          for (int j = 0; j < 8; ++j) vp[i][j] = __hip_atomic_load(po + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        float mb = M;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (p0 + i < nparts) mb = fmaxf(mb, mp[i]);
        const float fo = __builtin_amdgcn_exp2f(M - mb);
        L *= fo;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] *= fo;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float f = p0 + i < nparts ? __builtin_amdgcn_exp2f(mp[i] - mb) : 0.f;
          L += lp[i] * f;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += vp[i][j] * f;
        }
        M = mb;
      }
      const float inv = 1.f / L;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
      store8(out + ((long long)seq * Hq + kvh * G + qq) * D + d0, acc);
    }
  }
  if (lane == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  if (qrow0 >= qlen) return;  // padding tile (graph-captured prefill buckets): workgroup-uniform, before any barrier
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

// ---------------------------------------------------------------------------------------------
// Prefill, 32x32x16 MFMA (K4, default for GQA groups of 4k heads): same workgroup shape as the
// LDS-staged kernel above (4 query heads of one kv head x 64 query rows, 8 waves, every K/V tile read
// from the paged cache once per workgroup and double-buffered through LDS), with the per-wave math
// re-tiled for v_mfma_f32_32x32x16_bf16 (cdna_hip_programming.md §3, T12-T14):
//   * a wave owns 32 query rows of one head; per 64-key tile it issues 16 S^T MFMAs and 16 P.V MFMAs
//     (32 cycles each); the online softmax runs per 32-key subtile over 16 scores per lane;
//   * S^T = K . Q^T with the K rows permuted (row r loads key r with bits 2 and 3 swapped) so that
//     accumulator registers 8s..8s+7 of a lane hold 8 CONSECUTIVE keys: the bf16-packed accumulator
//     is directly the B operand of O^T += V^T . P^T, and the matching V^T fragment is one contiguous
//     16-byte LDS read (no transpose, no permute);
//   * the contraction over D is permuted the same way for Q/K: lane half hh covers dims 64hh..64hh+63,
//     so a lane's K fragment reads are 128 contiguous bytes of one key row;
//   * the row max crosses lane halves with one v_permlane32_swap; exp2 is the raw v_exp_f32 with the
//     1/sqrt(D)*log2(e) scale folded into one fma; masks are evaluated only on tiles that touch the
//     causal diagonal or the context end;
//   * deferred rescale (T13): the running max moves only when a tile's max exceeds it by > 8 (log2
//     units), so O and l are rescaled on a few tiles instead of every tile (P <= 2^8 before the bf16
//     cast: relative precision unchanged);
//   * the block-table reads of a tile are issued one tile ahead of its K/V loads (a dependent
//     table -> K/V load pair per tile exposed ~2 memory latencies per iteration: 2.5x slower);
//   * heavier tiles first: the engine orders the tiles by visible keys, descending, and the grid has the
//     kv head fastest, so the long causal rows of a sequence start in the first wave of workgroups
//     instead of forming the tail (1x4096: 241 -> 162 us).
// ---------------------------------------------------------------------------------------------
SYM_DEV f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

SYM_DEV float xhalf_max(float v) {  // max with the lane 32 apart (same query column, other key half)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

SYM_DEV float xhalf_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

constexpr float kRescaleThr = 8.f;  // T13 threshold, log2 units


// ---------------------------------------------------------------------------------------------
// Prefill, 32x32x16 MFMA, software-pipelined per 32-key subtile (K4 default).
// Same workgroup / wave decomposition and operand tricks as described above, restructured so
// that a wave's VALU work hides under its own MFMAs: the online-softmax update is per 32-key subtile
// and the loop body for subtile j is
//     [rescale decision for j]  ->  S(j+1) = K . Q^T MFMAs  ||  exp2 / bf16 pack / row-sum of S(j)
//                               ->  P(j) . V MFMAs         ||  row max of S(j+1)
// (an MFMA holds the wave's issue for 8 of its 32 cycles, so independent VALU placed between MFMAs
// runs in the remaining slots; cdna_hip_programming.md T15, MI355X_MICROARCH.md cycle constants).
// Masks apply only to the <= 2 subtiles of a wave that touch the causal diagonal / context end (a
// uniform branch).  K/V tiles are TRIPLE-buffered in LDS (107.5 KB, one workgroup per CU at this
// register budget anyway): tile t+1 is resident while tile t is consumed, so S(j+1) can cross a tile
// boundary, and tile t+2's global loads are in flight for a whole iteration.
// ---------------------------------------------------------------------------------------------
SYM_DEV void s_subtile(const bf16* __restrict__ sk, const bf16x8 (&qf)[8], f32x16& acc) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int pr = (r & 3) | ((r & 4) << 1) | ((r & 8) >> 1) | (r & 16);  // bits 2 <-> 3
  const bf16* kr = sk + pr * KST + 64 * hh;
  bf16x8 kf[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) kf[kk] = *reinterpret_cast<const bf16x8*>(kr + 8 * kk);
  acc = f32x16{};
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) acc = mfma32(kf[kk], qf[kk], acc);
}

SYM_DEV void mask_subtile(f32x16& s, int kbase, int mypos) {
  const int hh = (threadIdx.x & 63) >> 5;
  const int lim = mypos - kbase - 8 * hh;  // register i holds key kbase + 16 (i >> 3) + 8 hh + (i & 7)
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (16 * (i >> 3) + (i & 7) > lim) s[i] = -INFINITY;
}

SYM_DEV float subtile_max(const f32x16& s, float scale_log2) {
  float t = fmaxf(fmaxf(s[0], s[1]), s[2]);
#pragma unroll
  for (int i = 3; i < 15; i += 2) t = fmaxf(fmaxf(t, s[i]), s[i + 1]);
  t = fmaxf(t, s[15]);
  return xhalf_max(t) * scale_log2;
}

__global__ __launch_bounds__(512, 2) void attn_prefill_m32p_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ ctx_lens, const int* __restrict__ cu_q,
    const int* __restrict__ tiles, bf16* __restrict__ out, int Hq, int Hkv, int bs_shift, int max_blocks,
    float scale_log2) {
  const int BS = 1 << bs_shift, bs_mask = BS - 1;  // power-of-two blocks: no integer division per tile
  constexpr int HPW = 4, KROWS = 32, VROWS = 64;
  constexpr int TILE_ELEMS = 64 * KST + D * VST;  // one K tile + one V^T tile
  __shared__ bf16 smem[3 * TILE_ELEMS];
  const int tile = blockIdx.y, kvh = blockIdx.x;  // tiles arrive heaviest first (engine order)
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform to the compiler
  const int c = lane & 31, hh = lane >> 5;
  const int head = kvh * G + blockIdx.z * HPW + wid % HPW;
  const int half = wid / HPW;
  const int seq = tiles[2 * tile], qrow0 = tiles[2 * tile + 1];
  const int qstart = cu_q[seq], qlen = cu_q[seq + 1] - qstart;
  const int ctx = ctx_lens[seq];
  const int pos0 = ctx - qlen;
  if (qrow0 >= qlen) return;  // padding tile (graph-captured prefill buckets): workgroup-uniform, before any barrier
  const int* bt = block_tables + (long long)seq * max_blocks;
  const int row0 = qrow0 + 32 * half;
  const int kend_wg = min(ctx, pos0 + min(qrow0 + 64, qlen));
  const bool wave_live = row0 < qlen;
  const int kend_w = min(ctx, pos0 + min(row0 + 32, qlen));  // keys [0, kend_w) visible to some row
  const int minpos_w = pos0 + row0;                           // the wave's first query position
  const int nsub = wave_live ? (kend_w + 31) >> 5 : 0;        // 32-key subtiles this wave processes
  const int myrow = row0 + c;
  const bool row_ok = myrow < qlen;
  const int mypos = row_ok ? pos0 + myrow : ctx - 1;  // rows past the prompt attend like the last one

  bf16x8 qf[8];
  if (row_ok) {
    const bf16* qp = q + ((long long)(qstart + myrow) * Hq + head) * D + 64 * hh;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) qf[kk] = ld16(qp + 8 * kk);
  } else {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) qf[kk] = zero8();
  }
  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x16{};
  float m = -INFINITY, lsum = 0.f;

  // Cooperative tile staging: 2 x 16 B of K and of V per thread.  The paged-cache block ids of a tile are
  // fetched one tile AHEAD of its K/V loads, so issuing those loads never waits on a block-table read.
  // Keys past the context read the block of the last key (finite: the cache is zero-initialised and only
  // ever written with finite K/V; masked anyway).
  const int ck = threadIdx.x >> 4, pk = (threadIdx.x & 15) * 8;
  const int dv = threadIdx.x >> 3, tv8 = 8 * (threadIdx.x & 7);
  const long long kvoff = (long long)kvh * BS * D;
  const size_t bstride = (size_t)Hkv * BS * D;
  const int last = ctx - 1;
  const int ntiles = (kend_wg + 63) / 64;
  struct Ids { int k0, k1, v; };
  struct Stage { uint4 k0, k1, v0, v1; };
  auto fetch_ids = [&](int t0) {
    return Ids{bt[min(t0 + ck, last) >> bs_shift], bt[min(t0 + ck + KROWS, last) >> bs_shift],
               bt[min(t0 + tv8, last) >> bs_shift]};
  };
  // per-thread constant parts of the K / V addresses (elements)
  const bf16* kbase = k_cache + kvoff + pk;
  const bf16* vbase = v_cache + kvoff + (long long)dv * BS;
  auto issue = [&](int t0, const Ids& id) {
    const int k0 = min(t0 + ck, last), k1 = min(t0 + ck + KROWS, last), v0 = min(t0 + tv8, last & ~7);
    Stage st;
    st.k0 = *reinterpret_cast<const uint4*>(kbase + (size_t)(unsigned)id.k0 * bstride + ((k0 & bs_mask) << 7));
    st.k1 = *reinterpret_cast<const uint4*>(kbase + (size_t)(unsigned)id.k1 * bstride + ((k1 & bs_mask) << 7));
    const bf16* vb = vbase + (size_t)(unsigned)id.v * bstride + (v0 & bs_mask);
    st.v0 = *reinterpret_cast<const uint4*>(vb);
    st.v1 = *reinterpret_cast<const uint4*>(vb + VROWS * BS);
    return st;
  };
  auto store = [&](int t, const Stage& st) {
    bf16* sk = smem + (t % 3) * TILE_ELEMS;
    bf16* sv = sk + 64 * KST;
    *reinterpret_cast<uint4*>(sk + ck * KST + pk) = st.k0;
    *reinterpret_cast<uint4*>(sk + (ck + KROWS) * KST + pk) = st.k1;
    *reinterpret_cast<uint4*>(sv + dv * VST + tv8) = st.v0;
    *reinterpret_cast<uint4*>(sv + (dv + VROWS) * VST + tv8) = st.v1;
  };

  // prologue: tiles 0 and 1 loaded together (one memory round trip), tile 2's loads in flight
  Stage stg;
  Ids ids;
  if (ntiles > 0) {
    const Ids i0 = fetch_ids(0), i1 = fetch_ids(ntiles > 1 ? 64 : 0);
    stg = issue(0, i0);
    Stage s1;
    if (ntiles > 1) s1 = issue(64, i1);
    if (ntiles > 2) ids = fetch_ids(128);
    store(0, stg);
    if (ntiles > 1) store(1, s1);
  }
  __syncthreads();
  if (ntiles > 2) {
    stg = issue(128, ids);
    if (ntiles > 3) ids = fetch_ids(192);
  }

  f32x16 sa, sb;  // scores of the current / next subtile (named: static register allocation)
  float tmax = -INFINITY;
  if (nsub > 0) {
    s_subtile(smem, qf, sa);
    tmax = subtile_max(sa, scale_log2);
  }

  // one subtile step: j = 2 it + ST, current scores in SC, next into SN
#define SUBTILE_STEP(ST, SC, SN)                                                                          \
  do {                                                                                                    \
    const int j = 2 * it + (ST);                                                                          \
    if (j < nsub) {                                                                                       \
      if (32 * j + 31 > minpos_w) { /* diagonal / context-end subtile: mask, then its true max */         \
        mask_subtile(SC, 32 * j, mypos);                                                                  \
        tmax = subtile_max(SC, scale_log2);                                                               \
      }                                                                                                   \
      if (!__all(tmax <= m + kRescaleThr)) {                                                              \
        const float mn = fmaxf(m, tmax);                                                                  \
        const float alpha = __builtin_amdgcn_exp2f(m - mn); /* first subtile: m = -inf, alpha = 0 */      \
        m = mn;                                                                                           \
        lsum *= alpha;                                                                                    \
        _Pragma("unroll") for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;                                  \
      }                                                                                                   \
      /* branch-free from here: S(j+1) unconditionally (past the wave's last subtile it is an unused */   \
      /* stale-LDS product) so the exps of S(j) interleave with its MFMAs, and S(j+1)'s row max with */   \
      /* the P.V MFMAs (an upper bound until a masked subtile recomputes it above) */                    \
      s_subtile((ST) == 0 ? cur_k + 32 * KST : nxt_k, qf, SN);                                            \
      Pack8 pf[2];                                                                                        \
      float psum = 0.f;                                                                                   \
      _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                                    \
        const float p = __builtin_amdgcn_exp2f(fmaf(SC[i], scale_log2, -m));                              \
        psum += p;                                                                                        \
        pf[i >> 3].h[i & 7] = (bf16)p;                                                                    \
      }                                                                                                   \
      lsum += psum;                                                                                       \
      _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                                    \
        _Pragma("unroll") for (int dt = 0; dt < 4; ++dt) {                                                \
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(cur_v + (32 * dt + c) * VST + 32 * (ST) +    \
                                                             16 * ks + 8 * hh);                           \
          o[dt] = mfma32(vf, pf[ks].v, o[dt]);                                                            \
        }                                                                                                 \
      tmax = subtile_max(SN, scale_log2);                                                                 \
    }                                                                                                     \
  } while (0)

  for (int it = 0; it < ntiles; ++it) {
    const bf16* cur_k = smem + (it % 3) * TILE_ELEMS;
    const bf16* cur_v = cur_k + 64 * KST;
    const bf16* nxt_k = smem + ((it + 1) % 3) * TILE_ELEMS;
    SUBTILE_STEP(0, sa, sb);
    SUBTILE_STEP(1, sb, sa);
    if (it + 2 < ntiles) store(it + 2, stg);
    __syncthreads();
    if (it + 3 < ntiles) {
      stg = issue(64 * (it + 3), ids);
      if (it + 4 < ntiles) ids = fetch_ids(64 * (it + 4));
    }
  }
#undef SUBTILE_STEP
  const float l = xhalf_sum(lsum);
  if (!row_ok) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  bf16* op = out + ((long long)(qstart + myrow) * Hq + head) * D + 4 * hh;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (bf16)(o[dt][4 * g + e] * inv);
      *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * g) = v;
    }
}

}  // namespace

static int g_attn_stream_min = [] {
  const char* knob = getenv("SYMMETRY_ATTN_STREAM_MIN");
  return knob ? atoi(knob) : 1024;
}();

void set_attn_stream_min(int tokens) { g_attn_stream_min = tokens; }

// wide batches: the one-wave-per-(seq, kv head) kernel from this many units (seqs x kv heads) for block
// tables spanning at least this many tokens (and <= 64 blocks).  bench_attn_decode.py --wave 0 1
// (profiles/attn_decode_wave_r2.jsonl): at >= 128 sequences x 700-3000 tokens it streams K/V at 5.1-5.9 TB/s
// vs 4.3-5.0 for the grid / streaming kernels (-8..-20 %); at 64 sequences, or ~170-token contexts in the
// 512-token bucket, those stay ahead.  SYMMETRY_ATTN_WAVE_UNITS (0: never) / SYMMETRY_ATTN_WAVE_SPAN.
static int g_attn_wave_units = [] {
  const char* knob = getenv("SYMMETRY_ATTN_WAVE_UNITS");
  return knob ? atoi(knob) : 1024;
}();
static int g_attn_wave_span = [] {
  const char* knob = getenv("SYMMETRY_ATTN_WAVE_SPAN");
  return knob ? atoi(knob) : 513;
}();

void set_attn_wave(int min_units, int min_span) {
  g_attn_wave_units = min_units;
  g_attn_wave_span = min_span;
}

// A/B knob (partition length x ring depth of the streaming kernel): SYMMETRY_ATTN_STREAM_CFG
static int g_attn_stream_cfg = [] {
  const char* knob = getenv("SYMMETRY_ATTN_STREAM_CFG");
  return knob ? atoi(knob) : 0;
}();

void launch_attn_decode(const bf16* q, const bf16* k_cache, const bf16* v_cache, const int* block_tables,
                        const int* ctx_lens, bf16* out, float* tmp_o, float* tmp_ml, int* counters, int num_seqs,
                        int Hq, int Hkv, int BS, int max_blocks, int max_parts, float scale, hipStream_t s) {
  if (num_seqs == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  // block tables spanning >= g_attn_stream_min tokens (the graph's context bucket): the streaming
  // one-wave kernel
  const int span = max_blocks * BS;
  if (g_attn_wave_units > 0 && num_seqs * Hkv >= g_attn_wave_units && span >= g_attn_wave_span && G <= 16 &&
      max_blocks <= 64) {
    const int units = num_seqs * Hkv;
    attn_decode_wave_kernel<<<(units + WAVE_UNITS - 1) / WAVE_UNITS, WAVE_UNITS * 64, 0, s>>>(
        q, k_cache, v_cache, block_tables, ctx_lens, out, units, Hq, Hkv, BS, max_blocks, scale_log2);
    return;
  }
  if (g_attn_stream_min > 0 && span >= g_attn_stream_min && BS >= 32 && G <= 16) {
    // partitions of SG 32-token groups (>= 256 tokens: sparts <= max_parts, sized for 256-token ones)
    auto run = [&](auto kern, int sg) {
      const dim3 g(num_seqs, Hkv, (span + 32 * sg - 1) / (32 * sg));
      kern<<<g, 64, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml, counters, Hq, Hkv, BS,
                            max_blocks, max_parts, scale_log2);
    };
    switch (g_attn_stream_cfg) {
      case 1: run(attn_decode_stream_kernel<16, 8, 4>, 8); break;
      case 2: run(attn_decode_stream_kernel<16, 12, 2>, 12); break;
      case 3: run(attn_decode_stream_kernel<16, 24, 4>, 24); break;
      case 4: run(attn_decode_stream_kernel<16, 16, 4>, 16); break;
      case 5: run(attn_decode_stream_kernel<16, 8, 2>, 8); break;
      default: run(attn_decode_stream_kernel<16, 12, 4>, 12); break;
    }
    return;
  }
  dim3 grid(num_seqs, Hkv, max_parts);
  if (G <= 4)
    attn_decode_kernel<4><<<grid, DWAVES * 64, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml,
                                                       counters, Hq, Hkv, BS, max_blocks, max_parts, scale_log2);
  else if (G <= 8)
    attn_decode_kernel<8><<<grid, DWAVES * 64, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml,
                                                       counters, Hq, Hkv, BS, max_blocks, max_parts, scale_log2);
  else
    attn_decode_kernel<16><<<grid, DWAVES * 64, 0, s>>>(q, k_cache, v_cache, block_tables, ctx_lens, out, tmp_o, tmp_ml,
                                                        counters, Hq, Hkv, BS, max_blocks, max_parts, scale_log2);
}

void launch_attn_prefill(const bf16* q, const bf16* k_cache, const bf16* v_cache, const int* block_tables,
                         const int* ctx_lens, const int* cu_q, const int* tiles, int num_tiles, bf16* out, int Hq,
                         int Hkv, int BS, int max_blocks, float scale, hipStream_t s) {
  if (num_tiles == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  // A/B knob SYMMETRY_ATTN_PREFILL=lds: the previous 16x16x32 LDS kernel (profiles/attn_prefill_r1.jsonl)
  static const char* knob = getenv("SYMMETRY_ATTN_PREFILL");
  static const bool use_lds = knob && strstr(knob, "lds");
  if (!use_lds && BS >= 8 && (BS & (BS - 1)) == 0 && G % 4 == 0) {
    attn_prefill_m32p_kernel<<<dim3(Hkv, num_tiles, G / 4), 512, 0, s>>>(
        q, k_cache, v_cache, block_tables, ctx_lens, cu_q, tiles, out, Hq, Hkv, __builtin_ctz(BS), max_blocks,
        scale_log2);
    return;
  }
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
