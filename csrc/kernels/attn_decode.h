// Decode attention building blocks shared by the standalone split-KV kernel (attention.hip) and the
// fused QKV -> attention -> O-projection launch (decode_gemm.hip, decode_block_kernel).
// Math, layouts and the MFMA operand tricks are described at the top of attention.hip.
#pragma once
#include "common.h"

namespace {

constexpr int D = 128;
constexpr int DWAVES = 8;            // waves per decode workgroup
constexpr int PART = DWAVES * 32;    // tokens per decode partition (one 32-token group per wave): contexts
                                     // <= 256 need no combine; ~120 VGPRs -> two workgroups per CU, so one
                                     // unit's loads overlap another's finish (bench_attn_decode.py)

SYM_DEV bf16x8 ld16(const bf16* p) {
  Pack8 pk;
  pk.u = *reinterpret_cast<const uint4*>(p);
  return pk.v;
}

SYM_DEV bf16x8 zero8() {
  Pack8 pk;
  pk.u = make_uint4(0, 0, 0, 0);
  return pk.v;
}

// One 32-token group: S^T for two 16-token tiles, online softmax update, P.V.
// Split into a load phase (K and V fragments of the group to registers) and a compute phase so that
// callers can have the next group's loads in flight while computing the current one.
struct KVFrag {
  bf16x8 k[2][4];  // two 16-token S^T tiles x 4 D-slices
  bf16x8 v[8];     // 8 dim tiles of V^T
};

SYM_DEV void load_group(const bf16* __restrict__ kb, const bf16* __restrict__ vb, int BS, KVFrag& f) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, h = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int trow = (r16 >> 2) * 8 + 4 * a + (r16 & 3);
    const bf16* kr = kb + (long long)trow * D + 32 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) f.k[a][i] = ld16(kr + 8 * i);
  }
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) f.v[dt] = ld16(vb + (long long)(16 * dt + r16) * BS + 8 * h);
}

// `valid(a, r)` tells whether token (8h + 4a + r) of the group is visible to this lane's query column.
template <typename ValidFn>
SYM_DEV void compute_group(const KVFrag& f, const bf16x8 (&qf)[4], float scale_log2, ValidFn valid, f32x4 (&o)[8],
                           float& m, float& lsum) {
  f32x4 s[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = mfma16(f.k[a][i], qf[i], acc);
    s[a] = acc;
  }
  float x[8];
  float gmax = -INFINITY;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = valid(a, r) ? s[a][r] * scale_log2 : -INFINITY;
      x[4 * a + r] = v;
      gmax = fmaxf(gmax, v);
    }
  gmax = fmaxf(gmax, __shfl_xor(gmax, 16, 64));
  gmax = fmaxf(gmax, __shfl_xor(gmax, 32, 64));
  const float m_new = fmaxf(m, gmax);
  // m_new == -inf only if this column saw no visible token yet (causal prefill rows); keep zeros.
  // raw v_exp_f32 (the ocml exp2f adds a denormal range reduction softmax does not need)
  const float alpha = (m_new == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(m - m_new);
  Pack8 pf;
  float psum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float p = (m_new == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(x[j] - m_new);
    psum += p;
    pf.h[j] = (bf16)p;
  }
  lsum = lsum * alpha + psum;
  m = m_new;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    o[dt] *= alpha;
    o[dt] = mfma16(f.v[dt], pf.v, o[dt]);
  }
}

SYM_DEV void store8_sc1(bf16* p, const float* f) {
  // 16 B of bf16 as two 8-byte write-through (sc1) stores: read inside the same launch by another CU
  Pack8 pk;
#pragma unroll
  for (int i = 0; i < 8; ++i) pk.h[i] = (bf16)f[i];
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  __hip_atomic_store(q, ((unsigned long long)pk.u.y << 32) | pk.u.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, ((unsigned long long)pk.u.w << 32) | pk.u.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct AttnNoWait {
  SYM_DEV void operator()() const {}
};

// Cross-wave finish of one (seq, kv head, partition) unit: the 8 waves' online-softmax states are merged
// through LDS; a single-partition context writes its output rows, a multi-partition one publishes fp32
// partials and the last-arriving partition combines them (split-KV, flash-decoding, one launch).
// GMAX >= G query columns are staged (the fused block launch keeps LDS small with GMAX = 8).  kSc1:
// final rows are stored write-through (read by another CU of the same launch).  Returns true on the
// workgroup that stored final rows (uniform over the workgroup).
template <int GMAX, bool kSc1>
SYM_DEV bool attn_finish(const f32x4 (&o)[8], float m, float lsum, int ctx, int part_tokens, int seq, int kvh,
                         int part, int Hq, int Hkv, int max_parts, bf16* __restrict__ out, float* __restrict__ tmp_o,
                         float* __restrict__ tmp_ml, int* __restrict__ counters) {
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 15, h = lane >> 4;
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);

  __shared__ float sm_m[DWAVES][GMAX], sm_l[DWAVES][GMAX];
  __shared__ float sm_o[DWAVES][GMAX][D + 4];
  if (c < GMAX) {
    if (h == 0) {
      sm_m[wid][c] = m;
      sm_l[wid][c] = lsum;
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) sm_o[wid][c][16 * dt + 4 * h + r] = o[dt][r];
  }
  __syncthreads();

  // Combine the waves' partial softmax states: thread (qq, d0) owns 8 dims of query column qq.
  const int qq = threadIdx.x >> 4;        // 0..15 query column
  const int d0 = (threadIdx.x & 15) * 8;  // 8 dims per thread
  const bool active = qq < G && qq < GMAX;
  const int head = kvh * G + qq;
  const int nparts = (ctx + part_tokens - 1) / part_tokens;
  float M = -INFINITY, L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
#pragma unroll
    for (int w = 0; w < DWAVES; ++w) M = fmaxf(M, sm_m[w][qq]);
#pragma unroll
    for (int w = 0; w < DWAVES; ++w) {
      const float mw = sm_m[w][qq];
      const float f = (mw == -INFINITY) ? 0.f : exp2f(mw - M);
      L += sm_l[w][qq] * f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += sm_o[w][qq][d0 + j] * f;
    }
  }
  auto store_out = [&](float* a) {
    bf16* op = out + ((long long)seq * Hq + head) * D + d0;
    if constexpr (kSc1)
      store8_sc1(op, a);
    else
      store8(op, a);
  };
  if (nparts == 1) {  // uniform over the workgroup
    if (active) {
      const float inv = 1.f / L;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
      store_out(acc);
    }
    return true;
  }
  // Split-KV combine in the same launch (no reduce kernel): every partition publishes its partial
  // state with write-through (sc1) stores, drains them (vmcnt(0)), then bumps the (seq, kv head)
  // arrival counter; the workgroup whose add returns nparts - 1 reads all partials back with sc1
  // loads and writes the output, then re-arms the counter to 0 (graph-replay safe, no memset).
  // MI355X_MICROARCH.md hand-off table: sc1 stores + agent atomic add + sc1 loads, hipMalloc memory.
  const long long base = ((long long)seq * Hq + head) * max_parts;
  if (active) {
    float* po = tmp_o + (base + part) * D + d0;
#pragma unroll
    for (int j = 0; j < 8; ++j) __hip_atomic_store(po + j, acc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d0 == 0) {
      __hip_atomic_store(tmp_ml + (base + part) * 2, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(tmp_ml + (base + part) * 2 + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ int s_last;
  __syncthreads();
  int* cnt = counters + (long long)seq * Hkv + kvh;
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == nparts - 1;
  }
  __syncthreads();
  if (!s_last) return false;
  if (active) {
    // partials read 4 partitions at a time (40 independent loads in flight per batch) with an online
    // max: one memory round trip per 4 partitions instead of a dependent load chain per partition
    M = -INFINITY;
    L = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int p0 = 0; p0 < nparts; p0 += 4) {
      float mp[4], lp[4], vp[4][8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = min(p0 + i, nparts - 1);  // duplicates past the end are masked below
        mp[i] = __hip_atomic_load(tmp_ml + (base + p) * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lp[i] = __hip_atomic_load(tmp_ml + (base + p) * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float* po = tmp_o + (base + p) * D + d0;
#pragma unroll
        for (int j = 0; j < 8; ++j) vp[i][j] = __hip_atomic_load(po + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      float mb = M;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (p0 + i < nparts) mb = fmaxf(mb, mp[i]);
      const float fo = __builtin_amdgcn_exp2f(M - mb);  // M = -inf on the first batch: 0
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
    store_out(acc);
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

SYM_DEV void load_q(const bf16* __restrict__ q, int seq, int Hq, int kvh, int G, bf16x8 (&qf)[4]) {
  const int lane = threadIdx.x & 63;
  const int c = lane & 15, h = lane >> 4;
  if (c < G) {
    const bf16* qp = q + ((long long)seq * Hq + kvh * G + c) * D + 32 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = ld16(qp + 8 * i);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = zero8();
  }
}

// Standalone split-KV decode attention unit (seq, kv_head, partition) on an 8-wave workgroup: 8 waves x
// 64 tokens = one 512-token partition; the G = Hq/Hkv query heads of the kv head are the MFMA columns.
template <int GMAX>
SYM_DEV void attn_decode_unit(const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
                              const bf16* __restrict__ v_cache, const int* __restrict__ block_tables,
                              const int* __restrict__ ctx_lens, bf16* __restrict__ out, float* __restrict__ tmp_o,
                              float* __restrict__ tmp_ml, int* __restrict__ counters, int Hq, int Hkv, int BS,
                              int max_blocks, int max_parts, float scale_log2, int seq, int kvh, int part) {
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int h = lane >> 4;
  // The context length, this wave's block-table entries and the query fragments are independent
  // loads: issue all of them before the first use so the kernel pays one memory round trip before
  // the K/V stream instead of three (ctx -> block table -> K/V).  Entries past the context are
  // fetched (in-bounds: clamped to the row) but never dereferenced.
  const int* bt = block_tables + (long long)seq * max_blocks;
  const int tok0 = part * PART + wid * 32;
  const int bsh = __builtin_ctz(BS);  // block sizes are powers of two (launchers check)
  const int blk = bt[min(tok0 >> bsh, max_blocks - 1)];
  bf16x8 qf[4];
  load_q(q, seq, Hq, kvh, G, qf);
  const int ctx = ctx_lens[seq];
  if (part * PART >= ctx) return;
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  if (tok0 < ctx) {
    KVFrag f;
    const int boff = tok0 & (BS - 1);
    load_group(k_cache + (((long long)blk * Hkv + kvh) * BS + boff) * D,
               v_cache + ((long long)blk * Hkv + kvh) * (long long)D * BS + boff, BS, f);
    compute_group(f, qf, scale_log2, [&](int a, int r) { return tok0 + 8 * h + 4 * a + r < ctx; }, o, m, lsum);
  }
  attn_finish<GMAX, false>(o, m, lsum, ctx, PART, seq, kvh, part, Hq, Hkv, max_parts, out, tmp_o, tmp_ml, counters);
}

// Attention unit of the fused decode block launch (decode_gemm.hip, decode_block_kernel): 8 waves x ONE
// 32-token group = 256-token partitions, so a wave's whole K/V slice fits in registers next to the GEMM
// roles' budget and is loaded BEFORE `wait` (the poll for this kv group's QKV tiles): only the query and
// the group holding the newest token (written by this launch's QKV tiles) are read after it, so the
// attention phase costs one memory round trip after the QKV phase instead of three.
constexpr int PART_F = DWAVES * 32;

template <int GMAX, typename WaitFn>
SYM_DEV bool attn_fused_unit(const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
                             const bf16* __restrict__ v_cache, const int* __restrict__ block_tables,
                             const int* __restrict__ ctx_lens, bf16* __restrict__ out, float* __restrict__ tmp_o,
                             float* __restrict__ tmp_ml, int* __restrict__ counters, int Hq, int Hkv, int BS,
                             int max_blocks, int max_parts, float scale_log2, int seq, int kvh, int part,
                             WaitFn wait) {
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int h = lane >> 4;
  const int* bt = block_tables + (long long)seq * max_blocks;
  const int tok0 = part * PART_F + wid * 32;
  const int blk = bt[min(tok0 >> __builtin_ctz(BS), max_blocks - 1)];
  const int ctx = ctx_lens[seq];
  if (part * PART_F >= ctx) return false;
  const bool has = tok0 < ctx;
  const bool newest = has && ctx - 1 < tok0 + 32;  // this wave's group holds the token written this step
  const bf16* kb = k_cache + (((long long)blk * Hkv + kvh) * BS + (tok0 & (BS - 1))) * D;
  const bf16* vb = v_cache + ((long long)blk * Hkv + kvh) * (long long)D * BS + (tok0 & (BS - 1));
  KVFrag f;
  if (has && !newest) load_group(kb, vb, BS, f);  // bytes no workgroup of this launch writes
  wait();
  bf16x8 qf[4];
  load_q(q, seq, Hq, kvh, G, qf);
  if (newest) load_group(kb, vb, BS, f);
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  if (has) compute_group(f, qf, scale_log2, [&](int a, int r) { return tok0 + 8 * h + 4 * a + r < ctx; }, o, m, lsum);
  return attn_finish<GMAX, true>(o, m, lsum, ctx, PART_F, seq, kvh, part, Hq, Hkv, max_parts, out, tmp_o, tmp_ml,
                                 counters);
}

// ---------------------------------------------------------------------------------------------------
// Two 8-wave attention units per 16-wave workgroup: the attention role of the fused QKV + attention launch
// (decode_gemm.hip, decode_qkv_attn_kernel).  Half = wave / 8 runs unit u = 2 * pair + half (units numbered
// partition-major: (part, seq, kv head), 256-token partitions, one 32-token group per wave).
//   * before `wait` (the poll for "every QKV workgroup has stored its tiles"): the context length, the
//     block-table entry and the K/V of every group except the one holding the newest token -- bytes no
//     workgroup of this launch writes;
//   * after it: the query and the newest group's K/V, which the QKV epilogue stored write-through (sc1),
//     read with sc1 (L1-bypassing) loads -- every load of handed-off bytes is one, so no acquire fence is
//     needed (MI355X_MICROARCH.md hand-off table, first row) and an older group's line that shares a V
//     cache line with the newest token (64-token blocks) can never serve a stale copy from L1;
//   * the cross-wave merge and the split-KV combine of attn_finish, with every workgroup barrier executed
//     by both halves unconditionally (a unit past its context joins them with nothing to do), so two units
//     with different partition counts never disagree on the barrier count.
// ---------------------------------------------------------------------------------------------------
SYM_DEV bf16x8 ld16_sc1v(const bf16* p) {  // 16 B as two 8-byte sc1 loads
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  const unsigned long long lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  Pack8 pk;
  pk.u = make_uint4((unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32));
  return pk.v;
}

SYM_DEV void load_group_sc1(const bf16* __restrict__ kb, const bf16* __restrict__ vb, int BS, KVFrag& f) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, h = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int trow = (r16 >> 2) * 8 + 4 * a + (r16 & 3);
    const bf16* kr = kb + (long long)trow * D + 32 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) f.k[a][i] = ld16_sc1v(kr + 8 * i);
  }
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) f.v[dt] = ld16_sc1v(vb + (long long)(16 * dt + r16) * BS + 8 * h);
}

template <int GMAX, typename WaitFn>
SYM_DEV void attn_pair_units(const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
                             const bf16* __restrict__ v_cache, const int* __restrict__ block_tables,
                             const int* __restrict__ ctx_lens, bf16* __restrict__ out, float* __restrict__ tmp_o,
                             float* __restrict__ tmp_ml, int* __restrict__ counters, int Hq, int Hkv, int BS,
                             int max_blocks, int max_parts, float scale_log2, int M, int pair, WaitFn wait) {
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int half = wid >> 3, lw = wid & 7;
  const int c = lane & 15, h = lane >> 4;
  const int per_part = M * Hkv;
  const int u = 2 * pair + half;
  const bool valid = u < per_part * max_parts;
  const int part = valid ? u / per_part : 0;
  const int seq = valid ? (u % per_part) / Hkv : 0, kvh = valid ? u % Hkv : 0;
  const int* bt = block_tables + (long long)seq * max_blocks;
  const int tok0 = part * PART_F + lw * 32;
  const int blk = bt[min(tok0 >> __builtin_ctz(BS), max_blocks - 1)];
  const int ctx = valid ? ctx_lens[seq] : 0;
  const bool active = valid && part * PART_F < ctx;
  const bool has = active && tok0 < ctx;
  const bool newest = has && ctx - 1 < tok0 + 32;  // this wave's group holds the token written this step
  const bf16* kb = k_cache + (((long long)blk * Hkv + kvh) * BS + (tok0 & (BS - 1))) * D;
  const bf16* vb = v_cache + ((long long)blk * Hkv + kvh) * (long long)D * BS + (tok0 & (BS - 1));
  KVFrag f;
  if (has && !newest) load_group(kb, vb, BS, f);  // bytes no workgroup of this launch writes
  wait();
  bf16x8 qf[4];
  if (active && c < G) {
    const bf16* qp = q + ((long long)seq * Hq + kvh * G + c) * D + 32 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = ld16_sc1v(qp + 8 * i);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = zero8();
  }
  if (newest) load_group_sc1(kb, vb, BS, f);
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  if (has) compute_group(f, qf, scale_log2, [&](int a, int r) { return tok0 + 8 * h + 4 * a + r < ctx; }, o, m, lsum);
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);

  __shared__ float pm[2][DWAVES][GMAX], pl[2][DWAVES][GMAX];
  __shared__ float po[2][DWAVES][GMAX][D + 4];
  __shared__ int plast[2];
  if (c < GMAX) {
    if (h == 0) {
      pm[half][lw][c] = m;
      pl[half][lw][c] = lsum;
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) po[half][lw][c][16 * dt + 4 * h + r] = o[dt][r];
  }
  __syncthreads();
  const int tid = threadIdx.x & 511;  // thread within the half
  const int qq = tid >> 4, d0 = (tid & 15) * 8;
  const bool act = active && qq < G && qq < GMAX;
  const int head = kvh * G + qq;
  const int nparts = active ? (ctx + PART_F - 1) / PART_F : 1;
  float Mx = -INFINITY, L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (act) {
#pragma unroll
    for (int w = 0; w < DWAVES; ++w) Mx = fmaxf(Mx, pm[half][w][qq]);
#pragma unroll
    for (int w = 0; w < DWAVES; ++w) {
      const float mw = pm[half][w][qq];
      const float fw = (mw == -INFINITY) ? 0.f : exp2f(mw - Mx);
      L += pl[half][w][qq] * fw;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += po[half][w][qq][d0 + j] * fw;
    }
  }
  bf16* op = out + ((long long)seq * Hq + head) * D + d0;  // read by the next launch: plain stores
  const long long base = ((long long)seq * Hq + head) * max_parts;
  if (act && nparts == 1) {
    const float inv = 1.f / L;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
    store8(op, acc);
  } else if (act) {  // split-KV partial (write-through), combined by the last-arriving partition below
    float* pp = tmp_o + (base + part) * D + d0;
#pragma unroll
    for (int j = 0; j < 8; ++j) __hip_atomic_store(pp + j, acc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d0 == 0) {
      __hip_atomic_store(tmp_ml + (base + part) * 2, Mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(tmp_ml + (base + part) * 2 + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* cnt = counters + (long long)seq * Hkv + kvh;
  if (tid == 0)
    plast[half] = (active && nparts > 1)
                      ? __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nparts - 1
                      : 0;
  __syncthreads();
  if (!plast[half]) return;  // (no barrier below)
  if (act) {
    Mx = -INFINITY;
    L = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int p0 = 0; p0 < nparts; p0 += 4) {
      float mp[4], lp[4], vp[4][8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = min(p0 + i, nparts - 1);
        mp[i] = __hip_atomic_load(tmp_ml + (base + p) * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lp[i] = __hip_atomic_load(tmp_ml + (base + p) * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float* pp = tmp_o + (base + p) * D + d0;
#pragma unroll
        for (int j = 0; j < 8; ++j) vp[i][j] = __hip_atomic_load(pp + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      float mb = Mx;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (p0 + i < nparts) mb = fmaxf(mb, mp[i]);
      const float fo = __builtin_amdgcn_exp2f(Mx - mb);
      L *= fo;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= fo;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float fw = p0 + i < nparts ? __builtin_amdgcn_exp2f(mp[i] - mb) : 0.f;
        L += lp[i] * fw;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += vp[i][j] * fw;
      }
      Mx = mb;
    }
    const float inv = 1.f / L;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
    store8(op, acc);
  }
  if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


}  // namespace
