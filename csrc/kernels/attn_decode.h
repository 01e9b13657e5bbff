// Decode attention building blocks of the split-KV kernel (attention.hip).
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

// Cross-wave finish of one (seq, kv head, partition) unit: the 8 waves' online-softmax states are merged
// through LDS; a single-partition context writes its output rows, a multi-partition one publishes fp32
// partials and the last-arriving partition combines them (split-KV, flash-decoding, one launch).
// GMAX >= G query columns are staged.  Returns true on the workgroup that stored final rows (uniform over
// the workgroup).
template <int GMAX>
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
  attn_finish<GMAX>(o, m, lsum, ctx, PART, seq, kvh, part, Hq, Hkv, max_parts, out, tmp_o, tmp_ml, counters);
}


}  // namespace
