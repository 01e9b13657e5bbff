// Epilogues of the fused decode GEMMs (decode_gemm.hip) and of the medium-M GEMM's in-launch split-K
// reduction (mgemm.hip): one finished 16x16 accumulator tile in MFMA layout -- lane (r16, h) holds weight
// rows (output features) n0 + 4h .. n0 + 4h + 3 of token row m -- turned into the consumer's output
// (fp32 y, QKV RoPE + paged K/V write, residual add + next-norm prep, SwiGLU, fused sampling keys, or the
// xGMI push of a row-parallel projection under TP).
#pragma once

#include "common.h"
#include "launchers.h"
#include "xgmi_proto.h"

namespace {

SYM_DEV uint32_t ordered_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

SYM_DEV unsigned long long pack_key(float v, uint32_t idx) {
  return ((unsigned long long)ordered_bits(v) << 32) | (unsigned long long)(0xFFFFFFFFu - idx);
}

SYM_DEV void store4bf(bf16* p, float a, float b, float c, float d) {
  bf16x4 v;
  v[0] = (bf16)a;
  v[1] = (bf16)b;
  v[2] = (bf16)c;
  v[3] = (bf16)d;
  *reinterpret_cast<bf16x4*>(p) = v;
}

// Epilogue of one finished 16x16 accumulator tile (rows n0.., columns = token rows 16*mt..).
// Lane (r16, h) holds rows n0 + 4h .. n0 + 4h + 3 of token row m = 16 * mt + r16.
// 4 bf16 as one 8-byte write-through (sc1) store: visible to a consumer on another XCD once the
// storing wave's vmcnt has drained (MI355X_MICROARCH.md hand-off table)
SYM_DEV void store4bf_sc1(bf16* p, float a, float b, float c, float d) {
  Pack8 pk;
  pk.h[0] = (bf16)a;
  pk.h[1] = (bf16)b;
  pk.h[2] = (bf16)c;
  pk.h[3] = (bf16)d;
  const unsigned long long v = ((unsigned long long)pk.u.y << 32) | pk.u.x;
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- XAR (row-parallel projection under TP, all-reduced inside the GEMM launch) ----------------------------
// Granules of 8 B {fp32 value, u32 tag = collective epoch} in the XAR communicator's slot (parity, source):
// granule (m, n) at byte (m N + n) * 8.  A lane pushes its 4 values to every OTHER rank with 8-B stores (one
// single-copy-atomic write each, no flag, no ack wait), then polls the other ranks' granules of the same
// columns until their tags equal this epoch, and sums all ranks' values in rank order (its own from
// registers: the same fp32 bits the peers receive), so every rank gets bit-identical sums.  A stale granule
// (an older epoch of the same parity) never matches; the communicator carries nothing but XAR granules.
SYM_DEV long long xar_goff(int m, int N, int n) { return ((long long)m * N + n) * 8; }

SYM_DEV void xar_push(const XgmiArgs& c, const f32x4& v, long long goff, unsigned ep) {
  const int par = (int)(ep & 1u);
  for (int r = 0; r < c.world; ++r) {
    if (r == c.rank) continue;
    unsigned long long* d = reinterpret_cast<unsigned long long*>(c.bufs[r] + XG_FLAG_BYTES +
                                                                 ((long long)par * c.world + c.rank) * c.slot_bytes + goff);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __hip_atomic_store(d + i, ((unsigned long long)ep << 32) | __float_as_uint(v[i]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

SYM_DEV f32x4 xar_collect(const XgmiArgs& c, const f32x4& own, long long goff, unsigned ep) {
  const int par = (int)(ep & 1u);
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < c.world; ++s) {
    if (s == c.rank) {
      sum += own;
      continue;
    }
    const unsigned long long* g = reinterpret_cast<const unsigned long long*>(
        c.bufs[c.rank] + XG_FLAG_BYTES + ((long long)par * c.world + s) * c.slot_bytes + goff);
    unsigned long long q[4];
    const unsigned long long t0 = wall_clock64();
    int it = 0;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        q[i] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = ok && (unsigned)(q[i] >> 32) == ep;
      }
      if (ok || xg_fault_declared(c, ++it)) break;
      if (wall_clock64() - t0 > XG_WAIT_TICKS) {
        __hip_atomic_store(c.err, 1 + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    sum += f32x4{__uint_as_float((unsigned)q[0]), __uint_as_float((unsigned)q[1]), __uint_as_float((unsigned)q[2]),
                 __uint_as_float((unsigned)q[3])};
  }
  return sum;
}

template <int EPI>
SYM_DEV void epilogue(const DecodeEpi& e, f32x4 v, int tile, int m, bool mok, int h, int N, unsigned xep = 0) {
  const int n0 = tile * 16;
  if constexpr (EPI == DECODE_EPI_F32) {
    if (mok) *reinterpret_cast<float4*>(e.y + (long long)m * N + n0 + 4 * h) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (EPI == DECODE_EPI_XAR) {
    // the residual epilogue's own operands first (no peer involved), then push, collect, finish
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    uint2 wraw = make_uint2(0, 0);
    const long long goff = xar_goff(m, N, n0 + 4 * h);
    if (mok) {
      r = *reinterpret_cast<const float4*>(e.resid + (long long)m * N + n0 + 4 * h);
      wraw = *reinterpret_cast<const uint2*>(e.w_next + n0 + 4 * h);
      xar_push(e.xp, v, goff, xep);
    }
    const f32x4 t = mok ? xar_collect(e.xp, v, goff, xep) : f32x4{0.f, 0.f, 0.f, 0.f};
    float sq = 0.f;
    if (mok) {
      const float rr[4] = {r.x + t[0], r.y + t[1], r.z + t[2], r.w + t[3]};
      Pack8 wp;
      wp.u = make_uint4(wraw.x, wraw.y, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) sq += rr[i] * rr[i];
      *reinterpret_cast<float4*>(e.resid + (long long)m * N + n0 + 4 * h) = make_float4(rr[0], rr[1], rr[2], rr[3]);
      store4bf(e.xw_out + (long long)m * N + n0 + 4 * h, rr[0] * (float)wp.h[0], rr[1] * (float)wp.h[1],
               rr[2] * (float)wp.h[2], rr[3] * (float)wp.h[3]);
    }
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
    if (mok && h == 0) e.ss_out[(long long)m * (N / 16) + tile] = sq;
  } else if constexpr (EPI == DECODE_EPI_QKV) {
    const int D = 128;
    const int head = n0 / D, jj = (n0 % D) / 16;
    float p[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = __shfl_xor(v[i], 32, 64);
    if (!mok) return;
    const int pos = e.positions[m];
    const int slot = e.slots[m];
    const float* cs = e.cos_sin + (long long)pos * D;
    if (head < e.Hq + e.Hkv) {
      const bool lo = h < 2;
      const int dh = 8 * jj + 4 * (h & 1);  // dim within the half (0..63)
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float c = cs[dh + i], s = cs[64 + dh + i];
        o[i] = lo ? (v[i] * c - p[i] * s) : (v[i] * c + p[i] * s);
      }
      const int d = (lo ? 0 : 64) + dh;
      bf16* dst = nullptr;
      if (head < e.Hq) {
        dst = e.q_out + ((long long)m * e.Hq + head) * D + d;
      } else if (slot >= 0) {
        const long long blk = slot / e.BS, off = slot % e.BS;
        dst = e.k_cache + ((blk * e.Hkv + (head - e.Hq)) * e.BS + off) * D + d;
      }
      if (dst) {
        if (e.sc1)  // read by the attention role of the same (fused) launch
          store4bf_sc1(dst, o[0], o[1], o[2], o[3]);
        else
          store4bf(dst, o[0], o[1], o[2], o[3]);
      }
    } else if (slot >= 0) {
      const int vh = head - e.Hq - e.Hkv;
      const int d = 16 * jj + 4 * h;
      const long long blk = slot / e.BS, off = slot % e.BS;
      bf16* vp = e.v_cache + ((blk * e.Hkv + vh) * D + d) * e.BS + off;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (e.sc1) {
          const bf16 bv = (bf16)v[i];
          __hip_atomic_store(reinterpret_cast<unsigned short*>(vp + (long long)i * e.BS),
                             __builtin_bit_cast(unsigned short, bv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          vp[(long long)i * e.BS] = (bf16)v[i];
        }
      }
    }
  } else if constexpr (EPI == DECODE_EPI_RESID) {
    float sq = 0.f;
    if (mok) {
      float* rp = e.resid + (long long)m * N + n0 + 4 * h;
      float4 r;
      if (e.resid_sc1) {  // rewritten earlier in this launch (persistent MLP): bypass this CU's L1
        r.x = __hip_atomic_load(rp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.y = __hip_atomic_load(rp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.z = __hip_atomic_load(rp + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.w = __hip_atomic_load(rp + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        r = *reinterpret_cast<const float4*>(rp);
      }
      const float rr[4] = {r.x + v[0], r.y + v[1], r.z + v[2], r.w + v[3]};
      float wn[4];
      Pack8 wp;  // 4 bf16 of the next norm weight
      const uint2 raw = *reinterpret_cast<const uint2*>(e.w_next + n0 + 4 * h);
      wp.u = make_uint4(raw.x, raw.y, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        wn[i] = (float)wp.h[i];
        sq += rr[i] * rr[i];
      }
      bf16* xo = e.xw_out + (long long)m * N + n0 + 4 * h;
      if (e.sc1) {  // consumed inside the same persistent launch: write-through (sc1) stores
#pragma unroll
        for (int i = 0; i < 4; ++i) __hip_atomic_store(rp + i, rr[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        store4bf_sc1(xo, rr[0] * wn[0], rr[1] * wn[1], rr[2] * wn[2], rr[3] * wn[3]);
      } else {
        *reinterpret_cast<float4*>(rp) = make_float4(rr[0], rr[1], rr[2], rr[3]);
        store4bf(xo, rr[0] * wn[0], rr[1] * wn[1], rr[2] * wn[2], rr[3] * wn[3]);
      }
    }
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
    if (mok && h == 0) {
      float* sp = e.ss_out + (long long)m * (N / 16) + tile;
      if (e.sc1)
        __hip_atomic_store(sp, sq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        *sp = sq;
    }
  } else if constexpr (EPI == DECODE_EPI_SWIGLU) {
    float u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = __shfl_xor(v[i], 32, 64);
    if (mok && h < 2) {
      const int f = 8 * tile + 4 * h;
      bf16* ap = e.act + (long long)m * (N / 2) + f;
      if (e.sc1)
        store4bf_sc1(ap, silu(v[0]) * u[0], silu(v[1]) * u[1], silu(v[2]) * u[2], silu(v[3]) * u[3]);
      else
        store4bf(ap, silu(v[0]) * u[0], silu(v[1]) * u[1], silu(v[2]) * u[2], silu(v[3]) * u[3]);
    }
  } else {  // DECODE_EPI_ARGMAX
    const int mm = mok ? m : 0;
    const float t = e.temps ? e.temps[mm] : 0.f;
    const long long step = e.step ? *e.step : 0;
    unsigned long long best = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nl = n0 + 4 * h + i;
      const int gidx = e.n_offset + nl;
      float val = v[i];
      if (e.y && mok) e.y[(long long)m * N + nl] = val;
      if (t > 0.f) {
        const unsigned long long seed = e.seeds ? e.seeds[mm] : 0ull;
        const float uu = uniform01(seed ^ ((unsigned long long)step << 20), (unsigned long long)gidx);
        val = val / t - __logf(-__logf(uu));
      }
      const unsigned long long kk = pack_key(val, (uint32_t)gidx);
      best = kk > best ? kk : best;
    }
    unsigned long long o16 = __shfl_xor(best, 16, 64);
    best = o16 > best ? o16 : best;
    unsigned long long o32 = __shfl_xor(best, 32, 64);
    best = o32 > best ? o32 : best;
    if (h == 0 && mok) e.keys[(long long)m * (N / 16) + tile] = best;
  }
}


}  // namespace
