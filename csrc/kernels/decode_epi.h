// Epilogues of the fused decode GEMMs (decode_gemm.hip) and of the medium-M GEMM's in-launch split-K
// reduction (mgemm.hip): one finished 16x16 accumulator tile in MFMA layout -- lane (r16, h) holds weight
// rows (output features) n0 + 4h .. n0 + 4h + 3 of token row m -- turned into the consumer's output
// (fp32 y, QKV RoPE + paged K/V write, residual add + next-norm prep, SwiGLU, fused sampling keys, or the
// xGMI push of a row-parallel projection under TP).
#pragma once

#include "common.h"
#include "launchers.h"

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

// ---- XPUSH (row-parallel projection under TP, xgmi_ar.hip protocol): the collective's epoch is this
// rank's counter + 1 (read here, bumped by the reduce kernel that follows on the stream); tiles are stored
// into slot (epoch parity, this rank) of every rank's buffer, then flag (tile, this rank) is raised in
// every rank once the storing wave's stores are acknowledged (uncached buffers: no cache maintenance).
SYM_DEV unsigned xp_epoch(const XgmiPush& xp) {
  return __hip_atomic_load(reinterpret_cast<const unsigned*>(xp.bufs[xp.rank]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

SYM_DEV void xp_flag(const XgmiPush& xp, int r, int tile, unsigned epoch) {
  unsigned* f = reinterpret_cast<unsigned*>(xp.bufs[r] + XG_HDR_BYTES) + tile * XG_MAX_WORLD + xp.rank;
  __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int EPI>
SYM_DEV void epilogue(const DecodeEpi& e, f32x4 v, int tile, int m, bool mok, int h, int N, unsigned xep = 0) {
  const int n0 = tile * 16;
  if constexpr (EPI == DECODE_EPI_F32) {
    if (mok) *reinterpret_cast<float4*>(e.y + (long long)m * N + n0 + 4 * h) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (EPI == DECODE_EPI_XPUSH) {
    if (mok) {
      const long long off = XG_FLAG_BYTES + ((long long)(xep & 1u) * e.xp.world + e.xp.rank) * e.xp.slot_bytes +
                            ((long long)m * N + n0 + 4 * h) * 4;
      const float4 val = make_float4(v[0], v[1], v[2], v[3]);
      for (int r = 0; r < e.xp.world; ++r) *reinterpret_cast<float4*>(e.xp.bufs[r] + off) = val;
    }
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
