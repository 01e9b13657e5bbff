// K2 + K3: rotary embedding on Q/K fused with the paged KV-cache write.
//
// Input is the QKV projection output (LinOut: bf16 [T][(Hq+2Hkv)*D] or fp32
// split-K slabs), so the split-K reduce of the decode QKV GEMM happens here.
// Outputs:
//   q_out   bf16 [T][Hq][D]            rotated queries
//   k_cache bf16 [NB][Hkv][BS][D]      token-major K blocks (rotated)
//   v_cache bf16 [NB][Hkv][D][BS]      dim-major ("transposed") V blocks
// The V layout makes the P.V MFMA B-operand (8 consecutive tokens of one
// dim) a single 16-byte load in the attention kernels.
// rotate_half (NeoX/Llama) convention; cos/sin come from a host-built fp32
// table [max_pos][D] = [cos(0..D/2) | sin(0..D/2)] (no device trig).
#include "common.h"
#include "launchers.h"

namespace {

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void rope_cache_kernel(LinOut qkv, const int* __restrict__ positions,
                                                        const int* __restrict__ slots,
                                                        const float* __restrict__ cos_sin,
                                                        bf16* __restrict__ q_out, bf16* __restrict__ k_cache,
                                                        bf16* __restrict__ v_cache, int Hq, int Hkv, int D,
                                                        int BS, int perm) {
  const int t = blockIdx.x;
  const int N = (Hq + 2 * Hkv) * D;
  const long long row = (long long)t * N;
  const int pos = positions[t];
  const int slot = slots ? slots[t] : -1;
  const int half = D / 2;
  const int gpr = half / 8;  // 8-pair groups per head
  const float* cs = cos_sin + (long long)pos * D;
  const int rot_items = (Hq + Hkv) * gpr;
  const int v_items = Hkv * (D / 8);
  // gridDim.y workgroups per row: one item (8 dims of a head) per thread, one load round trip per row
  for (int it = blockIdx.y * NT + threadIdx.x; it < rot_items + v_items; it += gridDim.y * NT) {
    if (it < rot_items) {
      const int h = it / gpr;          // 0..Hq+Hkv-1 (q heads then k heads)
      const int i0 = (it % gpr) * 8;   // pair index within the half
      float x1[8], x2[8], c[8], s[8];
      // perm: rows of a q/k head are stored tile-interleaved (decode layout, decode_gemm.hip):
      // dims i0..i0+7 at 2*i0, dims half+i0.. at 2*i0 + 8
      const int p1 = perm ? 2 * i0 : i0, p2 = perm ? 2 * i0 + 8 : half + i0;
      linout_load8(qkv, row + (long long)h * D + p1, x1);
      linout_load8(qkv, row + (long long)h * D + p2, x2);
      load8f(cs + i0, c);
      load8f(cs + half + i0, s);
      float o1[8], o2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o1[j] = x1[j] * c[j] - x2[j] * s[j];
        o2[j] = x2[j] * c[j] + x1[j] * s[j];
      }
      if (h < Hq) {
        bf16* q = q_out + ((long long)t * Hq + h) * D;
        store8(q + i0, o1);
        store8(q + half + i0, o2);
      } else if (slot >= 0) {
        const int kh = h - Hq;
        const long long blk = slot / BS, off = slot % BS;
        bf16* k = k_cache + ((blk * Hkv + kh) * BS + off) * D;
        store8(k + i0, o1);
        store8(k + half + i0, o2);
      }
    } else if (slot >= 0) {
      const int vi = it - rot_items;
      const int kh = vi / (D / 8);
      const int d0 = (vi % (D / 8)) * 8;
      float x[8];
      linout_load8(qkv, row + (long long)(Hq + Hkv + kh) * D + d0, x);
      const long long blk = slot / BS, off = slot % BS;
      bf16* v = v_cache + ((blk * Hkv + kh) * D + d0) * BS + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[(long long)j * BS] = (bf16)x[j];
    }
  }
}

// Prefill form: grid (T / 8, 8).  Workgroup (g, y) rotates row 8 g + y (as above) and writes the V rows
// of kv heads y, y + 8, ... for the 8 rows of group g.  The dim-major V write -- 2-byte stores at a
// BS-element stride, one cache line touched per element, which made the plain kernel ~3x slower than its
// bytes (16.5 us at 1280 tokens) -- becomes one 16-byte store of 8 consecutive tokens per (kv head, dim)
// whenever the 8 rows fill 8 consecutive, 8-aligned slots of one block (a prefill chunk of one
// sequence); other groups fall back to per-token stores.  The 8 V loads per thread stay coalesced
// across the wave (consecutive dims of one row).
constexpr int RG = 8;

__global__ __launch_bounds__(NT) void rope_cache_grouped_kernel(LinOut qkv, const int* __restrict__ positions,
                                                                const int* __restrict__ slots,
                                                                const float* __restrict__ cos_sin,
                                                                bf16* __restrict__ q_out, bf16* __restrict__ k_cache,
                                                                bf16* __restrict__ v_cache, int T, int Hq, int Hkv,
                                                                int D, int BS, int perm) {
  const int t0 = blockIdx.x * RG;
  const int nt = min(RG, T - t0);
  const int N = (Hq + 2 * Hkv) * D;
  const int half = D / 2;
  const int gpr = half / 8;
  const int t = t0 + blockIdx.y;
  if (t < T) {  // rotation of one row (uniform over the workgroup)
    const long long row = (long long)t * N;
    const float* cs = cos_sin + (long long)positions[t] * D;
    const int slot = slots ? slots[t] : -1;
    for (int it = threadIdx.x; it < (Hq + Hkv) * gpr; it += NT) {
      const int h = it / gpr;
      const int i0 = (it % gpr) * 8;
      float x1[8], x2[8], c[8], sn[8];
      const int p1 = perm ? 2 * i0 : i0, p2 = perm ? 2 * i0 + 8 : half + i0;
      linout_load8(qkv, row + (long long)h * D + p1, x1);
      linout_load8(qkv, row + (long long)h * D + p2, x2);
      load8f(cs + i0, c);
      load8f(cs + half + i0, sn);
      float o1[8], o2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o1[j] = x1[j] * c[j] - x2[j] * sn[j];
        o2[j] = x2[j] * c[j] + x1[j] * sn[j];
      }
      if (h < Hq) {
        bf16* q = q_out + ((long long)t * Hq + h) * D;
        store8(q + i0, o1);
        store8(q + half + i0, o2);
      } else if (slot >= 0) {
        const int kh = h - Hq;
        const long long blk = slot / BS, off = slot % BS;
        bf16* k = k_cache + ((blk * Hkv + kh) * BS + off) * D;
        store8(k + i0, o1);
        store8(k + half + i0, o2);
      }
    }
  }
  if (!slots) return;
  // V of kv heads y, y + 8, ...: can this group go out as 16-byte token runs?  (uniform)
  const int s0 = slots[t0];
  bool run = nt == RG && s0 >= 0 && s0 % RG == 0 && BS % RG == 0;
  for (int j = 1; j < RG && run; ++j) run = slots[t0 + j] == s0 + j;
  const long long vbase = (long long)(Hq + Hkv) * D;
  for (int it = blockIdx.y * D + threadIdx.x; it < Hkv * D; it += RG * D) {
    if (threadIdx.x >= D) break;  // D threads per kv head
    const int kh = it / D, d = it % D;
    float x[RG];
#pragma unroll
    for (int j = 0; j < RG; ++j) x[j] = j < nt ? linout_load1(qkv, (long long)(t0 + j) * N + vbase + it) : 0.f;
    if (run) {
      const long long blk = s0 / BS, off = s0 % BS;
      store8(v_cache + ((blk * Hkv + kh) * D + d) * BS + off, x);
    } else {
      for (int j = 0; j < nt; ++j) {
        const int slot = slots[t0 + j];
        if (slot < 0) continue;
        const long long blk = slot / BS, off = slot % BS;
        v_cache[((blk * Hkv + kh) * D + d) * BS + off] = (bf16)x[j];
      }
    }
  }
}

}  // namespace

void launch_rope_cache(LinOut qkv, const int* positions, const int* slots, const float* cos_sin, bf16* q_out,
                       bf16* k_cache, bf16* v_cache, int T, int Hq, int Hkv, int D, int BS, hipStream_t s, int perm,
                       int decode) {
  if (T == 0) return;
  // decode rows belong to different sequences (no V token runs to gain): the per-row kernel with enough
  // workgroups per row that every thread handles one 8-dim item
  if (!decode && T >= 4 * RG && D <= NT) {  // prefill chunks: 8-row groups with 16-byte V token runs
    rope_cache_grouped_kernel<<<dim3((T + RG - 1) / RG, RG), NT, 0, s>>>(qkv, positions, slots, cos_sin, q_out,
                                                                          k_cache, v_cache, T, Hq, Hkv, D, BS, perm);
    return;
  }
  const int items = (Hq + Hkv) * (D / 16) + Hkv * (D / 8);
  rope_cache_kernel<<<dim3(T, (items + NT - 1) / NT), NT, 0, s>>>(qkv, positions, slots, cos_sin, q_out, k_cache,
                                                                   v_cache, Hq, Hkv, D, BS, perm);
}
