// R1 for decode: one-shot all-reduce over xGMI peer memory (§7.4 risk 4).
//
// A Llama-3-70B TP=8 decode step issues 160 all-reduces of 16 KiB x batch (fp32 partials: 32 KiB x
// batch).  At those sizes a collective is pure latency, and a ring (RCCL's default shape) pays 2(N-1)
// dependent hops over ONE of the seven point-to-point xGMI links.  Here every rank writes its partial
// straight into a slot of EVERY peer's buffer (seven links busy at once, one hop), raises a flag per
// (workgroup, source rank) in each peer, waits for the world's flags of its own chunk and reduces the
// slots in rank order -- so every rank computes bit-identical sums (TP ranks must agree on the sampled
// token).  The reduce can carry the decode epilogue of the row-parallel projections (residual add +
// next-norm prep, the `add_prep` of decode_gemm.hip), which removes a launch per all-reduce.
//
// Buffers: one per rank, hipExtMallocWithFlags(hipDeviceMallocUncached) so that stores arriving over
// xGMI are never hidden behind a stale L2 line of the reading GPU, exported with hipIpcGetMemHandle and
// opened by every peer (symmetry_amd/parallel/comm.py::XgmiComm).  Layout of a buffer:
//   header (local collective counter) | flags [XG_MAX_WG][XG_MAX_WORLD] u32 | data [2 parities][world][slot_bytes]
// Epochs: ONE counter per communicator numbers its collectives.  Every workgroup of a launch reads it on
// entry and counts itself in; the last one to arrive bumps it, after every workgroup has read it, and
// the next collective on the stream starts only after this launch retired -- so all workgroups of one
// collective share one epoch whatever the grid, and all ranks (running the same sequence of
// collectives) agree on it without host bookkeeping; a captured hipGraph replays correctly.  The data
// slots alternate by epoch parity.  A rank can finish collective e+1 only after every peer has entered
// e+1 (it waits for their flags), i.e. after every peer has finished reducing e: so a rank two
// collectives ahead can never overwrite the parity of e while a peer still reads it, however the two
// collectives split their bytes over workgroups (add_prep parts, all-reduce chunks and the keys
// collective all address the same slot bytes differently).  Flags are compared with a signed
// difference (a fast peer may already have raised a later epoch in the same flag word).
// Spins are bounded: a missing peer sets the error word and the kernel exits instead of hanging; every later
// spin sees that word and exits at once (xg_fault_declared).
#include "common.h"
#include "launchers.h"
#include "xgmi_proto.h"

namespace {

constexpr int XG_THREADS = 256;
// Push this workgroup's chunk (nvec vectors at byte offset `off`) into slot (parity, rank) of every rank's
// buffer (its own included, so the reduce reads all slots from one place), raise flag (wg, rank) in every
// rank, wait for every rank's flag (wg, src).  `wg` indexes flags only; `nwg` = workgroups of this rank in
// the launch (epoch accounting).  Returns the epoch parity (the slot set to reduce).
// `push(par)` stores this thread's part of the chunk into slot (par, rank) of every rank.
template <typename PushFn>
SYM_DEV int xg_exchange_fn(const XgmiArgs& c, int wg, int nwg, PushFn push, unsigned long long delay = 0) {
  const unsigned epoch = xg_epoch(c, nwg);
  xg_delay(delay);
  const int par = (int)(epoch & 1u);
  push(par);
  // Every wave waits for its slot stores to be acknowledged before the workgroup signals: the AMDGPU
  // memory model's system-scope release is `buffer_wbl2 sc0 sc1; s_waitcnt vmcnt(0)`, and the L2
  // write-back half has nothing to do here -- the buffers are uncached (MTYPE UC), so the stores never
  // sit in an L2 and the slot loads below never hit one (no acquire invalidate either).  A full
  // __threadfence_system() per collective costs an L2 write-back + invalidate of the whole XCD.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < c.world) {
    unsigned* f = reinterpret_cast<unsigned*>(c.bufs[threadIdx.x] + XG_HDR_BYTES) + wg * XG_MAX_WORLD + c.rank;
    __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* mine =
        reinterpret_cast<const unsigned*>(c.bufs[c.rank] + XG_HDR_BYTES) + wg * XG_MAX_WORLD + threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    int it = 0;
    while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if (xg_fault_declared(c, ++it)) break;
      if (wall_clock64() - t0 > XG_WAIT_TICKS) {  // error word: 1 + the source rank that never arrived
        __hip_atomic_store(c.err, 1 + (int)threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();  // the pollers saw every flag: the slot bytes behind them are in memory (uncached)
  return par;
}

template <typename V = uint4>
SYM_DEV int xg_exchange(const XgmiArgs& c, int wg, int nwg, const V* __restrict__ src, long long off, int nvec,
                        unsigned long long delay = 0) {
  return xg_exchange_fn(
      c, wg, nwg,
      [&](int par) {
        for (int v = threadIdx.x; v < nvec; v += XG_THREADS) {
          const V x = src[v];
          for (int r = 0; r < c.world; ++r) reinterpret_cast<V*>(xg_slot(c, r, par, c.rank) + off)[v] = x;
        }
      },
      delay);
}

// Plain all-reduce (sum) of n elements, in place or out of place; ELEM: 0 = fp32, 1 = bf16.
// Workgroup g of nwg owns elements [g * chunk, min(n, (g + 1) * chunk)), chunk a multiple of 8.
template <int ELEM>
SYM_DEV void xg_all_reduce_body(const XgmiArgs& c, int wg, int nwg, const void* in, void* out, long long n, int chunk,
                                unsigned long long delay = 0) {
  const long long e0 = (long long)wg * chunk;
  const int cnt = (int)min((long long)chunk, n - e0);
  constexpr int ESZ = ELEM == 0 ? 4 : 2;
  const int nvec = cnt * ESZ / 16;
  const long long off = e0 * ESZ;
  const int par = xg_exchange<uint4>(c, wg, nwg,
                                     reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(in) + off), off, nvec,
                                     delay);
  for (int v = threadIdx.x; v < nvec; v += XG_THREADS) {
    if constexpr (ELEM == 0) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < c.world; ++r) {
        const float4 x = reinterpret_cast<const float4*>(xg_slot(c, c.rank, par, r) + off)[v];
        acc[0] += x.x;
        acc[1] += x.y;
        acc[2] += x.z;
        acc[3] += x.w;
      }
      reinterpret_cast<float4*>(reinterpret_cast<char*>(out) + off)[v] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < c.world; ++r) {
        float f[8];
        load8(reinterpret_cast<const bf16*>(xg_slot(c, c.rank, par, r) + off) + 8 * v, f);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += f[i];
      }
      store8(reinterpret_cast<bf16*>(reinterpret_cast<char*>(out) + off) + 8 * v, acc);
    }
  }
}

// All-reduce of fp32 row partials [T][d] fused with the decode epilogue of a row-parallel projection
// (prep_kernel<1>): resid += sum; xw = bf16(resid * w); ss[row][part] = sum(resid^2) over the part's
// columns.  Workgroup (row, part) of T x P owns columns [part d / P, (part + 1) d / P) of its row.
SYM_DEV void xg_add_prep_body(const XgmiArgs& c, int row, int part, int T, int P, const float* __restrict__ y,
                              float* __restrict__ resid, const bf16* __restrict__ w, bf16* __restrict__ xw,
                              float* __restrict__ ss, int d, unsigned long long delay = 0) {
  __shared__ float scratch[XG_THREADS / 64];
  const int dp = d / P;
  const int wg = row * P + part;
  const long long rb = (long long)row * d + (long long)part * dp;
  const long long off = rb * 4;
  const bf16* wp = w + (long long)part * dp;
  float acc = 0.f;
  if (dp / 8 <= XG_THREADS) {
    // one 8-column vector per thread (every decode shape: d / P <= 2048): the partial, the residual and the
    // norm weight are loaded BEFORE the collective's epoch / flag round trips (none depends on a peer), so
    // their latency hides behind them; the partial is pushed from registers
    const int vi = threadIdx.x;
    const bool on = vi < dp / 8;
    float yv[8], r[8], g[8];
    if (on) {
      load8f(y + rb + vi * 8, yv);
      load8f(resid + rb + vi * 8, r);
      load8(wp + vi * 8, g);
    }
    const int par = xg_exchange_fn(
        c, wg, T * P,
        [&](int pr) {
          if (!on) return;
          const float4 a = make_float4(yv[0], yv[1], yv[2], yv[3]), b = make_float4(yv[4], yv[5], yv[6], yv[7]);
          for (int s = 0; s < c.world; ++s) {
            float4* dst = reinterpret_cast<float4*>(xg_slot(c, s, pr, c.rank) + off) + 2 * vi;
            dst[0] = a;
            dst[1] = b;
          }
        },
        delay);
    if (on) {
      float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < c.world; ++s) {  // the all-reduced delta first (rank order), then the residual add
        float dd[8];
        load8f(reinterpret_cast<const float*>(xg_slot(c, c.rank, par, s) + off) + vi * 8, dd);
#pragma unroll
        for (int i = 0; i < 8; ++i) sum[i] += dd[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] += sum[i];
      store8f(resid + rb + vi * 8, r);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc += r[i] * r[i];
        g[i] *= r[i];
      }
      store8(xw + rb + vi * 8, g);
    }
    acc = block_sum<XG_THREADS>(acc, scratch);
    if (threadIdx.x == 0) ss[row * P + part] = acc;
    return;
  }
  const int par = xg_exchange<uint4>(c, wg, T * P, reinterpret_cast<const uint4*>(y + rb), off, dp / 4, delay);
  for (int vi = threadIdx.x; vi < dp / 8; vi += XG_THREADS) {
    float r[8], g[8];
    float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < c.world; ++s) {  // the all-reduced delta first (rank order), then the residual add
      float dd[8];
      load8f(reinterpret_cast<const float*>(xg_slot(c, c.rank, par, s) + off) + vi * 8, dd);
#pragma unroll
      for (int i = 0; i < 8; ++i) sum[i] += dd[i];
    }
    load8f(resid + rb + vi * 8, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] += sum[i];
    store8f(resid + rb + vi * 8, r);
    load8(wp + vi * 8, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc += r[i] * r[i];
      g[i] *= r[i];
    }
    store8(xw + rb + vi * 8, g);
  }
  acc = block_sum<XG_THREADS>(acc, scratch);
  if (threadIdx.x == 0) ss[row * P + part] = acc;
}

// Vocab-parallel greedy / Gumbel sampling combine: every rank holds per-row packed u64 keys (order-
// preserving value bits | inverted vocabulary index) of its vocabulary shard; the max over ranks is the
// global argmax, and ids = 0xFFFFFFFF - low 32 bits.  One workgroup (rows <= 4096) on flag word XG_KEYS_WG.
SYM_DEV void xg_keys_max_body(const XgmiArgs& c, const unsigned long long* keys, int* __restrict__ ids, int B,
                              unsigned long long delay = 0) {
  const int par = xg_exchange<unsigned long long>(c, XG_KEYS_WG, 1, keys, 0, B, delay);
  for (int i = threadIdx.x; i < B; i += XG_THREADS) {
    unsigned long long best = 0;
    for (int r = 0; r < c.world; ++r) {
      const unsigned long long k = reinterpret_cast<const unsigned long long*>(xg_slot(c, c.rank, par, r))[i];
      best = k > best ? k : best;
    }
    ids[i] = (int)(0xFFFFFFFFu - (unsigned)(best & 0xFFFFFFFFull));
  }
}

__global__ __launch_bounds__(XG_THREADS) void xgmi_keys_max_kernel(XgmiArgs c, const unsigned long long* keys,
                                                                  int* __restrict__ ids, int B) {
  xg_keys_max_body(c, keys, ids, B);
}

template <int ELEM>
__global__ __launch_bounds__(XG_THREADS) void xgmi_all_reduce_kernel(XgmiArgs c, const void* in, void* out,
                                                                     long long n, int chunk) {
  xg_all_reduce_body<ELEM>(c, blockIdx.x, gridDim.x, in, out, n, chunk);
}

__global__ __launch_bounds__(XG_THREADS) void xgmi_add_prep_kernel(XgmiArgs c, const float* __restrict__ y,
                                                                  float* __restrict__ resid,
                                                                  const bf16* __restrict__ w,
                                                                  bf16* __restrict__ xw, float* __restrict__ ss,
                                                                  int d) {
  xg_add_prep_body(c, blockIdx.x, blockIdx.y, gridDim.x, gridDim.y, y, resid, w, xw, ss, d);
}

// Several ranks of ONE process in one launch (grid z = rank): the GPU test of the protocol on one device.
// Separate launches on separate streams are not guaranteed to be co-resident (streams may share a
// hardware queue), and every rank waits on the others; the slices of one grid are.  Slice
// m.delay_rank is held back by m.delay_ticks before it pushes (a slow peer).
SYM_DEV unsigned long long xg_multi_delay(const XgmiMulti& m, int r) {
  return r == m.delay_rank ? m.delay_ticks : 0ull;
}

template <int ELEM>
__global__ __launch_bounds__(XG_THREADS) void xgmi_all_reduce_multi_kernel(XgmiMulti m, long long n, int chunk) {
  const int r = blockIdx.z;
  xg_all_reduce_body<ELEM>(m.c[r], blockIdx.x, gridDim.x, m.in[r], m.out[r], n, chunk, xg_multi_delay(m, r));
}

__global__ __launch_bounds__(XG_THREADS) void xgmi_add_prep_multi_kernel(XgmiMulti m, int d) {
  const int r = blockIdx.z;
  xg_add_prep_body(m.c[r], blockIdx.x, blockIdx.y, gridDim.x, gridDim.y, reinterpret_cast<const float*>(m.in[r]),
                   reinterpret_cast<float*>(m.out[r]), m.w, reinterpret_cast<bf16*>(m.xw[r]), m.ss[r], d,
                   xg_multi_delay(m, r));
}


__global__ __launch_bounds__(XG_THREADS) void xgmi_keys_max_multi_kernel(XgmiMulti m, int B) {
  const int r = blockIdx.z;
  xg_keys_max_body(m.c[r], reinterpret_cast<const unsigned long long*>(m.in[r]), reinterpret_cast<int*>(m.out[r]), B,
                   xg_multi_delay(m, r));
}

// ---- R3: expert all-to-all, unpadded -----------------------------------------------------------------------
// Mixtral prefill under expert parallelism: rank r routes its token slice and groups the routed rows by owner
// rank into blocks of capacity `cap` (worst case: every row to one owner).  RCCL's all-to-all moves whole
// blocks -- N x the routed rows.  Here the counts stay on the device and each workgroup pushes only ITS share of
// the real rows of every block straight into the owner's slot for this rank (one hop over the owner's link),
// with the count and the rows' side ints (expert ids) beside them, raises flag (wg, rank) in the owner, waits
// for flag (wg, s) of every source s, and copies its share of every source's rows out of its own slot into the
// caller's buffer -- the same share rule on both ends (rows [wg n / G, (wg + 1) n / G) of an n-row block), so
// the flag a workgroup waits for covers exactly the rows it copies.  Epochs, parities, bounded spins and the
// declared-fault exit are the all-reduce's (xg_epoch, xg_fault_declared).
SYM_DEV long long xa_rows_off(int cap) { return (64 + 4LL * cap + 15) / 16 * 16; }

SYM_DEV void xg_a2a_body(const XgmiA2AArgs& a, int wg, int G, unsigned long long delay = 0) {
  const XgmiArgs& c = a.c;
  const unsigned epoch = xg_epoch(c, G);
  xg_delay(delay);
  const int par = (int)(epoch & 1u);
  const int tid = threadIdx.x, rb = a.row_bytes, cap = a.cap;
  const long long roff = xa_rows_off(cap);
  // push my share of every block to its owner
  for (int q = 0; q < c.world; ++q) {
    const int n = a.counts[q];
    const long long r0 = (long long)wg * n / G, r1 = (long long)(wg + 1) * n / G;
    char* slot = xg_slot(c, q, par, c.rank);
    const uint4* sp = reinterpret_cast<const uint4*>(a.src + ((long long)q * cap + r0) * rb);
    uint4* dp = reinterpret_cast<uint4*>(slot + roff + r0 * rb);
    const long long nv = (r1 - r0) * rb / 16;
    for (long long v = tid; v < nv; v += XG_THREADS) dp[v] = sp[v];
    if (a.side != nullptr)
      for (long long j = r0 + tid; j < r1; j += XG_THREADS)
        reinterpret_cast<int*>(slot + 64)[j] = a.side[(long long)q * cap + j];
    if (tid == 0) *reinterpret_cast<unsigned*>(slot) = (unsigned)n;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store acknowledged (uncached buffers: no L2 write-back)
  __syncthreads();
  if (tid < c.world) {
    unsigned* f = reinterpret_cast<unsigned*>(c.bufs[tid] + XG_HDR_BYTES) + wg * XG_MAX_WORLD + c.rank;
    __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* mine = reinterpret_cast<const unsigned*>(c.bufs[c.rank] + XG_HDR_BYTES) + wg * XG_MAX_WORLD + tid;
    const unsigned long long t0 = wall_clock64();
    int it = 0;
    while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if (xg_fault_declared(c, ++it)) break;
      if (wall_clock64() - t0 > XG_WAIT_TICKS) {
        __hip_atomic_store(c.err, 1 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  // copy my share of every source's rows out of my slot
  for (int s = 0; s < c.world; ++s) {
    const char* slot = xg_slot(c, c.rank, par, s);
    const int n = (int)min(*reinterpret_cast<const unsigned*>(slot), (unsigned)cap);
    const long long r0 = (long long)wg * n / G, r1 = (long long)(wg + 1) * n / G;
    const uint4* sp = reinterpret_cast<const uint4*>(slot + roff + r0 * rb);
    uint4* dp = reinterpret_cast<uint4*>(a.dst + ((long long)s * cap + r0) * rb);
    const long long nv = (r1 - r0) * rb / 16;
    for (long long v = tid; v < nv; v += XG_THREADS) dp[v] = sp[v];
    if (a.dst_side != nullptr) {
      int* ds = a.dst_side + (long long)s * cap;
      for (long long j = r0 + tid; j < r1; j += XG_THREADS) ds[j] = reinterpret_cast<const int*>(slot + 64)[j];
      const long long e0 = n + (long long)wg * (cap - n) / G, e1 = n + (long long)(wg + 1) * (cap - n) / G;
      for (long long j = e0 + tid; j < e1; j += XG_THREADS) ds[j] = -1;
    }
    if (a.dst_counts != nullptr && wg == 0 && tid == 0) a.dst_counts[s] = n;
  }
}

__global__ __launch_bounds__(XG_THREADS) void xgmi_a2a_kernel(XgmiA2AArgs a) { xg_a2a_body(a, blockIdx.x, gridDim.x); }

__global__ __launch_bounds__(XG_THREADS) void xgmi_a2a_multi_kernel(XgmiA2AMulti m) {
  const int r = blockIdx.y;
  xg_a2a_body(m.a[r], blockIdx.x, gridDim.x, r == m.delay_rank ? m.delay_ticks : 0ull);
}

}  // namespace

long long xgmi_a2a_slot_bytes(int cap, int row_bytes) {
  return (64 + 4LL * cap + 15) / 16 * 16 + (long long)cap * row_bytes;
}

void launch_xgmi_a2a(const XgmiA2AArgs& a, hipStream_t s) { xgmi_a2a_kernel<<<XA_WG, XG_THREADS, 0, s>>>(a); }

void launch_xgmi_a2a_multi(const XgmiA2AMulti& m, int world, hipStream_t s) {
  xgmi_a2a_multi_kernel<<<dim3(XA_WG, world), XG_THREADS, 0, s>>>(m);
}

long long xgmi_buffer_bytes(int world, long long slot_bytes) { return XG_FLAG_BYTES + 2LL * world * slot_bytes; }

int xgmi_chunk(long long n, long long max_wg) {
  // >= 1024 elements (4 KB of fp32) per workgroup, multiple of 8: the fused add_prep's sweep of
  // workgroups per row (profiles/xgmi_allreduce_local_r2.jsonl, 1-10 rows of 8192) was fastest with
  // 512-1024-element parts (4 ranks: 2048-element parts 5.8-6.4 us, 1024 5.0-5.3)
  long long chunk = (n + max_wg - 1) / max_wg;
  chunk = std::max<long long>(chunk, 1024);
  return (int)((chunk + 7) / 8 * 8);
}

void launch_xgmi_all_reduce(const XgmiArgs& c, const void* in, void* out, long long n, int elem, hipStream_t s) {
  if (n == 0) return;
  const int chunk = xgmi_chunk(n, XG_MAX_WG);
  const int grid = (int)((n + chunk - 1) / chunk);
  if (elem == 0)
    xgmi_all_reduce_kernel<0><<<grid, XG_THREADS, 0, s>>>(c, in, out, n, chunk);
  else
    xgmi_all_reduce_kernel<1><<<grid, XG_THREADS, 0, s>>>(c, in, out, n, chunk);
}

void launch_xgmi_add_prep(const XgmiArgs& c, const float* y, float* resid, const bf16* w, bf16* xw, float* ss, int T,
                          int d, int parts, hipStream_t s) {
  if (T == 0) return;
  xgmi_add_prep_kernel<<<dim3(T, parts), XG_THREADS, 0, s>>>(c, y, resid, w, xw, ss, d);
}

void launch_xgmi_keys_max(const XgmiArgs& c, const unsigned long long* keys, int* ids, int B, hipStream_t s) {
  if (B == 0) return;
  xgmi_keys_max_kernel<<<1, XG_THREADS, 0, s>>>(c, keys, ids, B);
}

void launch_xgmi_all_reduce_multi(const XgmiMulti& m, int world, long long n, int elem, hipStream_t s) {
  if (n == 0) return;
  const int chunk = xgmi_chunk(n, XG_MAX_WG);
  const dim3 grid((unsigned)((n + chunk - 1) / chunk), 1, (unsigned)world);
  if (elem == 0)
    xgmi_all_reduce_multi_kernel<0><<<grid, XG_THREADS, 0, s>>>(m, n, chunk);
  else
    xgmi_all_reduce_multi_kernel<1><<<grid, XG_THREADS, 0, s>>>(m, n, chunk);
}

void launch_xgmi_add_prep_multi(const XgmiMulti& m, int world, int T, int d, int parts, hipStream_t s) {
  if (T == 0) return;
  xgmi_add_prep_multi_kernel<<<dim3(T, parts, world), XG_THREADS, 0, s>>>(m, d);
}

void launch_xgmi_keys_max_multi(const XgmiMulti& m, int world, int B, hipStream_t s) {
  if (B == 0) return;
  xgmi_keys_max_multi_kernel<<<dim3(1, 1, world), XG_THREADS, 0, s>>>(m, B);
}
