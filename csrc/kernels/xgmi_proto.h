// Device side of the xGMI peer-memory protocol (xgmi_ar.hip): epochs, slots, bounded waits.  Shared by the
// collective kernels and by the decode GEMM's in-launch all-reduce epilogue (decode_gemm.hip, DECODE_EPI_XAR).
#pragma once
#include "common.h"
#include "launchers.h"

namespace {

// 30 s of the 100 MHz wall clock: a peer that never arrives is an error, not a hang.  Long enough for the
// first collectives of a provider start-up, where ranks can drift by the time each one spends loading
// library GEMM code objects before its first prefill.
constexpr unsigned long long XG_WAIT_TICKS = 3000000000ull;

// Fault containment: once the error word is set -- by an earlier collective that gave up on a peer, or by the
// host's health monitor that saw a rank die (parallel/health.py) -- no collective waits any more: the step
// finishes with garbage that the host discards, so a dead peer costs at most ONE wait limit per provider, not
// one per collective (a captured 70B TP=8 step holds 161).  The word is host-mapped (a PCIe round trip), so a
// spin reads it only after 16 polls and then every 256: a collective whose peers are on time never pays it.
SYM_DEV bool xg_fault_declared(const XgmiArgs& c, int it) {
  return (it & 255) == 16 && __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

SYM_DEV char* xg_slot(const XgmiArgs& c, int r, int par, int src) {
  return c.bufs[r] + XG_FLAG_BYTES + ((long long)par * c.world + src) * c.slot_bytes;
}

// This workgroup's epoch of the current collective (nwg workgroups per rank in the launch).
SYM_DEV unsigned xg_epoch(const XgmiArgs& c, int nwg) {
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) {
    // ONE returning atomic per workgroup on a packed {epoch (high 32), arrivals (low 32)} word: the add
    // counts this workgroup in and returns the epoch of the previous collective in the same round trip
    // (round 2 read the counter, waited, then counted in: two dependent round trips to uncached memory on
    // every collective).  The last arrival folds the arrivals back into an epoch increment -- the next
    // collective on the stream starts after this launch retired, so it finds {e, 0} -- and mirrors the
    // epoch into the u32 at byte 0 (diagnostics).
    unsigned long long* w = reinterpret_cast<unsigned long long*>(c.bufs[c.rank] + 64);
    const unsigned long long old = __hip_atomic_fetch_add(w, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned e = (unsigned)(old >> 32) + 1u;
    if ((unsigned)old == (unsigned)nwg - 1u) {  // last to arrive: every workgroup has counted itself in
      __hip_atomic_fetch_add(w, (1ull << 32) - (unsigned long long)nwg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<unsigned*>(c.bufs[c.rank]), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_epoch = e;
  }
  __syncthreads();
  return s_epoch;
}

// Test hook: hold this rank's workgroups back before they push (a slow peer), `delay` wall-clock ticks.
SYM_DEV void xg_delay(unsigned long long delay) {
  if (delay == 0) return;
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < delay) __builtin_amdgcn_s_sleep(8);
}

// Wait until flag (word, src) of this rank's buffer reached `epoch` (signed difference: a fast peer may already
// have raised a later epoch in the same word); bounded, and over at once once a fault was declared.
SYM_DEV void xg_wait_flag(const XgmiArgs& c, int word, int src, unsigned epoch) {
  const unsigned* f = reinterpret_cast<const unsigned*>(c.bufs[c.rank] + XG_HDR_BYTES) + word * XG_MAX_WORLD + src;
  const unsigned long long t0 = wall_clock64();
  int it = 0;
  while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
    if (xg_fault_declared(c, ++it)) break;
    if (wall_clock64() - t0 > XG_WAIT_TICKS) {  // error word: 1 + the source rank that never arrived
      __hip_atomic_store(c.err, 1 + src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Raise flag (word, this rank) in rank r's buffer.
SYM_DEV void xg_raise_flag(const XgmiArgs& c, int r, int word, unsigned epoch) {
  unsigned* f = reinterpret_cast<unsigned*>(c.bufs[r] + XG_HDR_BYTES) + word * XG_MAX_WORLD + c.rank;
  __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace
