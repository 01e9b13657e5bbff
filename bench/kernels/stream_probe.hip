// Weight-stream probe for the decode engine (csrc/kernels/decode_layers.hip): how fast can one workgroup per CU pull
// a per-CU weight share into registers with the engine's load shape (16 B buffer loads, 1 KB per wave instruction,
// pieces 8 KB apart), by cache policy, waves per CU and pieces in flight per wave?
//
//   hipcc --offload-arch=gfx950 -O3 -o build/stream_probe bench/kernels/stream_probe.hip && build/stream_probe
//
// Each launch: G workgroups, every wave loads `pieces` x 1 KB per round (all issued, then one wait), `rounds` rounds
// over fresh addresses (a 2 GiB buffer walked so no launch re-reads what an earlier one left in the caches); prints
// one JSON line per variant: chip GB/s and per-CU GB/s of the timed launches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int PIECES, int AUX>
__global__ void probe(const char* __restrict__ base, long long share_bytes, int rounds, int waves, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const char* mine = base + (long long)blockIdx.x * share_bytes * rounds;
  float acc = 0.f;
  for (int r = 0; r < rounds; ++r) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(mine + (long long)r * share_bytes),
                                                                  (short)0, (int)share_bytes, 0x00020000);
    u32x4 v[PIECES];
#pragma unroll
    for (int i = 0; i < PIECES; ++i)
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (w * 64 + lane) * 16,
                                                   __builtin_amdgcn_readfirstlane(i * waves * 1024), AUX);
#pragma unroll
    for (int i = 0; i < PIECES; ++i) acc += __uint_as_float(v[i].x ^ v[i].y ^ v[i].z ^ v[i].w);
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;  // keeps the loads; never true for the zero-filled buffer
}

template <int PIECES, int AUX>
void run(const char* name, char* buf, long long buf_bytes, int G, int waves, float* out) {
  const long long share = (long long)PIECES * waves * 1024;  // bytes per CU per round
  const int rounds = 8;
  const long long per_launch = share * rounds * G;
  const int launches = (int)(buf_bytes / per_launch);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // warm-up launch (code object, clocks)
  probe<PIECES, AUX><<<G, waves * 64>>>(buf, share, rounds, waves, out);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < launches; ++i)
    probe<PIECES, AUX><<<G, waves * 64>>>(buf + (long long)i * per_launch, share, rounds, waves, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)per_launch * launches;
  const double gbs = bytes / (ms * 1e-3) / 1e9;
  printf("{\"variant\": \"%s\", \"grid\": %d, \"waves\": %d, \"pieces_per_wave\": %d, \"kb_in_flight_per_cu\": %lld, "
         "\"chip_GBps\": %.0f, \"per_cu_GBps\": %.1f, \"us_per_round\": %.2f}\n",
         name, G, waves, PIECES, share / 1024, gbs, gbs / G, ms * 1e3 / launches / rounds);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const long long buf_bytes = 2LL << 30;
  char* buf = nullptr;
  float* out = nullptr;
  if (hipMalloc(&buf, buf_bytes) != hipSuccess || hipMalloc(&out, 4096 * sizeof(float)) != hipSuccess) return 1;
  hipMemset(buf, 0, buf_bytes);
  hipDeviceSynchronize();
  run<16, 2>("nt 8w x16", buf, buf_bytes, cus, 8, out);
  run<16, 0>("default 8w x16", buf, buf_bytes, cus, 8, out);
  run<16, 16>("sc1 8w x16", buf, buf_bytes, cus, 8, out);
  run<8, 2>("nt 8w x8", buf, buf_bytes, cus, 8, out);
  run<4, 2>("nt 8w x4", buf, buf_bytes, cus, 8, out);
  run<2, 2>("nt 8w x2", buf, buf_bytes, cus, 8, out);
  run<16, 2>("nt 4w x16", buf, buf_bytes, cus, 4, out);
  run<8, 2>("nt 16w x8", buf, buf_bytes, cus, 16, out);
  run<16, 2>("nt 8w x16 2/CU", buf, buf_bytes, 2 * cus, 8, out);
  run<7, 2>("nt 7w x7", buf, buf_bytes, cus, 7, out);
  hipFree(buf);
  hipFree(out);
  return 0;
}
