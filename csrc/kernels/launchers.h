// Host-side launch entry points of the symmetry_amd HIP kernels.
// Every launcher enqueues on the given stream, allocates nothing and never
// synchronises, so the calling op can be captured into a hipGraph.
// Shape/alignment preconditions are validated by the torch op layer
// (csrc/bindings/torch_ops.cpp) before any launch.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include "common.h"

// decode_gemm.hip -- fused decode projections (see the file header)
enum {
  DECODE_EPI_F32 = 0,
  DECODE_EPI_QKV = 1,
  DECODE_EPI_RESID = 2,
  DECODE_EPI_SWIGLU = 3,
  DECODE_EPI_ARGMAX = 4,
  // row-parallel projection under TP, all-reduced in the launch: every tile's values go to every other rank as
  // epoch-tagged granules, the tile's workgroup sums every rank's copy in rank order and runs the RESID
  // epilogue (residual add + next-norm prep, ss per 16-column tile) -- decode_epi.h, xar_push / xar_collect
  DECODE_EPI_XAR = 6,
  DECODE_EPI_BF16 = 7,  // plain bf16 [M][N] output (pgemm.hip only)
  DECODE_EPI_SWIGLU_SPLIT = 8,  // SwiGLU of [gate rows; up rows] halves (pgemm.hip grouped experts: act [M][N / 2])
  XAR_MAX_TILES = 32,  // output tiles per workgroup of an x-resident XAR launch (epoch slots in LDS)
};

// xGMI communicator buffer layout (xgmi_ar.hip): header (collective counter) | flags [XG_MAX_WG][XG_MAX_WORLD]
// u32 | data [2 parities][world][slot_bytes]
constexpr int XG_MAX_WORLD = 8;
constexpr int XG_MAX_WG = 4096;
constexpr int XG_KEYS_WG = XG_MAX_WG - 1;  // flag word of the sampling-keys collective (others stay below)
constexpr long long XG_HDR_BYTES = 256;   // [0] u32 epoch mirror, [64] u64 {epoch, arrivals} of the current collective
constexpr long long XG_FLAG_BYTES = XG_HDR_BYTES + (long long)XG_MAX_WG * XG_MAX_WORLD * 4;
// One xGMI communicator as seen by a kernel (xgmi_ar.hip protocol; also the DECODE_EPI_XAR target)
struct XgmiArgs {
  char* bufs[XG_MAX_WORLD] = {};  // every rank's comm buffer as mapped in this process (own one included; its
                                  // header holds this rank's collective counter)
  int* err = nullptr;             // local error word (a peer never arrived / a fault was declared; host-mapped)
  int rank = 0, world = 0;
  long long slot_bytes = 0;       // bytes of one (parity, source rank) data slot
};
struct DecodeEpi {
  // weight layout: 0 = row-major [N][K]; 1 = MFMA-preshuffled (models/layout.py::preshuffle): each
  // 16-row x 32-k block is 1 KB contiguous in lane order, so one load instruction reads 1 KB and a
  // wave's k-slice of a row tile is one contiguous stream
  int wshuf = 0;
  int wnt = 0;  // weight loads non-temporal (experiment knob, bench only)
  int sc1 = 0;  // RESID / SWIGLU outputs as write-through stores (consumed within a persistent launch)
  int resid_sc1 = 0;  // RESID reads the residual with L1-bypassing loads (written earlier in the launch)
  // prologue: RMSNorm row scale rsqrt(sum(ss_in[m][0..ss_tiles)) * inv_d + eps); ss_in == nullptr -> 1
  const float* ss_in = nullptr;
  int ss_tiles = 0;
  float inv_d = 0.f, eps = 0.f;
  float* y = nullptr;  // F32 output / ARGMAX optional logits
  bf16* out_bf = nullptr;  // BF16 output (pgemm.hip)
  // QKV: RoPE + paged cache write + q out
  const int* positions = nullptr;
  const int* slots = nullptr;
  const float* cos_sin = nullptr;
  bf16* q_out = nullptr;
  bf16* k_cache = nullptr;
  bf16* v_cache = nullptr;
  int Hq = 0, Hkv = 0, BS = 0;
  // RESID: resid += y; xw_out = bf16(resid * w_next); ss_out[m][tile] = sum(resid^2)
  float* resid = nullptr;
  const bf16* w_next = nullptr;
  bf16* xw_out = nullptr;
  float* ss_out = nullptr;
  // SWIGLU
  bf16* act = nullptr;
  // ARGMAX (fused sampling)
  const float* temps = nullptr;
  const unsigned long long* seeds = nullptr;
  const long long* step = nullptr;
  unsigned long long* keys = nullptr;
  int n_offset = 0;
  // XAR (row-parallel projection under TP): the all-reduce communicator (granule slots, decode_epi.h) and its
  // per-output-tile epoch counters (device memory, zero at creation): every XAR launch on a communicator covers
  // all N / 16 tiles, so tile t's counter is the same on every rank; the tile's workgroup bumps it with a plain
  // store (no atomics, no cross-workgroup fan-in), and kernel boundaries make it visible to the next launch
  XgmiArgs xp;
  unsigned* xar_ctr = nullptr;
  // split-K workspace of the x-resident decode GEMM (decode_gemm.hip, go_xres): ks_ws fp32 partial tiles
  // (256 floats per (tile, split)), ks_cnt one arrival counter per 16-row tile (zero, re-armed in-launch);
  // nullptr -> whole-K tiles only
  float* ks_ws = nullptr;
  int* ks_cnt = nullptr;
  long long ks_cap = 0;  // floats in ks_ws
  int ks_ncnt = 0;       // ints in ks_cnt
};
void set_decode_gemm_variant(int v);  // -1: default heuristic
void set_decode_ksplit(int on);       // x-resident decode GEMM remainder split over K (default off)
void set_decode_halves(int on);       // x-resident decode GEMM remainder tiles as row halves (default off)
void set_decode_gemm_nt(int on);      // non-temporal weight-stream loads (keeps the variant choice)
void launch_decode_gemm(int epi, const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e,
                        hipStream_t s);
// Row-parallel decode projection + xGMI all-reduce + residual add + next-norm prep in ONE launch
// (DECODE_EPI_XAR).  false (nothing launched): no variant whose whole grid is co-resident on this GPU (the
// workgroups wait on their peers' tiles) -- the caller runs the two-launch form.
bool launch_decode_gemm_xar(const bf16* x, const bf16* W, int M, int N, int K, const DecodeEpi& e, hipStream_t s);
// test-only: every rank of this process in ONE launch (grid z = rank; co-residency checked)
constexpr int XAR_MULTI_MAX = 8;
struct XarMulti {
  const bf16* x[XAR_MULTI_MAX];
  DecodeEpi e[XAR_MULTI_MAX];
  int delay_rank = -1;                 // test hook: this rank's workgroups start delay_ticks late (a slow peer)
  unsigned long long delay_ticks = 0;
};
bool launch_decode_gemm_xar_multi(const XarMulti& m, int world, const bf16* W, int M, int N, int K, int xres,
                                  hipStream_t s);
// ss: [T][parts] partial sums of squares, as launch_add_prep
void launch_embed_prep(const int* ids, const int* src, const int* prev, const bf16* table, float* resid, const bf16* w,
                       bf16* xw, float* ss, int T, int d, int parts, hipStream_t s);
// ss: [T][parts] partial sums of squares (parts column slices of each row, one workgroup each)
void launch_add_prep(LinOut delta, float* resid, const bf16* w, bf16* xw, float* ss, int T, int d, int parts,
                     hipStream_t s);
void launch_rownorm(const bf16* xw, const float* ss, int ss_tiles, float eps, bf16* out, int T, int d, hipStream_t s);

// mgemm.hip -- medium-M (65..256 tokens) projection into fp32 split-K slabs y[S][M][N]; W is the
// MFMA-preshuffled weight copy, 64 * rw | N, 64 * S | K
void launch_mgemm(const bf16* x, const bf16* Wshuf, float* y, int M, int N, int K, int S, int rw, hipStream_t s);
// mgemm with a fused consumer epilogue (DECODE_EPI_QKV / RESID / SWIGLU / F32 of decode_epi.h): y is the
// [S][M][N] fp32 slab scratch (S > 1: in-launch split-K reduction by the last workgroup of each column group),
// counters [N / (64 rw)] ints, zero before the first launch (re-armed by the kernel)
void launch_mgemm_epi(int epi, const bf16* x, const bf16* Wshuf, float* y, int M, int N, int K, int S, int rw,
                      const DecodeEpi& e, int* counters, hipStream_t s);
void set_mgemm_nt(int on);  // non-temporal weight DMA (A/B knob)

// pgemm.hip -- prefill projection GEMM (hundreds+ rows) on the MFMA-preshuffled weights: tile shape `cfg`
// (pgemm_cfg_shape: BM tokens x BN features per 512-thread block), S k-splits over grid.y (S > 1: slab
// [S][M][N] fp32 scratch + counters [tiles] ints zero before the first launch, re-armed by the kernel), fused
// epilogue `epi` (DECODE_EPI_F32 / BF16 / QKV / SWIGLU / RESID -- RESID writes ss_out [M][N / BN]).
// N % BN == 0, K % (64 S) == 0; rows past M are padded in-kernel.
int pgemm_cfg_shape(int cfg, int* bm, int* bn);
void launch_pgemm(int epi, int cfg, const bf16* x, const bf16* Wshuf, int M, int N, int K, int S, const DecodeEpi& e,
                  float* slab, int* counters, hipStream_t s);
// grouped (MoE expert) mode: expert e < E owns rows [offsets[e_lo + e], offsets[e_lo + e + 1]) of x [R][K] and of
// the output, weights Wshuf + e * wstride ([N][K] preshuffled per expert).  The grid covers ceil(R / BM) + E m-tiles
// per n-tile (segment bounds stay on the device: graph-capturable); blocks past the real tiles exit.  epi:
// DECODE_EPI_SWIGLU_SPLIT (act [R][N / 2]), BF16 (out_bf [R][N]) or F32 (y [R][N]; S > 1: slab [S][R][N]).
struct PgGroup {
  const int* offsets = nullptr;
  int e_lo = 0, E = 0;
  long long wstride = 0;
};
void launch_pgemm_grouped(int epi, int cfg, const bf16* x, const bf16* Wshuf, int R, int N, int K, int S,
                          const PgGroup& g, const DecodeEpi& e, float* slab, hipStream_t s);

// norm.hip
void launch_rms_norm(LinOut x, const bf16* w, bf16* out, int T, int d, float eps, hipStream_t s);
void launch_add_rms_norm(LinOut delta, float* residual, const bf16* w, bf16* out, int T, int d, float eps,
                         hipStream_t s);
void launch_embed_rms_norm(const int* ids, const bf16* table, float* residual, const bf16* w, bf16* out, int T,
                           int d, float eps, hipStream_t s, const int* src = nullptr, const int* prev = nullptr);

// rope_cache.hip
void launch_rope_cache(LinOut qkv, const int* positions, const int* slots, const float* cos_sin, bf16* q_out,
                       bf16* k_cache, bf16* v_cache, int T, int Hq, int Hkv, int D, int BS, hipStream_t s,
                       int perm = 0, int decode = 0);

// attention.hip
void launch_attn_decode(const bf16* q, const bf16* k_cache, const bf16* v_cache, const int* block_tables,
                        const int* ctx_lens, bf16* out, float* tmp_o, float* tmp_ml, int* counters, int num_seqs,
                        int Hq, int Hkv, int BS, int max_blocks, int max_parts, float scale, hipStream_t s);
// decode attention switches to the streaming long-context kernel from this block-table span (0: never)
void set_attn_stream_min(int tokens);
// wide batches: one wave per (seq, kv head) from min_units units for spans of >= min_span tokens
void set_attn_wave(int min_units, int min_span);
void launch_attn_prefill(const bf16* q, const bf16* k_cache, const bf16* v_cache, const int* block_tables,
                         const int* ctx_lens, const int* cu_q, const int* tiles, int num_tiles, bf16* out, int Hq,
                         int Hkv, int BS, int max_blocks, float scale, hipStream_t s);

// skinny_gemm.hip
void launch_skinny_gemm(const bf16* x, const bf16* W, float* y, int M, int N, int K, int S, hipStream_t s,
                        int variant = 0);
void launch_skinny_gemm_argmax(const bf16* x, const bf16* W, float* logits_or_null, int M, int N, int K,
                               const float* temps, const unsigned long long* seeds, const long long* step,
                               unsigned long long* tile_keys, int n_offset, hipStream_t s);
void launch_argmax_reduce(const unsigned long long* tile_keys, int M, int ntiles, unsigned long long* out_keys,
                          int* out_ids, hipStream_t s);

// sampling.hip: temperature + top-k + top-p over full-vocab fp32 logits [B, V]; rows without a
// filter (or greedy) keep out_ids untouched
void launch_sample_filtered(const float* logits, int B, int V, const float* temps, const int* top_k, const float* top_p,
                            const long long* seeds, const long long* step, int* out_ids, hipStream_t s);
// greedy / temperature (Gumbel-max) sampling over fp32 logits [B, V]: the fused lm_head
// epilogue's keys and RNG, for decode batches wider than the fused kernels
void launch_logits_argmax(const float* logits, int B, int V, const float* temps, const long long* seeds,
                          const long long* step, int n_offset, unsigned long long* out_keys, int* out_ids,
                          hipStream_t s);

// activation.hip
void launch_swiglu(LinOut gu, bf16* out, int T, int F, hipStream_t s, int interleaved = 0);

// moe.hip
void launch_moe_route(LinOut logits, int ld, int T, int E, int k, int* ids, float* w, hipStream_t s);
// fp32 logits [T][16] = x [T][d] . Wr[16][d]^T (router rows padded to 16), d % 128 == 0
void launch_moe_router(const bf16* x, const bf16* Wr, float* logits, int T, int d, hipStream_t s);
// dst (optional): each assignment's row in its segment (the scatter then runs with cursor == nullptr)
void launch_moe_align(const int* ids, int n, int E, int* counts, int* offsets, int* cursor, hipStream_t s,
                      int* dst = nullptr);
void launch_moe_scatter(const bf16* x, int T, int d, int k, int E, const int* ids, const int* offsets, int* cursor,
                        bf16* xs, int R, int* dst, int* src_tok, hipStream_t s);
// E_all: experts in the global numbering of `offsets` (sizes the streaming path's row blocks); 0 = E.
// pre: W MFMA-preshuffled per expert (the weight-streaming path only)
void launch_grouped_gemm(const bf16* xs, const bf16* W, const int* offsets, void* y, int R, int E, int e0, int N,
                         int K, int out, hipStream_t s, int E_all = 0, bool pre = false);
// grouped_gemm's weight-streaming path on row-major weights: 0 never, 1 where it measured faster (default),
// 2 always; + 10 x (2 | 4): weight tiles per wave
void set_grouped_stream_policy(int p);
void launch_grouped_skinny(const bf16* xs, const bf16* W, const int* offsets, float* y, int R, int E, int e0, int N,
                           int K, int S, hipStream_t s, bool wshuf = false);
void launch_moe_combine(LinOut y, int R, const int* dst, const int* ids, int e_lo, int e_hi, const float* w, int T, int k,
                        int d, float* out, int accumulate, hipStream_t s);
// decode (T <= 8, E <= 64, k <= 8, d <= 4096, d % 8 == 0): rms_norm + router + route + align + scatter as one launch
void launch_moe_decode_route(const float* resid, const bf16* lnw, float eps, const bf16* Wr, int T, int d, int E, int k,
                             int* ids, float* w, int* counts, int* offsets, int* cursor, bf16* xs, int* dst,
                             hipStream_t s);
// expert parallelism over replicated tokens (moe.hip): the weighted partial of each token's local experts pushed
// to its slice owner (cursor[N] zeroed by the caller), and the owner's rank-ordered sum as bf16 [S][d]
void launch_moe_owner_pack(LinOut y, int R, const int* dst, const int* ids, const float* w, int e_lo, int e_hi, int T,
                           int k, int d, int S, int cap, int* cursor, float* send, int* side, hipStream_t s);
void launch_moe_owner_combine(const float* recv, const int* side, const int* rcnt, int N, int cap, int S, int Tr,
                              int d, int* pos, bf16* out, hipStream_t s);
// decode, every expert local: moe_combine + add_prep as one launch (ss [T, parts]: partials over column parts)
void launch_moe_combine_prep(LinOut y, int R, const int* dst, const int* ids, int E, const float* w, int T, int k, int d,
                             float* resid, const bf16* w_next, bf16* xw, float* ss, int parts, hipStream_t s);

// xgmi_ar.hip: one-shot all-reduce over xGMI peer memory (IPC-mapped buffers of every TP rank); the
// constants and the push descriptor live at the top of this header (the decode GEMMs push into the slots)
long long xgmi_buffer_bytes(int world, long long slot_bytes);
int xgmi_chunk(long long n, long long max_wg);
void launch_xgmi_all_reduce(const XgmiArgs& c, const void* in, void* out, long long n, int elem, hipStream_t s);
void launch_xgmi_keys_max(const XgmiArgs& c, const unsigned long long* keys, int* ids, int B, hipStream_t s);
void launch_xgmi_add_prep(const XgmiArgs& c, const float* y, float* resid, const bf16* w, bf16* xw, float* ss, int T,
                          int d, int parts, hipStream_t s);
// test-only: the ranks of one process as grid slices of ONE launch (co-resident by construction).
// add_prep: in = y, out = resid, xw, ss per rank; w shared
constexpr int XG_MULTI_MAX = 8;
constexpr int XG_MULTI_MAX_GROUPS = 1024;  // all slices co-resident (they wait on each other)
struct XgmiMulti {
  XgmiArgs c[XG_MULTI_MAX];
  const void* in[XG_MULTI_MAX];
  void* out[XG_MULTI_MAX];
  void* xw[XG_MULTI_MAX];
  float* ss[XG_MULTI_MAX];
  const bf16* w;
  int delay_rank;                  // this slice waits delay_ticks (100 MHz wall clock) before pushing (-1: none)
  unsigned long long delay_ticks;
};
void launch_xgmi_all_reduce_multi(const XgmiMulti& m, int world, long long n, int elem, hipStream_t s);
void launch_xgmi_add_prep_multi(const XgmiMulti& m, int world, int T, int d, int parts, hipStream_t s);
void launch_xgmi_keys_max_multi(const XgmiMulti& m, int world, int B, hipStream_t s);
// R3: unpadded expert all-to-all over xGMI peer memory (xgmi_ar.hip, xgmi_a2a_kernel).  Block q of `src` (rows
// [q cap, q cap + counts[q]), counts read on the DEVICE) lands as block `rank` of rank q's `dst`; only routed rows
// cross the links (no worst-case capacity padding on the wire).  Slot (parity, source) of the communicator's
// buffer: [0, 64) row count | side ints [cap] | rows [cap][row_bytes] (16-B aligned).
constexpr int XA_WG = 128;  // workgroups per rank in one all-to-all launch (flag words wg x source)
struct XgmiA2AArgs {
  XgmiArgs c;
  const char* src = nullptr;    // [world * cap][row_bytes]
  const int* counts = nullptr;  // [world] rows of block q for rank q
  const int* side = nullptr;    // optional [world * cap] int travelling with each row
  char* dst = nullptr;          // [world * cap][row_bytes]: block s <- rank s (rows past its count untouched)
  int* dst_side = nullptr;      // optional [world * cap]: received side ints, -1 past each block's count
  int* dst_counts = nullptr;    // optional [world]: rows received from each rank
  int cap = 0, row_bytes = 0;
};
long long xgmi_a2a_slot_bytes(int cap, int row_bytes);
void launch_xgmi_a2a(const XgmiA2AArgs& a, hipStream_t s);
// test-only: every rank of this process in one launch (grid y = rank), rank `delay_rank` held back delay_ticks
struct XgmiA2AMulti {
  XgmiA2AArgs a[XG_MULTI_MAX];
  int delay_rank;
  unsigned long long delay_ticks;
};
void launch_xgmi_a2a_multi(const XgmiA2AMulti& m, int world, hipStream_t s);
