// Host-side launch entry points of the symmetry_amd HIP kernels.
// Every launcher enqueues on the given stream, allocates nothing and never
// synchronises, so the calling op can be captured into a hipGraph.
// Shape/alignment preconditions are validated by the torch op layer
// (csrc/bindings/torch_ops.cpp) before any launch.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include "common.h"

// norm.hip
void launch_rms_norm(LinOut x, const bf16* w, bf16* out, int T, int d, float eps, hipStream_t s);
void launch_add_rms_norm(LinOut delta, float* residual, const bf16* w, bf16* out, int T, int d, float eps,
                         hipStream_t s);
void launch_embed_rms_norm(const int* ids, const bf16* table, float* residual, const bf16* w, bf16* out, int T,
                           int d, float eps, hipStream_t s);

// rope_cache.hip
void launch_rope_cache(LinOut qkv, const int* positions, const int* slots, const float* cos_sin, bf16* q_out,
                       bf16* k_cache, bf16* v_cache, int T, int Hq, int Hkv, int D, int BS, hipStream_t s);

// attention.hip
void launch_attn_decode(const bf16* q, const bf16* k_cache, const bf16* v_cache, const int* block_tables,
                        const int* ctx_lens, bf16* out, float* tmp_o, float* tmp_ml, int num_seqs, int Hq, int Hkv,
                        int BS, int max_blocks, int max_parts, float scale, hipStream_t s);
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

// activation.hip
void launch_swiglu(LinOut gu, bf16* out, int T, int F, hipStream_t s);

// moe.hip
void launch_moe_route(LinOut logits, int ld, int T, int E, int k, int* ids, float* w, hipStream_t s);
void launch_moe_align(const int* ids, int n, int E, int* counts, int* offsets, int* cursor, hipStream_t s);
void launch_moe_scatter(const bf16* x, int T, int d, int k, const int* ids, const int* offsets, int* cursor,
                        bf16* xs, int* dst, int* src_tok, hipStream_t s);
void launch_grouped_skinny(const bf16* xs, const bf16* W, const int* offsets, float* y, int R, int E, int e0, int N,
                           int K, int S, hipStream_t s);
void launch_moe_combine(LinOut y, int R, const int* dst, const int* ids, int e_lo, int e_hi, const float* w, int T, int k,
                        int d, float* out, int accumulate, hipStream_t s);
