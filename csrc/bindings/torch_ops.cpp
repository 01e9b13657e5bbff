// TORCH_LIBRARY registration of the symmetry_amd CDNA4 kernels.
//
// Every op is out-parameter style (the caller pre-allocates), allocates
// nothing, and launches on torch's current HIP stream, so the model runner can
// capture a whole decode step into a hipGraph.  All shape / dtype / layout
// preconditions the kernels and their grids assume are checked here, on the
// host, before any launch.
//
// Note on names: ROCm builds of PyTorch report HIP tensors with the device
// type spelled "cuda" (c10::DeviceType::CUDA); that is torch's enum, not a
// compatibility layer in this code.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "launchers.h"

namespace {

using at::Tensor;

hipStream_t cur_stream(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.get_device()).stream(); }

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.device().type() == c10::DeviceType::CUDA, name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_dtype(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}

template <typename T>
T* ptr(const Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}

// bf16 [T][N] or fp32 slabs [S][T][N] (or fp32 [T][N] == one slab).
LinOut linout(const Tensor& t, int64_t T, int64_t N, const char* name) {
  check_gpu(t, name);
  LinOut L{};
  L.ptr = t.data_ptr();
  if (t.scalar_type() == at::kBFloat16) {
    TORCH_CHECK(t.dim() == 2 && t.size(0) == T && t.size(1) == N, name, ": expected bf16 [", T, ",", N, "], got ",
                t.sizes());
    L.is_f32 = 0;
    L.nsplit = 1;
    L.split_stride = 0;
  } else {
    check_dtype(t, at::kFloat, name);
    if (t.dim() == 2) {
      TORCH_CHECK(t.size(0) == T && t.size(1) == N, name, ": expected [", T, ",", N, "], got ", t.sizes());
      L.nsplit = 1;
    } else {
      TORCH_CHECK(t.dim() == 3 && t.size(1) == T && t.size(2) == N, name, ": expected [S,", T, ",", N, "], got ",
                  t.sizes());
      L.nsplit = (int)t.size(0);
    }
    L.is_f32 = 1;
    L.split_stride = T * N;
  }
  return L;
}

int64_t rows_of(const Tensor& t) { return t.dim() == 3 ? t.size(1) : t.size(0); }
int64_t cols_of(const Tensor& t) { return t.size(t.dim() - 1); }

// ----------------------------------------------------------------------------------------------
void rms_norm(const Tensor& x, const Tensor& w, double eps, Tensor& out) {
  const int64_t T = rows_of(x), d = cols_of(x);
  check_gpu(w, "w");
  check_gpu(out, "out");
  check_dtype(w, at::kBFloat16, "w");
  check_dtype(out, at::kBFloat16, "out");
  TORCH_CHECK(d % 8 == 0 && d <= 16384, "rms_norm: d must be a multiple of 8 and <= 16384");
  TORCH_CHECK(w.numel() == d && out.numel() == T * d, "rms_norm: shape mismatch");
  const at::OptionalDeviceGuard g(x.device());
  launch_rms_norm(linout(x, T, d, "x"), ptr<bf16>(w), ptr<bf16>(out), (int)T, (int)d, (float)eps, cur_stream(x));
}

void add_rms_norm(const Tensor& delta, Tensor& residual, const Tensor& w, double eps, Tensor& out) {
  check_gpu(residual, "residual");
  check_dtype(residual, at::kFloat, "residual");
  TORCH_CHECK(residual.dim() == 2, "residual must be [T, d]");
  const int64_t T = residual.size(0), d = residual.size(1);
  check_gpu(w, "w");
  check_gpu(out, "out");
  check_dtype(w, at::kBFloat16, "w");
  check_dtype(out, at::kBFloat16, "out");
  TORCH_CHECK(d % 8 == 0 && d <= 16384, "add_rms_norm: d must be a multiple of 8 and <= 16384");
  TORCH_CHECK(w.numel() == d && out.numel() == T * d, "add_rms_norm: shape mismatch");
  const at::OptionalDeviceGuard g(residual.device());
  launch_add_rms_norm(linout(delta, T, d, "delta"), ptr<float>(residual), ptr<bf16>(w), ptr<bf16>(out), (int)T,
                      (int)d, (float)eps, cur_stream(residual));
}

void embed_rms_norm(const Tensor& ids, const Tensor& table, Tensor& residual, const Tensor& w, double eps,
                    Tensor& out, const c10::optional<Tensor>& src, const c10::optional<Tensor>& prev) {
  check_gpu(ids, "ids");
  check_gpu(table, "table");
  check_gpu(residual, "residual");
  check_dtype(ids, at::kInt, "ids");
  check_dtype(table, at::kBFloat16, "table");
  check_dtype(residual, at::kFloat, "residual");
  check_dtype(out, at::kBFloat16, "out");
  const int64_t T = ids.numel(), d = table.size(1);
  TORCH_CHECK(residual.numel() == T * d && out.numel() == T * d && w.numel() == d, "embed_rms_norm: shape mismatch");
  TORCH_CHECK(d % 8 == 0 && d <= 16384, "embed_rms_norm: bad d");
  TORCH_CHECK(src.has_value() == prev.has_value(), "embed_rms_norm: src and prev go together");
  const int* sp = nullptr;
  const int* pp = nullptr;
  if (src.has_value()) {
    check_gpu(*src, "src");
    check_gpu(*prev, "prev");
    check_dtype(*src, at::kInt, "src");
    check_dtype(*prev, at::kInt, "prev");
    TORCH_CHECK(src->numel() >= T, "embed_rms_norm: src shorter than ids");
    sp = ptr<int>(*src);
    pp = ptr<int>(*prev);
  }
  const at::OptionalDeviceGuard g(ids.device());
  launch_embed_rms_norm(ptr<int>(ids), ptr<bf16>(table), ptr<float>(residual), ptr<bf16>(w), ptr<bf16>(out), (int)T,
                        (int)d, (float)eps, cur_stream(ids), sp, pp);
}

void rope_cache(const Tensor& qkv, const Tensor& positions, const Tensor& slots, const Tensor& cos_sin,
                Tensor& q_out, Tensor& k_cache, Tensor& v_cache, int64_t Hq, int64_t Hkv, bool perm, bool decode) {
  check_gpu(positions, "positions");
  check_gpu(slots, "slots");
  check_gpu(cos_sin, "cos_sin");
  check_gpu(q_out, "q_out");
  check_gpu(k_cache, "k_cache");
  check_gpu(v_cache, "v_cache");
  check_dtype(positions, at::kInt, "positions");
  check_dtype(slots, at::kInt, "slots");
  check_dtype(cos_sin, at::kFloat, "cos_sin");
  check_dtype(q_out, at::kBFloat16, "q_out");
  check_dtype(k_cache, at::kBFloat16, "k_cache");
  check_dtype(v_cache, at::kBFloat16, "v_cache");
  const int64_t T = positions.numel();
  TORCH_CHECK(k_cache.dim() == 4, "k_cache must be [NB, Hkv, BS, D]");
  const int64_t BS = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(k_cache.size(1) == Hkv, "k_cache head count mismatch");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(0) == k_cache.size(0) && v_cache.size(1) == Hkv &&
                  v_cache.size(2) == D && v_cache.size(3) == BS,
              "v_cache must be [NB, Hkv, D, BS]");
  TORCH_CHECK(D % 16 == 0, "head dim must be a multiple of 16");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == D, "cos_sin must be [max_pos, D]");
  TORCH_CHECK(slots.numel() == T, "slots must have T entries");
  TORCH_CHECK(q_out.numel() == T * Hq * D, "q_out shape mismatch");
  const at::OptionalDeviceGuard g(positions.device());
  launch_rope_cache(linout(qkv, T, (Hq + 2 * Hkv) * D, "qkv"), ptr<int>(positions), ptr<int>(slots),
                    ptr<float>(cos_sin), ptr<bf16>(q_out), ptr<bf16>(k_cache), ptr<bf16>(v_cache), (int)T, (int)Hq,
                    (int)Hkv, (int)D, (int)BS, cur_stream(positions), perm ? 1 : 0, decode ? 1 : 0);
}

void check_cache(const Tensor& k_cache, const Tensor& v_cache) {
  check_gpu(k_cache, "k_cache");
  check_gpu(v_cache, "v_cache");
  check_dtype(k_cache, at::kBFloat16, "k_cache");
  check_dtype(v_cache, at::kBFloat16, "v_cache");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(3) == 128, "attention kernels require head_dim == 128");
  TORCH_CHECK(k_cache.size(2) % 32 == 0 && (k_cache.size(2) & (k_cache.size(2) - 1)) == 0,
              "attention kernels require a power-of-two block_size >= 32");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(2) == 128 && v_cache.size(3) == k_cache.size(2),
              "v_cache must be [NB, Hkv, D, BS]");
}

void attn_decode(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                 const Tensor& ctx_lens, Tensor& out, Tensor& tmp_o, Tensor& tmp_ml, Tensor& counters, double scale) {
  check_gpu(q, "q");
  check_dtype(q, at::kBFloat16, "q");
  check_cache(k_cache, v_cache);
  check_gpu(block_tables, "block_tables");
  check_gpu(ctx_lens, "ctx_lens");
  check_dtype(block_tables, at::kInt, "block_tables");
  check_dtype(ctx_lens, at::kInt, "ctx_lens");
  check_gpu(out, "out");
  check_dtype(out, at::kBFloat16, "out");
  TORCH_CHECK(q.dim() == 3 && q.size(2) == 128, "q must be [num_seqs, Hq, 128]");
  const int64_t S = q.size(0), Hq = q.size(1), Hkv = k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0 && Hq / Hkv <= 16, "GQA group must divide and be <= 16");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= S, "block_tables must be [>=num_seqs, max_blocks]");
  TORCH_CHECK(ctx_lens.numel() >= S, "ctx_lens too short");
  TORCH_CHECK(out.numel() == S * Hq * 128, "out shape mismatch");
  check_gpu(tmp_o, "tmp_o");
  check_gpu(tmp_ml, "tmp_ml");
  TORCH_CHECK(tmp_o.dim() == 4 && tmp_o.size(0) >= S && tmp_o.size(1) == Hq && tmp_o.size(3) == 128,
              "tmp_o must be [>=num_seqs, Hq, max_parts, 128]");
  const int64_t max_parts = tmp_o.size(2);
  TORCH_CHECK(tmp_ml.numel() >= S * Hq * max_parts * 2, "tmp_ml too small");
  const int64_t BS = k_cache.size(2), max_blocks = block_tables.size(1);
  TORCH_CHECK(max_parts * 256 >= max_blocks * BS, "tmp_o has too few partitions for the block table span");
  check_gpu(counters, "counters");
  check_dtype(counters, at::kInt, "counters");
  TORCH_CHECK(counters.numel() >= S * Hkv, "counters must hold num_seqs * Hkv zero-initialised ints");
  const at::OptionalDeviceGuard g(q.device());
  launch_attn_decode(ptr<bf16>(q), ptr<bf16>(k_cache), ptr<bf16>(v_cache), ptr<int>(block_tables), ptr<int>(ctx_lens),
                     ptr<bf16>(out), ptr<float>(tmp_o), ptr<float>(tmp_ml), ptr<int>(counters), (int)S, (int)Hq,
                     (int)Hkv, (int)BS, (int)max_blocks, (int)max_parts, (float)scale, cur_stream(q));
}

void attn_prefill(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                  const Tensor& ctx_lens, const Tensor& cu_q, const Tensor& tiles, Tensor& out, double scale) {
  check_gpu(q, "q");
  check_dtype(q, at::kBFloat16, "q");
  check_cache(k_cache, v_cache);
  for (auto* t : {&block_tables, &ctx_lens, &cu_q, &tiles}) {
    check_gpu(*t, "index tensor");
    check_dtype(*t, at::kInt, "index tensor");
  }
  check_gpu(out, "out");
  check_dtype(out, at::kBFloat16, "out");
  TORCH_CHECK(q.dim() == 3 && q.size(2) == 128, "q must be [T, Hq, 128]");
  const int64_t Hq = q.size(1), Hkv = k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0, "GQA group must divide");
  TORCH_CHECK(tiles.dim() == 2 && tiles.size(1) == 2, "tiles must be [n, 2]");
  TORCH_CHECK(out.numel() == q.numel(), "out shape mismatch");
  TORCH_CHECK(cu_q.numel() == ctx_lens.numel() + 1, "cu_q must have num_seqs + 1 entries");
  const at::OptionalDeviceGuard g(q.device());
  launch_attn_prefill(ptr<bf16>(q), ptr<bf16>(k_cache), ptr<bf16>(v_cache), ptr<int>(block_tables),
                      ptr<int>(ctx_lens), ptr<int>(cu_q), ptr<int>(tiles), (int)tiles.size(0), ptr<bf16>(out),
                      (int)Hq, (int)Hkv, (int)k_cache.size(2), (int)block_tables.size(1), (float)scale, cur_stream(q));
}

void skinny_gemm(const Tensor& x, const Tensor& w, Tensor& y, int64_t variant) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_gpu(y, "y");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(w, at::kBFloat16, "w");
  check_dtype(y, at::kFloat, "y");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 3, "skinny_gemm: x [M,K], w [N,K], y [S,M,N]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0), S = y.size(0);
  TORCH_CHECK(w.size(1) == K, "skinny_gemm: K mismatch");
  TORCH_CHECK(M >= 1 && M <= 64, "skinny_gemm: M must be in [1, 64]");
  TORCH_CHECK(N % 16 == 0, "skinny_gemm: N must be a multiple of 16");
  TORCH_CHECK(S >= 1 && K % (S * 256) == 0, "skinny_gemm: K must be a multiple of 256 * nsplit");
  TORCH_CHECK(y.size(1) == M && y.size(2) == N, "skinny_gemm: y shape mismatch");
  const at::OptionalDeviceGuard g(x.device());
  TORCH_CHECK(variant != 3 || N % 32 == 0, "variant 3 needs N % 32 == 0");
  launch_skinny_gemm(ptr<bf16>(x), ptr<bf16>(w), ptr<float>(y), (int)M, (int)N, (int)K, (int)S, cur_stream(x),
                     (int)variant);
}

// Medium-M projection (65..256 rows) into fp32 split-K slabs; w is the MFMA-preshuffled weight copy.
void mgemm(const Tensor& x, const Tensor& w, Tensor& y, int64_t rw) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_gpu(y, "y");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(w, at::kBFloat16, "w");
  check_dtype(y, at::kFloat, "y");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 3, "mgemm: x [M,K], w [N,K], y [S,M,N]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0), S = y.size(0);
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && y.is_contiguous(), "mgemm: contiguous operands");
  TORCH_CHECK(w.size(1) == K, "mgemm: K mismatch");
  TORCH_CHECK(M >= 1 && M <= 256, "mgemm: M must be in [1, 256]");
  TORCH_CHECK(rw >= 1 && rw <= 4 && (M <= 128 || rw <= 2), "mgemm: rw in 1..4 (<= 2 above 128 rows)");
  TORCH_CHECK(N % (64 * rw) == 0, "mgemm: N must be a multiple of 64 * rw");
  TORCH_CHECK(S >= 1 && K % (S * 64) == 0, "mgemm: K must be a multiple of 64 * nsplit");
  // 32-bit buffer offsets (x rows are addressed up to 16 * ceil(M / 16) * K * 2 bytes)
  TORCH_CHECK((M + 255) * K * 2 < (1LL << 31) && N * K * 2 < (1LL << 31), "mgemm: operands exceed 2 GB");
  TORCH_CHECK(y.size(1) == M && y.size(2) == N, "mgemm: y shape mismatch");
  const at::OptionalDeviceGuard g(x.device());
  launch_mgemm(ptr<bf16>(x), ptr<bf16>(w), ptr<float>(y), (int)M, (int)N, (int)K, (int)S, (int)rw, cur_stream(x));
}

// ---- prefill projection GEMM (pgemm.hip) ------------------------------------------------------------
// Checks shared by every pgemm entry: tile config, split, 32-bit buffer offsets, optional split-K scratch.
struct PgShape {
  int64_t M, N, K, S, bm, bn;
};

PgShape pg_check(const Tensor& x, const Tensor& w, int64_t cfg, int64_t S, const c10::optional<Tensor>& slab,
                 const c10::optional<Tensor>& counters) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(w, at::kBFloat16, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "pgemm: x [M,K], w [N,K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  int bm = 0, bn = 0;
  TORCH_CHECK(pgemm_cfg_shape((int)cfg, &bm, &bn), "pgemm: unknown tile config ", cfg);
  TORCH_CHECK(M >= 1 && N % bn == 0, "pgemm: N must be a multiple of the tile width ", bn);
  TORCH_CHECK(S >= 1 && K % (64 * S) == 0, "pgemm: K must be a multiple of 64 * S");
  const int64_t mpad = (M + bm - 1) / bm * bm;
  TORCH_CHECK(mpad * K * 2 < (1LL << 31) && N * K * 2 < (1LL << 31), "pgemm: operands exceed 2 GB");
  const int64_t tiles = mpad / bm * (N / bn);
  TORCH_CHECK(tiles < (1LL << 31) / 8, "pgemm: too many tiles");
  if (S > 1 && counters.has_value()) {  // in-launch reduction (without counters: y itself is the slab array)
    TORCH_CHECK(slab.has_value(), "pgemm: the in-launch split-K reduction needs a slab");
    check_gpu(*slab, "slab");
    check_dtype(*slab, at::kFloat, "slab");
    check_gpu(*counters, "counters");
    check_dtype(*counters, at::kInt, "counters");
    TORCH_CHECK(slab->numel() >= S * M * N, "pgemm: slab must hold [S, M, N] fp32");
    TORCH_CHECK(counters->numel() >= tiles, "pgemm: counters must hold one int per output tile");
  }
  return {M, N, K, S, bm, bn};
}

float* opt_f32(const c10::optional<Tensor>& t) { return t.has_value() ? ptr<float>(*t) : nullptr; }
int* opt_i32(const c10::optional<Tensor>& t) { return t.has_value() ? ptr<int>(*t) : nullptr; }

// y [M, N] bf16 or fp32 = x @ w^T (w MFMA-preshuffled).  S > 1 with counters: the k splits are summed in-launch
// (slab scratch); S > 1 without counters: y is fp32 [S, M, N], one partial slab per split (LinOut consumers sum).
void pgemm(const Tensor& x, const Tensor& w, Tensor& y, int64_t cfg, int64_t S, const c10::optional<Tensor>& slab,
           const c10::optional<Tensor>& counters) {
  const auto sh = pg_check(x, w, cfg, S, slab, counters);
  check_gpu(y, "y");
  if (S > 1 && !counters.has_value()) {
    check_dtype(y, at::kFloat, "y");
    TORCH_CHECK(y.dim() == 3 && y.size(0) == S && y.size(1) == sh.M && y.size(2) == sh.N, "pgemm: y must be [S, M, N]");
    DecodeEpi e;
    e.wshuf = 1;
    const at::OptionalDeviceGuard g(x.device());
    launch_pgemm(DECODE_EPI_F32, (int)cfg, ptr<bf16>(x), ptr<bf16>(w), (int)sh.M, (int)sh.N, (int)sh.K, (int)S, e,
                 ptr<float>(y), nullptr, cur_stream(x));
    return;
  }
  TORCH_CHECK(y.numel() == sh.M * sh.N, "pgemm: y must be [M, N]");
  DecodeEpi e;
  e.wshuf = 1;
  int epi = DECODE_EPI_F32;
  if (y.scalar_type() == at::kBFloat16) {
    epi = DECODE_EPI_BF16;
    e.out_bf = ptr<bf16>(y);
  } else {
    check_dtype(y, at::kFloat, "y");
    e.y = ptr<float>(y);
  }
  const at::OptionalDeviceGuard g(x.device());
  launch_pgemm(epi, (int)cfg, ptr<bf16>(x), ptr<bf16>(w), (int)sh.M, (int)sh.N, (int)sh.K, (int)S, e, opt_f32(slab),
               opt_i32(counters), cur_stream(x));
}

// pgemm with a fused epilogue (S = 1): QKV (RoPE + paged K/V write + q out), SWIGLU (tile-interleaved gate/up rows
// -> act [M, N / 2]), RESID (resid += y; xw = bf16(resid * w_next); ss_out [M, N / BN] one partial per row and
// block column).  ss_in: the producer's sum-of-squares partials of x's rows (deferred RMSNorm) or none.
void pg_norm_in(DecodeEpi& e, const c10::optional<Tensor>& ss_in, int64_t M, int64_t K, double eps) {
  if (!ss_in.has_value()) return;
  check_gpu(*ss_in, "ss_in");
  check_dtype(*ss_in, at::kFloat, "ss_in");
  TORCH_CHECK(ss_in->dim() == 2 && ss_in->size(0) >= M && ss_in->size(1) >= 1, "ss_in must be [>=M, P]");
  e.ss_in = ptr<float>(*ss_in);
  e.ss_tiles = (int)ss_in->size(1);
  e.inv_d = 1.f / (float)K;
  e.eps = (float)eps;
}

void pg_qkv(const Tensor& x, const Tensor& W, const c10::optional<Tensor>& ss_in, double eps, const Tensor& positions,
            const Tensor& slots, const Tensor& cos_sin, Tensor& q_out, Tensor& k_cache, Tensor& v_cache, int64_t Hq,
            int64_t Hkv, int64_t cfg) {
  const auto sh = pg_check(x, W, cfg, 1, c10::nullopt, c10::nullopt);
  for (auto* t : {&positions, &slots}) {
    check_gpu(*t, "index tensor");
    check_dtype(*t, at::kInt, "index tensor");
  }
  check_gpu(cos_sin, "cos_sin");
  check_dtype(cos_sin, at::kFloat, "cos_sin");
  check_cache(k_cache, v_cache);
  check_gpu(q_out, "q_out");
  check_dtype(q_out, at::kBFloat16, "q_out");
  TORCH_CHECK(sh.N == (Hq + 2 * Hkv) * 128, "pg_qkv: N must be (Hq + 2 Hkv) * 128");
  TORCH_CHECK(k_cache.size(1) == Hkv, "pg_qkv: cache head count");
  TORCH_CHECK(positions.numel() >= sh.M && slots.numel() >= sh.M, "pg_qkv: positions/slots too short");
  TORCH_CHECK(q_out.numel() >= sh.M * Hq * 128, "pg_qkv: q_out too small");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == 128, "pg_qkv: cos_sin [max_pos, 128]");
  DecodeEpi e;
  e.wshuf = 1;
  pg_norm_in(e, ss_in, sh.M, sh.K, eps);
  e.positions = ptr<int>(positions);
  e.slots = ptr<int>(slots);
  e.cos_sin = ptr<float>(cos_sin);
  e.q_out = ptr<bf16>(q_out);
  e.k_cache = ptr<bf16>(k_cache);
  e.v_cache = ptr<bf16>(v_cache);
  e.Hq = (int)Hq;
  e.Hkv = (int)Hkv;
  e.BS = (int)k_cache.size(2);
  const at::OptionalDeviceGuard g(x.device());
  launch_pgemm(DECODE_EPI_QKV, (int)cfg, ptr<bf16>(x), ptr<bf16>(W), (int)sh.M, (int)sh.N, (int)sh.K, 1, e, nullptr,
               nullptr, cur_stream(x));
}

void pg_swiglu(const Tensor& x, const Tensor& W, const c10::optional<Tensor>& ss_in, double eps, Tensor& act,
               int64_t cfg) {
  const auto sh = pg_check(x, W, cfg, 1, c10::nullopt, c10::nullopt);
  check_gpu(act, "act");
  check_dtype(act, at::kBFloat16, "act");
  TORCH_CHECK(act.numel() == sh.M * sh.N / 2, "pg_swiglu: act must be [M, N / 2]");
  DecodeEpi e;
  e.wshuf = 1;
  pg_norm_in(e, ss_in, sh.M, sh.K, eps);
  e.act = ptr<bf16>(act);
  const at::OptionalDeviceGuard g(x.device());
  launch_pgemm(DECODE_EPI_SWIGLU, (int)cfg, ptr<bf16>(x), ptr<bf16>(W), (int)sh.M, (int)sh.N, (int)sh.K, 1, e, nullptr,
               nullptr, cur_stream(x));
}

// grouped experts (MoE prefill): W [E, N, K] preshuffled per expert, xs [R, K] rows permuted into expert segments
// (offsets [>= e_lo + E + 1] int32 on the device, global expert numbering), expert e < E of W = global e_lo + e.
// epi SWIGLU_SPLIT: y = act [R, N / 2] bf16 (W rows [gate; up]); BF16: y [R, N] bf16; F32: y [R, N] fp32, or
// [S, R, N] fp32 partial slabs for S > 1.  Rows outside the E segments are not written.
void pg_grouped(const Tensor& xs, const Tensor& W, const Tensor& offsets, int64_t e_lo, Tensor& y, int64_t epi,
                int64_t cfg, int64_t S) {
  check_gpu(xs, "xs");
  check_gpu(W, "W");
  check_gpu(offsets, "offsets");
  check_gpu(y, "y");
  check_dtype(xs, at::kBFloat16, "xs");
  check_dtype(W, at::kBFloat16, "W");
  check_dtype(offsets, at::kInt, "offsets");
  TORCH_CHECK(xs.dim() == 2 && W.dim() == 3 && W.size(2) == xs.size(1), "pg_grouped: xs [R, K], W [E, N, K]");
  const int64_t R = xs.size(0), K = xs.size(1), E = W.size(0), N = W.size(1);
  TORCH_CHECK(offsets.numel() >= e_lo + E + 1, "pg_grouped: offsets too short");
  int bm = 0, bn = 0;
  TORCH_CHECK(pgemm_cfg_shape((int)cfg, &bm, &bn), "pg_grouped: unknown tile config ", cfg);
  TORCH_CHECK(R >= 1 && N % bn == 0, "pg_grouped: N must be a multiple of the tile width ", bn);
  TORCH_CHECK(S >= 1 && K % (64 * S) == 0, "pg_grouped: K must be a multiple of 64 * S");
  TORCH_CHECK(S == 1 || epi == DECODE_EPI_F32, "pg_grouped: split-K slabs are fp32 only");
  TORCH_CHECK((int64_t)bm * K * 2 < (1LL << 31) && N * K * 2 < (1LL << 31) && R * N < (1LL << 31),
              "pg_grouped: operands exceed 2 GB");
  TORCH_CHECK(((R + bm - 1) / bm + E) * (N / bn) < (1LL << 31) / 8, "pg_grouped: too many tiles");
  DecodeEpi e;
  e.wshuf = 1;
  if (epi == DECODE_EPI_SWIGLU_SPLIT) {
    check_dtype(y, at::kBFloat16, "act");
    TORCH_CHECK(y.dim() == 2 && y.size(0) == R && y.size(1) == N / 2, "pg_grouped: act must be [R, N / 2]");
    e.act = ptr<bf16>(y);
  } else if (epi == DECODE_EPI_BF16) {
    check_dtype(y, at::kBFloat16, "y");
    TORCH_CHECK(y.dim() == 2 && y.size(0) == R && y.size(1) == N, "pg_grouped: y must be [R, N]");
    e.out_bf = ptr<bf16>(y);
  } else {
    TORCH_CHECK(epi == DECODE_EPI_F32, "pg_grouped: epi must be SWIGLU_SPLIT, BF16 or F32");
    check_dtype(y, at::kFloat, "y");
    TORCH_CHECK(y.numel() == S * R * N && y.size(-1) == N, "pg_grouped: y must be [S, R, N] fp32");
    e.y = ptr<float>(y);
  }
  TORCH_CHECK(xs.is_contiguous() && W.is_contiguous() && y.is_contiguous(), "pg_grouped: contiguous tensors");
  PgGroup g;
  g.offsets = ptr<int>(offsets);
  g.e_lo = (int)e_lo;
  g.E = (int)E;
  g.wstride = N * K;
  const at::OptionalDeviceGuard dg(xs.device());
  launch_pgemm_grouped((int)epi, (int)cfg, ptr<bf16>(xs), ptr<bf16>(W), (int)R, (int)N, (int)K, (int)S, g, e,
                       ptr<float>(y), cur_stream(xs));
}

void pg_resid(const Tensor& x, const Tensor& W, Tensor& resid, const Tensor& w_next, Tensor& xw_out, Tensor& ss_out,
              int64_t cfg) {
  const auto sh = pg_check(x, W, cfg, 1, c10::nullopt, c10::nullopt);
  check_gpu(resid, "resid");
  check_dtype(resid, at::kFloat, "resid");
  check_gpu(w_next, "w_next");
  check_dtype(w_next, at::kBFloat16, "w_next");
  check_gpu(xw_out, "xw_out");
  check_dtype(xw_out, at::kBFloat16, "xw_out");
  check_gpu(ss_out, "ss_out");
  check_dtype(ss_out, at::kFloat, "ss_out");
  TORCH_CHECK(resid.numel() == sh.M * sh.N && xw_out.numel() == sh.M * sh.N && w_next.numel() == sh.N,
              "pg_resid: shape mismatch");
  TORCH_CHECK(ss_out.dim() == 2 && ss_out.size(0) >= sh.M && ss_out.size(1) == sh.N / sh.bn,
              "pg_resid: ss_out must be [M, N / BN]");
  DecodeEpi e;
  e.wshuf = 1;
  e.resid = ptr<float>(resid);
  e.w_next = ptr<bf16>(w_next);
  e.xw_out = ptr<bf16>(xw_out);
  e.ss_out = ptr<float>(ss_out);
  const at::OptionalDeviceGuard g(x.device());
  launch_pgemm(DECODE_EPI_RESID, (int)cfg, ptr<bf16>(x), ptr<bf16>(W), (int)sh.M, (int)sh.N, (int)sh.K, 1, e, nullptr,
               nullptr, cur_stream(x));
}

void lm_head_sample(const Tensor& x, const Tensor& w, const Tensor& temps, const Tensor& seeds, const Tensor& step,
                    Tensor& tile_keys, Tensor& out_keys, Tensor& out_ids, int64_t n_offset,
                    const c10::optional<Tensor>& logits) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(w, at::kBFloat16, "w");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "lm_head_sample: K mismatch");
  TORCH_CHECK(M >= 1 && M <= 64, "lm_head_sample: M must be in [1, 64]");
  TORCH_CHECK(N % 16 == 0 && K % 256 == 0, "lm_head_sample: N % 16 and K % 256 required");
  check_gpu(temps, "temps");
  check_dtype(temps, at::kFloat, "temps");
  check_gpu(seeds, "seeds");
  check_dtype(seeds, at::kLong, "seeds");
  check_gpu(step, "step");
  check_dtype(step, at::kLong, "step");
  TORCH_CHECK(temps.numel() >= M && seeds.numel() >= M && step.numel() >= 1, "lm_head_sample: sampling params");
  check_gpu(tile_keys, "tile_keys");
  check_dtype(tile_keys, at::kLong, "tile_keys");
  TORCH_CHECK(tile_keys.numel() >= M * (N / 16), "tile_keys too small");
  check_gpu(out_keys, "out_keys");
  check_dtype(out_keys, at::kLong, "out_keys");
  check_gpu(out_ids, "out_ids");
  check_dtype(out_ids, at::kInt, "out_ids");
  TORCH_CHECK(out_keys.numel() >= M && out_ids.numel() >= M, "outputs too small");
  float* lp = nullptr;
  if (logits.has_value()) {
    check_gpu(*logits, "logits");
    check_dtype(*logits, at::kFloat, "logits");
    TORCH_CHECK(logits->numel() == M * N, "logits shape mismatch");
    lp = ptr<float>(*logits);
  }
  const at::OptionalDeviceGuard g(x.device());
  hipStream_t s = cur_stream(x);
  auto* tk = reinterpret_cast<unsigned long long*>(tile_keys.data_ptr());
  launch_skinny_gemm_argmax(ptr<bf16>(x), ptr<bf16>(w), lp, (int)M, (int)N, (int)K, ptr<float>(temps),
                            reinterpret_cast<const unsigned long long*>(seeds.data_ptr()),
                            reinterpret_cast<const long long*>(step.data_ptr()), tk, (int)n_offset, s);
  launch_argmax_reduce(tk, (int)M, (int)(N / 16), reinterpret_cast<unsigned long long*>(out_keys.data_ptr()),
                       ptr<int>(out_ids), s);
}

void swiglu(const Tensor& gu, Tensor& out, bool interleaved) {
  check_gpu(out, "out");
  check_dtype(out, at::kBFloat16, "out");
  TORCH_CHECK(out.dim() == 2, "out must be [T, F]");
  const int64_t T = out.size(0), F = out.size(1);
  TORCH_CHECK(F % 8 == 0, "swiglu: F must be a multiple of 8");
  const at::OptionalDeviceGuard g(out.device());
  TORCH_CHECK(!interleaved || F % 8 == 0, "swiglu: interleaved layout needs F % 8");
  launch_swiglu(linout(gu, T, 2 * F, "gu"), ptr<bf16>(out), (int)T, (int)F, cur_stream(out), interleaved ? 1 : 0);
}

// ---- MoE -----------------------------------------------------------------------------------------
// Routing: logits LinOut [T][E] -> ids/w [T][k], counts [E] (zeroed here), offsets [E+1],
// then rows scattered into expert segments of xs [T*k][d]; dst [T][k] row of each assignment.
void moe_route_permute(const Tensor& logits, const Tensor& x, int64_t k, int64_t E_, Tensor& ids, Tensor& w,
                       Tensor& counts, Tensor& offsets, Tensor& cursor, Tensor& xs, Tensor& dst) {
  check_gpu(x, "x");
  check_dtype(x, at::kBFloat16, "x");
  const int64_t T = x.size(0), d = x.size(1);
  const int64_t E = E_;
  TORCH_CHECK(counts.numel() >= E, "moe: counts too small");
  TORCH_CHECK(E >= 1 && E <= 64 && k >= 1 && k <= 8 && k <= E, "moe: need 1 <= k <= E <= 64, k <= 8");
  TORCH_CHECK(d % 8 == 0, "moe: d % 8");
  for (auto* t : {&ids, &counts, &offsets, &cursor, &dst}) {
    check_gpu(*t, "index tensor");
    check_dtype(*t, at::kInt, "index tensor");
  }
  check_gpu(w, "w");
  check_dtype(w, at::kFloat, "w");
  check_gpu(xs, "xs");
  check_dtype(xs, at::kBFloat16, "xs");
  TORCH_CHECK(ids.numel() >= T * k && w.numel() >= T * k && dst.numel() >= T * k, "moe: [T, k] outputs too small");
  TORCH_CHECK(offsets.numel() >= E + 1 && cursor.numel() >= E, "moe: offsets/cursor too small");
  TORCH_CHECK(xs.numel() >= T * k * d, "moe: xs too small");
  const at::OptionalDeviceGuard g(x.device());
  hipStream_t s = cur_stream(x);
  const int64_t ld = logits.size(logits.dim() - 1);
  TORCH_CHECK(ld >= E, "moe: logits narrower than E");
  launch_moe_route(linout(logits, T, ld, "logits"), (int)ld, (int)T, (int)E, (int)k, ptr<int>(ids), ptr<float>(w), s);
  // rows placed by the align kernel (LDS atomics): the scatter is a plain copy
  launch_moe_align(ptr<int>(ids), (int)(T * k), (int)E, ptr<int>(counts), ptr<int>(offsets), ptr<int>(cursor), s,
                   ptr<int>(dst));
  launch_moe_scatter(ptr<bf16>(x), (int)T, (int)d, (int)k, (int)E, ptr<int>(ids), ptr<int>(offsets), nullptr,
                     ptr<bf16>(xs), (int)(T * k), ptr<int>(dst), nullptr, s);
}

// Router logits: fp32 [T, 16] = x [T, d] @ Wr[16, d]^T (router rows padded to 16).
void moe_router(const Tensor& x, const Tensor& Wr, Tensor& logits) {
  check_gpu(x, "x");
  check_gpu(Wr, "Wr");
  check_gpu(logits, "logits");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(Wr, at::kBFloat16, "Wr");
  check_dtype(logits, at::kFloat, "logits");
  TORCH_CHECK(x.dim() == 2 && Wr.dim() == 2 && Wr.size(0) == 16 && Wr.size(1) == x.size(1),
              "moe_router: x [T, d], Wr [16, d]");
  TORCH_CHECK(x.size(1) % 128 == 0, "moe_router: d % 128");
  TORCH_CHECK(logits.numel() == x.size(0) * 16 && logits.is_contiguous(), "moe_router: logits [T, 16]");
  TORCH_CHECK(x.is_contiguous() && Wr.is_contiguous(), "moe_router: contiguous inputs");
  const at::OptionalDeviceGuard g(x.device());
  launch_moe_router(ptr<bf16>(x), ptr<bf16>(Wr), ptr<float>(logits), (int)x.size(0), (int)x.size(1), cur_stream(x));
}

// Routing only: logits LinOut [T][E] -> top-k ids [T*k] + softmax-renormalised weights [T*k].
void moe_route(const Tensor& logits, int64_t T, int64_t k, int64_t E, Tensor& ids, Tensor& w) {
  check_gpu(ids, "ids");
  check_dtype(ids, at::kInt, "ids");
  check_gpu(w, "w");
  check_dtype(w, at::kFloat, "w");
  TORCH_CHECK(E >= 1 && E <= 64 && k >= 1 && k <= 8 && k <= E, "moe_route: need 1 <= k <= E <= 64, k <= 8");
  TORCH_CHECK(ids.numel() >= T * k && w.numel() >= T * k, "moe_route: outputs too small");
  const int64_t ld = logits.size(logits.dim() - 1);
  TORCH_CHECK(ld >= E, "moe_route: logits narrower than E");
  const at::OptionalDeviceGuard g(ids.device());
  launch_moe_route(linout(logits, T, ld, "logits"), (int)ld, (int)T, (int)E, (int)k, ptr<int>(ids), ptr<float>(w),
                   cur_stream(ids));
}

// Segment ids into groups: counts [G] + offsets [G+1] (exclusive prefix sum) + cursor [G] zeroed, from
// ids [n] (ids outside [0, G) ignored).
void moe_align(const Tensor& ids, int64_t G, Tensor& counts, Tensor& offsets, Tensor& cursor) {
  for (const Tensor* t : std::initializer_list<const Tensor*>{&ids, &counts, &offsets, &cursor}) {
    check_gpu(*t, "moe_align tensor");
    check_dtype(*t, at::kInt, "moe_align tensor");
  }
  TORCH_CHECK(G >= 1 && G <= 64 && counts.numel() >= G && offsets.numel() >= G + 1 && cursor.numel() >= G,
              "moe_align: 1 <= G <= 64 groups");
  const at::OptionalDeviceGuard g(ids.device());
  launch_moe_align(ptr<int>(ids), (int)ids.numel(), (int)G, ptr<int>(counts), ptr<int>(offsets), ptr<int>(cursor),
                   cur_stream(ids));
}

// Row scatter into group segments: for assignment a = t * k + j with group g = ids[a] in [0, G):
// row = offsets[g] + (running count of g); xs[row] = x[t]; dst[a] = row (src_tok[row] = t if given).
// Assignments with g outside [0, G) are skipped (dst[a] left as is).  cursor [G] must be zero; the
// segments may be any fixed starts (e.g. one capacity block per destination rank), rows past xs are dropped.
void moe_scatter(const Tensor& x, const Tensor& ids, int64_t k, int64_t G, const Tensor& offsets, Tensor& cursor,
                 Tensor& xs, Tensor& dst, const c10::optional<Tensor>& src_tok) {
  check_gpu(x, "x");
  check_dtype(x, at::kBFloat16, "x");
  check_gpu(xs, "xs");
  check_dtype(xs, at::kBFloat16, "xs");
  for (const Tensor* t : std::initializer_list<const Tensor*>{&ids, &offsets, &cursor, &dst}) {
    check_gpu(*t, "moe_scatter index");
    check_dtype(*t, at::kInt, "moe_scatter index");
  }
  TORCH_CHECK(x.dim() == 2 && xs.dim() == 2 && xs.size(1) == x.size(1), "moe_scatter: x [T, d], xs [R, d]");
  const int64_t T = x.size(0), d = x.size(1);
  TORCH_CHECK(d % 8 == 0 && k >= 1 && ids.numel() >= T * k && dst.numel() >= T * k, "moe_scatter: shapes");
  TORCH_CHECK(G >= 1 && offsets.numel() >= G + 1 && cursor.numel() >= G, "moe_scatter: offsets / cursor");
  int* st = nullptr;
  if (src_tok.has_value()) {
    check_gpu(*src_tok, "src_tok");
    check_dtype(*src_tok, at::kInt, "src_tok");
    TORCH_CHECK(src_tok->numel() >= xs.size(0), "moe_scatter: src_tok too small");
    st = ptr<int>(*src_tok);
  }
  const at::OptionalDeviceGuard g(x.device());
  launch_moe_scatter(ptr<bf16>(x), (int)T, (int)d, (int)k, (int)G, ptr<int>(ids), ptr<int>(offsets), ptr<int>(cursor),
                     ptr<bf16>(xs), (int)xs.size(0), ptr<int>(dst), st, cur_stream(x));
}

// Grouped MFMA GEMM over expert segments (any routed row count; segment bounds read on the device).
// mode 0: y bf16 [R, N]; 1: y fp32 [R, N]; 2: SwiGLU, W [E, 2N, K] = [gate; up] rows, y = act bf16 [R, N].
void grouped_gemm(const Tensor& xs, const Tensor& W, const Tensor& offsets, int64_t e0, Tensor& y, int64_t mode) {
  check_gpu(xs, "xs");
  check_gpu(W, "W");
  check_gpu(offsets, "offsets");
  check_gpu(y, "y");
  check_dtype(xs, at::kBFloat16, "xs");
  check_dtype(W, at::kBFloat16, "W");
  check_dtype(offsets, at::kInt, "offsets");
  const bool pre = (mode & 4) != 0;  // W MFMA-preshuffled per expert (models/layout.py::preshuffle)
  mode &= 3;
  check_dtype(y, mode == 1 ? at::kFloat : at::kBFloat16, "y");
  TORCH_CHECK(mode >= 0 && mode <= 2, "grouped_gemm: mode 0 (bf16), 1 (fp32), 2 (SwiGLU) [+4: preshuffled W]");
  TORCH_CHECK(W.dim() == 3 && xs.dim() == 2 && y.dim() == 2 && xs.is_contiguous() && W.is_contiguous() &&
                  y.is_contiguous(), "grouped_gemm: W [E, N, K], xs [R, K], y [R, N], contiguous");
  const int64_t E = W.size(0), K = W.size(2), R = xs.size(0);
  const int64_t N = mode == 2 ? W.size(1) / 2 : W.size(1);
  TORCH_CHECK(xs.size(1) == K && y.size(0) >= R && y.size(1) == N, "grouped_gemm: shape mismatch");
  TORCH_CHECK(K % 64 == 0 && (mode == 2 ? N % 64 == 0 : N % 128 == 0), "grouped_gemm: K % 64, N % 128 (SwiGLU: F % 64)");
  TORCH_CHECK(E >= 1 && E <= 64 && e0 >= 0 && offsets.numel() >= e0 + E + 1, "grouped_gemm: offsets must cover e0..e0+E");
  TORCH_CHECK(!pre || (E <= 8 && K % 256 == 0),
              "grouped_gemm: preshuffled weights take the streaming path (<= 8 local experts, K % 256)");
  const at::OptionalDeviceGuard g(xs.device());
  launch_grouped_gemm(ptr<bf16>(xs), ptr<bf16>(W), ptr<int>(offsets), y.data_ptr(), (int)R, (int)E, (int)e0, (int)N,
                      (int)K, (int)mode, cur_stream(xs), (int)(offsets.numel() - 1), pre);
}

// Dense medium-M projection on the weight-streaming kernel: mode 1 -> fp32 slabs y [S, M, N]; mode 3 -> SwiGLU of
// the decode layout's tile-interleaved gate/up rows, y = act bf16 [M, N / 2].  W MFMA-preshuffled [N, K].

void grouped_skinny(const Tensor& xs, const Tensor& W, const Tensor& offsets, int64_t e0, Tensor& y, bool wshuf) {
  check_gpu(xs, "xs");
  check_gpu(W, "W");
  check_gpu(offsets, "offsets");
  check_gpu(y, "y");
  check_dtype(xs, at::kBFloat16, "xs");
  check_dtype(W, at::kBFloat16, "W");
  check_dtype(offsets, at::kInt, "offsets");
  check_dtype(y, at::kFloat, "y");
  TORCH_CHECK(W.dim() == 3 && xs.dim() == 2 && y.dim() == 3, "grouped_skinny: W [E,N,K], xs [R,K], y [S,R,N]");
  const int64_t E = W.size(0), N = W.size(1), K = W.size(2), R = xs.size(0), S = y.size(0);
  TORCH_CHECK(xs.size(1) == K && y.size(1) == R && y.size(2) == N, "grouped_skinny: shape mismatch");
  TORCH_CHECK(e0 >= 0 && offsets.numel() >= e0 + E + 1, "grouped_skinny: offsets must cover experts e0..e0+E");
  TORCH_CHECK(N % 16 == 0 && K % (256 * S) == 0, "grouped_skinny: N % 16 and K % (256 S)");
  TORCH_CHECK(R <= 64, "grouped_skinny: at most 64 routed rows on this path (larger batches use library GEMMs)");
  const at::OptionalDeviceGuard g(xs.device());
  TORCH_CHECK(!wshuf || K % 32 == 0, "grouped_skinny: preshuffled weights need K % 32");
  launch_grouped_skinny(ptr<bf16>(xs), ptr<bf16>(W), ptr<int>(offsets), ptr<float>(y), (int)R, (int)E, (int)e0,
                        (int)N, (int)K, (int)S, cur_stream(xs), wshuf);
}

void moe_combine(const Tensor& y, const Tensor& dst, const Tensor& ids, int64_t e_lo, int64_t e_hi, const Tensor& w,
                 int64_t k, Tensor& out, bool accumulate) {
  check_gpu(out, "out");
  check_dtype(out, at::kFloat, "out");
  check_gpu(dst, "dst");
  check_dtype(dst, at::kInt, "dst");
  check_gpu(w, "w");
  check_dtype(w, at::kFloat, "w");
  TORCH_CHECK(out.dim() == 2, "out must be [T, d]");
  const int64_t T = out.size(0), d = out.size(1);
  const int64_t R = y.dim() == 3 ? y.size(1) : y.size(0);
  check_gpu(ids, "ids");
  check_dtype(ids, at::kInt, "ids");
  TORCH_CHECK(dst.numel() >= T * k && w.numel() >= T * k && ids.numel() >= T * k, "moe_combine: dst/w too small");
  TORCH_CHECK(d % 8 == 0, "moe_combine: d % 8");
  const at::OptionalDeviceGuard g(out.device());
  launch_moe_combine(linout(y, R, d, "y"), (int)R, ptr<int>(dst), ptr<int>(ids), (int)e_lo, (int)e_hi, ptr<float>(w), (int)T,
                     (int)k, (int)d, ptr<float>(out), accumulate ? 1 : 0, cur_stream(out));
}

// Expert parallelism over replicated tokens (moe.hip moe_owner_*): y = the expert outputs of this rank's routed
// rows ([R, d] or fp32 slabs), dst / ids / w [T*k] of ALL T tokens; send fp32 [N*cap, d], side int32 [N*cap],
// cursor int32 [N] (zeroed here): the weighted partial of every token with a local expert, grouped by slice owner.
void moe_owner_pack(const Tensor& y, const Tensor& dst, const Tensor& ids, const Tensor& w, int64_t e_lo, int64_t e_hi,
                    int64_t k, int64_t S, Tensor& cursor, Tensor& send, Tensor& side) {
  for (const Tensor* t : {&dst, &ids, (const Tensor*)&cursor, (const Tensor*)&side}) {
    check_gpu(*t, "moe_owner_pack index");
    check_dtype(*t, at::kInt, "moe_owner_pack index");
  }
  check_gpu(w, "w");
  check_dtype(w, at::kFloat, "w");
  check_gpu(send, "send");
  check_dtype(send, at::kFloat, "send");
  TORCH_CHECK(send.dim() == 2 && send.is_contiguous(), "moe_owner_pack: send [N * cap, d]");
  const int64_t N = cursor.numel(), d = send.size(1), T = dst.numel() / k;
  TORCH_CHECK(N >= 1 && send.size(0) % N == 0 && side.numel() >= send.size(0), "moe_owner_pack: send / side blocks");
  const int64_t cap = send.size(0) / N;
  TORCH_CHECK(S >= 1 && cap >= S && N * S >= T && d % 8 == 0, "moe_owner_pack: capacity / slice shapes");
  TORCH_CHECK(ids.numel() >= T * k && w.numel() >= T * k, "moe_owner_pack: ids / w too small");
  const int64_t R = y.dim() == 3 ? y.size(1) : y.size(0);
  TORCH_CHECK((y.dim() == 3 ? y.size(2) : y.size(1)) == d, "moe_owner_pack: y width");
  const at::OptionalDeviceGuard g(send.device());
  (void)hipMemsetAsync(cursor.data_ptr(), 0, N * sizeof(int), cur_stream(send));
  launch_moe_owner_pack(linout(y, R, d, "y"), (int)R, ptr<int>(dst), ptr<int>(ids), ptr<float>(w), (int)e_lo, (int)e_hi,
                        (int)T, (int)k, (int)d, (int)S, (int)cap, ptr<int>(cursor), ptr<float>(send), ptr<int>(side),
                        cur_stream(send));
}

// The slice owner's combine: recv fp32 [N*cap, d] (block s: source s's rows, rcnt[s] of them, side ints = slice
// token), pos int32 [N*S] scratch, out bf16 [S, d] = rank-ordered sums, rows >= Tr zero.
void moe_owner_combine(const Tensor& recv, const Tensor& side, const Tensor& rcnt, int64_t Tr, Tensor& pos,
                       Tensor& out) {
  check_gpu(recv, "recv");
  check_dtype(recv, at::kFloat, "recv");
  check_gpu(out, "out");
  check_dtype(out, at::kBFloat16, "out");
  for (const Tensor* t : {&side, &rcnt, (const Tensor*)&pos}) {
    check_gpu(*t, "moe_owner_combine index");
    check_dtype(*t, at::kInt, "moe_owner_combine index");
  }
  TORCH_CHECK(recv.dim() == 2 && out.dim() == 2 && out.size(1) == recv.size(1) && out.is_contiguous(),
              "moe_owner_combine: recv [N * cap, d], out [S, d]");
  const int64_t N = rcnt.numel(), d = recv.size(1), S = out.size(0);
  TORCH_CHECK(N >= 1 && recv.size(0) % N == 0 && side.numel() >= recv.size(0), "moe_owner_combine: blocks");
  const int64_t cap = recv.size(0) / N;
  TORCH_CHECK(pos.numel() >= N * S && Tr >= 0 && Tr <= S && d % 8 == 0, "moe_owner_combine: shapes");
  const at::OptionalDeviceGuard g(out.device());
  launch_moe_owner_combine(ptr<float>(recv), ptr<int>(side), ptr<int>(rcnt), (int)N, (int)cap, (int)S, (int)Tr, (int)d,
                           ptr<int>(pos), ptr<bf16>(out), cur_stream(out));
}

// Decode MoE routing in one launch: resid fp32 [T, d] (T <= 16) -> ids / w [T*k], counts / offsets / cursor,
// xs [T*k, d] (the normalised rows, expert segments in token order), dst [T*k]
void moe_decode_route(const Tensor& resid, const Tensor& lnw, double eps, const Tensor& Wr, int64_t k, Tensor& ids,
                      Tensor& w, Tensor& counts, Tensor& offsets, Tensor& cursor, Tensor& xs, Tensor& dst) {
  check_gpu(resid, "resid");
  check_dtype(resid, at::kFloat, "resid");
  check_gpu(lnw, "lnw");
  check_dtype(lnw, at::kBFloat16, "lnw");
  check_gpu(Wr, "Wr");
  check_dtype(Wr, at::kBFloat16, "Wr");
  TORCH_CHECK(resid.dim() == 2 && resid.is_contiguous() && Wr.dim() == 2 && Wr.is_contiguous() &&
                  Wr.size(1) == resid.size(1) && lnw.numel() == resid.size(1),
              "moe_decode_route: resid [T, d], Wr [E, d], lnw [d]");
  const int64_t T = resid.size(0), d = resid.size(1), E = Wr.size(0);
  TORCH_CHECK(T <= 8 && E >= 1 && E <= 64 && k >= 1 && k <= 8 && k <= E && d % 8 == 0 && d <= 4096,
              "moe_decode_route: T <= 8, k <= E <= 64, k <= 8, d <= 4096, d % 8 == 0");
  for (auto* t : {&ids, &counts, &offsets, &cursor, &dst}) {
    check_gpu(*t, "index tensor");
    check_dtype(*t, at::kInt, "index tensor");
  }
  check_gpu(w, "w");
  check_dtype(w, at::kFloat, "w");
  check_gpu(xs, "xs");
  check_dtype(xs, at::kBFloat16, "xs");
  TORCH_CHECK(ids.numel() >= T * k && w.numel() >= T * k && dst.numel() >= T * k && counts.numel() >= E &&
                  offsets.numel() >= E + 1 && cursor.numel() >= E && xs.numel() >= T * k * d,
              "moe_decode_route: outputs too small");
  const at::OptionalDeviceGuard g(resid.device());
  launch_moe_decode_route(ptr<float>(resid), ptr<bf16>(lnw), (float)eps, ptr<bf16>(Wr), (int)T, (int)d, (int)E, (int)k,
                          ptr<int>(ids), ptr<float>(w), ptr<int>(counts), ptr<int>(offsets), ptr<int>(cursor),
                          ptr<bf16>(xs), ptr<int>(dst), cur_stream(resid));
}

// moe_combine over every expert + add_prep (resid += combined; xw = bf16(resid * w_next); ss[t] = sum resid^2)
void moe_combine_prep(const Tensor& y, const Tensor& dst, const Tensor& ids, int64_t E, const Tensor& w, int64_t k,
                      Tensor& resid, const Tensor& w_next, Tensor& xw, Tensor& ss) {
  check_gpu(resid, "resid");
  check_dtype(resid, at::kFloat, "resid");
  check_gpu(xw, "xw");
  check_dtype(xw, at::kBFloat16, "xw");
  check_gpu(w_next, "w_next");
  check_dtype(w_next, at::kBFloat16, "w_next");
  check_gpu(ss, "ss");
  check_dtype(ss, at::kFloat, "ss");
  check_gpu(dst, "dst");
  check_dtype(dst, at::kInt, "dst");
  check_gpu(ids, "ids");
  check_dtype(ids, at::kInt, "ids");
  check_gpu(w, "w");
  check_dtype(w, at::kFloat, "w");
  TORCH_CHECK(resid.dim() == 2 && resid.is_contiguous(), "resid must be [T, d]");
  const int64_t T = resid.size(0), d = resid.size(1);
  const int64_t R = y.dim() == 3 ? y.size(1) : y.size(0);
  // ss [T, P]: one sum-of-squares partial per column part (P divides d / 8)
  TORCH_CHECK(ss.dim() == 2 && ss.size(0) >= T && ss.is_contiguous(), "moe_combine_prep: ss must be [T, P]");
  const int64_t P = ss.size(1);
  TORCH_CHECK(xw.numel() >= T * d && w_next.numel() == d && d % 8 == 0 && P >= 1 && (d / 8) % P == 0,
              "moe_combine_prep: shape mismatch");
  TORCH_CHECK(dst.numel() >= T * k && w.numel() >= T * k && ids.numel() >= T * k, "moe_combine_prep: dst/w too small");
  const at::OptionalDeviceGuard g(resid.device());
  launch_moe_combine_prep(linout(y, R, d, "y"), (int)R, ptr<int>(dst), ptr<int>(ids), (int)E, ptr<float>(w), (int)T,
                          (int)k, (int)d, ptr<float>(resid), ptr<bf16>(w_next), ptr<bf16>(xw), ptr<float>(ss), (int)P,
                          cur_stream(resid));
}

// ---- fused decode projections (decode_gemm.hip) ----------------------------------------------------
struct DGShape {
  int64_t M, N, K;
};

DGShape dg_check(const Tensor& x, const Tensor& W, bool mg = false) {
  check_gpu(x, "x");
  check_gpu(W, "W");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(W, at::kBFloat16, "W");
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && x.size(1) == W.size(1), "decode_gemm: x [M,K], W [N,K]");
  const int64_t M = x.size(0), K = x.size(1), N = W.size(0);
  TORCH_CHECK(M >= 1 && M <= (mg ? 256 : 64), "decode_gemm: M must be in [1, 64] (mgemm: 256)");
  TORCH_CHECK(N % 16 == 0, "decode_gemm: N % 16");
  TORCH_CHECK(K % (mg ? 64 : 256) == 0, "decode_gemm: K must be a multiple of 256 (4 waves x 64)");
  return {M, N, K};
}

// mg_slab [S, M, N] selects the medium-M GEMM; a 1-D fp32 mg_slab is the decode GEMM's split-K workspace
bool is_mg(const c10::optional<Tensor>& slab) { return slab.has_value() && slab->dim() == 3; }

// The decode GEMM (M <= 64) or, with an mgemm slab given, the medium-M GEMM with the same fused epilogue
// (in-launch split-K reduction; weights MFMA-preshuffled): slab [S, M, N] fp32 scratch, counters [N / (64 rw)]
// ints zeroed once (re-armed by the kernel).  With a 1-D slab (fp32 workspace) + counters (ints, zeroed once)
// the decode GEMM may split K across workgroups (decode_gemm.hip, go_xres).
void launch_dg(int epi, const Tensor& x, const Tensor& W, const DGShape& sh, DecodeEpi& e,
               const c10::optional<Tensor>& slab, const c10::optional<Tensor>& counters, int64_t rw) {
  const at::OptionalDeviceGuard g(x.device());
  if (!is_mg(slab)) {
    if (slab.has_value()) {
      TORCH_CHECK(counters.has_value(), "decode split-K workspace: counters required");
      check_gpu(*slab, "ks_ws");
      check_dtype(*slab, at::kFloat, "ks_ws");
      check_gpu(*counters, "ks_cnt");
      check_dtype(*counters, at::kInt, "ks_cnt");
      TORCH_CHECK(slab->is_contiguous() && counters->is_contiguous(), "decode split-K workspace: contiguous");
      e.ks_ws = ptr<float>(*slab);
      e.ks_cap = slab->numel();
      e.ks_cnt = ptr<int>(*counters);
      e.ks_ncnt = (int)counters->numel();
    }
    launch_decode_gemm(epi, ptr<bf16>(x), ptr<bf16>(W), (int)sh.M, (int)sh.N, (int)sh.K, e, cur_stream(x));
    return;
  }
  TORCH_CHECK(e.wshuf, "mgemm epilogue: the weights must be the MFMA-preshuffled copy");
  TORCH_CHECK(counters.has_value(), "mgemm epilogue: counters required");
  check_gpu(*slab, "slab");
  check_dtype(*slab, at::kFloat, "slab");
  check_gpu(*counters, "counters");
  check_dtype(*counters, at::kInt, "counters");
  const int64_t S = slab->dim() == 3 ? slab->size(0) : 0;
  TORCH_CHECK(S >= 1 && slab->size(1) == sh.M && slab->size(2) == sh.N && slab->is_contiguous(),
              "mgemm epilogue: slab [S, M, N]");
  TORCH_CHECK(rw >= 1 && rw <= 4 && (sh.M <= 128 || rw <= 2) && sh.N % (64 * rw) == 0 && sh.K % (S * 64) == 0,
              "mgemm epilogue: rw / split shape");
  TORCH_CHECK(counters->numel() >= sh.N / (64 * rw), "mgemm epilogue: counters too small");
  TORCH_CHECK((sh.M + 255) * sh.K * 2 < (1LL << 31) && sh.N * sh.K * 2 < (1LL << 31), "mgemm: operands exceed 2 GB");
  launch_mgemm_epi(epi, ptr<bf16>(x), ptr<bf16>(W), ptr<float>(*slab), (int)sh.M, (int)sh.N, (int)sh.K, (int)S,
                   (int)rw, e, ptr<int>(*counters), cur_stream(x));
}

void dg_norm_in(DecodeEpi& e, const c10::optional<Tensor>& ss_in, int64_t M, int64_t K, double eps) {
  if (!ss_in.has_value()) return;
  check_gpu(*ss_in, "ss_in");
  check_dtype(*ss_in, at::kFloat, "ss_in");
  TORCH_CHECK(ss_in->dim() == 2 && ss_in->size(0) >= M, "ss_in must be [>=M, tiles]");
  e.ss_in = ptr<float>(*ss_in);
  e.ss_tiles = (int)ss_in->size(1);
  e.inv_d = 1.f / (float)K;
  e.eps = (float)eps;
}

void dg_f32(const Tensor& x, const Tensor& W, const c10::optional<Tensor>& ss_in, double eps, Tensor& y, bool wshuf) {
  auto sh = dg_check(x, W);
  check_gpu(y, "y");
  check_dtype(y, at::kFloat, "y");
  TORCH_CHECK(y.numel() == sh.M * sh.N, "dg_f32: y must be [M, N]");
  DecodeEpi e;
  e.wshuf = wshuf ? 1 : 0;
  dg_norm_in(e, ss_in, sh.M, sh.K, eps);
  e.y = ptr<float>(y);
  const at::OptionalDeviceGuard g(x.device());
  launch_decode_gemm(DECODE_EPI_F32, ptr<bf16>(x), ptr<bf16>(W), (int)sh.M, (int)sh.N, (int)sh.K, e, cur_stream(x));
}

void dg_qkv(const Tensor& x, const Tensor& W, const c10::optional<Tensor>& ss_in, double eps, const Tensor& positions,
            const Tensor& slots, const Tensor& cos_sin, Tensor& q_out, Tensor& k_cache, Tensor& v_cache, int64_t Hq,
            int64_t Hkv, bool wshuf, const c10::optional<Tensor>& mg_slab, const c10::optional<Tensor>& mg_counters,
            int64_t mg_rw) {
  auto sh = dg_check(x, W, is_mg(mg_slab));
  for (auto* t : {&positions, &slots}) {
    check_gpu(*t, "index tensor");
    check_dtype(*t, at::kInt, "index tensor");
  }
  check_gpu(cos_sin, "cos_sin");
  check_dtype(cos_sin, at::kFloat, "cos_sin");
  check_cache(k_cache, v_cache);
  check_gpu(q_out, "q_out");
  check_dtype(q_out, at::kBFloat16, "q_out");
  TORCH_CHECK(sh.N == (Hq + 2 * Hkv) * 128, "dg_qkv: N must be (Hq + 2 Hkv) * 128");
  TORCH_CHECK(k_cache.size(1) == Hkv, "dg_qkv: cache head count");
  TORCH_CHECK(positions.numel() >= sh.M && slots.numel() >= sh.M, "dg_qkv: positions/slots too short");
  TORCH_CHECK(q_out.numel() >= sh.M * Hq * 128, "dg_qkv: q_out too small");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == 128, "dg_qkv: cos_sin [max_pos, 128]");
  DecodeEpi e;
  e.wshuf = wshuf ? 1 : 0;
  dg_norm_in(e, ss_in, sh.M, sh.K, eps);
  e.positions = ptr<int>(positions);
  e.slots = ptr<int>(slots);
  e.cos_sin = ptr<float>(cos_sin);
  e.q_out = ptr<bf16>(q_out);
  e.k_cache = ptr<bf16>(k_cache);
  e.v_cache = ptr<bf16>(v_cache);
  e.Hq = (int)Hq;
  e.Hkv = (int)Hkv;
  e.BS = (int)k_cache.size(2);
  launch_dg(DECODE_EPI_QKV, x, W, sh, e, mg_slab, mg_counters, mg_rw);
}

void dg_resid(const Tensor& x, const Tensor& W, Tensor& resid, const Tensor& w_next, Tensor& xw_out, Tensor& ss_out, bool wshuf,
              const c10::optional<Tensor>& mg_slab, const c10::optional<Tensor>& mg_counters, int64_t mg_rw) {
  auto sh = dg_check(x, W, is_mg(mg_slab));
  check_gpu(resid, "resid");
  check_dtype(resid, at::kFloat, "resid");
  check_gpu(w_next, "w_next");
  check_dtype(w_next, at::kBFloat16, "w_next");
  check_gpu(xw_out, "xw_out");
  check_dtype(xw_out, at::kBFloat16, "xw_out");
  check_gpu(ss_out, "ss_out");
  check_dtype(ss_out, at::kFloat, "ss_out");
  TORCH_CHECK(resid.numel() == sh.M * sh.N && xw_out.numel() == sh.M * sh.N && w_next.numel() == sh.N,
              "dg_resid: shape mismatch");
  TORCH_CHECK(ss_out.dim() == 2 && ss_out.size(0) >= sh.M && ss_out.size(1) == sh.N / 16, "dg_resid: ss_out [M, N/16]");
  DecodeEpi e;
  e.wshuf = wshuf ? 1 : 0;
  e.resid = ptr<float>(resid);
  e.w_next = ptr<bf16>(w_next);
  e.xw_out = ptr<bf16>(xw_out);
  e.ss_out = ptr<float>(ss_out);
  launch_dg(DECODE_EPI_RESID, x, W, sh, e, mg_slab, mg_counters, mg_rw);
}

void dg_swiglu(const Tensor& x, const Tensor& W, const c10::optional<Tensor>& ss_in, double eps, Tensor& act, bool wshuf,
               const c10::optional<Tensor>& mg_slab, const c10::optional<Tensor>& mg_counters, int64_t mg_rw) {
  auto sh = dg_check(x, W, is_mg(mg_slab));
  check_gpu(act, "act");
  check_dtype(act, at::kBFloat16, "act");
  TORCH_CHECK(act.numel() == sh.M * sh.N / 2, "dg_swiglu: act must be [M, N/2]");
  DecodeEpi e;
  e.wshuf = wshuf ? 1 : 0;
  dg_norm_in(e, ss_in, sh.M, sh.K, eps);
  e.act = ptr<bf16>(act);
  launch_dg(DECODE_EPI_SWIGLU, x, W, sh, e, mg_slab, mg_counters, mg_rw);
}

void dg_argmax(const Tensor& x, const Tensor& W, const c10::optional<Tensor>& ss_in, double eps, const Tensor& temps,
               const Tensor& seeds, const Tensor& step, Tensor& tile_keys, Tensor& out_keys, Tensor& out_ids,
               int64_t n_offset, const c10::optional<Tensor>& logits, bool wshuf) {
  auto sh = dg_check(x, W);
  check_gpu(temps, "temps");
  check_dtype(temps, at::kFloat, "temps");
  check_gpu(seeds, "seeds");
  check_dtype(seeds, at::kLong, "seeds");
  check_gpu(step, "step");
  check_dtype(step, at::kLong, "step");
  check_gpu(tile_keys, "tile_keys");
  check_dtype(tile_keys, at::kLong, "tile_keys");
  check_gpu(out_keys, "out_keys");
  check_dtype(out_keys, at::kLong, "out_keys");
  check_gpu(out_ids, "out_ids");
  check_dtype(out_ids, at::kInt, "out_ids");
  TORCH_CHECK(temps.numel() >= sh.M && seeds.numel() >= sh.M, "dg_argmax: sampling params");
  TORCH_CHECK(tile_keys.numel() >= sh.M * (sh.N / 16), "dg_argmax: tile_keys too small");
  TORCH_CHECK(out_keys.numel() >= sh.M && out_ids.numel() >= sh.M, "dg_argmax: outputs too small");
  DecodeEpi e;
  e.wshuf = wshuf ? 1 : 0;
  dg_norm_in(e, ss_in, sh.M, sh.K, eps);
  if (logits.has_value()) {
    check_gpu(*logits, "logits");
    check_dtype(*logits, at::kFloat, "logits");
    TORCH_CHECK(logits->numel() == sh.M * sh.N, "dg_argmax: logits [M, N]");
    e.y = ptr<float>(*logits);
  }
  e.temps = ptr<float>(temps);
  e.seeds = reinterpret_cast<const unsigned long long*>(seeds.data_ptr());
  e.step = reinterpret_cast<const long long*>(step.data_ptr());
  e.keys = reinterpret_cast<unsigned long long*>(tile_keys.data_ptr());
  e.n_offset = (int)n_offset;
  const at::OptionalDeviceGuard g(x.device());
  hipStream_t s = cur_stream(x);
  launch_decode_gemm(DECODE_EPI_ARGMAX, ptr<bf16>(x), ptr<bf16>(W), (int)sh.M, (int)sh.N, (int)sh.K, e, s);
  launch_argmax_reduce(e.keys, (int)sh.M, (int)(sh.N / 16), reinterpret_cast<unsigned long long*>(out_keys.data_ptr()),
                       ptr<int>(out_ids), s);
}

void embed_prep(const Tensor& ids, const Tensor& table, Tensor& resid, const Tensor& w, Tensor& xw, Tensor& ss,
                const c10::optional<Tensor>& src, const c10::optional<Tensor>& prev) {
  check_gpu(ids, "ids");
  check_dtype(ids, at::kInt, "ids");
  check_gpu(table, "table");
  check_dtype(table, at::kBFloat16, "table");
  const int64_t T = ids.numel(), d = table.size(1);
  check_gpu(resid, "resid");
  check_dtype(resid, at::kFloat, "resid");
  check_gpu(xw, "xw");
  check_dtype(xw, at::kBFloat16, "xw");
  check_gpu(ss, "ss");
  check_dtype(ss, at::kFloat, "ss");
  // ss [>=T] / [>=T, 1]: one sum per row; [>=T, P]: P per-row partials over column slices (as add_prep)
  const int64_t P = ss.dim() == 2 ? ss.size(1) : 1;
  TORCH_CHECK(ss.is_contiguous() && P >= 1 && P <= 16 && d % (8 * P) == 0, "embed_prep: ss parts must divide d / 8");
  TORCH_CHECK(resid.numel() == T * d && xw.numel() == T * d && w.numel() == d && ss.numel() >= T * P && d % 8 == 0,
              "embed_prep: shape mismatch");
  const int* sp = nullptr;
  const int* pp = nullptr;
  TORCH_CHECK(src.has_value() == prev.has_value(), "embed_prep: src and prev go together");
  if (src.has_value()) {
    check_gpu(*src, "src");
    check_gpu(*prev, "prev");
    check_dtype(*src, at::kInt, "src");
    check_dtype(*prev, at::kInt, "prev");
    TORCH_CHECK(src->numel() >= T, "embed_prep: src must have one entry per row");
    sp = ptr<int>(*src);
    pp = ptr<int>(*prev);
  }
  const at::OptionalDeviceGuard g(ids.device());
  launch_embed_prep(ptr<int>(ids), sp, pp, ptr<bf16>(table), ptr<float>(resid), ptr<bf16>(w), ptr<bf16>(xw),
                    ptr<float>(ss), (int)T, (int)d, (int)P, cur_stream(ids));
}

void add_prep(const Tensor& delta, Tensor& resid, const Tensor& w, Tensor& xw, Tensor& ss) {
  check_gpu(resid, "resid");
  check_dtype(resid, at::kFloat, "resid");
  TORCH_CHECK(resid.dim() == 2, "add_prep: resid [T, d]");
  const int64_t T = resid.size(0), d = resid.size(1);
  check_gpu(xw, "xw");
  check_dtype(xw, at::kBFloat16, "xw");
  check_gpu(ss, "ss");
  check_dtype(ss, at::kFloat, "ss");
  // ss [>=T] / [>=T, 1]: one sum per row; [>=T, P]: P per-row partials over column slices
  const int64_t P = ss.dim() == 2 ? ss.size(1) : 1;
  TORCH_CHECK(ss.is_contiguous() && P >= 1 && P <= 16 && d % (8 * P) == 0, "add_prep: ss parts must divide d / 8");
  TORCH_CHECK(xw.numel() == T * d && w.numel() == d && ss.numel() >= T * P && d % 8 == 0, "add_prep: shape mismatch");
  const at::OptionalDeviceGuard g(resid.device());
  launch_add_prep(linout(delta, T, d, "delta"), ptr<float>(resid), ptr<bf16>(w), ptr<bf16>(xw), ptr<float>(ss), (int)T,
                  (int)d, (int)P, cur_stream(resid));
}

void sample_filtered(const Tensor& logits, const Tensor& temps, const Tensor& top_k, const Tensor& top_p,
                     const Tensor& seeds, const Tensor& step, Tensor& out_ids) {
  check_gpu(logits, "logits");
  check_dtype(logits, at::kFloat, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "sample_filtered: logits [B, V] contiguous");
  const int64_t B = logits.size(0), V = logits.size(1);
  for (const Tensor* t : {&temps, &top_k, &top_p, &seeds, &step, static_cast<const Tensor*>(&out_ids)})
    check_gpu(*t, "sampling tensor");
  check_dtype(temps, at::kFloat, "temps");
  check_dtype(top_k, at::kInt, "top_k");
  check_dtype(top_p, at::kFloat, "top_p");
  check_dtype(seeds, at::kLong, "seeds");
  check_dtype(step, at::kLong, "step");
  check_dtype(out_ids, at::kInt, "out_ids");
  TORCH_CHECK(temps.numel() >= B && top_k.numel() >= B && top_p.numel() >= B && seeds.numel() >= B &&
                  out_ids.numel() >= B && step.numel() >= 1,
              "sample_filtered: per-row tensors too short");
  const at::OptionalDeviceGuard g(logits.device());
  launch_sample_filtered(ptr<float>(logits), (int)B, (int)V, ptr<float>(temps), ptr<int>(top_k), ptr<float>(top_p),
                         reinterpret_cast<const long long*>(seeds.data_ptr()),
                         reinterpret_cast<const long long*>(step.data_ptr()), ptr<int>(out_ids), cur_stream(logits));
}

void logits_argmax(const Tensor& logits, const Tensor& temps, const Tensor& seeds, const Tensor& step, int64_t n_offset,
                   Tensor& out_keys, Tensor& out_ids) {
  check_gpu(logits, "logits");
  check_dtype(logits, at::kFloat, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits_argmax: logits [B, V] contiguous");
  const int64_t B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(n_offset >= 0 && n_offset + V < (1LL << 31), "logits_argmax: vocab index range");
  for (const Tensor* t : {&temps, &seeds, &step, static_cast<const Tensor*>(&out_keys),
                          static_cast<const Tensor*>(&out_ids)})
    check_gpu(*t, "sampling tensor");
  check_dtype(temps, at::kFloat, "temps");
  check_dtype(seeds, at::kLong, "seeds");
  check_dtype(step, at::kLong, "step");
  check_dtype(out_keys, at::kLong, "out_keys");
  check_dtype(out_ids, at::kInt, "out_ids");
  TORCH_CHECK(temps.numel() >= B && seeds.numel() >= B && out_keys.numel() >= B && out_ids.numel() >= B &&
                  step.numel() >= 1,
              "logits_argmax: per-row tensors too short");
  const at::OptionalDeviceGuard g(logits.device());
  launch_logits_argmax(ptr<float>(logits), (int)B, (int)V, ptr<float>(temps),
                       reinterpret_cast<const long long*>(seeds.data_ptr()),
                       reinterpret_cast<const long long*>(step.data_ptr()), (int)n_offset,
                       reinterpret_cast<unsigned long long*>(out_keys.data_ptr()), ptr<int>(out_ids), cur_stream(logits));
}

// Replay a captured decode hipGraph (torch.cuda.CUDAGraph.raw_cuda_graph_exec()) on the current stream WITHOUT
// releasing the GIL: torch's CUDAGraph.replay() drops it, and on a provider whose event-loop thread is busy with
// the clients' sockets the engine thread then waits out the interpreter's switch interval to get it back (TP=2
// client-end run: 2.06 ms of "launch" per step).  Our graphs hold no torch RNG state, so replay() would do
// nothing else.
void graph_launch(int64_t exec, int64_t device) {
  TORCH_CHECK(exec != 0, "graph_launch: null graph exec");
  const hipStream_t s = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream();
  const hipError_t e = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(exec), s);
  TORCH_CHECK(e == hipSuccess, "hipGraphLaunch: ", hipGetErrorString(e));
}

// Async copy of n bytes between a pinned host buffer and device memory on the current stream of `device`, with the
// GIL held (the per-step metadata H2D and sampled-ids D2H of the engine loop; torch's copy_ releases the GIL --
// see graph_launch).
void copy_async(Tensor& dst, const Tensor& src, int64_t nbytes, int64_t device) {
  TORCH_CHECK(nbytes >= 0 && nbytes <= dst.numel() * dst.element_size() && nbytes <= src.numel() * src.element_size(),
              "copy_async: byte count exceeds a tensor");
  TORCH_CHECK(dst.is_contiguous() && src.is_contiguous(), "copy_async: contiguous tensors only");
  if (nbytes == 0) return;
  const hipStream_t s = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream();
  const hipError_t e = hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), (size_t)nbytes, hipMemcpyDefault, s);
  TORCH_CHECK(e == hipSuccess, "hipMemcpyAsync: ", hipGetErrorString(e));
}

void rownorm(const Tensor& xw, const Tensor& ss, double eps, Tensor& out) {
  check_gpu(xw, "xw");
  check_dtype(xw, at::kBFloat16, "xw");
  check_gpu(ss, "ss");
  check_dtype(ss, at::kFloat, "ss");
  check_gpu(out, "out");
  check_dtype(out, at::kBFloat16, "out");
  TORCH_CHECK(xw.dim() == 2 && ss.dim() == 2 && ss.size(0) >= xw.size(0) && out.numel() == xw.numel(),
              "rownorm: shape mismatch");
  const at::OptionalDeviceGuard g(xw.device());
  launch_rownorm(ptr<bf16>(xw), ptr<float>(ss), (int)ss.size(1), (float)eps, ptr<bf16>(out), (int)xw.size(0),
                 (int)xw.size(1), cur_stream(xw));
}

}  // namespace

TORCH_LIBRARY(symmetry_amd, m) {
  m.def("graph_launch(int exec, int device) -> ()", &graph_launch);
  m.def("copy_async(Tensor(a!) dst, Tensor src, int nbytes, int device) -> ()", &copy_async);
  m.def(
      "moe_decode_route(Tensor resid, Tensor lnw, float eps, Tensor Wr, int k, Tensor(a!) ids, Tensor(b!) w, "
      "Tensor(c!) counts, Tensor(d!) offsets, Tensor(e!) cursor, Tensor(f!) xs, Tensor(g!) dst) -> ()",
      &moe_decode_route);
  m.def(
      "moe_combine_prep(Tensor y, Tensor dst, Tensor ids, int E, Tensor w, int k, Tensor(a!) resid, Tensor w_next, "
      "Tensor(b!) xw, Tensor(c!) ss) -> ()",
      &moe_combine_prep);
  m.def("rms_norm(Tensor x, Tensor w, float eps, Tensor(a!) out) -> ()", &rms_norm);
  m.def("add_rms_norm(Tensor delta, Tensor(a!) residual, Tensor w, float eps, Tensor(b!) out) -> ()", &add_rms_norm);
  m.def("embed_rms_norm(Tensor ids, Tensor table, Tensor(a!) residual, Tensor w, float eps, Tensor(b!) out, "
        "Tensor? src=None, Tensor? prev=None) -> ()",
        &embed_rms_norm);
  m.def(
      "rope_cache(Tensor qkv, Tensor positions, Tensor slots, Tensor cos_sin, Tensor(a!) q_out, Tensor(b!) k_cache, "
      "Tensor(c!) v_cache, int Hq, int Hkv, bool perm=False, bool decode=False) -> ()",
      &rope_cache);
  m.def(
      "attn_decode(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor ctx_lens, Tensor(a!) out, "
      "Tensor(b!) tmp_o, Tensor(c!) tmp_ml, Tensor(d!) counters, float scale) -> ()",
      &attn_decode);
  m.def(
      "attn_prefill(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor ctx_lens, Tensor cu_q, "
      "Tensor tiles, Tensor(a!) out, float scale) -> ()",
      &attn_prefill);
  m.def("skinny_gemm(Tensor x, Tensor w, Tensor(a!) y, int variant=0) -> ()", &skinny_gemm);
  m.def("mgemm(Tensor x, Tensor w, Tensor(a!) y, int rw) -> ()", &mgemm);
  m.def("mgemm_nt(int on) -> ()", [](int64_t on) { set_mgemm_nt((int)on); });
  m.def("pgemm(Tensor x, Tensor w, Tensor(a!) y, int cfg, int S, Tensor? slab, Tensor? counters) -> ()", &pgemm);
  m.def(
      "pg_qkv(Tensor x, Tensor W, Tensor? ss_in, float eps, Tensor positions, Tensor slots, Tensor cos_sin, "
      "Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, int Hq, int Hkv, int cfg) -> ()",
      &pg_qkv);
  m.def("pg_swiglu(Tensor x, Tensor W, Tensor? ss_in, float eps, Tensor(a!) act, int cfg) -> ()", &pg_swiglu);
  m.def("pg_resid(Tensor x, Tensor W, Tensor(a!) resid, Tensor w_next, Tensor(b!) xw_out, Tensor(c!) ss_out, int cfg) -> ()",
        &pg_resid);
  m.def("pg_grouped(Tensor xs, Tensor W, Tensor offsets, int e_lo, Tensor(a!) y, int epi, int cfg, int S) -> ()",
        &pg_grouped);
  m.def("pgemm_shape(int cfg) -> int[]", [](int64_t cfg) {
    int bm = 0, bn = 0;
    if (!pgemm_cfg_shape((int)cfg, &bm, &bn)) return std::vector<int64_t>{};
    return std::vector<int64_t>{bm, bn};
  });
  m.def("decode_halves(int on) -> ()", [](int64_t on) { set_decode_halves((int)on); });
  m.def("attn_stream_min(int tokens) -> ()", [](int64_t t) { set_attn_stream_min((int)t); });
  m.def("attn_wave(int min_units, int min_span) -> ()",
        [](int64_t u, int64_t span) { set_attn_wave((int)u, (int)span); });
  m.def(
      "lm_head_sample(Tensor x, Tensor w, Tensor temps, Tensor seeds, Tensor step, Tensor(a!) tile_keys, "
      "Tensor(b!) out_keys, Tensor(c!) out_ids, int n_offset, Tensor(d!)? logits) -> ()",
      &lm_head_sample);
  m.def("swiglu(Tensor gu, Tensor(a!) out, bool interleaved=False) -> ()", &swiglu);
  m.def(
      "moe_router(Tensor x, Tensor Wr, Tensor(a!) logits) -> ()", &moe_router);
  m.def(
      "moe_route_permute(Tensor logits, Tensor x, int k, int E, Tensor(a!) ids, Tensor(b!) w, Tensor(c!) counts, "
      "Tensor(d!) offsets, Tensor(e!) cursor, Tensor(f!) xs, Tensor(g!) dst) -> ()",
      &moe_route_permute);
  m.def("dg_f32(Tensor x, Tensor W, Tensor? ss_in, float eps, Tensor(a!) y, bool wshuf=False) -> ()", &dg_f32);
  m.def(
      "dg_qkv(Tensor x, Tensor W, Tensor? ss_in, float eps, Tensor positions, Tensor slots, Tensor cos_sin, "
      "Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, int Hq, int Hkv, bool wshuf=False, "
      "Tensor(d!)? mg_slab=None, Tensor(e!)? mg_counters=None, int mg_rw=0) -> ()",
      &dg_qkv);
  m.def(
      "dg_resid(Tensor x, Tensor W, Tensor(a!) resid, Tensor w_next, Tensor(b!) xw_out, Tensor(c!) ss_out, "
      "bool wshuf=False, Tensor(d!)? mg_slab=None, Tensor(e!)? mg_counters=None, int mg_rw=0) -> ()",
      &dg_resid);
  m.def(
      "dg_swiglu(Tensor x, Tensor W, Tensor? ss_in, float eps, Tensor(a!) act, bool wshuf=False, "
      "Tensor(d!)? mg_slab=None, Tensor(e!)? mg_counters=None, int mg_rw=0) -> ()",
      &dg_swiglu);
  m.def(
      "dg_argmax(Tensor x, Tensor W, Tensor? ss_in, float eps, Tensor temps, Tensor seeds, Tensor step, "
      "Tensor(a!) tile_keys, Tensor(b!) out_keys, Tensor(c!) out_ids, int n_offset, Tensor(d!)? logits, bool wshuf=False) -> ()",
      &dg_argmax);
  m.def("embed_prep(Tensor ids, Tensor table, Tensor(a!) resid, Tensor w, Tensor(b!) xw, Tensor(c!) ss, "
        "Tensor? src=None, Tensor? prev=None) -> ()",
        &embed_prep);
  m.def("add_prep(Tensor delta, Tensor(a!) resid, Tensor w, Tensor(b!) xw, Tensor(c!) ss) -> ()", &add_prep);
  m.def("rownorm(Tensor xw, Tensor ss, float eps, Tensor(a!) out) -> ()", &rownorm);
  m.def(
      "sample_filtered(Tensor logits, Tensor temps, Tensor top_k, Tensor top_p, Tensor seeds, Tensor step, "
      "Tensor(a!) out_ids) -> ()",
      &sample_filtered);
  m.def(
      "logits_argmax(Tensor logits, Tensor temps, Tensor seeds, Tensor step, int n_offset, Tensor(a!) out_keys, "
      "Tensor(b!) out_ids) -> ()",
      &logits_argmax);
  m.def("decode_gemm_variant(int v) -> ()", [](int64_t v) { set_decode_gemm_variant((int)v); });
  m.def("decode_ksplit(int on) -> ()", [](int64_t on) { set_decode_ksplit((int)on); });
  m.def("decode_gemm_nt(int on) -> ()", [](int64_t on) { set_decode_gemm_nt((int)on); });
  m.def("grouped_skinny(Tensor xs, Tensor W, Tensor offsets, int e0, Tensor(a!) y, bool wshuf=False) -> ()",
        &grouped_skinny);
  m.def("grouped_gemm(Tensor xs, Tensor W, Tensor offsets, int e0, Tensor(a!) y, int mode) -> ()", &grouped_gemm);
  m.def("grouped_stream_policy(int p) -> ()", [](int64_t p) { set_grouped_stream_policy((int)p); });
  m.def("moe_route(Tensor logits, int T, int k, int E, Tensor(a!) ids, Tensor(b!) w) -> ()", &moe_route);
  m.def("moe_align(Tensor ids, int G, Tensor(a!) counts, Tensor(b!) offsets, Tensor(c!) cursor) -> ()", &moe_align);
  m.def(
      "moe_scatter(Tensor x, Tensor ids, int k, int G, Tensor offsets, Tensor(a!) cursor, Tensor(b!) xs, Tensor(c!) dst, "
      "Tensor(d!)? src_tok=None) -> ()",
      &moe_scatter);
  m.def("moe_owner_pack(Tensor y, Tensor dst, Tensor ids, Tensor w, int e_lo, int e_hi, int k, int S, "
        "Tensor(a!) cursor, Tensor(b!) send, Tensor(c!) side) -> ()", &moe_owner_pack);
  m.def("moe_owner_combine(Tensor recv, Tensor side, Tensor rcnt, int Tr, Tensor(a!) pos, Tensor(b!) out) -> ()",
        &moe_owner_combine);
  m.def(
      "moe_combine(Tensor y, Tensor dst, Tensor ids, int e_lo, int e_hi, Tensor w, int k, Tensor(a!) out, "
      "bool accumulate) -> ()",
      &moe_combine);
}
