// Host side of the one-shot xGMI all-reduce (csrc/kernels/xgmi_ar.hip): buffer lifetime, IPC export /
// import of the peers' buffers, and the torch ops.
//
// Each TP rank allocates ONE uncached device buffer (flags + two parities x world data slots), exports it
// with hipIpcGetMemHandle and maps every peer's buffer with hipIpcOpenMemHandle; the handles travel over
// the gloo bootstrap group (symmetry_amd/parallel/comm.py::XgmiComm).  The collectives launch on torch's
// current HIP stream, so they are captured into the decode hipGraph like every other kernel.
// `xgmi_connect_local` maps buffers of the SAME process instead of IPC handles: several "ranks" on one
// GPU in one process, for the kernel-level GPU test.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <vector>

#include "launchers.h"

namespace {

using at::Tensor;

#define HIP_OK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    TORCH_CHECK(e_ == hipSuccess, "HIP error ", hipGetErrorString(e_), " at " #x);  \
  } while (0)

struct Xgmi {
  XgmiArgs args{};
  volatile int* err_host = nullptr;  // host-mapped error word: polled after every step without a sync
  unsigned* xar_ctr = nullptr;       // per-output-tile epoch counters of the fused GEMM + all-reduce (XAR_CTR)
  char* own = nullptr;
  std::vector<char*> opened;  // IPC mappings to close
  int device = 0;
  long long bytes = 0;
  bool connected = false;
};

constexpr int XAR_CTR = XG_MAX_WG;  // output tiles (N / 16) a communicator's XAR launches may cover
std::mutex g_mu;
std::vector<Xgmi*> g_x;
// Uncached buffers are never returned to the runtime: memory freed from a hipDeviceMallocUncached
// allocation and handed out again to ordinary hipMalloc users (the torch caching allocator) was seen
// to lose or mix plain stores of later kernels on gfx950 (a round-2 probe: outputs written after
// a communicator was destroyed read back differently from the GPU and from the host).  A destroyed
// communicator's buffer waits here for the next communicator of the same size.
std::vector<std::pair<long long, char*>> g_uc_pool;

Xgmi* get(int64_t h) {
  std::lock_guard<std::mutex> g(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_x.size() && g_x[h] != nullptr, "invalid xgmi communicator");
  return g_x[h];
}

int64_t xgmi_create(int64_t slot_bytes, int64_t world, int64_t rank, int64_t device) {
  TORCH_CHECK(world >= 1 && world <= XG_MAX_WORLD, "xgmi: world must be 1..", XG_MAX_WORLD);
  TORCH_CHECK(rank >= 0 && rank < world, "xgmi: bad rank");
  TORCH_CHECK(slot_bytes > 0 && slot_bytes % 256 == 0, "xgmi: slot bytes must be a positive multiple of 256");
  auto* x = new Xgmi();
  x->device = (int)device;
  HIP_OK(hipSetDevice(x->device));
  x->bytes = xgmi_buffer_bytes((int)world, slot_bytes);
  void* p = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    for (size_t i = 0; i < g_uc_pool.size(); ++i)
      if (g_uc_pool[i].first == x->bytes) {
        p = g_uc_pool[i].second;
        g_uc_pool.erase(g_uc_pool.begin() + i);
        break;
      }
  }
  if (p == nullptr) HIP_OK(hipExtMallocWithFlags(&p, (size_t)x->bytes, hipDeviceMallocUncached));
  HIP_OK(hipMemset(p, 0, (size_t)x->bytes));
  x->own = (char*)p;
  void* eh = nullptr;
  HIP_OK(hipHostMalloc(&eh, 64, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(eh, 0, 64);
  void* ed = nullptr;
  HIP_OK(hipHostGetDevicePointer(&ed, eh, 0));
  HIP_OK(hipDeviceSynchronize());
  x->err_host = (volatile int*)eh;
  HIP_OK(hipMalloc(&x->xar_ctr, XAR_CTR * sizeof(unsigned)));
  HIP_OK(hipMemset(x->xar_ctr, 0, XAR_CTR * sizeof(unsigned)));
  HIP_OK(hipDeviceSynchronize());
  x->args.err = (int*)ed;
  x->args.rank = (int)rank;
  x->args.world = (int)world;
  x->args.slot_bytes = slot_bytes;
  for (int r = 0; r < XG_MAX_WORLD; ++r) x->args.bufs[r] = nullptr;
  x->args.bufs[rank] = x->own;
  std::lock_guard<std::mutex> g(g_mu);
  g_x.push_back(x);
  return (int64_t)g_x.size() - 1;
}

Tensor xgmi_ipc_handle(int64_t h) {
  Xgmi* x = get(h);
  hipIpcMemHandle_t ih;
  HIP_OK(hipIpcGetMemHandle(&ih, x->own));
  auto t = at::empty({(int64_t)sizeof(ih)}, at::kByte);
  std::memcpy(t.data_ptr(), &ih, sizeof(ih));
  return t;
}

// handles: uint8 [world, sizeof(hipIpcMemHandle_t)] gathered from every rank (own row ignored)
void xgmi_open(int64_t h, const Tensor& handles) {
  Xgmi* x = get(h);
  const int world = x->args.world;
  auto hc = handles.cpu().contiguous();
  TORCH_CHECK(hc.scalar_type() == at::kByte && hc.dim() == 2 && hc.size(0) == world &&
                  hc.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
              "xgmi_open: handles must be uint8 [world, ", sizeof(hipIpcMemHandle_t), "]");
  HIP_OK(hipSetDevice(x->device));
  for (int r = 0; r < world; ++r) {
    if (r == x->args.rank) continue;
    hipIpcMemHandle_t ih;
    std::memcpy(&ih, hc.data_ptr<uint8_t>() + r * sizeof(ih), sizeof(ih));
    void* p = nullptr;
    HIP_OK(hipIpcOpenMemHandle(&p, ih, hipIpcMemLazyEnablePeerAccess));
    x->args.bufs[r] = (char*)p;
    x->opened.push_back((char*)p);
  }
  x->connected = true;
}

// same-process "ranks" (kernel test): rank r's buffer is communicator peers[r]'s own buffer
void xgmi_connect_local(int64_t h, std::vector<int64_t> peers) {
  Xgmi* x = get(h);
  TORCH_CHECK((int)peers.size() == x->args.world, "xgmi_connect_local: one communicator per rank");
  for (int r = 0; r < x->args.world; ++r) {
    Xgmi* p = get(peers[r]);
    TORCH_CHECK(p->args.rank == r && p->args.world == x->args.world && p->args.slot_bytes == x->args.slot_bytes,
                "xgmi_connect_local: peer ", r, " has a different layout");
    x->args.bufs[r] = p->own;
  }
  x->connected = true;
}

void check_ready(Xgmi* x, const Tensor& t) {
  TORCH_CHECK(x->connected, "xgmi communicator is not connected to its peers");
  TORCH_CHECK(t.device().type() == c10::DeviceType::CUDA && t.get_device() == x->device,
              "xgmi: tensor must live on the communicator's GPU");
  TORCH_CHECK(t.is_contiguous(), "xgmi: tensor must be contiguous");
}

hipStream_t stream_of(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.get_device()).stream(); }

// out = sum over ranks of `in` (fp32 or bf16; out may alias in)
void xgmi_all_reduce(const Tensor& in, Tensor& out, int64_t h) {
  Xgmi* x = get(h);
  check_ready(x, in);
  check_ready(x, out);
  TORCH_CHECK(in.scalar_type() == out.scalar_type() && in.numel() == out.numel(), "xgmi_all_reduce: in/out mismatch");
  const int elem = in.scalar_type() == at::kFloat ? 0 : in.scalar_type() == at::kBFloat16 ? 1 : -1;
  TORCH_CHECK(elem >= 0, "xgmi_all_reduce: fp32 or bf16 only");
  const long long n = in.numel();
  TORCH_CHECK(n % 8 == 0, "xgmi_all_reduce: element count must be a multiple of 8");
  TORCH_CHECK(n * (long long)in.element_size() <= x->args.slot_bytes, "xgmi_all_reduce: message of ",
              n * in.element_size(), " B exceeds the ", x->args.slot_bytes, " B slot");
  const int chunk = xgmi_chunk(n, XG_MAX_WG);
  TORCH_CHECK((n + chunk - 1) / chunk < XG_KEYS_WG, "xgmi_all_reduce: too many chunks");
  launch_xgmi_all_reduce(x->args, in.data_ptr(), out.data_ptr(), n, elem, stream_of(in));
}

// resid += all_reduce(y); xw = bf16(resid * w); ss[row][part] = sum(resid^2) per column part
void xgmi_add_prep(const Tensor& y, Tensor& resid, const Tensor& w, Tensor& xw, Tensor& ss, int64_t h) {
  Xgmi* x = get(h);
  for (const Tensor* t : std::initializer_list<const Tensor*>{&y, &resid, &w, &xw, &ss}) check_ready(x, *t);
  TORCH_CHECK(y.scalar_type() == at::kFloat && resid.scalar_type() == at::kFloat && ss.scalar_type() == at::kFloat,
              "xgmi_add_prep: y, resid, ss fp32");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && xw.scalar_type() == at::kBFloat16, "xgmi_add_prep: w, xw bf16");
  TORCH_CHECK(resid.dim() == 2, "xgmi_add_prep: resid [T, d]");
  const int64_t T = resid.size(0), d = resid.size(1);
  TORCH_CHECK(y.numel() == T * d && xw.numel() == T * d && w.numel() == d, "xgmi_add_prep: shape mismatch");
  const int64_t P = ss.dim() == 2 ? ss.size(1) : 1;
  TORCH_CHECK(ss.numel() >= T * P && P >= 1 && P <= 16 && d % (8 * P) == 0, "xgmi_add_prep: ss parts must divide d / 8");
  TORCH_CHECK(T * P < XG_KEYS_WG, "xgmi_add_prep: too many rows");
  TORCH_CHECK(T * d * 4 <= x->args.slot_bytes, "xgmi_add_prep: message exceeds the slot");
  launch_xgmi_add_prep(x->args, y.data_ptr<float>(), resid.data_ptr<float>(),
                       reinterpret_cast<const bf16*>(w.data_ptr()), reinterpret_cast<bf16*>(xw.data_ptr()),
                       ss.data_ptr<float>(), (int)T, (int)d, (int)P, stream_of(y));
}

// vocab-parallel sampling combine: ids[i] = global argmax from every rank's packed u64 keys [B]
void xgmi_keys_max(const Tensor& keys, Tensor& ids, int64_t h) {
  Xgmi* x = get(h);
  check_ready(x, keys);
  check_ready(x, ids);
  TORCH_CHECK(keys.scalar_type() == at::kLong && ids.scalar_type() == at::kInt, "xgmi_keys_max: keys int64, ids int32");
  const int64_t B = keys.numel();
  TORCH_CHECK(ids.numel() >= B && B <= 4096 && B * 8 <= x->args.slot_bytes, "xgmi_keys_max: shapes");
  launch_xgmi_keys_max(x->args, reinterpret_cast<const unsigned long long*>(keys.data_ptr()), ids.data_ptr<int>(),
                       (int)B, stream_of(keys));
}

// ---- row-parallel projection + all-reduce + residual + next-norm prep in ONE launch (DECODE_EPI_XAR) -------
DecodeEpi xar_epi(Xgmi* x, const Tensor& a, const Tensor& W, bool wshuf, Tensor& resid, const Tensor& w_next,
                  Tensor& xw, Tensor& ss) {
  check_ready(x, a);
  check_ready(x, W);
  for (const Tensor* t : std::initializer_list<const Tensor*>{&resid, &w_next, &xw, &ss}) check_ready(x, *t);
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16 && w_next.scalar_type() == at::kBFloat16 &&
                  xw.scalar_type() == at::kBFloat16, "xgmi_gemm_ar_resid: x, W, w_next, xw bf16");
  TORCH_CHECK(resid.scalar_type() == at::kFloat && ss.scalar_type() == at::kFloat, "xgmi_gemm_ar_resid: resid, ss fp32");
  TORCH_CHECK(a.dim() == 2 && W.dim() == 2 && a.size(1) == W.size(1), "xgmi_gemm_ar_resid: x [M, K], W [N, K]");
  const int64_t M = a.size(0), N = W.size(0);
  TORCH_CHECK(resid.dim() == 2 && resid.size(0) == M && resid.size(1) == N && xw.numel() == M * N &&
                  w_next.numel() == N, "xgmi_gemm_ar_resid: resid / xw [M, N], w_next [N]");
  TORCH_CHECK(ss.dim() == 2 && ss.size(0) >= M && ss.size(1) == N / 16, "xgmi_gemm_ar_resid: ss [M, N / 16]");
  TORCH_CHECK(M * N * 8 <= x->args.slot_bytes, "xgmi_gemm_ar_resid: output granules exceed the slot");
  TORCH_CHECK(N / 16 <= XAR_CTR, "xgmi_gemm_ar_resid: too many output tiles");
  DecodeEpi e;
  e.wshuf = wshuf ? 1 : 0;
  e.xp = x->args;
  e.xar_ctr = x->xar_ctr;
  e.resid = resid.data_ptr<float>();
  e.w_next = reinterpret_cast<const bf16*>(w_next.data_ptr());
  e.xw_out = reinterpret_cast<bf16*>(xw.data_ptr());
  e.ss_out = ss.data_ptr<float>();
  return e;
}

// resid += all_reduce(x @ W^T); xw = bf16(resid * w_next); ss[m][tile] = sum(resid^2) over each 16 columns.
// Returns false (nothing launched) where no co-resident decomposition exists: run GEMM + add_prep instead.
bool xgmi_gemm_ar_resid(const Tensor& a, const Tensor& W, bool wshuf, Tensor& resid, const Tensor& w_next, Tensor& xw,
                        Tensor& ss, int64_t h) {
  Xgmi* x = get(h);
  const DecodeEpi e = xar_epi(x, a, W, wshuf, resid, w_next, xw, ss);
  TORCH_CHECK(a.size(1) % 256 == 0 && W.size(0) % 16 == 0, "xgmi_gemm_ar_resid: K % 256, N % 16");
  return launch_decode_gemm_xar(reinterpret_cast<const bf16*>(a.data_ptr()), reinterpret_cast<const bf16*>(W.data_ptr()),
                                (int)a.size(0), (int)W.size(0), (int)a.size(1), e, stream_of(a));
}

// test-only: every rank of this process in one launch (grid z = rank); xres: the x-resident walk
bool xgmi_gemm_ar_resid_multi(std::vector<Tensor> xs, const Tensor& W, bool wshuf, std::vector<Tensor> resids,
                              const Tensor& w_next, std::vector<Tensor> xws, std::vector<Tensor> sss,
                              std::vector<int64_t> comms, bool xres, int64_t delay_rank, int64_t delay_us) {
  const int world = (int)comms.size();
  TORCH_CHECK(world >= 1 && world <= XAR_MULTI_MAX && (int)xs.size() == world && (int)resids.size() == world &&
                  (int)xws.size() == world && (int)sss.size() == world, "xgmi_gemm_ar_resid_multi: one set per rank");
  XarMulti m{};
  m.delay_rank = (int)delay_rank;
  m.delay_ticks = (unsigned long long)std::max<int64_t>(delay_us, 0) * 100ull;  // 100 MHz wall clock
  for (int r = 0; r < world; ++r) {
    Xgmi* x = get(comms[r]);
    TORCH_CHECK(x->args.rank == r && x->args.world == world, "xgmi_gemm_ar_resid_multi: communicator order");
    m.e[r] = xar_epi(x, xs[r], W, wshuf, resids[r], w_next, xws[r], sss[r]);
    m.x[r] = reinterpret_cast<const bf16*>(xs[r].data_ptr());
  }
  return launch_decode_gemm_xar_multi(m, world, reinterpret_cast<const bf16*>(W.data_ptr()), (int)xs[0].size(0),
                                      (int)W.size(0), (int)xs[0].size(1), xres ? 1 : 0, stream_of(xs[0]));
}

// test-only: every rank of this process in one launch (grid slice per rank; see xgmi_ar.hip)
void xgmi_all_reduce_multi(std::vector<Tensor> ins, std::vector<Tensor> outs, std::vector<int64_t> comms,
                           int64_t delay_rank, int64_t delay_us) {
  const int world = (int)comms.size();
  TORCH_CHECK(world >= 1 && world <= XG_MULTI_MAX && (int)ins.size() == world && (int)outs.size() == world,
              "xgmi_all_reduce_multi: one input, output and communicator per rank (<= ", XG_MULTI_MAX, ")");
  XgmiMulti m{};
  m.delay_rank = (int)delay_rank;
  m.delay_ticks = (unsigned long long)std::max<int64_t>(delay_us, 0) * 100ull;  // 100 MHz wall clock
  const long long n = ins[0].numel();
  int elem = -1;
  for (int r = 0; r < world; ++r) {
    Xgmi* x = get(comms[r]);
    TORCH_CHECK(x->args.rank == r && x->args.world == world, "xgmi_all_reduce_multi: communicator ", r, " is not rank ", r);
    check_ready(x, ins[r]);
    check_ready(x, outs[r]);
    TORCH_CHECK(ins[r].numel() == n && outs[r].numel() == n && ins[r].scalar_type() == ins[0].scalar_type() &&
                    outs[r].scalar_type() == ins[0].scalar_type(), "xgmi_all_reduce_multi: shape / dtype mismatch");
    TORCH_CHECK(n * (long long)ins[r].element_size() <= x->args.slot_bytes, "xgmi_all_reduce_multi: message exceeds the slot");
    m.c[r] = x->args;
    m.in[r] = ins[r].data_ptr();
    m.out[r] = outs[r].data_ptr();
  }
  elem = ins[0].scalar_type() == at::kFloat ? 0 : ins[0].scalar_type() == at::kBFloat16 ? 1 : -1;
  TORCH_CHECK(elem >= 0 && n % 8 == 0, "xgmi_all_reduce_multi: fp32 / bf16, element count % 8");
  // the slices wait on each other: they must all be resident at once (256 CUs x a few 256-thread groups)
  const int chunk = xgmi_chunk(n, XG_MAX_WG);
  TORCH_CHECK(world * ((n + chunk - 1) / chunk) <= XG_MULTI_MAX_GROUPS, "xgmi_all_reduce_multi: ",
              world * ((n + chunk - 1) / chunk), " workgroups would not be co-resident");
  launch_xgmi_all_reduce_multi(m, world, n, elem, stream_of(ins[0]));
}

void xgmi_add_prep_multi(std::vector<Tensor> ys, std::vector<Tensor> resids, const Tensor& w, std::vector<Tensor> xws,
                         std::vector<Tensor> sss, std::vector<int64_t> comms, int64_t delay_rank, int64_t delay_us) {
  const int world = (int)comms.size();
  TORCH_CHECK(world >= 1 && world <= XG_MULTI_MAX && (int)ys.size() == world && (int)resids.size() == world &&
                  (int)xws.size() == world && (int)sss.size() == world,
              "xgmi_add_prep_multi: one set of tensors per rank");
  XgmiMulti m{};
  m.delay_rank = (int)delay_rank;
  m.delay_ticks = (unsigned long long)std::max<int64_t>(delay_us, 0) * 100ull;
  const int64_t T = resids[0].size(0), d = resids[0].size(1);
  const int64_t P = sss[0].dim() == 2 ? sss[0].size(1) : 1;
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.numel() == d && w.is_contiguous(), "xgmi_add_prep_multi: w bf16 [d]");
  TORCH_CHECK(P >= 1 && P <= 16 && d % (8 * P) == 0 && T * P < XG_KEYS_WG, "xgmi_add_prep_multi: bad parts");
  TORCH_CHECK(world * T * P <= XG_MULTI_MAX_GROUPS, "xgmi_add_prep_multi: ", world * T * P,
              " workgroups would not be co-resident");
  for (int r = 0; r < world; ++r) {
    Xgmi* x = get(comms[r]);
    TORCH_CHECK(x->args.rank == r && x->args.world == world, "xgmi_add_prep_multi: communicator ", r, " is not rank ", r);
    for (const Tensor* t : std::initializer_list<const Tensor*>{&ys[r], &resids[r], &xws[r], &sss[r]}) check_ready(x, *t);
    TORCH_CHECK(ys[r].scalar_type() == at::kFloat && resids[r].scalar_type() == at::kFloat &&
                    sss[r].scalar_type() == at::kFloat && xws[r].scalar_type() == at::kBFloat16,
                "xgmi_add_prep_multi: dtypes");
    TORCH_CHECK(ys[r].numel() == T * d && resids[r].numel() == T * d && xws[r].numel() == T * d &&
                    sss[r].numel() >= T * P, "xgmi_add_prep_multi: shapes");
    TORCH_CHECK(T * d * 4 <= x->args.slot_bytes, "xgmi_add_prep_multi: message exceeds the slot");
    m.c[r] = x->args;
    m.in[r] = ys[r].data_ptr();
    m.out[r] = resids[r].data_ptr();
    m.xw[r] = xws[r].data_ptr();
    m.ss[r] = sss[r].data_ptr<float>();
  }
  m.w = reinterpret_cast<const bf16*>(w.data_ptr());
  launch_xgmi_add_prep_multi(m, world, (int)T, (int)d, (int)P, stream_of(ys[0]));
}

void xgmi_keys_max_multi(std::vector<Tensor> keys, std::vector<Tensor> ids, std::vector<int64_t> comms,
                         int64_t delay_rank, int64_t delay_us) {
  const int world = (int)comms.size();
  TORCH_CHECK(world >= 1 && world <= XG_MULTI_MAX && (int)keys.size() == world && (int)ids.size() == world,
              "xgmi_keys_max_multi: one keys / ids tensor and communicator per rank");
  XgmiMulti m{};
  m.delay_rank = (int)delay_rank;
  m.delay_ticks = (unsigned long long)std::max<int64_t>(delay_us, 0) * 100ull;
  const int64_t B = keys[0].numel();
  for (int r = 0; r < world; ++r) {
    Xgmi* x = get(comms[r]);
    TORCH_CHECK(x->args.rank == r && x->args.world == world, "xgmi_keys_max_multi: communicator ", r, " is not rank ", r);
    check_ready(x, keys[r]);
    check_ready(x, ids[r]);
    TORCH_CHECK(keys[r].scalar_type() == at::kLong && ids[r].scalar_type() == at::kInt && keys[r].numel() == B &&
                    ids[r].numel() >= B && B <= 4096 && B * 8 <= x->args.slot_bytes,
                "xgmi_keys_max_multi: keys int64 [B], ids int32 [>= B]");
    m.c[r] = x->args;
    m.in[r] = keys[r].data_ptr();
    m.out[r] = ids[r].data_ptr();
  }
  launch_xgmi_keys_max_multi(m, world, (int)B, stream_of(keys[0]));
}

// ---- R3: unpadded expert all-to-all (xgmi_a2a_kernel) ------------------------------------------------------
XgmiA2AArgs a2a_args(Xgmi* x, const Tensor& src, const Tensor& counts, const c10::optional<Tensor>& side, Tensor& dst,
                     const c10::optional<Tensor>& dst_side, const c10::optional<Tensor>& dst_counts, int64_t cap) {
  const int world = x->args.world;
  check_ready(x, src);
  check_ready(x, dst);
  check_ready(x, counts);
  TORCH_CHECK(counts.scalar_type() == at::kInt && counts.numel() == world, "xgmi_a2a: counts int32 [world]");
  TORCH_CHECK(cap >= 1 && src.size(0) == world * cap && dst.size(0) == world * cap,
              "xgmi_a2a: src / dst must be [world * cap, ...]");
  TORCH_CHECK(src.scalar_type() == dst.scalar_type() && src.numel() == dst.numel(), "xgmi_a2a: src / dst mismatch");
  const int64_t rb = src.numel() / src.size(0) * src.element_size();
  TORCH_CHECK(rb % 16 == 0, "xgmi_a2a: row bytes must be a multiple of 16");
  TORCH_CHECK(xgmi_a2a_slot_bytes((int)cap, (int)rb) <= x->args.slot_bytes, "xgmi_a2a: ", cap, " rows of ", rb,
              " B exceed the communicator's ", x->args.slot_bytes, " B slot");
  XgmiA2AArgs a;
  a.c = x->args;
  a.src = reinterpret_cast<const char*>(src.data_ptr());
  a.counts = counts.data_ptr<int>();
  a.dst = reinterpret_cast<char*>(dst.data_ptr());
  a.cap = (int)cap;
  a.row_bytes = (int)rb;
  if (side.has_value()) {
    check_ready(x, *side);
    TORCH_CHECK(side->scalar_type() == at::kInt && side->numel() == world * cap, "xgmi_a2a: side int32 [world * cap]");
    a.side = side->data_ptr<int>();
  }
  if (dst_side.has_value()) {
    check_ready(x, *dst_side);
    TORCH_CHECK(dst_side->scalar_type() == at::kInt && dst_side->numel() == world * cap,
                "xgmi_a2a: dst_side int32 [world * cap]");
    a.dst_side = dst_side->data_ptr<int>();
  }
  if (dst_counts.has_value()) {
    check_ready(x, *dst_counts);
    TORCH_CHECK(dst_counts->scalar_type() == at::kInt && dst_counts->numel() == world, "xgmi_a2a: dst_counts int32 [world]");
    a.dst_counts = dst_counts->data_ptr<int>();
  }
  return a;
}

// rows [q cap, q cap + counts[q]) of src -> rows [rank cap, ...) of rank q's dst (+ side ints, received counts)
void xgmi_a2a(const Tensor& src, const Tensor& counts, const c10::optional<Tensor>& side, Tensor& dst,
              const c10::optional<Tensor>& dst_side, const c10::optional<Tensor>& dst_counts, int64_t cap, int64_t h) {
  Xgmi* x = get(h);
  launch_xgmi_a2a(a2a_args(x, src, counts, side, dst, dst_side, dst_counts, cap), stream_of(src));
}

// test-only: every rank of this process in one launch (grid slice per rank)
void xgmi_a2a_multi(std::vector<Tensor> srcs, std::vector<Tensor> counts, std::vector<Tensor> sides,
                    std::vector<Tensor> dsts, std::vector<Tensor> dst_sides, std::vector<Tensor> dst_counts,
                    int64_t cap, std::vector<int64_t> comms, int64_t delay_rank, int64_t delay_us) {
  const int world = (int)comms.size();
  TORCH_CHECK(world >= 1 && world <= XG_MULTI_MAX && (int)srcs.size() == world && (int)counts.size() == world &&
                  (int)sides.size() == world && (int)dsts.size() == world && (int)dst_sides.size() == world &&
                  (int)dst_counts.size() == world, "xgmi_a2a_multi: one set of tensors per rank");
  TORCH_CHECK(world * XA_WG <= XG_MULTI_MAX_GROUPS, "xgmi_a2a_multi: slices would not be co-resident");
  XgmiA2AMulti m{};
  m.delay_rank = (int)delay_rank;
  m.delay_ticks = (unsigned long long)std::max<int64_t>(delay_us, 0) * 100ull;
  for (int r = 0; r < world; ++r) {
    Xgmi* x = get(comms[r]);
    TORCH_CHECK(x->args.rank == r && x->args.world == world, "xgmi_a2a_multi: communicator order");
    m.a[r] = a2a_args(x, srcs[r], counts[r], sides[r], dsts[r], dst_sides[r], dst_counts[r], cap);
  }
  launch_xgmi_a2a_multi(m, world, stream_of(srcs[0]));
}

int64_t xgmi_a2a_slot(int64_t cap, int64_t row_bytes) { return xgmi_a2a_slot_bytes((int)cap, (int)row_bytes); }

// reads the error word: 1 + the source rank that never signalled within the wait limit, or the code the host
// declared (xgmi_set_error).  Sticky: a communicator that lost a peer stays failed (every later collective
// skips its waits), the provider exits and a supervisor starts fresh ranks.  Host-mapped memory: no device
// synchronisation; a kernel still running may set it later.
int64_t xgmi_error(int64_t h) { return *get(h)->err_host; }

// the host's health monitor declares a fault (e.g. 1 + the rank whose process died): spinning collectives
// stop waiting within a few polls; code 0 clears the word (tests)
void xgmi_set_error(int64_t h, int64_t code) {
  Xgmi* x = get(h);
  *x->err_host = (int)code;
  std::atomic_thread_fence(std::memory_order_seq_cst);
}

int64_t xgmi_slot_bytes(int64_t h) { return get(h)->args.slot_bytes; }

void xgmi_destroy(int64_t h) {
  Xgmi* x = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (h < 0 || h >= (int64_t)g_x.size() || g_x[h] == nullptr) return;
    x = g_x[h];
    g_x[h] = nullptr;
  }
  (void)hipSetDevice(x->device);
  (void)hipDeviceSynchronize();
  for (char* p : x->opened) (void)hipIpcCloseMemHandle(p);
  (void)hipHostFree((void*)x->err_host);
  (void)hipFree(x->xar_ctr);
  {
    std::lock_guard<std::mutex> g(g_mu);
    g_uc_pool.emplace_back(x->bytes, x->own);
  }
  delete x;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(symmetry_amd, m) {
  m.def("xgmi_create(int slot_bytes, int world, int rank, int device) -> int", &xgmi_create);
  m.def("xgmi_ipc_handle(int comm) -> Tensor", &xgmi_ipc_handle);
  m.def("xgmi_open(int comm, Tensor handles) -> ()", &xgmi_open);
  m.def("xgmi_connect_local(int comm, int[] peers) -> ()", &xgmi_connect_local);
  m.def("xgmi_all_reduce(Tensor input, Tensor(a!) out, int comm) -> ()", &xgmi_all_reduce);
  m.def("xgmi_add_prep(Tensor y, Tensor(a!) resid, Tensor w, Tensor(b!) xw, Tensor(c!) ss, int comm) -> ()",
        &xgmi_add_prep);
  m.def("xgmi_all_reduce_multi(Tensor[] inputs, Tensor(a!)[] outs, int[] comms, int delay_rank=-1, int delay_us=0) -> ()",
        &xgmi_all_reduce_multi);
  m.def(
      "xgmi_add_prep_multi(Tensor[] ys, Tensor(a!)[] resids, Tensor w, Tensor(b!)[] xws, Tensor(c!)[] sss, int[] comms, "
      "int delay_rank=-1, int delay_us=0) -> ()",
      &xgmi_add_prep_multi);
  m.def("xgmi_keys_max(Tensor keys, Tensor(a!) ids, int comm) -> ()", &xgmi_keys_max);
  m.def(
      "xgmi_gemm_ar_resid(Tensor x, Tensor W, bool wshuf, Tensor(a!) resid, Tensor w_next, Tensor(b!) xw, "
      "Tensor(c!) ss, int comm) -> bool",
      &xgmi_gemm_ar_resid);
  m.def(
      "xgmi_gemm_ar_resid_multi(Tensor[] xs, Tensor W, bool wshuf, Tensor(a!)[] resids, Tensor w_next, "
      "Tensor(b!)[] xws, Tensor(c!)[] sss, int[] comms, bool xres, int delay_rank=-1, int delay_us=0) -> bool",
      &xgmi_gemm_ar_resid_multi);
  m.def("xgmi_keys_max_multi(Tensor[] keys, Tensor(a!)[] ids, int[] comms, int delay_rank=-1, int delay_us=0) -> ()",
        &xgmi_keys_max_multi);
  m.def(
      "xgmi_a2a(Tensor src, Tensor counts, Tensor? side, Tensor(a!) dst, Tensor(b!)? dst_side, Tensor(c!)? dst_counts, "
      "int cap, int comm) -> ()",
      &xgmi_a2a);
  m.def(
      "xgmi_a2a_multi(Tensor[] srcs, Tensor[] counts, Tensor[] sides, Tensor(a!)[] dsts, Tensor(b!)[] dst_sides, "
      "Tensor(c!)[] dst_counts, int cap, int[] comms, int delay_rank=-1, int delay_us=0) -> ()",
      &xgmi_a2a_multi);
  m.def("xgmi_a2a_slot(int cap, int row_bytes) -> int", &xgmi_a2a_slot);
  m.def("xgmi_error(int comm) -> int", &xgmi_error);
  m.def("xgmi_set_error(int comm, int code) -> ()", &xgmi_set_error);
  m.def("xgmi_slot_bytes(int comm) -> int", &xgmi_slot_bytes);
  m.def("xgmi_destroy(int comm) -> ()", &xgmi_destroy);
}
