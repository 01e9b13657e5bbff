// RCCL communicators for tensor / expert parallelism.
//
// One ncclComm_t per process group, created from a unique id that rank 0
// broadcasts over torch.distributed (the TCPStore / gloo plane).  Collectives
// are enqueued on torch's current HIP stream and are therefore captured into
// the decode hipGraph together with the kernels around them -- the reason
// this wrapper exists instead of torch.distributed's own RCCL calls.  On the
// MI355X node RCCL rides xGMI (7 point-to-point links per GPU).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <mutex>
#include <vector>

namespace {

std::mutex g_mu;
std::vector<ncclComm_t> g_comms;

#define RCCL_CHECK(x)                                                                     \
  do {                                                                                    \
    ncclResult_t r_ = (x);                                                                \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error ", ncclGetErrorString(r_), " at " #x);     \
  } while (0)

at::Tensor rccl_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  auto t = at::empty({(int64_t)sizeof(id)}, at::kByte);
  std::memcpy(t.data_ptr(), &id, sizeof(id));
  return t;
}

int64_t rccl_init(const at::Tensor& uid, int64_t world, int64_t rank) {
  TORCH_CHECK(uid.numel() == sizeof(ncclUniqueId) && uid.scalar_type() == at::kByte, "bad unique id tensor");
  ncclUniqueId id;
  std::memcpy(&id, uid.cpu().data_ptr(), sizeof(id));
  ncclComm_t comm;
  RCCL_CHECK(ncclCommInitRank(&comm, (int)world, id, (int)rank));
  std::lock_guard<std::mutex> g(g_mu);
  g_comms.push_back(comm);
  return (int64_t)g_comms.size() - 1;
}

ncclComm_t get(int64_t h) {
  std::lock_guard<std::mutex> g(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr, "invalid RCCL communicator");
  return g_comms[h];
}

ncclDataType_t dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
}

ncclRedOp_t op_of(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  TORCH_CHECK(false, "unsupported reduce op ", op);
}

hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.get_device()).stream(); }

void rccl_all_reduce(at::Tensor& t, int64_t h, const std::string& op) {
  TORCH_CHECK(t.is_contiguous(), "all_reduce needs a contiguous tensor");
  RCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), op_of(op), get(h), stream_of(t)));
}

void rccl_all_gather(const at::Tensor& in, at::Tensor& out, int64_t h) {
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "all_gather needs contiguous tensors");
  RCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), dtype_of(in), get(h), stream_of(in)));
}

void rccl_broadcast(at::Tensor& t, int64_t root, int64_t h) {
  RCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), (int)root, get(h), stream_of(t)));
}

// all-to-all-v on rows: send_counts / recv_counts in rows (host lists), row = `row_elems` elements.
void rccl_all_to_all(const at::Tensor& send, at::Tensor& recv, std::vector<int64_t> send_counts,
                     std::vector<int64_t> recv_counts, int64_t row_elems, int64_t h) {
  ncclComm_t comm = get(h);
  int world = 0;
  RCCL_CHECK(ncclCommCount(comm, &world));
  TORCH_CHECK((int)send_counts.size() == world && (int)recv_counts.size() == world, "count lists must be world-sized");
  const auto dt = dtype_of(send);
  const size_t esz = send.element_size();
  hipStream_t s = stream_of(send);
  const char* sp = (const char*)send.data_ptr();
  char* rp = (char*)recv.data_ptr();
  int64_t so = 0, ro = 0;
  RCCL_CHECK(ncclGroupStart());
  for (int p = 0; p < world; ++p) {
    if (send_counts[p]) RCCL_CHECK(ncclSend(sp + so * row_elems * esz, send_counts[p] * row_elems, dt, p, comm, s));
    if (recv_counts[p]) RCCL_CHECK(ncclRecv(rp + ro * row_elems * esz, recv_counts[p] * row_elems, dt, p, comm, s));
    so += send_counts[p];
    ro += recv_counts[p];
  }
  RCCL_CHECK(ncclGroupEnd());
}

void rccl_destroy(int64_t h) {
  std::lock_guard<std::mutex> g(g_mu);
  if (h >= 0 && h < (int64_t)g_comms.size() && g_comms[h]) {
    ncclCommDestroy(g_comms[h]);
    g_comms[h] = nullptr;
  }
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(symmetry_amd, m) {
  m.def("rccl_unique_id() -> Tensor", &rccl_unique_id);
  m.def("rccl_init(Tensor uid, int world, int rank) -> int", &rccl_init);
  m.def("rccl_all_reduce(Tensor(a!) t, int comm, str op) -> ()", &rccl_all_reduce);
  m.def("rccl_all_gather(Tensor input, Tensor(a!) out, int comm) -> ()", &rccl_all_gather);
  m.def("rccl_broadcast(Tensor(a!) t, int root, int comm) -> ()", &rccl_broadcast);
  m.def(
      "rccl_all_to_all(Tensor send, Tensor(a!) recv, int[] send_counts, int[] recv_counts, int row_elems, int comm) "
      "-> ()",
      &rccl_all_to_all);
  m.def("rccl_destroy(int comm) -> ()", &rccl_destroy);
}
