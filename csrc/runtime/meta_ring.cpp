// R4: the rank-0 -> worker step-metadata plane of a tensor-parallel provider.
//
// Rank 0 owns the scheduler; every TP worker must enqueue the same step (same packed int32 metadata:
// token ids, positions, slots, block tables, sampling params) on its own GPU.  Round 2 pushed that
// with two gloo broadcasts per step over TCP and made each worker synchronise its stream after every
// step, so rank 0's first xGMI collective of a step spun while the workers' hosts were still receiving.
// Here the metadata goes through a single-producer / multi-consumer ring in POSIX shared memory (all
// ranks of a provider live on one node): rank 0 appends a step with one memcpy and a release store and
// goes on to the next step; every worker polls its own read cursor, so a worker enqueues step N+1 while
// its GPU still runs step N (pipelined TP decode).  The ring is bounded (nslots steps), and rank 0 only
// blocks if a worker falls nslots steps behind.
//
// Layout of the mapping:  Header | slot[nslots] where slot = {u64 seq, u32 bytes, u32 pad, payload}.
// A slot is published by storing its seq (release) after the payload; a reader owns message k when
// slot[k % nslots].seq == k + 1 (acquire), and releases it by advancing its cursor (release).
//
// Back-channel (fault containment): every process registers its pid in the header; a worker that fails
// stores a nonzero error code in its own word before it exits.  Rank 0's health monitor reads
// `faults()` -- reported codes, plus readers whose process is gone (killed: no chance to report) -- so a
// dead peer is noticed on the host within one poll instead of by the device collectives' wait limit, and a
// worker notices a dead rank 0 the same way (pop returns None).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <atomic>
#include <cerrno>
#include <csignal>
#include <cstdio>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <stdexcept>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <time.h>
#include <unistd.h>

#if defined(__x86_64__)
#include <immintrin.h>
#define RING_PAUSE() _mm_pause()
#else
#define RING_PAUSE() std::atomic_signal_fence(std::memory_order_seq_cst)
#endif

namespace py = pybind11;

namespace {

constexpr uint64_t kMagic = 0x53594d4d52494e47ull;  // "SYMMRING"
constexpr int kMaxReaders = 16;

struct alignas(64) Cursor {
  std::atomic<uint64_t> v;
  char pad[64 - sizeof(std::atomic<uint64_t>)];
};

struct Header {
  uint64_t magic;
  uint64_t slot_bytes;  // payload capacity of one slot
  uint64_t nslots;
  uint64_t readers;
  alignas(64) std::atomic<uint64_t> written;  // messages published
  alignas(64) std::atomic<uint32_t> closed;   // the producer shut the ring down
  Cursor read[kMaxReaders];                   // messages consumed, per reader
  alignas(64) std::atomic<int32_t> rerr[kMaxReaders];  // worker -> rank 0 error codes (0 = healthy)
  std::atomic<int32_t> rpid[kMaxReaders];              // reader pids (0 = not registered)
  std::atomic<int32_t> wpid;                           // producer pid
};

struct SlotHdr {
  std::atomic<uint64_t> seq;
  uint32_t bytes;
  uint32_t pad;
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory atomics must be lock-free");

// false once `pid` has exited (gone, or a zombie its parent has not reaped yet)
bool pid_alive(int pid) {
  if (pid <= 0) return true;
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  FILE* f = std::fopen(path, "r");
  if (f == nullptr) return true;  // no procfs: trust kill()
  char buf[512];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* rp = std::strrchr(buf, ')');  // "pid (comm) S ...": the state follows the last ')'
  return !(rp != nullptr && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X'));
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Spin hard for the first `spin_s`, then nap in growing steps (idle provider: ~no CPU).
class Backoff {
 public:
  explicit Backoff(double spin_s) : t0_(now_s()), spin_s_(spin_s) {}
  // returns the elapsed seconds
  double wait() {
    const double el = now_s() - t0_;
    if (el < spin_s_) {
      for (int i = 0; i < 32; ++i) RING_PAUSE();
      return el;
    }
    const long ns = el < 0.05 ? 20000 : el < 1.0 ? 200000 : 1000000;
    timespec ts{0, ns};
    nanosleep(&ts, nullptr);
    return el;
  }

 private:
  double t0_, spin_s_;
};

class MetaRing {
 public:
  MetaRing(const std::string& name, int64_t slot_bytes, int64_t nslots, int64_t readers, bool create)
      : name_(name), owner_(create) {
    if (readers < 0 || readers > kMaxReaders) throw std::invalid_argument("MetaRing: 0..16 readers");
    if (create && (slot_bytes <= 0 || nslots <= 0)) throw std::invalid_argument("MetaRing: slot_bytes, nslots > 0");
    int fd = -1;
    if (create) {
      fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("MetaRing: shm_open(create " + name + "): " + std::strerror(errno));
      slot_stride_ = (sizeof(SlotHdr) + (uint64_t)slot_bytes + 63) / 64 * 64;
      bytes_ = sizeof(Header) + slot_stride_ * (uint64_t)nslots;
      if (ftruncate(fd, (off_t)bytes_) != 0) {
        const int e = errno;
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error(std::string("MetaRing: ftruncate: ") + std::strerror(e));
      }
    } else {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("MetaRing: shm_open(" + name + "): " + std::strerror(errno));
      struct stat st {};
      fstat(fd, &st);
      bytes_ = (uint64_t)st.st_size;
      if (bytes_ < sizeof(Header)) {
        close(fd);
        throw std::runtime_error("MetaRing: " + name + " is not initialised");
      }
    }
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error(std::string("MetaRing: mmap: ") + std::strerror(errno));
    base_ = static_cast<char*>(p);
    h_ = reinterpret_cast<Header*>(base_);
    if (create) {
      std::memset(base_, 0, sizeof(Header));
      h_->slot_bytes = (uint64_t)slot_bytes;
      h_->nslots = (uint64_t)nslots;
      h_->readers = (uint64_t)readers;
      for (uint64_t i = 0; i < (uint64_t)nslots; ++i) slot(i)->seq.store(0, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      h_->magic = kMagic;
    } else {
      if (h_->magic != kMagic) throw std::runtime_error("MetaRing: bad magic in " + name);
      slot_stride_ = (sizeof(SlotHdr) + h_->slot_bytes + 63) / 64 * 64;
    }
  }

  ~MetaRing() { release(); }

  int64_t slot_bytes() const { return (int64_t)h_->slot_bytes; }
  int64_t nslots() const { return (int64_t)h_->nslots; }
  int64_t written() const { return (int64_t)h_->written.load(std::memory_order_acquire); }

  // Producer: append one message (any C-contiguous buffer).  Blocks (GIL released) while the slowest
  // reader is nslots messages behind; raises after `timeout_s` (< 0: wait forever).
  void push(py::buffer buf, double timeout_s) {
    check_open();
    py::buffer_info info = buf.request();
    const uint64_t n = (uint64_t)info.size * (uint64_t)info.itemsize;
    if (n > h_->slot_bytes)
      throw std::invalid_argument("MetaRing.push: " + std::to_string(n) + " B message > " +
                                  std::to_string(h_->slot_bytes) + " B slot");
    const uint64_t k = h_->written.load(std::memory_order_relaxed);
    // Release the GIL only when the ring is full and we must wait: an idle release hands the GIL to the
    // provider's event-loop thread, and the engine thread then waits out the interpreter's switch interval
    // to get it back (the TP client-end run measured ~2 ms of "launch" per step from exactly that)
    if (k - min_read() >= h_->nslots) {
      py::gil_scoped_release nogil;
      Backoff bo(0.002);
      int it = 0;
      while (k - min_read() >= h_->nslots) {
        if (bo.wait() > timeout_s && timeout_s >= 0)
          throw std::runtime_error("MetaRing.push: a reader is " + std::to_string(h_->nslots) +
                                   " messages behind and made no progress");
        if ((++it & 1023) == 0 && first_fault() >= 0)
          throw std::runtime_error("MetaRing.push: a reader failed (see faults())");
      }
    }
    SlotHdr* s = slot(k % h_->nslots);
    std::memcpy(reinterpret_cast<char*>(s) + sizeof(SlotHdr), info.ptr, n);
    s->bytes = (uint32_t)n;
    s->seq.store(k + 1, std::memory_order_release);
    h_->written.store(k + 1, std::memory_order_release);
  }

  // Reader `r`: the next message as int32 (None once the producer closed the ring AND it is drained).
  // Waits with the GIL released; raises TimeoutError after `timeout_s` (< 0: wait forever).
  py::object pop(int64_t r, double timeout_s) {
    check_open();
    if (r < 0 || (uint64_t)r >= h_->readers) throw std::invalid_argument("MetaRing.pop: bad reader index");
    const uint64_t k = h_->read[r].v.load(std::memory_order_relaxed);
    SlotHdr* s = slot(k % h_->nslots);
    bool closed = false, timed_out = false;
    {
      py::gil_scoped_release nogil;
      Backoff bo(0.005);
      int it = 0;
      while (s->seq.load(std::memory_order_acquire) != k + 1) {
        const bool gone = (++it & 1023) == 0 && !pid_alive(h_->wpid.load(std::memory_order_relaxed));
        if (gone || h_->closed.load(std::memory_order_acquire)) {
          // the producer may have published message k between our seq load and its shut(): the closed
          // flag was stored after that seq (release), so this acquire re-load sees it if it exists
          closed = s->seq.load(std::memory_order_acquire) != k + 1;
          break;
        }
        if (bo.wait() > timeout_s && timeout_s >= 0) {
          timed_out = true;
          break;
        }
      }
    }
    if (timed_out) {
      PyErr_SetString(PyExc_TimeoutError, "MetaRing.pop: timed out");
      throw py::error_already_set();
    }
    if (closed) return py::none();
    const uint32_t n = s->bytes;
    py::array_t<int32_t> out((py::ssize_t)(n / 4));
    std::memcpy(out.mutable_data(), reinterpret_cast<char*>(s) + sizeof(SlotHdr), n);
    h_->read[r].v.store(k + 1, std::memory_order_release);
    return std::move(out);
  }

  // Producer: wake every reader with "closed" (their pop returns None once the ring is drained).
  void shut() {
    check_open();
    h_->closed.store(1, std::memory_order_release);
  }

  // Register this process as reader r (r < 0: the producer) for the liveness checks.
  void register_pid(int64_t r, int64_t pid) {
    check_open();
    if (r < 0) {
      h_->wpid.store((int32_t)pid, std::memory_order_release);
      return;
    }
    if ((uint64_t)r >= h_->readers) throw std::invalid_argument("MetaRing.register_pid: bad reader index");
    h_->rpid[r].store((int32_t)pid, std::memory_order_release);
  }

  // Reader r reports a failure (code != 0) to the producer before it exits.
  void report(int64_t r, int64_t code) {
    check_open();
    if (r < 0 || (uint64_t)r >= h_->readers) throw std::invalid_argument("MetaRing.report: bad reader index");
    h_->rerr[r].store(code ? (int32_t)code : 1, std::memory_order_release);
  }

  // Producer: [(reader, code)] of every faulted reader: its reported code, or -1 if its process is gone.
  py::list faults() const {
    check_open();
    py::list out;
    for (uint64_t r = 0; r < h_->readers; ++r) {
      const int code = fault_of(r);
      if (code != 0) out.append(py::make_tuple((int64_t)r, (int64_t)code));
    }
    return out;
  }

  void unlink() {
    if (!name_.empty()) shm_unlink(name_.c_str());
  }

  void release() {
    if (base_ != nullptr) {
      munmap(base_, bytes_);
      base_ = nullptr;
      h_ = nullptr;
    }
  }

 private:
  SlotHdr* slot(uint64_t i) const {
    return reinterpret_cast<SlotHdr*>(base_ + sizeof(Header) + i * slot_stride_);
  }
  int fault_of(uint64_t r) const {
    const int code = h_->rerr[r].load(std::memory_order_acquire);
    if (code != 0) return code;
    return pid_alive(h_->rpid[r].load(std::memory_order_acquire)) ? 0 : -1;
  }
  int first_fault() const {
    for (uint64_t r = 0; r < h_->readers; ++r)
      if (fault_of(r) != 0) return (int)r;
    return -1;
  }
  uint64_t min_read() const {
    uint64_t m = UINT64_MAX;
    for (uint64_t r = 0; r < h_->readers; ++r) {
      const uint64_t v = h_->read[r].v.load(std::memory_order_acquire);
      m = v < m ? v : m;
    }
    return h_->readers ? m : h_->written.load(std::memory_order_relaxed);
  }
  void check_open() const {
    if (h_ == nullptr) throw std::runtime_error("MetaRing: released");
  }

  std::string name_;
  bool owner_ = false;
  char* base_ = nullptr;
  Header* h_ = nullptr;
  uint64_t bytes_ = 0;
  uint64_t slot_stride_ = 0;
};

}  // namespace

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "symmetry_amd native runtime: shared-memory step-metadata ring for TP workers (R4)";
  py::class_<MetaRing>(m, "MetaRing")
      .def(py::init<const std::string&, int64_t, int64_t, int64_t, bool>(), py::arg("name"), py::arg("slot_bytes"),
           py::arg("nslots"), py::arg("readers"), py::arg("create"))
      .def("push", &MetaRing::push, py::arg("buf"), py::arg("timeout_s") = 60.0)
      .def("pop", &MetaRing::pop, py::arg("reader"), py::arg("timeout_s") = -1.0)
      .def("shut", &MetaRing::shut)
      .def("register_pid", &MetaRing::register_pid, py::arg("reader"), py::arg("pid"))
      .def("report", &MetaRing::report, py::arg("reader"), py::arg("code"))
      .def("faults", &MetaRing::faults)
      .def("unlink", &MetaRing::unlink)
      .def("release", &MetaRing::release)
      .def_property_readonly("slot_bytes", &MetaRing::slot_bytes)
      .def_property_readonly("nslots", &MetaRing::nslots)
      .def_property_readonly("written", &MetaRing::written);
}
