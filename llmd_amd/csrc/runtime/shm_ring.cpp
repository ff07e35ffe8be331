// Shared-memory broadcast ring: one writer (the TP driver), N readers (its
// followers on the same host) - the per-step plan channel of TP replicas
// (engine/tp_worker.py; the role vLLM's shm MessageQueue plays for its TP
// workers). Replaces two gloo broadcasts (size, then payload, ~100-300 us of
// loopback TCP per step) by a memcpy and one release store.
//
// Layout (one POSIX shm object):
//   Header: magic, slots, slot_bytes, readers, write_seq, read_seq[r] (each on
//           its own 64-B line, so readers never false-share);
//   slots x (u64 length + payload).
// Message k lives in slot k % slots. The writer may reuse a slot only when
// every reader has consumed the message that used it (read_seq[r] >= k -
// slots + 1); it publishes by storing write_seq = k + 1 (release), readers
// acquire-load write_seq and publish their progress the same way. Waits spin
// briefly, then yield, then sleep in 20-50 us steps (an idle follower costs
// ~nothing), always with the GIL released.
#include <fcntl.h>
#include <pybind11/pybind11.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace {

constexpr uint64_t MAGIC = 0x6c6c6d6452494e47ULL;  // "llmdRING"
constexpr int MAX_READERS = 31;

struct alignas(64) Line {
  std::atomic<uint64_t> v;
  char pad[56];
};

struct Header {
  uint64_t magic;
  uint64_t slots;
  uint64_t slot_bytes;
  uint64_t readers;
  char pad0[32];
  Line write_seq;
  Line read_seq[MAX_READERS];
};

class ShmRing {
 public:
  ShmRing(const std::string& name, bool create, int readers, int64_t slots, int64_t slot_bytes)
      : name_(name), owner_(create) {
    if (create) {
      if (readers < 1 || readers > MAX_READERS || slots < 1 || slot_bytes < 64)
        throw std::invalid_argument("ShmRing: bad geometry");
      size_ = sizeof(Header) + (size_t)slots * ((size_t)slot_bytes + 8);
      fd_ = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("ShmRing: shm_open(create) failed for " + name);
      if (ftruncate(fd_, (off_t)size_) != 0) {
        close(fd_);
        shm_unlink(name.c_str());
        throw std::runtime_error("ShmRing: ftruncate failed");
      }
    } else {
      fd_ = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("ShmRing: shm_open failed for " + name);
      struct stat st;
      if (fstat(fd_, &st) != 0 || (size_t)st.st_size < sizeof(Header)) {
        close(fd_);
        throw std::runtime_error("ShmRing: bad shm object");
      }
      size_ = (size_t)st.st_size;
    }
    base_ = (char*)mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) {
      close(fd_);
      if (create) shm_unlink(name.c_str());
      throw std::runtime_error("ShmRing: mmap failed");
    }
    h_ = reinterpret_cast<Header*>(base_);
    if (create) {
      h_->slots = (uint64_t)slots;
      h_->slot_bytes = (uint64_t)slot_bytes;
      h_->readers = (uint64_t)readers;
      h_->write_seq.v.store(0, std::memory_order_relaxed);
      for (int r = 0; r < MAX_READERS; ++r) h_->read_seq[r].v.store(0, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      h_->magic = MAGIC;
    } else if (h_->magic != MAGIC) {
      munmap(base_, size_);
      close(fd_);
      throw std::runtime_error("ShmRing: not a ring (magic)");
    }
  }

  ~ShmRing() { close_(); }

  int64_t slot_bytes() const { return (int64_t)h_->slot_bytes; }
  int readers() const { return (int)h_->readers; }

  // false if the message does not fit a slot (the caller uses its fallback channel)
  bool write(py::bytes data, double timeout_s) {
    std::string_view v = data;
    if (v.size() > h_->slot_bytes) return false;
    const uint64_t k = h_->write_seq.v.load(std::memory_order_relaxed);
    {
      py::gil_scoped_release nogil;
      if (k >= h_->slots) {
        const uint64_t need = k - h_->slots + 1;
        for (uint64_t r = 0; r < h_->readers; ++r)
          wait_([&] { return h_->read_seq[r].v.load(std::memory_order_acquire) >= need; }, timeout_s,
                "ShmRing.write: reader did not drain");
      }
      char* slot = slot_(k);
      const uint64_t n = v.size();
      std::memcpy(slot, &n, 8);
      std::memcpy(slot + 8, v.data(), n);
      h_->write_seq.v.store(k + 1, std::memory_order_release);
    }
    return true;
  }

  py::bytes read(int reader, double timeout_s) {
    if (reader < 0 || (uint64_t)reader >= h_->readers) throw std::out_of_range("ShmRing.read: reader id");
    const uint64_t k = h_->read_seq[reader].v.load(std::memory_order_relaxed);
    std::string out;
    {
      py::gil_scoped_release nogil;
      wait_([&] { return h_->write_seq.v.load(std::memory_order_acquire) > k; }, timeout_s,
            "ShmRing.read: no message");
      const char* slot = slot_(k);
      uint64_t n;
      std::memcpy(&n, slot, 8);
      if (n > h_->slot_bytes) throw std::runtime_error("ShmRing.read: corrupt length");
      out.assign(slot + 8, n);
      h_->read_seq[reader].v.store(k + 1, std::memory_order_release);
    }
    return py::bytes(out);
  }

  void unlink() {
    if (owner_ && !unlinked_) {
      shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

  void close_() {
    if (base_ != nullptr && base_ != MAP_FAILED) munmap(base_, size_);
    base_ = nullptr;
    if (fd_ >= 0) close(fd_);
    fd_ = -1;
    unlink();
  }

 private:
  char* slot_(uint64_t k) const {
    return base_ + sizeof(Header) + (size_t)(k % h_->slots) * ((size_t)h_->slot_bytes + 8);
  }

  template <class F>
  void wait_(F ready, double timeout_s, const char* what) {
    if (ready()) return;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0;; ++i) {
      if (ready()) return;
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (timeout_s > 0 && el > timeout_s) throw std::runtime_error(what);
      if (el < 50e-6) continue;                       // spin: a step plan usually arrives within us
      if (el < 2e-3) sched_yield();                   // yield while the writer is mid-step
      else std::this_thread::sleep_for(std::chrono::microseconds(el < 1.0 ? 20 : 50));
    }
  }

  std::string name_;
  bool owner_;
  bool unlinked_ = false;
  int fd_ = -1;
  size_t size_ = 0;
  char* base_ = nullptr;
  Header* h_ = nullptr;
};

}  // namespace

void register_shm_ring(py::module_& m) {
  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, bool, int, int64_t, int64_t>(), py::arg("name"), py::arg("create"),
           py::arg("readers") = 1, py::arg("slots") = 4, py::arg("slot_bytes") = 4 << 20)
      .def("write", &ShmRing::write, py::arg("data"), py::arg("timeout_s") = 0.0,
           "publish one message to every reader; False if it exceeds slot_bytes")
      .def("read", &ShmRing::read, py::arg("reader"), py::arg("timeout_s") = 0.0)
      .def("unlink", &ShmRing::unlink, "remove the name (mappings stay valid)")
      .def("close", &ShmRing::close_)
      .def_property_readonly("slot_bytes", &ShmRing::slot_bytes)
      .def_property_readonly("readers", &ShmRing::readers);
}
