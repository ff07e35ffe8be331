// Filesystem KV tier (the llmd-fs-connector role). One file per
// KV block under <root>/<key[0:2]>/<key>.kv, written by a native thread pool
// (write to a temp file + fsync-less atomic rename, so readers never see a
// torn block; "the directory is the index"). Survives engine restarts.
//
// Asynchronous I/O on two pools (the reference offloader's n_read_threads /
// n_write_threads, docs/architecture/advanced/kv-management/kv-offloader.md):
//   * write_async(name, ptr, bytes, ticket): the worker writes straight from the
//     caller's (pinned host-tier) buffer, no copy on the engine thread; the
//     caller keeps the buffer unchanged until poll_writes() returns the ticket;
//   * read_async(name, ptr, bytes, ticket): a read worker fills the caller's
//     pinned buffer; poll_reads() returns (ticket, ok). Blocks still queued for
//     writing are served from the writer's source buffer.
// write()/read() are the synchronous forms. Per-direction byte and time
// counters feed vllm:kv_offload_* metrics.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <functional>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <memory>
#include <mutex>
#include <string>
#include <sys/stat.h>
#include <sys/types.h>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

class FsStore {
 public:
  FsStore(const std::string& root, int threads, int read_threads) : root_(root) {
    ::mkdir(root_.c_str(), 0755);
    for (int i = 0; i < std::max(1, threads); ++i) workers_.emplace_back([this] { run_writes(); });
    for (int i = 0; i < std::max(1, read_threads); ++i) workers_.emplace_back([this] { run_reads(); });
  }
  ~FsStore() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    rcv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  // synchronous-source write: the bytes are copied now (small / test use)
  void write(const std::string& name, py::array_t<uint8_t, py::array::c_style> data) {
    auto own = std::make_shared<std::vector<uint8_t>>(data.data(), data.data() + data.size());
    enqueue_write(name, Job{own->data(), own->size(), -1, own});
  }

  // zero-copy write from a caller-owned buffer that stays valid until `ticket` is polled
  void write_async(const std::string& name, uintptr_t ptr, int64_t bytes, int64_t ticket) {
    enqueue_write(name, Job{reinterpret_cast<const uint8_t*>(ptr), (size_t)bytes, ticket, nullptr});
  }

  std::vector<int64_t> poll_writes() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int64_t> out;
    out.swap(wdone_);
    return out;
  }

  bool exists(const std::string& name) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (pending_.count(name)) return true;
    }
    struct stat st;
    return ::stat(path(name).c_str(), &st) == 0;
  }

  bool read(const std::string& name, py::array_t<uint8_t, py::array::c_style> out) {
    uint8_t* dst = out.mutable_data();
    const size_t n = (size_t)out.size();
    py::gil_scoped_release nogil;
    return read_into(name, dst, n);
  }

  void read_async(const std::string& name, uintptr_t ptr, int64_t bytes, int64_t ticket) {
    {
      std::lock_guard<std::mutex> g(mu_);
      rq_.push_back(RJob{name, reinterpret_cast<uint8_t*>(ptr), (size_t)bytes, ticket});
    }
    rcv_.notify_one();
  }

  std::vector<std::pair<int64_t, bool>> poll_reads() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::pair<int64_t, bool>> out;
    out.swap(rdone_);
    return out;
  }

  void flush() {
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [this] { return q_.empty() && in_flight_ == 0 && rq_.empty() && r_in_flight_ == 0; });
  }

  bool remove(const std::string& name) { return ::unlink(path(name).c_str()) == 0; }

  int64_t written() const { return written_.load(); }
  // {bytes_written, write_seconds, bytes_read, read_seconds}
  std::vector<double> io_stats() const {
    return {(double)wbytes_.load(), wns_.load() * 1e-9, (double)rbytes_.load(), rns_.load() * 1e-9};
  }

 private:
  struct Job {
    const uint8_t* data;
    size_t size;
    int64_t ticket;                               // -1: synchronous-source write (owns its copy)
    std::shared_ptr<std::vector<uint8_t>> own;
  };
  struct RJob {
    std::string name;
    uint8_t* dst;
    size_t size;
    int64_t ticket;
  };

  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }

  std::string path(const std::string& name) const {
    const std::string d = root_ + "/" + name.substr(0, 2);
    return d + "/" + name + ".kv";
  }

  // Per name at most one job is QUEUED (not yet picked by a worker) and at most
  // one RUNNING. A new write replaces only the queued one, whose ticket is then
  // reported as done (superseded: no worker ever read its buffer); a running job
  // keeps its buffer until its own worker reports its ticket. Writes of one name
  // are serialized (the finishing worker re-queues the name), so renames land in
  // enqueue order and an older block can never overwrite a newer one.
  void enqueue_write(const std::string& name, Job job) {
    {
      std::lock_guard<std::mutex> g(mu_);
      Entry& e = pending_[name];
      const bool queued = e.has_queued;
      if (queued && e.queued.ticket >= 0) wdone_.push_back(e.queued.ticket);  // superseded, never read
      e.queued = job;
      e.has_queued = true;
      if (!queued && !e.running) q_.push_back(name);
    }
    cv_.notify_one();
  }

  bool read_into(const std::string& name, uint8_t* dst, size_t n) {
    const int64_t t0 = now_ns();
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = pending_.find(name);
      if (it != pending_.end()) {  // queued or being written: copy from the newest source buffer
        const Job& j = it->second.has_queued ? it->second.queued : it->second.running_job;
        if (j.size != n) return false;
        std::memcpy(dst, j.data, n);
        return true;
      }
    }
    int fd = ::open(path(name).c_str(), O_RDONLY);
    if (fd < 0) return false;
    size_t off = 0;
    while (off < n) {
      ssize_t r = ::read(fd, dst + off, n - off);
      if (r <= 0) break;
      off += (size_t)r;
    }
    ::close(fd);
    if (off == n) {
      rbytes_ += (int64_t)n;
      rns_ += now_ns() - t0;
    }
    return off == n;
  }

  void run_reads() {
    for (;;) {
      RJob job;
      {
        std::unique_lock<std::mutex> g(mu_);
        rcv_.wait(g, [this] { return stop_ || !rq_.empty(); });
        if (stop_ && rq_.empty()) return;
        job = rq_.front();
        rq_.pop_front();
        ++r_in_flight_;
      }
      const bool ok = read_into(job.name, job.dst, job.size);
      {
        std::lock_guard<std::mutex> g(mu_);
        rdone_.emplace_back(job.ticket, ok);
        --r_in_flight_;
      }
      done_cv_.notify_all();
    }
  }

  void run_writes() {
    for (;;) {
      std::string name;
      Job job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        name = q_.front();
        q_.pop_front();
        auto it = pending_.find(name);
        if (it == pending_.end() || !it->second.has_queued || it->second.running) continue;
        Entry& e = it->second;
        job = e.queued;
        e.running_job = e.queued;
        e.has_queued = false;
        e.running = true;
        ++in_flight_;
      }
      const int64_t t0 = now_ns();
      const std::string d = root_ + "/" + name.substr(0, 2);
      ::mkdir(d.c_str(), 0755);
      const std::string fin = path(name);
      const std::string tmp = fin + ".tmp" + std::to_string((uintptr_t)job.data) + "." +
                              std::to_string((uintptr_t)std::hash<std::thread::id>{}(std::this_thread::get_id()));
      int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
      bool ok = fd >= 0;
      if (ok) {
        size_t off = 0;
        while (off < job.size) {
          ssize_t w = ::write(fd, job.data + off, job.size - off);
          if (w <= 0) {
            ok = false;
            break;
          }
          off += (size_t)w;
        }
        ::close(fd);
        if (ok) ok = ::rename(tmp.c_str(), fin.c_str()) == 0;
        if (!ok) ::unlink(tmp.c_str());
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        auto it = pending_.find(name);
        bool requeue = false;
        if (it != pending_.end()) {
          it->second.running = false;
          if (it->second.has_queued) requeue = true;  // a newer block arrived while this one was written
          else pending_.erase(it);
        }
        if (requeue) q_.push_back(name);
        if (job.ticket >= 0) wdone_.push_back(job.ticket);
        --in_flight_;
        if (ok) {
          ++written_;
          wbytes_ += (int64_t)job.size;
          wns_ += now_ns() - t0;
        }
      }
      done_cv_.notify_all();
      cv_.notify_one();
    }
  }

  std::string root_;
  std::mutex mu_;
  std::condition_variable cv_, rcv_, done_cv_;
  std::deque<std::string> q_;
  std::deque<RJob> rq_;
  struct Entry {
    Job queued{nullptr, 0, -1, nullptr};
    Job running_job{nullptr, 0, -1, nullptr};
    bool has_queued = false, running = false;
  };
  std::unordered_map<std::string, Entry> pending_;
  std::vector<int64_t> wdone_;
  std::vector<std::pair<int64_t, bool>> rdone_;
  std::vector<std::thread> workers_;
  bool stop_ = false;
  int in_flight_ = 0, r_in_flight_ = 0;
  std::atomic<int64_t> written_{0}, wbytes_{0}, wns_{0}, rbytes_{0}, rns_{0};
};

}  // namespace

void register_fs_store(py::module_& m) {
  py::class_<FsStore>(m, "FsStore")
      .def(py::init<const std::string&, int, int>(), py::arg("root"), py::arg("threads") = 8,
           py::arg("read_threads") = 8)
      .def("write", &FsStore::write)
      .def("write_async", &FsStore::write_async)
      .def("poll_writes", &FsStore::poll_writes)
      .def("exists", &FsStore::exists)
      .def("read", &FsStore::read)
      .def("read_async", &FsStore::read_async)
      .def("poll_reads", &FsStore::poll_reads)
      .def("io_stats", &FsStore::io_stats)
      .def("flush", &FsStore::flush, py::call_guard<py::gil_scoped_release>())
      .def("remove", &FsStore::remove)
      .def_property_readonly("written", &FsStore::written);
}
