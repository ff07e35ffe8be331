// Filesystem KV tier (the llmd-fs-connector role). One file per
// KV block under <root>/<key[0:2]>/<key>.kv, written by a native thread pool
// (write to a temp file + fsync-less atomic rename, so readers never see a
// torn block; "the directory is the index"). Reads are synchronous into a
// caller-provided (pinned) buffer; blocks still queued for writing are served
// from the queue. Survives engine restarts.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <atomic>
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
  FsStore(const std::string& root, int threads) : root_(root) {
    ::mkdir(root_.c_str(), 0755);
    for (int i = 0; i < std::max(1, threads); ++i) workers_.emplace_back([this] { run(); });
  }
  ~FsStore() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  void write(const std::string& name, py::array_t<uint8_t, py::array::c_style> data) {
    auto buf = std::make_shared<std::vector<uint8_t>>(data.data(), data.data() + data.size());
    {
      std::lock_guard<std::mutex> g(mu_);
      pending_[name] = buf;
      q_.push_back(name);
    }
    cv_.notify_one();
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
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = pending_.find(name);
      if (it != pending_.end()) {
        if ((py::ssize_t)it->second->size() != out.size()) return false;
        std::memcpy(out.mutable_data(), it->second->data(), it->second->size());
        return true;
      }
    }
    py::gil_scoped_release nogil;
    int fd = ::open(path(name).c_str(), O_RDONLY);
    if (fd < 0) return false;
    size_t off = 0, n = (size_t)out.size();
    uint8_t* dst = out.mutable_data();
    while (off < n) {
      ssize_t r = ::read(fd, dst + off, n - off);
      if (r <= 0) break;
      off += (size_t)r;
    }
    ::close(fd);
    return off == n;
  }

  void flush() {
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [this] { return q_.empty() && in_flight_ == 0; });
  }

  bool remove(const std::string& name) { return ::unlink(path(name).c_str()) == 0; }

  int64_t written() const { return written_.load(); }

 private:
  std::string path(const std::string& name) const {
    const std::string d = root_ + "/" + name.substr(0, 2);
    return d + "/" + name + ".kv";
  }

  void run() {
    for (;;) {
      std::string name;
      std::shared_ptr<std::vector<uint8_t>> buf;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        name = q_.front();
        q_.pop_front();
        buf = pending_[name];
        ++in_flight_;
      }
      const std::string d = root_ + "/" + name.substr(0, 2);
      ::mkdir(d.c_str(), 0755);
      const std::string fin = path(name);
      const std::string tmp = fin + ".tmp" + std::to_string((uintptr_t)buf.get());
      int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
      bool ok = fd >= 0;
      if (ok) {
        size_t off = 0;
        while (off < buf->size()) {
          ssize_t w = ::write(fd, buf->data() + off, buf->size() - off);
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
        if (it != pending_.end() && it->second == buf) pending_.erase(it);
        --in_flight_;
        if (ok) ++written_;
      }
      done_cv_.notify_all();
    }
  }

  std::string root_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<std::string> q_;
  std::unordered_map<std::string, std::shared_ptr<std::vector<uint8_t>>> pending_;
  std::vector<std::thread> workers_;
  bool stop_ = false;
  int in_flight_ = 0;
  std::atomic<int64_t> written_{0};
};

}  // namespace

void register_fs_store(py::module_& m) {
  py::class_<FsStore>(m, "FsStore")
      .def(py::init<const std::string&, int>(), py::arg("root"), py::arg("threads") = 8)
      .def("write", &FsStore::write)
      .def("exists", &FsStore::exists)
      .def("read", &FsStore::read)
      .def("flush", &FsStore::flush, py::call_guard<py::gil_scoped_release>())
      .def("remove", &FsStore::remove)
      .def_property_readonly("written", &FsStore::written);
}
