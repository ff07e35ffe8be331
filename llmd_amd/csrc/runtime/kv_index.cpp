// Router-side prefix indexes (reference semantics in
// docs/architecture/advanced/kv-management/kv-indexer.md:65-151 and
// prefix-cache-aware-routing.md:18-24).
//
// KVBlockIndex  - precise index fed by engine KV events: two-level LRU
//                 (block key -> {pod -> tier mask | speculative expiry}),
//                 longest *consecutive* prefix scoring with tier weights
//                 (max weight over tiers holding the block), speculative
//                 entries with a TTL closing the route->event blind spot.
// ApproxIndex   - approximate index: per-server LRU of block hashes the
//                 router itself has sent there (learn-on-route).
// Both are hot paths (every request x every pod x every block), so they are
// native; Python only passes arrays of 64-bit keys.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <cstdint>
#include <list>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

struct PodEntry {
  uint32_t tiers = 0;      // bit per tier (0 = gpu, 1 = cpu, 2 = disk ...)
  double spec_expiry = 0;  // >0: speculative until this time
};

struct KeyEntry {
  std::vector<std::pair<int32_t, PodEntry>> pods;  // small inner map
  std::list<uint64_t>::iterator lru_it;
};

class KVBlockIndex {
 public:
  KVBlockIndex(int64_t max_keys, int pod_cap) : max_keys_(max_keys), pod_cap_(pod_cap) {}

  int pod_id(const std::string& pod) {
    auto it = pod_ids_.find(pod);
    if (it != pod_ids_.end()) return it->second;
    int id = (int)pod_names_.size();
    pod_ids_.emplace(pod, id);
    pod_names_.push_back(pod);
    return id;
  }
  int tier_id(const std::string& tier) {
    std::string t;
    for (char c : tier) t.push_back((char)std::tolower(c));
    if (t == "gpu" || t == "hbm" || t.empty()) return 0;
    if (t == "cpu" || t == "cpu_pinned" || t == "dram") return 1;
    if (t == "disk" || t == "fs" || t == "storage") return 2;
    auto it = tier_ids_.find(t);
    if (it != tier_ids_.end()) return it->second;
    int id = 3 + (int)tier_ids_.size();
    tier_ids_.emplace(t, id);
    return id;
  }

  void add(const std::string& pod, const std::vector<uint64_t>& keys, const std::string& tier) {
    std::lock_guard<std::mutex> g(mu_);
    const int p = pod_id(pod), t = tier_id(tier);
    for (uint64_t k : keys) {
      PodEntry& e = entry(k, p);
      e.tiers |= (1u << t);
      e.spec_expiry = 0;
    }
  }

  void add_speculative(const std::string& pod, const std::vector<uint64_t>& keys, double ttl) {
    std::lock_guard<std::mutex> g(mu_);
    const int p = pod_id(pod);
    const double exp = now_s() + ttl;
    for (uint64_t k : keys) {
      PodEntry& e = entry(k, p);
      if (e.tiers == 0) e.spec_expiry = exp;
    }
  }

  void remove(const std::string& pod, const std::vector<uint64_t>& keys, const std::string& tier) {
    std::lock_guard<std::mutex> g(mu_);
    auto pit = pod_ids_.find(pod);
    if (pit == pod_ids_.end()) return;
    const int p = pit->second, t = tier_id(tier);
    for (uint64_t k : keys) {
      auto it = map_.find(k);
      if (it == map_.end()) continue;
      auto& v = it->second.pods;
      for (size_t i = 0; i < v.size(); ++i) {
        if (v[i].first != p) continue;
        v[i].second.tiers &= ~(1u << t);
        if (v[i].second.tiers == 0 && v[i].second.spec_expiry == 0) v.erase(v.begin() + i);
        break;
      }
      if (v.empty()) {
        lru_.erase(it->second.lru_it);
        map_.erase(it);
      }
    }
  }

  void clear_pod(const std::string& pod) {
    std::lock_guard<std::mutex> g(mu_);
    auto pit = pod_ids_.find(pod);
    if (pit == pod_ids_.end()) return;
    const int p = pit->second;
    for (auto it = map_.begin(); it != map_.end();) {
      auto& v = it->second.pods;
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i].first == p) {
          v.erase(v.begin() + i);
          break;
        }
      if (v.empty()) {
        lru_.erase(it->second.lru_it);
        it = map_.erase(it);
      } else {
        ++it;
      }
    }
  }

  // pod -> weighted length of the longest consecutive cached prefix (in blocks)
  std::unordered_map<std::string, double> score(const std::vector<uint64_t>& keys,
                                                const std::vector<std::string>& pods,
                                                const std::vector<double>& tier_w,
                                                double spec_weight) {
    std::lock_guard<std::mutex> g(mu_);
    const double now = now_s();
    std::vector<int> pidx;
    std::unordered_map<std::string, double> out;
    for (auto& s : pods) {
      auto it = pod_ids_.find(s);
      pidx.push_back(it == pod_ids_.end() ? -1 : it->second);
      out[s] = 0.0;
    }
    std::vector<char> alive(pods.size(), 1);
    size_t n_alive = pods.size();
    for (uint64_t k : keys) {
      if (n_alive == 0) break;
      auto it = map_.find(k);
      if (it == map_.end()) break;
      touch(it->second);
      auto& v = it->second.pods;
      for (size_t j = 0; j < pods.size(); ++j) {
        if (!alive[j]) continue;
        double w = 0;
        if (pidx[j] >= 0) {
          for (auto& pe : v) {
            if (pe.first != pidx[j]) continue;
            for (size_t t = 0; t < tier_w.size() && t < 32; ++t)
              if (pe.second.tiers & (1u << t)) w = std::max(w, tier_w[t]);
            if (w == 0 && pe.second.spec_expiry > now) w = spec_weight;
          }
        }
        if (w <= 0) {
          alive[j] = 0;
          --n_alive;
        } else {
          out[pods[j]] += w;
        }
      }
    }
    return out;
  }

  int64_t size() const { return (int64_t)map_.size(); }

 private:
  PodEntry& entry(uint64_t k, int p) {
    auto it = map_.find(k);
    if (it == map_.end()) {
      if ((int64_t)map_.size() >= max_keys_ && !lru_.empty()) {
        map_.erase(lru_.back());
        lru_.pop_back();
      }
      lru_.push_front(k);
      KeyEntry e;
      e.lru_it = lru_.begin();
      it = map_.emplace(k, std::move(e)).first;
    } else {
      touch(it->second);
    }
    auto& v = it->second.pods;
    for (auto& pe : v)
      if (pe.first == p) return pe.second;
    if ((int)v.size() >= pod_cap_) v.erase(v.begin());  // inner LRU-ish: drop oldest
    v.emplace_back(p, PodEntry{});
    return v.back().second;
  }
  void touch(KeyEntry& e) {
    lru_.splice(lru_.begin(), lru_, e.lru_it);
  }

  int64_t max_keys_;
  int pod_cap_;
  std::mutex mu_;
  std::unordered_map<uint64_t, KeyEntry> map_;
  std::list<uint64_t> lru_;
  std::unordered_map<std::string, int> pod_ids_;
  std::vector<std::string> pod_names_;
  std::unordered_map<std::string, int> tier_ids_;
};

class ApproxIndex {
 public:
  explicit ApproxIndex(int64_t cap_per_server) : cap_(cap_per_server) {}

  void insert(const std::string& server, const std::vector<uint64_t>& keys) {
    std::lock_guard<std::mutex> g(mu_);
    auto& s = servers_[server];
    const int64_t cap = s.cap > 0 ? s.cap : cap_;
    for (uint64_t k : keys) {
      auto it = s.map.find(k);
      if (it != s.map.end()) {
        s.lru.splice(s.lru.begin(), s.lru, it->second);
        continue;
      }
      if ((int64_t)s.map.size() >= cap && !s.lru.empty()) {
        s.map.erase(s.lru.back());
        s.lru.pop_back();
      }
      s.lru.push_front(k);
      s.map.emplace(k, s.lru.begin());
    }
  }

  // server -> number of leading keys present (consecutive)
  std::unordered_map<std::string, int> match(const std::vector<uint64_t>& keys,
                                             const std::vector<std::string>& servers) {
    std::lock_guard<std::mutex> g(mu_);
    std::unordered_map<std::string, int> out;
    for (auto& name : servers) {
      int n = 0;
      auto sit = servers_.find(name);
      if (sit != servers_.end()) {
        for (uint64_t k : keys) {
          if (!sit->second.map.count(k)) break;
          ++n;
        }
      }
      out[name] = n;
    }
    return out;
  }

  void remove_server(const std::string& s) {
    std::lock_guard<std::mutex> g(mu_);
    servers_.erase(s);
  }
  // Per-server LRU capacity (autoTune: the server's real KV capacity in
  // producer blocks); shrinking evicts the least recently used keys at once.
  void set_capacity(const std::string& server, int64_t cap) {
    std::lock_guard<std::mutex> g(mu_);
    auto& s = servers_[server];
    s.cap = cap;
    const int64_t c = cap > 0 ? cap : cap_;
    while ((int64_t)s.map.size() > c && !s.lru.empty()) {
      s.map.erase(s.lru.back());
      s.lru.pop_back();
    }
  }
  int64_t server_size(const std::string& server) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = servers_.find(server);
    return it == servers_.end() ? 0 : (int64_t)it->second.map.size();
  }
  int64_t size() const {
    int64_t n = 0;
    for (auto& kv : servers_) n += (int64_t)kv.second.map.size();
    return n;
  }

 private:
  struct S {
    int64_t cap = -1;  // < 0: the index-wide default
    std::list<uint64_t> lru;
    std::unordered_map<uint64_t, std::list<uint64_t>::iterator> map;
  };
  int64_t cap_;
  std::mutex mu_;
  std::unordered_map<std::string, S> servers_;
};

// Rolling hash chain over character blocks (approximate producer). FNV-1a
// over the block bytes chained with the parent.
std::vector<uint64_t> char_block_hashes(const std::string& text, int block_chars, uint64_t seed,
                                        int max_blocks) {
  std::vector<uint64_t> out;
  uint64_t parent = seed;
  const size_t n = text.size();
  for (size_t off = 0; off + (size_t)block_chars <= n; off += (size_t)block_chars) {
    if (max_blocks > 0 && (int)out.size() >= max_blocks) break;
    uint64_t h = 0xcbf29ce484222325ull ^ parent;
    for (int i = 0; i < block_chars; ++i) {
      h ^= (uint8_t)text[off + i];
      h *= 0x100000001b3ull;
    }
    h ^= h >> 29;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 32;
    out.push_back(h);
    parent = h;
  }
  return out;
}

}  // namespace

void register_kv_index(py::module_& m) {
  py::class_<KVBlockIndex>(m, "KVBlockIndex")
      .def(py::init<int64_t, int>(), py::arg("max_keys") = 100000000, py::arg("pod_cap") = 10)
      .def("add", &KVBlockIndex::add, py::arg("pod"), py::arg("keys"), py::arg("tier") = "gpu")
      .def("add_speculative", &KVBlockIndex::add_speculative, py::arg("pod"), py::arg("keys"),
           py::arg("ttl") = 2.0)
      .def("remove", &KVBlockIndex::remove, py::arg("pod"), py::arg("keys"), py::arg("tier") = "gpu")
      .def("clear_pod", &KVBlockIndex::clear_pod)
      .def("score", &KVBlockIndex::score, py::arg("keys"), py::arg("pods"),
           py::arg("tier_weights") = std::vector<double>{1.0, 0.8, 0.5}, py::arg("spec_weight") = 1.0)
      .def("size", &KVBlockIndex::size);
  py::class_<ApproxIndex>(m, "ApproxIndex")
      .def(py::init<int64_t>(), py::arg("cap_per_server") = 31250)
      .def("insert", &ApproxIndex::insert)
      .def("match", &ApproxIndex::match)
      .def("remove_server", &ApproxIndex::remove_server)
      .def("set_capacity", &ApproxIndex::set_capacity, py::arg("server"), py::arg("cap"))
      .def("server_size", &ApproxIndex::server_size)
      .def("size", &ApproxIndex::size);
  m.def("char_block_hashes", &char_block_hashes, py::arg("text"), py::arg("block_chars"),
        py::arg("seed") = 0, py::arg("max_blocks") = 0);
}
