// Paged KV block manager with automatic prefix caching (APC) and KV events.
//
// Native equivalent of the engine-side KV manager the reference's recipes rely
// on (vLLM APC + `--kv-events-config`):
//   * fixed pool of `num_blocks` GPU blocks of `block_size` tokens;
//   * per-sequence block tables;
//   * full blocks are content-addressed by a chained hash (hashing.h) and stay
//     cached after their sequence finishes, evictable in LRU order;
//   * every store / eviction / reset emits an event (BlockStored with parent
//     hash + tokens, BlockRemoved, AllBlocksCleared) drained by the publisher;
//   * evicted blocks are reported so an offload tier can save them first.
// Sliding-window groups (engine/hybrid_kv.py, the hybrid KV-cache manager):
//   * `reserved` leading blocks are never handed out; block 0 then serves as
//     the null block that replaces released table entries;
//   * release_before() drops a sequence's blocks that lie entirely before the
//     first key any future query can attend (they stay cached / evictable);
//   * acquire_window() takes a cached prefix whose LAST window of blocks is
//     resident (earlier entries are null): a windowed layer never reads older
//     keys, so they need not be cached.
// Single-threaded by design: the engine scheduler owns it.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "hashing.h"

namespace py = pybind11;
using namespace llmd_rt;

namespace {

struct Block {
  int32_t ref = 0;
  uint64_t hash = 0;     // 0 = not content-addressed
  uint64_t parent = 0;
  std::list<int32_t>::iterator lru_it;
  bool in_lru = false;
};

struct Seq {
  std::vector<int32_t> blocks;
  int32_t committed = 0;  // number of leading blocks already hashed/registered
  uint64_t last_hash = kRootHash;
  uint64_t extra = 0;
  int32_t released = 0;   // leading entries replaced by the null block
};

struct Event {
  int kind;  // 0 stored, 1 removed, 2 all cleared
  uint64_t hash;
  uint64_t parent;
  int32_t block;
  std::vector<int32_t> tokens;
};

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool prefix_caching, bool emit_events, int reserved = 0)
      : bs_(block_size), caching_(prefix_caching), events_on_(emit_events), reserved_(reserved),
        blocks_(num_blocks) {
    if (num_blocks <= reserved || block_size <= 0 || reserved < 0) throw std::invalid_argument("bad pool");
    free_.reserve(num_blocks);
    for (int i = num_blocks - 1; i >= reserved; --i) free_.push_back(i);
    for (int i = 0; i < reserved; ++i) blocks_[i].ref = 1;  // pinned forever
  }

  int block_size() const { return bs_; }
  int num_blocks() const { return (int)blocks_.size() - reserved_; }
  int num_free() const { return (int)(free_.size() + lru_.size()); }
  int num_cached() const { return (int)cache_.size(); }
  double usage() const { return 1.0 - (double)num_free() / (double)num_blocks(); }

  // Number of leading prompt tokens already in the cache (multiple of bs).
  // Never matches the whole prompt: at least one token must be computed.
  int lookup(py::array_t<int32_t, py::array::c_style | py::array::forcecast> toks,
             uint64_t extra) const {
    if (!caching_) return 0;
    auto r = toks.unchecked<1>();
    const int n = (int)r.shape(0);
    const int32_t* p = toks.data();
    uint64_t h = kRootHash;
    int hit = 0;
    for (int b = 0; (b + 1) * bs_ <= n - 1; ++b) {
      h = hash_block(h, extra, p + b * bs_, bs_);
      if (!cache_.count(h)) break;
      hit = (b + 1) * bs_;
    }
    return hit;
  }

  // Register a new sequence and take references on its cached prefix blocks
  // (at most max_tokens of them when max_tokens >= 0).
  int acquire(int64_t seq_id, py::array_t<int32_t, py::array::c_style | py::array::forcecast> toks,
              uint64_t extra, int max_tokens = -1) {
    if (seqs_.count(seq_id)) throw std::runtime_error("acquire: sequence exists");
    Seq s;
    s.extra = extra;
    const int n = (int)toks.shape(0);
    const int32_t* p = toks.data();
    if (caching_) {
      uint64_t h = kRootHash;
      for (int b = 0; (b + 1) * bs_ <= n - 1 && (max_tokens < 0 || (b + 1) * bs_ <= max_tokens); ++b) {
        const uint64_t nh = hash_block(h, extra, p + b * bs_, bs_);
        auto it = cache_.find(nh);
        if (it == cache_.end()) break;
        take_ref(it->second);
        s.blocks.push_back(it->second);
        h = nh;
      }
      s.committed = (int)s.blocks.size();
      s.last_hash = h;
      hits_ += (int64_t)s.blocks.size() * bs_;
    }
    queries_ += n;
    const int hit = (int)s.blocks.size() * bs_;
    seqs_.emplace(seq_id, std::move(s));
    return hit;
  }

  // Windowed group: the longest cached prefix of at most max_tokens tokens
  // (multiple of bs) whose blocks [lo, k) are all cached, lo = first block a
  // query at position k*bs can reach with a `window`-token window; entries
  // before lo become the null block (block 0, requires reserved >= 1).
  int acquire_window(int64_t seq_id, py::array_t<int32_t, py::array::c_style | py::array::forcecast> toks,
                     uint64_t extra, int max_tokens, int window) {
    if (seqs_.count(seq_id)) throw std::runtime_error("acquire_window: sequence exists");
    if (reserved_ < 1) throw std::runtime_error("acquire_window needs a reserved null block");
    Seq s;
    s.extra = extra;
    const int n = (int)toks.shape(0);
    const int32_t* p = toks.data();
    int best = 0;
    std::vector<uint64_t> hs;
    if (caching_) {
      uint64_t h = kRootHash;
      for (int b = 0; (b + 1) * bs_ <= n - 1 && (b + 1) * bs_ <= max_tokens; ++b) {
        h = hash_block(h, extra, p + b * bs_, bs_);
        hs.push_back(h);
      }
      // candidate k from the longest down: blocks [lo(k), k) must be cached
      for (int k = (int)hs.size(); k > 0; --k) {
        const int lo = std::max(0, (k * bs_ - window + 1) / bs_);
        bool ok = true;
        for (int b = lo; b < k && ok; ++b) ok = cache_.count(hs[b]) > 0;
        if (ok) {
          best = k;
          break;
        }
      }
      if (best > 0) {
        const int lo = std::max(0, (best * bs_ - window + 1) / bs_);
        for (int b = 0; b < lo; ++b) s.blocks.push_back(0);
        for (int b = lo; b < best; ++b) {
          const int32_t blk = cache_.find(hs[b])->second;
          take_ref(blk);
          s.blocks.push_back(blk);
        }
        s.released = lo;
        s.committed = best;
        s.last_hash = hs[best - 1];
      }
      hits_ += (int64_t)best * bs_;
    }
    queries_ += n;
    seqs_.emplace(seq_id, std::move(s));
    return best * bs_;
  }

  // Release every block of the sequence that lies entirely before token
  // position `first_needed` (never attended again by a windowed layer); the
  // table entries become the null block. Returns the number released.
  int release_before(int64_t seq_id, int first_needed) {
    if (reserved_ < 1) throw std::runtime_error("release_before needs a reserved null block");
    Seq& s = get(seq_id);
    const int upto = std::min<int>((int)s.blocks.size(), std::max(0, first_needed) / bs_);
    int n = 0;
    for (int b = s.released; b < upto; ++b) {
      if (s.blocks[b] != 0) {
        drop_ref(s.blocks[b]);
        s.blocks[b] = 0;
        ++n;
      }
    }
    s.released = std::max(s.released, upto);
    return n;
  }

  // Can `extra_blocks` more blocks be obtained right now?
  bool can_allocate(int extra_blocks) const { return extra_blocks <= num_free(); }

  // Ensure the sequence owns ceil(total_tokens / bs) blocks. Returns false
  // (and changes nothing) if the pool cannot satisfy it.
  bool grow(int64_t seq_id, int total_tokens) {
    Seq& s = get(seq_id);
    const int need = (total_tokens + bs_ - 1) / bs_ - (int)s.blocks.size();
    if (need <= 0) return true;
    if (need > num_free()) return false;
    for (int i = 0; i < need; ++i) s.blocks.push_back(pop_free());
    return true;
  }

  // Hash + register every full block whose tokens are all computed.
  void commit(int64_t seq_id, py::array_t<int32_t, py::array::c_style | py::array::forcecast> toks,
              int num_computed) {
    if (!caching_) return;
    Seq& s = get(seq_id);
    const int32_t* p = toks.data();
    const int n = std::min<int>((int)toks.shape(0), num_computed);
    const int full = std::min<int>(n / bs_, (int)s.blocks.size());
    for (int b = s.committed; b < full; ++b) {
      const uint64_t h = hash_block(s.last_hash, s.extra, p + b * bs_, bs_);
      const int32_t blk = s.blocks[b];
      auto it = cache_.find(h);
      if (blk < reserved_) {  // a released (null) entry: keep the hash chain, register nothing
        s.last_hash = h;
        s.committed = b + 1;
        continue;
      }
      if (it == cache_.end()) {
        Block& B = blocks_[blk];
        B.hash = h;
        B.parent = s.last_hash;
        cache_.emplace(h, blk);
        if (events_on_) events_.push_back(Event{0, h, s.last_hash, blk, std::vector<int32_t>(p + b * bs_, p + (b + 1) * bs_)});
      }
      // duplicate content computed concurrently: keep ours private (unhashed)
      s.last_hash = h;
      s.committed = b + 1;
    }
  }

  void free(int64_t seq_id) {
    auto it = seqs_.find(seq_id);
    if (it == seqs_.end()) return;
    // release in reverse so the tail of a prefix is evicted before its head
    const int rel = it->second.released;
    const auto& bl = it->second.blocks;
    for (int b = (int)bl.size() - 1; b >= rel; --b) drop_ref(bl[b]);
    seqs_.erase(it);
  }

  bool has_seq(int64_t seq_id) const { return seqs_.count(seq_id) > 0; }

  std::vector<int32_t> block_table(int64_t seq_id) const {
    auto it = seqs_.find(seq_id);
    if (it == seqs_.end()) throw std::runtime_error("block_table: unknown sequence");
    return it->second.blocks;
  }
  int num_seq_blocks(int64_t seq_id) const { return (int)get_c(seq_id).blocks.size(); }

  // Fill rows of a [n, width] int32 numpy block table in one call.
  void fill_block_tables(const std::vector<int64_t>& ids,
                         py::array_t<int32_t, py::array::c_style> out) {
    auto m = out.mutable_unchecked<2>();
    const int width = (int)m.shape(1);
    for (size_t i = 0; i < ids.size(); ++i) {
      const Seq& s = get_c(ids[i]);
      const int n = std::min<int>(width, (int)s.blocks.size());
      for (int j = 0; j < n; ++j) m(i, j) = s.blocks[j];
    }
  }

  // Blocks for an externally produced KV (P/D): allocate `n` fresh blocks for a
  // new sequence without any prefix reuse (the sender fills them). window > 0
  // (windowed group of a hybrid cache): only the blocks the decoder's first query
  // can reach are allocated. That query RECOMPUTES the last prompt token (position
  // num_tokens - 1, scheduler.py: num_computed = prompt_len - 1), so it attends keys
  // >= num_tokens - window, one more than a query at num_tokens would; earlier
  // entries are the null block (requires reserved >= 1).
  std::vector<int32_t> allocate_remote(int64_t seq_id, int num_tokens, uint64_t extra, int window) {
    if (seqs_.count(seq_id)) throw std::runtime_error("allocate_remote: sequence exists");
    if (window > 0 && reserved_ < 1) throw std::runtime_error("allocate_remote(window) needs a reserved null block");
    const int nb = (num_tokens + bs_ - 1) / bs_;
    const int lo = window > 0 ? std::min(nb, std::max(0, num_tokens - window) / bs_) : 0;
    if (nb - lo > num_free()) return {};
    Seq s;
    s.extra = extra;
    for (int i = 0; i < lo; ++i) s.blocks.push_back(0);
    for (int i = lo; i < nb; ++i) s.blocks.push_back(pop_free());
    s.released = lo;
    auto out = s.blocks;
    seqs_.emplace(seq_id, std::move(s));
    return out;
  }

  void reset_prefix_cache() {
    for (auto& kv : cache_) {
      Block& B = blocks_[kv.second];
      B.hash = 0;
      if (B.ref == 0 && B.in_lru) {
        lru_.erase(B.lru_it);
        B.in_lru = false;
        free_.push_back(kv.second);
      }
    }
    cache_.clear();
    for (auto& kv : seqs_) {
      kv.second.committed = 0;
      kv.second.last_hash = kRootHash;
    }
    if (events_on_) events_.push_back(Event{2, 0, 0, -1, {}});
  }

  py::list take_events() {
    py::list out;
    for (auto& e : events_) {
      out.append(py::make_tuple(e.kind, e.hash, e.parent, e.block, e.tokens));
    }
    events_.clear();
    return out;
  }

  // Blocks evicted from the cache since the last call (for the offload tier):
  // list of (block_id, hash).
  std::vector<std::pair<int32_t, uint64_t>> take_evicted() {
    auto out = std::move(evicted_);
    evicted_.clear();
    return out;
  }

  std::pair<int64_t, int64_t> prefix_stats() const { return {hits_, queries_}; }

  int64_t cached_block_for(uint64_t h) const {
    auto it = cache_.find(h);
    return it == cache_.end() ? -1 : it->second;
  }

  // Blocks reloaded from an offload tier are hashed by the request's next
  // `commit` (its committed index still points before them).
  void check_invariants() const {
    int refd = 0;
    for (size_t i = (size_t)reserved_; i < blocks_.size(); ++i)
      if (blocks_[i].ref > 0) ++refd;
    if ((size_t)(refd + free_.size() + lru_.size() + reserved_) != blocks_.size())
      throw std::runtime_error("block conservation violated");
  }

 private:
  Seq& get(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::runtime_error("unknown sequence");
    return it->second;
  }
  const Seq& get_c(int64_t id) const {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::runtime_error("unknown sequence");
    return it->second;
  }
  void take_ref(int32_t b) {
    Block& B = blocks_[b];
    if (B.ref == 0 && B.in_lru) {
      lru_.erase(B.lru_it);
      B.in_lru = false;
    }
    ++B.ref;
  }
  void drop_ref(int32_t b) {
    Block& B = blocks_[b];
    if (--B.ref > 0) return;
    if (B.hash != 0 && caching_) {
      lru_.push_back(b);
      B.lru_it = std::prev(lru_.end());
      B.in_lru = true;
    } else {
      B.hash = 0;
      free_.push_back(b);
    }
  }
  int32_t pop_free() {
    int32_t b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else {
      b = lru_.front();
      lru_.pop_front();
      Block& B = blocks_[b];
      B.in_lru = false;
      cache_.erase(B.hash);
      evicted_.emplace_back(b, B.hash);
      if (events_on_) events_.push_back(Event{1, B.hash, B.parent, b, {}});
      B.hash = 0;
    }
    blocks_[b].ref = 1;
    return b;
  }

  int bs_;
  bool caching_, events_on_;
  int reserved_ = 0;
  std::vector<Block> blocks_;
  std::vector<int32_t> free_;
  std::list<int32_t> lru_;
  std::unordered_map<uint64_t, int32_t> cache_;
  std::unordered_map<int64_t, Seq> seqs_;
  std::vector<Event> events_;
  std::vector<std::pair<int32_t, uint64_t>> evicted_;
  int64_t hits_ = 0, queries_ = 0;
};

uint64_t py_hash_block(uint64_t parent, uint64_t extra,
                       py::array_t<int32_t, py::array::c_style | py::array::forcecast> toks) {
  return hash_block(parent, extra, toks.data(), (size_t)toks.shape(0));
}

std::vector<uint64_t> py_hash_blocks(py::array_t<int32_t, py::array::c_style | py::array::forcecast> toks,
                                     int bs, uint64_t extra) {
  std::vector<uint64_t> out;
  const int n = (int)toks.shape(0);
  const int32_t* p = toks.data();
  uint64_t h = kRootHash;
  for (int b = 0; (b + 1) * bs <= n; ++b) {
    h = hash_block(h, extra, p + b * bs, bs);
    out.push_back(h);
  }
  return out;
}

}  // namespace

void register_block_manager(py::module_& m) {
  m.attr("ROOT_HASH") = py::int_(kRootHash);
  m.def("hash_block", &py_hash_block, "chained 64-bit block key");
  m.def("hash_blocks", &py_hash_blocks, py::arg("tokens"), py::arg("block_size"),
        py::arg("extra") = 0, "chained keys of every full block of a token sequence");
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool, bool, int>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("prefix_caching") = true, py::arg("emit_events") = false, py::arg("reserved") = 0)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def("num_free", &BlockManager::num_free)
      .def("num_cached", &BlockManager::num_cached)
      .def("usage", &BlockManager::usage)
      .def("lookup", &BlockManager::lookup)
      .def("acquire", &BlockManager::acquire, py::arg("seq_id"), py::arg("tokens"), py::arg("extra"),
           py::arg("max_tokens") = -1)
      .def("acquire_window", &BlockManager::acquire_window)
      .def("release_before", &BlockManager::release_before)
      .def("can_allocate", &BlockManager::can_allocate)
      .def("grow", &BlockManager::grow)
      .def("commit", &BlockManager::commit)
      .def("free", &BlockManager::free)
      .def("has_seq", &BlockManager::has_seq)
      .def("block_table", &BlockManager::block_table)
      .def("num_seq_blocks", &BlockManager::num_seq_blocks)
      .def("fill_block_tables", &BlockManager::fill_block_tables)
      .def("allocate_remote", &BlockManager::allocate_remote, py::arg("seq_id"), py::arg("num_tokens"),
           py::arg("extra"), py::arg("window") = 0)
      .def("reset_prefix_cache", &BlockManager::reset_prefix_cache)
      .def("take_events", &BlockManager::take_events)
      .def("take_evicted", &BlockManager::take_evicted)
      .def("prefix_stats", &BlockManager::prefix_stats)
      .def("cached_block_for", &BlockManager::cached_block_for)
      .def("check_invariants", &BlockManager::check_invariants);
}
