// Gradient-boosted regression trees for the latency predictor (SURVEY C20;
// reference: docs/architecture/advanced/latency-predictor.md:18-100 trains two
// XGBoost regressors, TTFT and TPOT, on a sliding window). xgboost is not
// available, so this is a compact native replacement:
//   * squared-error boosting, depth-limited trees, shrinkage;
//   * histogram split finding on per-feature quantile bins (fast retrain on a
//     few 10k samples, the sliding-window size the predictor uses);
//   * optional quantile objective (pinball loss) for p90-style predictions;
//   * flat serialisation so prediction servers load the trainer's model from a
//     shared file (the reference's training/prediction server split).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct Node {
  int feat = -1;       // -1 = leaf
  float thr = 0.f;     // go left if x[feat] <= thr
  int left = -1, right = -1;
  float value = 0.f;
};

struct Tree {
  std::vector<Node> nodes;
  float predict(const float* x) const {
    int i = 0;
    while (nodes[i].feat >= 0) i = x[nodes[i].feat] <= nodes[i].thr ? nodes[i].left : nodes[i].right;
    return nodes[i].value;
  }
};

class GBDT {
 public:
  GBDT(int n_trees, int max_depth, double lr, int min_leaf, int n_bins, double quantile)
      : n_trees_(n_trees), depth_(max_depth), lr_(lr), min_leaf_(min_leaf), n_bins_(n_bins),
        quantile_(quantile) {}

  void fit(py::array_t<float, py::array::c_style | py::array::forcecast> X,
           py::array_t<float, py::array::c_style | py::array::forcecast> y) {
    if (X.ndim() != 2 || y.ndim() != 1 || X.shape(0) != y.shape(0)) throw std::invalid_argument("shapes");
    const int n = (int)X.shape(0), f = (int)X.shape(1);
    if (n == 0) throw std::invalid_argument("empty");
    nf_ = f;
    if (n_bins_ > 255) n_bins_ = 255;
    if (n_bins_ < 2) n_bins_ = 2;
    const float* xp = X.data();
    const float* yp = y.data();
    // --- bin edges (quantiles per feature)
    edges_.assign(f, {});
    std::vector<float> col(n);
    for (int j = 0; j < f; ++j) {
      for (int i = 0; i < n; ++i) col[i] = xp[(size_t)i * f + j];
      std::sort(col.begin(), col.end());
      std::vector<float>& e = edges_[j];
      for (int b = 1; b < n_bins_; ++b) {
        float v = col[std::min(n - 1, (int)((int64_t)b * n / n_bins_))];
        if (e.empty() || v > e.back()) e.push_back(v);
      }
    }
    // --- binned matrix
    std::vector<uint8_t> bins((size_t)n * f);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < f; ++j) {
        const auto& e = edges_[j];
        bins[(size_t)i * f + j] = (uint8_t)(std::lower_bound(e.begin(), e.end(), xp[(size_t)i * f + j]) - e.begin());
      }
    // --- boosting
    if (quantile_ > 0) {
      std::vector<float> s(yp, yp + n);
      std::nth_element(s.begin(), s.begin() + (size_t)(quantile_ * (n - 1)), s.end());
      base_ = s[(size_t)(quantile_ * (n - 1))];
    } else {
      base_ = (float)(std::accumulate(yp, yp + n, 0.0) / n);
    }
    std::vector<float> pred(n, base_), grad(n);
    trees_.clear();
    std::vector<int> idx(n);
    for (int t = 0; t < n_trees_; ++t) {
      for (int i = 0; i < n; ++i) {
        const float r = yp[i] - pred[i];
        grad[i] = quantile_ > 0 ? (r > 0 ? (float)quantile_ : (float)(quantile_ - 1.0)) : r;
      }
      std::iota(idx.begin(), idx.end(), 0);
      Tree tr;
      tr.nodes.emplace_back();
      build(tr, 0, idx, 0, n, bins, grad, 0);
      if (quantile_ > 0) refit_quantile_leaves(tr, xp, yp, pred, n);
      for (int i = 0; i < n; ++i) pred[i] += (float)lr_ * tr.predict(xp + (size_t)i * f);
      trees_.push_back(std::move(tr));
    }
  }

  py::array_t<float> predict(py::array_t<float, py::array::c_style | py::array::forcecast> X) const {
    if (X.ndim() != 2 || (int)X.shape(1) != nf_) throw std::invalid_argument("feature count");
    const int n = (int)X.shape(0);
    py::array_t<float> out(n);
    float* o = out.mutable_data();
    const float* xp = X.data();
    for (int i = 0; i < n; ++i) {
      float v = base_;
      for (auto& t : trees_) v += (float)lr_ * t.predict(xp + (size_t)i * nf_);
      o[i] = v;
    }
    return out;
  }

  py::bytes serialize() const {
    std::string s;
    auto put = [&](const void* p, size_t n) { s.append((const char*)p, n); };
    const uint32_t magic = 0x47424454;  // "GBDT"
    put(&magic, 4);
    put(&nf_, 4);
    put(&base_, 4);
    put(&lr_, 8);
    const uint32_t nt = (uint32_t)trees_.size();
    put(&nt, 4);
    for (auto& t : trees_) {
      const uint32_t nn = (uint32_t)t.nodes.size();
      put(&nn, 4);
      put(t.nodes.data(), nn * sizeof(Node));
    }
    return py::bytes(s);
  }

  void deserialize(const std::string& s) {
    size_t off = 0;
    auto get = [&](void* p, size_t n) {
      if (off + n > s.size()) throw std::runtime_error("truncated model");
      std::memcpy(p, s.data() + off, n);
      off += n;
    };
    uint32_t magic;
    get(&magic, 4);
    if (magic != 0x47424454) throw std::runtime_error("bad model magic");
    get(&nf_, 4);
    get(&base_, 4);
    get(&lr_, 8);
    uint32_t nt;
    get(&nt, 4);
    trees_.assign(nt, {});
    for (auto& t : trees_) {
      uint32_t nn;
      get(&nn, 4);
      t.nodes.resize(nn);
      get(t.nodes.data(), nn * sizeof(Node));
    }
  }

  int num_trees() const { return (int)trees_.size(); }
  int num_features() const { return nf_; }

 private:
  void build(Tree& tr, int node, std::vector<int>& idx, int lo, int hi, const std::vector<uint8_t>& bins,
             const std::vector<float>& g, int depth) {
    const int n = hi - lo;
    double sum = 0;
    for (int i = lo; i < hi; ++i) sum += g[idx[i]];
    tr.nodes[node].value = (float)(sum / std::max(1, n));
    if (depth >= depth_ || n < 2 * min_leaf_) return;
    // histogram per feature
    int best_f = -1, best_b = -1;
    double best_gain = 1e-12;
    const double parent = sum * sum / n;
    std::vector<double> hs(n_bins_ + 1);
    std::vector<int> hc(n_bins_ + 1);
    for (int j = 0; j < nf_; ++j) {
      const int nb = (int)edges_[j].size() + 1;
      std::fill(hs.begin(), hs.begin() + nb, 0.0);
      std::fill(hc.begin(), hc.begin() + nb, 0);
      for (int i = lo; i < hi; ++i) {
        const int b = bins[(size_t)idx[i] * nf_ + j];
        hs[b] += g[idx[i]];
        hc[b] += 1;
      }
      double ls = 0;
      int lc = 0;
      for (int b = 0; b < nb - 1; ++b) {
        ls += hs[b];
        lc += hc[b];
        const int rc = n - lc;
        if (lc < min_leaf_ || rc < min_leaf_) continue;
        const double rs = sum - ls;
        const double gain = ls * ls / lc + rs * rs / rc - parent;
        if (gain > best_gain) {
          best_gain = gain;
          best_f = j;
          best_b = b;
        }
      }
    }
    if (best_f < 0) return;
    auto mid = std::partition(idx.begin() + lo, idx.begin() + hi,
                              [&](int i) { return bins[(size_t)i * nf_ + best_f] <= best_b; });
    const int m = (int)(mid - idx.begin());
    Node& nd = tr.nodes[node];
    nd.feat = best_f;
    nd.thr = edges_[best_f][best_b];
    const int l = (int)tr.nodes.size();
    tr.nodes.emplace_back();
    const int r = (int)tr.nodes.size();
    tr.nodes.emplace_back();
    tr.nodes[node].left = l;
    tr.nodes[node].right = r;
    build(tr, l, idx, lo, m, bins, g, depth + 1);
    build(tr, r, idx, m, hi, bins, g, depth + 1);
  }

  // For the pinball loss the optimal leaf value is the q-quantile of the
  // residuals that reach the leaf (gradient step only gives the sign).
  void refit_quantile_leaves(Tree& tr, const float* xp, const float* yp, const std::vector<float>& pred, int n) {
    std::vector<std::vector<float>> res(tr.nodes.size());
    for (int i = 0; i < n; ++i) {
      int k = 0;
      const float* x = xp + (size_t)i * nf_;
      while (tr.nodes[k].feat >= 0) k = x[tr.nodes[k].feat] <= tr.nodes[k].thr ? tr.nodes[k].left : tr.nodes[k].right;
      res[k].push_back(yp[i] - pred[i]);
    }
    for (size_t k = 0; k < tr.nodes.size(); ++k) {
      if (tr.nodes[k].feat >= 0 || res[k].empty()) continue;
      auto& r = res[k];
      const size_t q = (size_t)(quantile_ * (r.size() - 1));
      std::nth_element(r.begin(), r.begin() + q, r.end());
      tr.nodes[k].value = r[q];
    }
  }

  int n_trees_, depth_;
  double lr_;
  int min_leaf_, n_bins_;
  double quantile_;
  int nf_ = 0;
  float base_ = 0.f;
  std::vector<std::vector<float>> edges_;
  std::vector<Tree> trees_;
};

}  // namespace

void register_gbdt(py::module_& m) {
  py::class_<GBDT>(m, "GBDT")
      .def(py::init<int, int, double, int, int, double>(), py::arg("n_trees") = 100,
           py::arg("max_depth") = 6, py::arg("learning_rate") = 0.1, py::arg("min_samples_leaf") = 5,
           py::arg("n_bins") = 64, py::arg("quantile") = 0.0)
      .def("fit", &GBDT::fit)
      .def("predict", &GBDT::predict)
      .def("serialize", &GBDT::serialize)
      .def("deserialize", [](GBDT& g, py::bytes b) { g.deserialize(std::string(b)); })
      .def_property_readonly("num_trees", &GBDT::num_trees)
      .def_property_readonly("num_features", &GBDT::num_features);
}
