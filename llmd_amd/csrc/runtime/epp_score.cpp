// EPP scoring hot path: the weighted sum of a profile's scorer
// columns and the picker, in one native call per profile run. The reference's EPP
// runs its scheduler in Go; in this EPP the per-endpoint x per-scorer accumulation
// and the max-score sort were ~40 % of a decision's Python time at 32 endpoints
// (profiles/epp_decision_r6.txt). Scorer semantics stay in the (pluggable) Python
// scorers, which now hand over one list per scorer aligned with the candidates.
//
//   combine_pick(cols, weights, n_pick, picker, seed) -> (totals, picked indices)
//     value v of a column contributes w * clamp(v, 0, 1) (NaN / None-as-0 -> 0)
//     picker 0 = max-score (uniform random tie-break, the reference's max-score-picker),
//            1 = weighted random without replacement (lottery), 2 = uniform random
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <cstdint>
#include <vector>

namespace py = pybind11;

namespace {

struct Rng {  // splitmix64: seeded per call from Python's random, so runs stay reproducible
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

py::tuple combine_pick(const std::vector<std::vector<double>>& cols, const std::vector<double>& w, int n_pick,
                       int picker, uint64_t seed) {
  const size_t n = cols.empty() ? 0 : cols[0].size();
  std::vector<double> tot(n, 0.0);
  for (size_t c = 0; c < cols.size(); ++c) {
    if (cols[c].size() != n) throw std::invalid_argument("combine_pick: ragged columns");
    const double wc = c < w.size() ? w[c] : 1.0;
    const double* v = cols[c].data();
    for (size_t i = 0; i < n; ++i) {
      double x = v[i];
      if (!(x > 0.0)) continue;  // <= 0 and NaN
      tot[i] += wc * (x > 1.0 ? 1.0 : x);
    }
  }
  Rng rng{seed};
  std::vector<int> picked;
  const int want = n_pick < 0 ? 0 : std::min<int>(n_pick, (int)n);
  std::vector<char> used(n, 0);
  for (int k = 0; k < want; ++k) {
    int pick = -1;
    if (picker == 0) {  // max score, reservoir tie-break over the equal maxima
      double best = -INFINITY;
      int ties = 0;
      for (size_t i = 0; i < n; ++i) {
        if (used[i]) continue;
        if (tot[i] > best) {
          best = tot[i];
          pick = (int)i;
          ties = 1;
        } else if (tot[i] == best) {
          ++ties;
          if (rng.uniform() * ties < 1.0) pick = (int)i;
        }
      }
    } else if (picker == 1) {  // lottery: probability proportional to score
      double sum = 0.0;
      int left = 0;
      for (size_t i = 0; i < n; ++i)
        if (!used[i]) {
          sum += tot[i] > 0.0 ? tot[i] : 0.0;
          ++left;
        }
      if (sum <= 0.0) {
        int r = (int)(rng.uniform() * left);
        for (size_t i = 0; i < n; ++i)
          if (!used[i] && r-- == 0) {
            pick = (int)i;
            break;
          }
      } else {
        const double r = rng.uniform() * sum;
        double acc = 0.0;
        for (size_t i = 0; i < n; ++i) {
          if (used[i]) continue;
          pick = (int)i;
          acc += tot[i] > 0.0 ? tot[i] : 0.0;
          if (r <= acc) break;
        }
      }
    } else {  // uniform
      int left = 0;
      for (size_t i = 0; i < n; ++i) left += !used[i];
      int r = (int)(rng.uniform() * left);
      for (size_t i = 0; i < n; ++i)
        if (!used[i] && r-- == 0) {
          pick = (int)i;
          break;
        }
    }
    if (pick < 0) break;
    used[pick] = 1;
    picked.push_back(pick);
  }
  return py::make_tuple(tot, picked);
}

}  // namespace

void register_epp_score(py::module_& m) {
  m.def("combine_pick", &combine_pick, py::arg("cols"), py::arg("weights"), py::arg("n_pick"), py::arg("picker"),
        py::arg("seed"),
        "weighted sum of clamped scorer columns + max-score / weighted-random / random pick (EPP hot path)");
}
