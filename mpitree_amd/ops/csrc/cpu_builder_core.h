// Exact depth-first host tree builder (no Python dependency).
//
// Shared by the ``mpitree_amd._cpu`` extension (cpu_builder.cpp) and the
// host-sanitizer harness (tests/native/asan_driver.cpp, built with
// -fsanitize=address,undefined by tests/test_sanitizers.py). Reference
// semantics: mpitree/tree/decision_tree.py:93-166 (stopping rules, split
// search, recursion), with the integer-form criterion of criterion.h so the
// host and gfx950 builders produce identical trees.
#pragma once

#include <algorithm>
#include <cstdint>
#include <limits>
#include <vector>

#include "criterion.h"

#ifdef _OPENMP
#include <omp.h>
#endif

namespace mt {
namespace host {

inline int thread_id() {
#ifdef _OPENMP
  return omp_get_thread_num();
#else
  return 0;
#endif
}

struct Params {
  int crit;
  int max_depth;  // -1 = none
  int64_t mss;
  int64_t msl;
  int C;          // classes (classification); 2 for regression stats
  bool reg;
};

template <typename CodeT>
struct Builder {
  const CodeT* codes;
  int64_t n, F;
  const int32_t* ylab;   // classification labels 0..C-1
  const int64_t* yfix;   // regression fixed-point targets
  const int32_t* nbins;
  Params p;
  std::vector<int32_t> idx, tmp;
  // outputs
  std::vector<int32_t> feat, bin, depth;
  std::vector<int64_t> left, right, nsamp;
  std::vector<int64_t> stats;  // [N][C] counts or [N][2] (count, sum)

  int64_t add_node(int d, int64_t m, const int64_t* st) {
    const int64_t id = (int64_t)feat.size();
    feat.push_back(-1);
    bin.push_back(-1);
    depth.push_back(d);
    left.push_back(-1);
    right.push_back(-1);
    nsamp.push_back(m);
    const int S = p.reg ? 2 : p.C;
    for (int c = 0; c < S; ++c) stats.push_back(st[c]);
    return id;
  }

  double term_cls(const int64_t* cnt, const int32_t* present, int np, int64_t m) const {
    if (p.crit == mt::kEntropy) {
      double acc = 0.0;
      for (int i = 0; i < np; ++i) acc = acc + mt::xlog2x((uint64_t)cnt[i]);
      return mt::xlog2x((uint64_t)m) - acc;
    }
    int64_t sq = 0;
    for (int i = 0; i < np; ++i) sq += cnt[i] * cnt[i];
    return mt::gini_term(m, sq);
  }

  struct Best {
    double gain = -std::numeric_limits<double>::infinity();
    int f = -1, b = -1;
  };

  // Best split of one feature over rows [s, s+m).
  void scan_feature_cls(int f, int64_t s, int64_t m, const std::vector<int32_t>& present,
                        const std::vector<int32_t>& cls_pos, const std::vector<int64_t>& tot,
                        double pterm, Best& best, std::vector<int64_t>& work,
                        std::vector<uint64_t>& pairs) const {
    const int np = (int)present.size();
    const int nb = nbins[f];
    std::vector<int64_t> L(np, 0), R(np);
    double best_cost = std::numeric_limits<double>::infinity();
    int best_b = -1;
    const double tu = tie_unit(xlog2x((uint64_t)m), m);  // canonical ties (criterion.h)
    const double tinv = 1.0 / tu;
    auto eval = [&](int b, int64_t ml) {
      const int64_t mr = m - ml;
      if (ml < p.msl || mr < p.msl || ml <= 0 || mr <= 0) return;
      for (int i = 0; i < np; ++i) R[i] = tot[i] - L[i];
      const double cost = tie_round(term_cls(L.data(), present.data(), np, ml) +
                                        term_cls(R.data(), present.data(), np, mr),
                                    tinv, tu);
      if (cost < best_cost) {
        best_cost = cost;
        best_b = b;
      }
    };
    if ((int64_t)nb * np <= 4 * m) {
      // dense per-bin class counts
      work.assign((size_t)nb * np, 0);
      for (int64_t r = 0; r < m; ++r) {
        const int32_t row = idx[s + r];
        work[(size_t)codes[row * F + f] * np + cls_pos[ylab[row]]]++;
      }
      int64_t ml = 0;
      for (int b = 0; b < nb; ++b) {
        int64_t any = 0;
        for (int i = 0; i < np; ++i) {
          const int64_t v = work[(size_t)b * np + i];
          L[i] += v;
          ml += v;
          any |= v;
        }
        if (any) eval(b, ml);
      }
    } else {
      pairs.resize(m);
      for (int64_t r = 0; r < m; ++r) {
        const int32_t row = idx[s + r];
        pairs[r] = ((uint64_t)codes[row * F + f] << 32) | (uint32_t)cls_pos[ylab[row]];
      }
      std::sort(pairs.begin(), pairs.end());
      int64_t ml = 0;
      for (int64_t r = 0; r < m;) {
        const uint32_t code = (uint32_t)(pairs[r] >> 32);
        while (r < m && (uint32_t)(pairs[r] >> 32) == code) {
          L[(uint32_t)pairs[r]]++;
          ++ml;
          ++r;
        }
        eval((int)code, ml);
      }
    }
    if (best_b >= 0) {
      const double g = pterm - best_cost;
      if (g > best.gain) {  // features visited in order: strict > keeps the lowest
        best.gain = g;
        best.f = f;
        best.b = best_b;
      }
    }
  }

  void scan_feature_reg(int f, int64_t s, int64_t m, int64_t S, double pterm, Best& best,
                        std::vector<int64_t>& work, std::vector<uint64_t>& pairs) const {
    const int nb = nbins[f];
    double best_cost = std::numeric_limits<double>::infinity();
    int best_b = -1;
    auto eval = [&](int b, int64_t ml, int64_t sl) {
      const int64_t mr = m - ml;
      if (ml < p.msl || mr < p.msl || ml <= 0 || mr <= 0) return;
      const double cost = mt::mse_term(ml, sl) + mt::mse_term(mr, S - sl);
      if (cost < best_cost) {
        best_cost = cost;
        best_b = b;
      }
    };
    if (nb <= 4 * m) {
      work.assign((size_t)nb * 2, 0);
      for (int64_t r = 0; r < m; ++r) {
        const int32_t row = idx[s + r];
        const int c = codes[row * F + f];
        work[2 * c] += 1;
        work[2 * c + 1] += yfix[row];
      }
      int64_t ml = 0, sl = 0;
      for (int b = 0; b < nb; ++b) {
        if (!work[2 * b]) continue;
        ml += work[2 * b];
        sl += work[2 * b + 1];
        eval(b, ml, sl);
      }
    } else {
      pairs.resize(m);
      for (int64_t r = 0; r < m; ++r) {
        const int32_t row = idx[s + r];
        pairs[r] = ((uint64_t)codes[row * F + f] << 32) | (uint32_t)r;
      }
      std::sort(pairs.begin(), pairs.end());
      int64_t ml = 0, sl = 0;
      for (int64_t r = 0; r < m;) {
        const uint32_t code = (uint32_t)(pairs[r] >> 32);
        while (r < m && (uint32_t)(pairs[r] >> 32) == code) {
          ml += 1;
          sl += yfix[idx[s + (uint32_t)pairs[r]]];
          ++r;
        }
        eval((int)code, ml, sl);
      }
    }
    if (best_b >= 0) {
      const double g = pterm - best_cost;
      if (g > best.gain) {
        best.gain = g;
        best.f = f;
        best.b = best_b;
      }
    }
  }

  void run(int n_threads) {
    idx.resize(n);
    tmp.resize(n);
    for (int64_t i = 0; i < n; ++i) idx[i] = (int32_t)i;
    struct Item {
      int64_t s, m, parent;
      int side, d;
    };
    std::vector<Item> stack;
    stack.push_back({0, n, -1, 0, 0});
    const int Cs = p.reg ? 2 : p.C;
    std::vector<int64_t> st(Cs), cntbuf(p.reg ? 0 : p.C);
    std::vector<int32_t> present, cls_pos(p.reg ? 0 : p.C, -1);
    std::vector<int64_t> tot;
    std::vector<std::vector<int64_t>> works(n_threads);
    std::vector<std::vector<uint64_t>> pairss(n_threads);
    while (!stack.empty()) {
      Item it = stack.back();
      stack.pop_back();
      const int64_t s = it.s, m = it.m;
      bool pure;
      int64_t S = 0;
      if (p.reg) {
        int64_t mn = std::numeric_limits<int64_t>::max(), mx = std::numeric_limits<int64_t>::min();
        for (int64_t r = 0; r < m; ++r) {
          const int64_t v = yfix[idx[s + r]];
          S += v;
          mn = std::min(mn, v);
          mx = std::max(mx, v);
        }
        st[0] = m;
        st[1] = S;
        pure = m == 0 || mn == mx;
      } else {
        std::fill(cntbuf.begin(), cntbuf.end(), 0);
        for (int64_t r = 0; r < m; ++r) cntbuf[ylab[idx[s + r]]]++;
        present.clear();
        for (int c = 0; c < p.C; ++c) {
          st[c] = cntbuf[c];
          if (cntbuf[c]) present.push_back(c);
        }
        pure = present.size() <= 1;
      }
      const int64_t id = add_node(it.d, m, st.data());
      if (it.parent >= 0) (it.side == 0 ? left : right)[it.parent] = id;
      if (pure || (p.max_depth >= 0 && it.d >= p.max_depth) || m < p.mss || m < 2 * p.msl)
        continue;
      Best best;
      double pterm;
      if (p.reg) {
        pterm = mt::mse_term(m, S);
      } else {
        tot.assign(present.size(), 0);
        for (size_t i = 0; i < present.size(); ++i) {
          cls_pos[present[i]] = (int32_t)i;
          tot[i] = cntbuf[present[i]];
        }
        pterm = term_cls(tot.data(), present.data(), (int)present.size(), m);
      }
      const bool par = n_threads > 1 && m * F >= 65536;
      if (par) {
        std::vector<Best> bests(F);
#pragma omp parallel for num_threads(n_threads) schedule(dynamic)
        for (int64_t f = 0; f < F; ++f) {
          Best b;
          const int t = thread_id();
          if (p.reg)
            scan_feature_reg((int)f, s, m, S, pterm, b, works[t], pairss[t]);
          else
            scan_feature_cls((int)f, s, m, present, cls_pos, tot, pterm, b, works[t], pairss[t]);
          bests[f] = b;
        }
        for (int64_t f = 0; f < F; ++f)
          if (bests[f].f >= 0 && bests[f].gain > best.gain) best = bests[f];
      } else {
        for (int64_t f = 0; f < F; ++f) {
          if (p.reg)
            scan_feature_reg((int)f, s, m, S, pterm, best, works[0], pairss[0]);
          else
            scan_feature_cls((int)f, s, m, present, cls_pos, tot, pterm, best, works[0],
                             pairss[0]);
        }
      }
      if (best.f < 0) continue;
      feat[id] = best.f;
      bin[id] = best.b;
      // stable partition of the segment
      int64_t nl = 0;
      for (int64_t r = 0; r < m; ++r)
        if ((int)codes[(int64_t)idx[s + r] * F + best.f] <= best.b) tmp[nl++] = idx[s + r];
      int64_t k = nl;
      for (int64_t r = 0; r < m; ++r)
        if ((int)codes[(int64_t)idx[s + r] * F + best.f] > best.b) tmp[k++] = idx[s + r];
      std::copy(tmp.begin(), tmp.begin() + m, idx.begin() + s);
      stack.push_back({s + nl, m - nl, id, 1, it.d + 1});
      stack.push_back({s, nl, id, 0, it.d + 1});
    }
  }
};

}  // namespace host
}  // namespace mt
