// Native host side of mpitree_amd (module ``mpitree_amd._cpu``, built with g++).
//
// * build_tree: exact depth-first tree builder for CPU fits (the reference's
//   own execution model: mpitree/tree/decision_tree.py:93-166), sharing the
//   integer-form criterion of criterion.h with the gfx950 kernels so both
//   produce identical trees. Per node and feature it scans the node's
//   distinct codes in ascending order (dense per-bin counts when the node is
//   large relative to the bin count, a sort of (code, class) pairs
//   otherwise), so cost is O(m log m + distinct_codes * present_classes) --
//   the reference's O(F^2 m^2) masking loop is gone while the candidate set,
//   tie-breaking and stopping rules are the same.
// * preorder / node_terms: vectorised helpers for tree assembly.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <limits>
#include <vector>

#include "cpu_builder_core.h"
#include "criterion.h"

namespace py = pybind11;
using mt::Criterion;

namespace {

using mt::host::Builder;
using mt::host::Params;

template <typename CodeT>
py::dict build_impl(py::array codes_a, py::array y_a, py::array_t<int32_t> nbins_a, int C,
                    int crit, int max_depth, int64_t mss, int64_t msl, int n_threads) {
  auto codes = codes_a.cast<py::array_t<CodeT, py::array::c_style | py::array::forcecast>>();
  Builder<CodeT> b;
  b.codes = codes.data();
  b.n = codes.shape(0);
  b.F = codes.shape(1);
  b.p = Params{crit, max_depth, mss, std::max<int64_t>(1, msl), C, crit == mt::kSquaredError};
  py::array_t<int32_t, py::array::c_style | py::array::forcecast> ylab;
  py::array_t<int64_t, py::array::c_style | py::array::forcecast> yfix;
  if (b.p.reg) {
    yfix = y_a.cast<decltype(yfix)>();
    b.yfix = yfix.data();
    b.ylab = nullptr;
  } else {
    ylab = y_a.cast<decltype(ylab)>();
    b.ylab = ylab.data();
    b.yfix = nullptr;
  }
  auto nb = nbins_a.cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
  b.nbins = nb.data();
  {
    py::gil_scoped_release rel;
    b.run(std::max(1, n_threads));
  }
  const int64_t N = (int64_t)b.feat.size();
  const int S = b.p.reg ? 2 : C;
  py::array_t<int32_t> feat(N), bin(N), depth(N);
  py::array_t<int64_t> left(N), right(N), nsamp(N);
  py::array_t<int64_t> stats({N, (int64_t)S});
  std::copy(b.feat.begin(), b.feat.end(), feat.mutable_data());
  std::copy(b.bin.begin(), b.bin.end(), bin.mutable_data());
  std::copy(b.depth.begin(), b.depth.end(), depth.mutable_data());
  std::copy(b.left.begin(), b.left.end(), left.mutable_data());
  std::copy(b.right.begin(), b.right.end(), right.mutable_data());
  std::copy(b.nsamp.begin(), b.nsamp.end(), nsamp.mutable_data());
  std::copy(b.stats.begin(), b.stats.end(), stats.mutable_data());
  py::dict out;
  out["feature"] = feat;
  out["bin"] = bin;
  out["depth"] = depth;
  out["left"] = left;
  out["right"] = right;
  out["nsamp"] = nsamp;
  out["stats"] = stats;
  return out;
}

py::dict build_tree(py::array codes, py::array y, py::array_t<int32_t> nbins, int C, int crit,
                    int max_depth, int64_t mss, int64_t msl, int n_threads) {
  if (codes.ndim() != 2) throw std::invalid_argument("codes must be 2-D");
  if (py::isinstance<py::array_t<uint8_t>>(codes))
    return build_impl<uint8_t>(codes, y, nbins, C, crit, max_depth, mss, msl, n_threads);
  if (py::isinstance<py::array_t<uint32_t>>(codes))  // exact mode, > 65536 unique values
    return build_impl<uint32_t>(codes, y, nbins, C, crit, max_depth, mss, msl, n_threads);
  return build_impl<uint16_t>(codes, y, nbins, C, crit, max_depth, mss, msl, n_threads);
}

// Pre-order renumbering of an arbitrary node table (root `root`).
py::tuple preorder(py::array_t<int32_t, py::array::c_style | py::array::forcecast> feature,
                   py::array_t<int64_t, py::array::c_style | py::array::forcecast> left,
                   py::array_t<int64_t, py::array::c_style | py::array::forcecast> right,
                   int64_t root) {
  const int64_t n = feature.shape(0);
  const int32_t* f = feature.data();
  const int64_t* l = left.data();
  const int64_t* r = right.data();
  std::vector<int64_t> order;
  std::vector<int32_t> dep(n, 0);
  order.reserve(n);
  std::vector<int64_t> stack{root};
  while (!stack.empty()) {
    const int64_t i = stack.back();
    stack.pop_back();
    order.push_back(i);
    if (f[i] >= 0) {
      dep[l[i]] = dep[i] + 1;
      dep[r[i]] = dep[i] + 1;
      stack.push_back(r[i]);
      stack.push_back(l[i]);
    }
  }
  py::array_t<int64_t> o((int64_t)order.size());
  std::copy(order.begin(), order.end(), o.mutable_data());
  py::array_t<int32_t> d(n);
  std::copy(dep.begin(), dep.end(), d.mutable_data());
  return py::make_tuple(o, d);
}

// x*log2(x) for small counts (same function, same bits as the kernels).
const std::vector<double>& xlog_table() {
  static const std::vector<double> tab = [] {
    std::vector<double> t(1 << 16);
    for (size_t x = 0; x < t.size(); ++x) t[x] = mt::xlog2x(x);
    return t;
  }();
  return tab;
}

inline double tabled_xlog(const std::vector<double>& tab, int64_t x) {
  return x < (int64_t)tab.size() ? tab[x] : mt::xlog2x((uint64_t)x);
}

// Node term of one node: c = C class counts, or (count, fixed-point sum).
inline double node_term(const int64_t* c, int64_t C, int crit, const std::vector<double>& tab) {
  if (crit == mt::kSquaredError) return mt::mse_term(c[0], c[1]);
  if (crit == mt::kEntropy) {
    double acc = 0.0;
    int64_t m = 0;
    for (int64_t k = 0; k < C; ++k) {
      acc = acc + tabled_xlog(tab, c[k]);
      m += c[k];
    }
    return tabled_xlog(tab, m) - acc;
  }
  int64_t m = 0, sq = 0;
  for (int64_t k = 0; k < C; ++k) {
    m += c[k];
    sq += c[k] * c[k];
  }
  return mt::gini_term(m, sq);
}

// Pre-order re-numbering + column emission shared by both assembly entry
// points. f/b/l/r: split feature, bin and child ids of N nodes; ns(i) and
// st(i, c) read a node's row count and statistics. Optional outputs: split
// thresholds from a padded [F, EB] edge table, node terms for ``crit``.
template <typename NsFn, typename StFn>
py::dict assemble_core(int64_t n, const int32_t* f, const int32_t* b, const int64_t* l,
                       const int64_t* r, NsFn ns, StFn st, int64_t C, int64_t root,
                       const double* ed, int64_t EB, int crit, int n_threads) {
  using clk = std::chrono::steady_clock;
  const auto t_begin = clk::now();
  auto ms = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  const bool want_thr = ed != nullptr;
  const bool want_term = crit >= 0;
  const std::vector<double>& tab = xlog_table();
  std::vector<int64_t> new_id(n, -1);
  std::vector<int32_t> depv(n, 0);
  int64_t k = 0;
  // Every builder creates children after their parent (child id > parent id),
  // so subtree sizes come from one backward sweep and pre-order positions from
  // one forward sweep: sequential reads, scattered writes, no DFS stack.
  bool topo = root == 0;
  for (int64_t i = 0; i < n && topo; ++i)
    if (f[i] >= 0 && (l[i] <= i || r[i] <= i || l[i] >= n || r[i] >= n)) topo = false;
  if (topo) {
    std::vector<int64_t> size(n, 1);
    for (int64_t i = n - 1; i >= 0; --i)
      if (f[i] >= 0) size[i] = 1 + size[l[i]] + size[r[i]];
    k = n ? size[0] : 0;
    if (n) new_id[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (new_id[i] < 0 || f[i] < 0) continue;
      new_id[l[i]] = new_id[i] + 1;
      new_id[r[i]] = new_id[i] + 1 + size[l[i]];
      depv[l[i]] = depv[i] + 1;
      depv[r[i]] = depv[i] + 1;
    }
  } else {  // general tables: explicit DFS
    std::vector<int64_t> stack{root};
    while (!stack.empty()) {
      const int64_t i = stack.back();
      stack.pop_back();
      new_id[i] = k++;
      if (f[i] >= 0) {
        depv[l[i]] = depv[i] + 1;
        depv[r[i]] = depv[i] + 1;
        stack.push_back(r[i]);
        stack.push_back(l[i]);
      }
    }
  }
  const auto t_order = clk::now();
  py::array_t<int32_t> of(k), ob(k), od(k), ol(k), orr(k);
  py::array_t<int64_t> on(k), oo(k);
  py::array_t<int64_t> os({k, C});
  py::array_t<double> othr(want_thr ? k : 0), oterm(want_term ? k : 0);
  int32_t *pf = of.mutable_data(), *pb = ob.mutable_data(), *pd = od.mutable_data();
  int32_t *pl = ol.mutable_data(), *pr = orr.mutable_data();
  int64_t *pn = on.mutable_data(), *po = oo.mutable_data(), *ps = os.mutable_data();
  double* pt = want_thr ? othr.mutable_data() : nullptr;
  double* pm = want_term ? oterm.mutable_data() : nullptr;
  const double nan = std::numeric_limits<double>::quiet_NaN();
  // scatter node i to its pre-order slot (independent per node)
#pragma omp parallel for num_threads(n_threads) schedule(static) if (n > 32768)
  for (int64_t i = 0; i < n; ++i) {
    const int64_t j = new_id[i];
    if (j < 0) continue;
    po[j] = i;
    pf[j] = f[i];
    pd[j] = depv[i];
    pn[j] = ns(i);
    int64_t cs[64];
    const int64_t cc = C < 64 ? C : 64;
    for (int64_t c = 0; c < C; ++c) {
      const int64_t v = st(i, c);
      ps[j * C + c] = v;
      if (c < cc) cs[c] = v;
    }
    if (want_term) {
      if (C <= 64) {
        pm[j] = node_term(cs, C, crit, tab);
      } else {
        std::vector<int64_t> tmp(C);
        for (int64_t c = 0; c < C; ++c) tmp[c] = st(i, c);
        pm[j] = node_term(tmp.data(), C, crit, tab);
      }
    }
    if (f[i] >= 0) {
      pb[j] = b[i];
      pl[j] = (int32_t)new_id[l[i]];
      pr[j] = (int32_t)new_id[r[i]];
      if (want_thr) pt[j] = ed[(int64_t)f[i] * EB + b[i]];
    } else {
      pb[j] = -1;
      pl[j] = -1;
      pr[j] = -1;
      if (want_thr) pt[j] = nan;
    }
  }
  const auto t_end = clk::now();
  py::dict out;
  out["order"] = oo;
  out["feature"] = of;
  out["bin"] = ob;
  out["left"] = ol;
  out["right"] = orr;
  out["depth"] = od;
  out["nsamp"] = on;
  out["stats"] = os;
  if (want_thr) out["threshold"] = othr;
  if (want_term) out["term"] = oterm;
  out["ms_order"] = ms(t_begin, t_order);
  out["ms_scatter"] = ms(t_order, t_end);
  return out;
}

using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
using F64 = py::array_t<double, py::array::c_style | py::array::forcecast>;

// Re-number one node table into pre-order (see assemble_core).
py::dict assemble(I32 feature, I32 tbin, I64 left, I64 right, I64 nsamp, I64 stats, int64_t root,
                  F64 edges, int crit, int n_threads) {
  const int64_t n = feature.shape(0);
  const int64_t C = stats.ndim() == 2 ? stats.shape(1) : 1;
  const int64_t* ns = nsamp.data();
  const int64_t* st = stats.data();
  const bool thr = edges.ndim() == 2 && edges.size() > 0;
  return assemble_core(
      n, feature.data(), tbin.data(), left.data(), right.data(),
      [&](int64_t i) { return ns[i]; }, [&](int64_t i, int64_t c) { return st[i * C + c]; }, C,
      root, thr ? edges.data() : nullptr, thr ? edges.shape(1) : 0, crit, n_threads);
}

// Tree assembly after a level-wise fit whose deferred nodes were grown by the
// subtree finisher: the level table (n1 nodes) plus the finisher's compact node
// table ``fin`` ([T, 6] = feature, bin, left, right, depth, n; links index
// ``fin``) with class statistics ``fin_stats`` [T, C]. Deferred node did[j]
// continues as finisher root roots[j] (the root's own row becomes unreachable).
// One pass builds the joined table and renumbers it (no Python-side splice).
py::dict assemble_tree(I32 feature, I32 tbin, I64 left, I64 right, I64 nsamp, I64 stats, I32 fin,
                       I64 fin_stats, I64 did, I64 roots, F64 edges, int crit, int n_threads) {
  const int64_t n1 = feature.shape(0);
  const int64_t C = stats.ndim() == 2 ? stats.shape(1) : 1;
  const int64_t T = fin.ndim() == 2 ? fin.shape(0) : 0;
  if (T && fin.shape(1) != 6) throw std::invalid_argument("fin must be [T, 6]");
  if (T && (fin_stats.ndim() != 2 || fin_stats.shape(0) != T || fin_stats.shape(1) != C))
    throw std::invalid_argument("fin_stats must be [T, C]");
  const int64_t J = did.size();
  if (roots.size() != J) throw std::invalid_argument("did/roots length mismatch");
  const int64_t n = n1 + T;
  std::vector<int32_t> f(n), b(n);
  std::vector<int64_t> l(n), r(n);
  std::copy(feature.data(), feature.data() + n1, f.begin());
  std::copy(tbin.data(), tbin.data() + n1, b.begin());
  std::copy(left.data(), left.data() + n1, l.begin());
  std::copy(right.data(), right.data() + n1, r.begin());
  const int32_t* fi = T ? fin.data() : nullptr;
  for (int64_t t = 0; t < T; ++t) {
    const int32_t* R = fi + t * 6;
    f[n1 + t] = R[0];
    b[n1 + t] = R[1];
    l[n1 + t] = R[0] >= 0 ? n1 + R[2] : -1;
    r[n1 + t] = R[0] >= 0 ? n1 + R[3] : -1;
  }
  const int64_t* dp = did.data();
  const int64_t* rp = roots.data();
  for (int64_t j = 0; j < J; ++j) {
    const int64_t d = dp[j], rt = n1 + rp[j];
    if (d < 0 || d >= n1 || rt < n1 || rt >= n) throw std::out_of_range("bad deferred link");
    if (f[rt] < 0) continue;
    f[d] = f[rt];
    b[d] = b[rt];
    l[d] = l[rt];
    r[d] = r[rt];
  }
  const int64_t* ns = nsamp.data();
  const int64_t* st = stats.data();
  const int64_t* fs = T ? fin_stats.data() : nullptr;
  const bool thr = edges.ndim() == 2 && edges.size() > 0;
  return assemble_core(
      n, f.data(), b.data(), l.data(), r.data(),
      [&](int64_t i) { return i < n1 ? ns[i] : (int64_t)fi[(i - n1) * 6 + 5]; },
      [&](int64_t i, int64_t c) {
        return i < n1 ? st[i * C + c] : fs[(i - n1) * C + c];
      },
      C, 0, thr ? edges.data() : nullptr, thr ? edges.shape(1) : 0, crit, n_threads);
}

// Node terms for every node: stats [N, C] class counts, or [N, 2] (count, sum).
py::array_t<double> node_terms(py::array_t<int64_t, py::array::c_style | py::array::forcecast> st,
                               int crit) {
  const int64_t N = st.shape(0), C = st.shape(1);
  const int64_t* s = st.data();
  py::array_t<double> out(N);
  double* o = out.mutable_data();
  const std::vector<double>& tab = xlog_table();
  for (int64_t i = 0; i < N; ++i) o[i] = node_term(s + i * C, C, crit, tab);
  return out;
}

py::array_t<double> xlog2x_np(py::array_t<int64_t, py::array::c_style | py::array::forcecast> x) {
  py::array_t<double> out(x.size());
  for (py::ssize_t i = 0; i < x.size(); ++i) out.mutable_data()[i] = mt::xlog2x((uint64_t)x.data()[i]);
  return out;
}

}  // namespace

PYBIND11_MODULE(_cpu, m) {
  m.doc() = "mpitree_amd native host builder and tree helpers";
  m.def("build_tree", &build_tree);
  m.def("preorder", &preorder);
  m.def("assemble", &assemble, py::arg("feature"), py::arg("tbin"), py::arg("left"),
        py::arg("right"), py::arg("nsamp"), py::arg("stats"), py::arg("root") = 0,
        py::arg("edges") = py::array_t<double>(), py::arg("crit") = -1,
        py::arg("n_threads") = 1);
  m.def("assemble_tree", &assemble_tree, py::arg("feature"), py::arg("tbin"), py::arg("left"),
        py::arg("right"), py::arg("nsamp"), py::arg("stats"), py::arg("fin"),
        py::arg("fin_stats"), py::arg("did"), py::arg("roots"),
        py::arg("edges") = py::array_t<double>(), py::arg("crit") = -1,
        py::arg("n_threads") = 1);
  m.def("node_terms", &node_terms);
  m.def("xlog2x", &xlog2x_np);
}
