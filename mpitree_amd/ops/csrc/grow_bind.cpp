// Host-side level enqueue of the device level loop (ops/device_grower.py).
//
// The loop's kernels read their work counts from device memory, so the host
// only enqueues a fixed chain per level: histogram items -> slab reduction ->
// (regression: sibling derivation) -> scan / select -> planner -> partition
// (-> regression purity). Issued from Python that chain is ~8 pybind calls
// with 15-25 arguments each, tens of microseconds of host time per level --
// comparable to a level's GPU time at the deep, small levels, so the GPU can
// drain the queue and wait on the host. A GrowCtx holds every pointer and
// bound of a fit once; a level is one call that issues the same launches from
// C++ (the Python loop keeps the lagged termination read, checkpoints,
// failure checks, and the multi-rank variants with collectives between the
// kernels).
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>

#include "common.h"
#include "grow.h"

namespace py = pybind11;

namespace mt {

void launch_hist(hipStream_t, const void*, int, int64_t, const uint32_t*, const void*, int,
                 const int64_t*, int, void*, void*, int, int, int, int, bool, int,
                 const int32_t*, const int64_t*, int, const int32_t*);
void launch_hist_reduce(hipStream_t, const int64_t*, int, int, const void*, void*, int, int, int,
                        bool, const int32_t*);
void launch_hist_reduce_tasks(hipStream_t, const int64_t*, int, const int64_t*, int, const void*,
                              void*, int, int, int, const int32_t*, const int32_t*, bool);
void launch_hist_derive(hipStream_t, const int64_t*, int, const void*, void*, int64_t, bool,
                        const int32_t*);
void launch_scan(hipStream_t, const void*, const int64_t*, int, const int32_t*, int, int, int,
                 int, int, int, double*, int32_t*, int64_t*, const double*, int,
                 const int32_t*, const int64_t*, const void*, const int32_t*, int32_t*,
                 int32_t*, const int32_t*);
void launch_grow_plan(hipStream_t, const PlanArgs&);
void launch_partition(hipStream_t, const void*, int, int64_t, uint32_t*, uint32_t*, uint32_t,
                      const int64_t*, int, const int64_t*, int32_t*, const int32_t*, bool);
void launch_seg_minmax(hipStream_t, const uint32_t*, const int64_t*, const int64_t*, int, int64_t*,
                       const int32_t*);

namespace {

template <typename T>
T* ptr(int64_t v) {
  return reinterpret_cast<T*>((uintptr_t)v);
}

LevelLists lists_of(const py::dict& d) {
  auto g = [&](const char* k) { return d[k].cast<int64_t>(); };
  return LevelLists{ptr<int64_t>(g("pos")),    ptr<int64_t>(g("start")), ptr<int32_t>(g("cnt")),
                    ptr<int32_t>(g("depth")),  ptr<int32_t>(g("stats")), ptr<int64_t>(g("items")),
                    ptr<int64_t>(g("red")),    ptr<int64_t>(g("der")),   ptr<int64_t>(g("tasks")),
                    ptr<int32_t>(g("ctl")),    ptr<int64_t>(g("stats64")),
                    ptr<int64_t>(g("minmax")), ptr<int64_t>(g("mitems")),
                    ptr<int32_t>(g("gcnt")),   ptr<int32_t>(g("src"))};
}

// One fit's level-loop arguments (the single-rank and subtree-ownership paths:
// no collective between the kernels).
struct GrowCtx {
  LevelLists L[2]{};
  void* hist[2]{};
  uint32_t* rows[2]{};  // the two row permutation buffers (levels alternate)
  const void* codes_rm = nullptr;
  const void* codes_fm = nullptr;
  const void* y = nullptr;
  void* slab = nullptr;
  int64_t* rec = nullptr;
  double* cost = nullptr;
  int32_t* bins = nullptr;
  int64_t* ident = nullptr;
  int64_t* split = nullptr;
  int64_t* pitems = nullptr;
  int32_t* cursors = nullptr;
  int64_t* jobs = nullptr;
  int32_t* job_count = nullptr;
  int32_t* pos_rec = nullptr;
  void* pos_st = nullptr;
  const int32_t* nbins = nullptr;
  const double* xtab = nullptr;
  int32_t* host_ctl = nullptr;  // 64 host-mapped slots of 16 int32
  // fused selection (two classes, <= 256 bins): [KMAX][F_h][2] left counts and
  // [KMAX][2] class totals from the scan; null: the select kernel runs
  int32_t* sel_left = nullptr;
  int32_t* sel_tot = nullptr;
  int xtab_n = 0;
  int cb = 1, lab_shift = 0, F_h = 0, f_lo = 0, B = 0, C = 0, reg = 0, crit = 0;
  int md = -1, n_cu = 256, lds_budget = 0;
  uint32_t row_mask = 0xFFFFFFFFu;
  int64_t row_bytes = 0, n_codes = 0, n_loc = 0, E = 0;
  int64_t KMAX = 0, IMAX = 0, TMAX = 0, RMAX = 0, PMAX = 0, MMAX = 0;
  int64_t mss = 2, msl = 1, fr = 0;
  int32_t tag0 = 0;
  int derive_free = 0;
  OwnArgs own{0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, 0};

  void level(hipStream_t s, int lvl) {
    const int par = lvl & 1;
    const LevelLists& cur = L[par];
    const LevelLists& nxt = L[par ^ 1];
    void* H = hist[par];
    void* Hp = hist[par ^ 1];
    uint32_t* src = rows[par];
    uint32_t* dst = rows[par ^ 1];
    int32_t* ctl = cur.ctl;
    const int64_t kb = std::min<int64_t>((int64_t)1 << std::min(lvl, 40), KMAX);
    const int ib = (int)std::min<int64_t>(IMAX, kb + n_loc / 1024 + 2 * n_cu + 1);
    const int rb = (int)std::min<int64_t>(kb, RMAX);
    // histogram items (classification: the launch also zeroes the multi-item
    // slots the slab reduction adds into)
    launch_hist(s, codes_rm, cb, row_bytes, src, y, lab_shift, cur.items, ib, H, slab, F_h, f_lo,
                B, C, reg != 0, lds_budget, ctl + 2, reg ? nullptr : cur.red, reg ? 0 : rb,
                reg ? nullptr : ctl + 3);
    if (reg)
      launch_hist_reduce(s, cur.red, rb, 1, slab, H, F_h, B, C, true, ctl + 3);
    else
      launch_hist_reduce_tasks(s, cur.red, rb, cur.tasks,
                               (int)std::min<int64_t>(TMAX, rb + ib / 16 + 1), slab, H, F_h, B,
                               C, ctl + 3, ctl + 7, false);
    // classification: the scan derives the larger siblings (parent - built)
    const bool fuse = lvl > 0 && !reg;
    if (lvl > 0 && reg) launch_hist_derive(s, cur.der, (int)kb, Hp, H, E, true, ctl + 4);
    launch_scan(s, H, ident, (int)kb, nbins, F_h, f_lo, B, C, crit, (int)msl, cost, bins, rec,
                xtab, xtab_n, ctl, fuse ? cur.der : nullptr, fuse ? Hp : nullptr,
                fuse ? ctl + 1 : nullptr, sel_left, sel_tot, reg ? nullptr : cur.stats);
    PlanArgs a{cur,       nxt,        rec,        split,
               pitems,    cursors,    ctl + 5,    pos_rec,
               reg ? nullptr : (int32_t*)pos_st,  reg ? (int64_t*)pos_st : nullptr,
               reg,       par ^ 1,    jobs,       job_count,
               C,         md,         n_cu,       mss,
               msl,       fr,         host_ctl + (lvl % 64) * 16,
               tag0 + (lvl % 4096) + 1, 0, own};
    a.derive_free = derive_free;
    if (sel_left) {
      a.sel_cost = cost;
      a.sel_bins = bins;
      a.sel_left = sel_left;
      a.sel_tot = sel_tot;
      a.sel_F = F_h;
      a.crit = crit;
    }
    launch_grow_plan(s, a);
    const int pb = (int)std::min<int64_t>(PMAX, n_loc / 1024 + kb + 1);
    launch_partition(s, codes_fm, cb, n_codes, src, dst, row_mask, pitems, pb, split, cursors,
                     ctl + 6, false);
    if (reg)  // purity of the next frontier, read by the next planner
      launch_seg_minmax(s, dst, (const int64_t*)y, nxt.mitems,
                        (int)std::min<int64_t>(MMAX, 2 * kb + n_loc / 4096 + 1), nxt.minmax,
                        nxt.ctl + 8);
  }
};

}  // namespace

void bind_grow(py::module_& m) {
  py::class_<GrowCtx>(m, "GrowCtx")
      .def(py::init([](py::dict d, py::dict l0, py::dict l1, py::dict own) {
        auto g = [&](const char* k) { return d[k].cast<int64_t>(); };
        GrowCtx c;
        c.L[0] = lists_of(l0);
        c.L[1] = lists_of(l1);
        c.hist[0] = ptr<void>(g("hist0"));
        c.hist[1] = ptr<void>(g("hist1"));
        c.rows[0] = ptr<uint32_t>(g("idx"));
        c.rows[1] = ptr<uint32_t>(g("tmp"));
        c.codes_rm = ptr<void>(g("codes_rm"));
        c.codes_fm = ptr<void>(g("codes_fm"));
        c.y = ptr<void>(g("y"));
        c.slab = ptr<void>(g("slab"));
        c.rec = ptr<int64_t>(g("rec"));
        c.cost = ptr<double>(g("cost"));
        c.bins = ptr<int32_t>(g("bins"));
        c.ident = ptr<int64_t>(g("ident"));
        c.split = ptr<int64_t>(g("split"));
        c.pitems = ptr<int64_t>(g("pitems"));
        c.cursors = ptr<int32_t>(g("cursors"));
        c.jobs = ptr<int64_t>(g("jobs"));
        c.job_count = ptr<int32_t>(g("job_count"));
        c.pos_rec = ptr<int32_t>(g("pos_rec"));
        c.pos_st = ptr<void>(g("pos_st"));
        c.nbins = ptr<int32_t>(g("nbins"));
        c.xtab = ptr<double>(g("xtab"));
        c.xtab_n = (int)g("xtab_n");
        c.host_ctl = ptr<int32_t>(g("host_ctl"));
        c.cb = (int)g("cb");
        c.row_bytes = g("row_bytes");
        c.lab_shift = (int)g("lab_shift");
        c.row_mask = (uint32_t)g("row_mask");
        c.n_codes = g("n_codes");
        c.n_loc = g("n_loc");
        c.F_h = (int)g("F_h");
        c.f_lo = (int)g("f_lo");
        c.B = (int)g("B");
        c.C = (int)g("C");
        c.reg = (int)g("reg");
        c.crit = (int)g("crit");
        c.E = g("E");
        c.md = (int)g("max_depth");
        c.mss = g("mss");
        c.msl = g("msl");
        c.fr = g("fr");
        c.n_cu = (int)g("n_cu");
        c.lds_budget = (int)g("lds_budget");
        c.KMAX = g("KMAX");
        c.IMAX = g("IMAX");
        c.TMAX = g("TMAX");
        c.RMAX = g("RMAX");
        c.PMAX = g("PMAX");
        c.MMAX = g("MMAX");
        c.tag0 = (int32_t)g("tag0");
        c.derive_free = d.contains("derive_free") ? (int)g("derive_free") : 0;
        if (d.contains("sel_left")) {
          c.sel_left = ptr<int32_t>(g("sel_left"));
          c.sel_tot = ptr<int32_t>(g("sel_tot"));
        }
        if (own.size()) {
          auto o = [&](const char* k) { return own[k].cast<int64_t>(); };
          c.own = OwnArgs{(int)o("P"), (int)o("rank"), (int)o("min_units"), (int)o("cap"),
                          ptr<int32_t>(o("state")), ptr<int64_t>(o("ranges")),
                          ptr<int32_t>(o("node_owner")), ptr<int32_t>(o("job_owner")),
                          own.contains("jobs_at_switch") ? (int)o("jobs_at_switch") : 0,
                          own.contains("segs") ? ptr<int64_t>(o("segs")) : nullptr,
                          own.contains("build_all") ? (int)o("build_all") : 0};
        }
        return c;
      }), py::arg("args"), py::arg("l0"), py::arg("l1"), py::arg("own") = py::dict())
      // a context reused by the next fit of the same workspace: only the host
      // slot tag changes (the caller checks every other field is unchanged)
      .def("set_tag0", [](GrowCtx& c, int64_t tag0) { c.tag0 = (int32_t)tag0; })
      .def("level", [](GrowCtx& c, uintptr_t s, int lvl) {
        c.level(reinterpret_cast<hipStream_t>(s), lvl);
      });
}

}  // namespace mt
