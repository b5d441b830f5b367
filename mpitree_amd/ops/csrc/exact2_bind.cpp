// Host bindings of the exact-threshold engine v2 (exact2.hip).
//
// A fit builds one XeCtx from a dict of device pointers and sizes; per level
// the host then only calls ctx methods with the level index (the list buffers
// and level-list sets alternate by level parity), so enqueueing a level costs
// a few microseconds of host time and no device synchronisation.
#include <pybind11/pybind11.h>

#include "exact2.h"

namespace py = pybind11;

namespace mt {

namespace {

template <typename T>
T* ptr(uintptr_t v) {
  return reinterpret_cast<T*>(v);
}

hipStream_t stream_of(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

struct XeCtx {
  XeArgs a{};
  XeLists L[2]{};
  uint32_t* Eb[2]{};
  int64_t* Yb[2]{};
  XePlanArgs p{};
  uint32_t seq = 1;  // fit sequence number: look-back status tags differ per (fit, level)
  int32_t* sitem = nullptr;  // two-class chunk totals counted by the partition (or null)
  int first = 0;  // first level this process runs (a resumed fit: > 0)

  XeArgs args(int lvl) const {
    XeArgs x = a;
    const int c = lvl & 1;
    x.tag = (uint32_t)((((uint64_t)seq << 12) + (uint64_t)(lvl & 4095)) % 0x3FFFFFFFull) + 1u;
    x.E = Eb[c];
    x.D = Eb[c ^ 1];
    x.Y = Yb[c];
    x.DY = Yb[c ^ 1];
    x.sitem = sitem;
    x.nctl = sitem ? L[c ^ 1].ctl : nullptr;
    // (the level a resumed fit starts at recounts its chunk totals: the saved
    // state holds no partition-counted ones)
    x.tot_ready = sitem != nullptr && lvl > first;
    return x;
  }
};

XeLists lists_of(const py::dict& d) {
  auto g = [&](const char* k) { return d[k].cast<uintptr_t>(); };
  XeLists L;
  L.pos = ptr<int64_t>(g("pos"));
  L.start = ptr<int64_t>(g("start"));
  L.cnt = ptr<int32_t>(g("cnt"));
  L.depth = ptr<int32_t>(g("depth"));
  L.stats = ptr<int64_t>(g("stats"));
  L.minmax = ptr<int64_t>(g("minmax"));
  L.items = ptr<int64_t>(g("items"));
  L.ifirst = ptr<int32_t>(g("ifirst"));
  L.ctl = ptr<int32_t>(g("ctl"));
  return L;
}

}  // namespace

void bind_exact2(py::module_& m) {
  m.def("xe_chunk", &xe_chunk);
  m.def("xe_part_units", &xe_part_units);
  m.def("xe_local_max", &xe_local_max);
  m.def("xe_max_classes", &xe_max_classes);
  m.def("xe_packed_classes", &xe_packed_classes);
  m.def("xe_rec_width", [](int C) { return xe_rec_width(C); });

  py::class_<XeCtx>(m, "XeCtx")
      .def(py::init([](py::dict d, py::dict l0, py::dict l1) {
        auto g = [&](const char* k) { return d[k].cast<int64_t>(); };
        auto u = [&](const char* k) { return (uintptr_t)d[k].cast<int64_t>(); };
        XeCtx c;
        c.L[0] = lists_of(l0);
        c.L[1] = lists_of(l1);
        c.Eb[0] = ptr<uint32_t>(u("E0"));
        c.Eb[1] = ptr<uint32_t>(u("E1"));
        c.Yb[0] = ptr<int64_t>(u("Y0"));
        c.Yb[1] = ptr<int64_t>(u("Y1"));
        XeArgs& a = c.a;
        a.rank_of = nullptr;
        a.X = ptr<void>(u("X"));
        a.x64 = (int)g("x64");
        a.n = g("n");
        a.F = (int)g("F");
        a.f_lo = (int)g("f_lo");
        a.F_loc = (int)g("F_loc");
        a.C = (int)g("C");
        a.ylab = d.contains("ylab") ? ptr<int32_t>(u("ylab")) : nullptr;
        a.crit = (int)g("crit");
        a.msl = g("msl");
        a.xtab = ptr<double>(u("xtab"));
        a.xtab_n = (int)g("xtab_n");
        a.tot = ptr<int64_t>(u("tot"));
        a.carry = ptr<int64_t>(u("carry"));
        a.cmm = ptr<int64_t>(u("cmm"));
        a.cbest = ptr<uint64_t>(u("cbest"));
        a.cmin = d.contains("cmin") ? ptr<uint32_t>(u("cmin")) : nullptr;
        a.nmin = d.contains("nmin") ? ptr<uint32_t>(u("nmin")) : nullptr;
        a.gthr = d.contains("gthr") ? ptr<float>(u("gthr")) : nullptr;
        a.rec = ptr<int64_t>(u("rec"));
        a.split = ptr<int64_t>(u("split"));
        a.pitems = ptr<int64_t>(u("pitems"));
        a.pfirst = ptr<int32_t>(u("pfirst"));
        a.flag = ptr<uint32_t>(u("flag"));
        a.flagb = d.contains("flagb") ? ptr<uint8_t>(u("flagb")) : nullptr;
        a.pstat = ptr<uint64_t>(u("pstat"));
        a.tick = ptr<int32_t>(u("tick"));
        a.tag = 1;
        // (two classes: the partition counts the next level's chunk totals)
        c.sitem = (a.C > 0 && a.C <= 2 && d.contains("sitem")) ? ptr<int32_t>(u("sitem")) : nullptr;
        a.sitem = nullptr;
        a.nctl = nullptr;
        a.tot_ready = 0;
        XePlanArgs& p = c.p;
        p.rec = a.rec;
        p.split = a.split;
        p.pitems = a.pitems;
        p.pfirst = a.pfirst;
        p.pos_rec = ptr<int32_t>(u("pos_rec"));
        p.pos_st = ptr<void>(u("pos_st"));
        p.pos_thr = ptr<double>(u("pos_thr"));
        p.X = a.X;
        p.x64 = a.x64;
        p.F = a.F;
        p.C = a.C;
        p.jobs = ptr<int64_t>(u("jobs"));
        p.job_count = ptr<int32_t>(u("job_count"));
        p.max_depth = (int)g("max_depth");
        p.mss = g("mss");
        p.msl = g("msl");
        p.fr = g("fr");
        p.tick = a.tick;
        p.sitem = c.sitem;
        return c;
      }))
      .def("begin", [](XeCtx& c, int64_t seq) { c.seq = (uint32_t)seq; })
      .def("resume_at", [](XeCtx& c, int lvl) { c.first = lvl; })
      .def("init", [](XeCtx& c, uintptr_t s, uintptr_t root) {
        xe_init(stream_of(s), c.L[0], c.a.n, c.a.C > 0 ? c.a.C : 2, ptr<int64_t>(root),
                c.p.job_count);
      })
      .def("level_scan", [](XeCtx& c, uintptr_t s, int lvl, int items_bound, int slots_bound) {
        xe_level_scan(stream_of(s), c.args(lvl), c.L[lvl & 1], items_bound, slots_bound);
      })
      .def("plan", [](XeCtx& c, uintptr_t s, int lvl, uintptr_t host_ctl, int tag) {
        XePlanArgs p = c.p;
        p.cur = c.L[lvl & 1];
        p.nxt = c.L[(lvl + 1) & 1];
        p.out_buf = (lvl + 1) & 1;
        p.host_ctl = ptr<int32_t>(host_ctl);
        p.host_tag = tag;
        xe_plan(stream_of(s), p);
      })
      .def("flag", [](XeCtx& c, uintptr_t s, int lvl, int pitems_bound, int write_right) {
        xe_flag(stream_of(s), c.args(lvl), c.L[lvl & 1], pitems_bound, write_right);
      })
      .def("partition", [](XeCtx& c, uintptr_t s, int lvl, int pitems_bound, int splits_bound) {
        xe_partition(stream_of(s), c.args(lvl), c.L[lvl & 1], pitems_bound, splits_bound);
      });

  m.def("xe_local_codes", [](uintptr_t s, uintptr_t E0, uintptr_t E1, uintptr_t Y0, uintptr_t Y1,
                             uintptr_t X, int x64, int F, int fg_lo, int64_t n, int F_loc,
                             int f_lo, uintptr_t jobs, int J, int JW, uintptr_t codes_fm,
                             uintptr_t ent, uintptr_t yv, uintptr_t ylab, uintptr_t codes_rm,
                             int row_bytes) {
    xe_local_codes(stream_of(s), ptr<uint32_t>(E0), ptr<uint32_t>(E1), ptr<int64_t>(Y0),
                   ptr<int64_t>(Y1), ptr<void>(X), x64, F, fg_lo, n, F_loc, f_lo,
                   ptr<int64_t>(jobs), J, JW, ptr<uint8_t>(codes_fm), ptr<uint8_t>(codes_rm),
                   row_bytes, ptr<uint32_t>(ent),
                   ptr<int64_t>(yv), ptr<int32_t>(ylab));
  }, py::arg("s"), py::arg("E0"), py::arg("E1"), py::arg("Y0"), py::arg("Y1"), py::arg("X"),
     py::arg("x64"), py::arg("F"), py::arg("fg_lo"), py::arg("n"), py::arg("F_loc"),
     py::arg("f_lo"), py::arg("jobs"), py::arg("J"), py::arg("JW"), py::arg("codes_fm"),
     py::arg("ent"), py::arg("yv"), py::arg("ylab") = 0, py::arg("codes_rm") = 0,
     py::arg("row_bytes") = 0);
  m.def("xe_codes_rm", [](uintptr_t s, uintptr_t codes_fm, int64_t n, int F, int row_bytes,
                          uintptr_t jobs, int J, int JW, uintptr_t codes_rm) {
    xe_codes_rm(stream_of(s), ptr<uint8_t>(codes_fm), n, F, row_bytes, ptr<int64_t>(jobs), J, JW,
                ptr<uint8_t>(codes_rm));
  });
  m.def("xe_fix", [](uintptr_t s, uintptr_t E0, uintptr_t E1, uintptr_t X, int x64, int F,
                     int64_t n, int f_lo, int F_loc, uintptr_t jobs, int J, int JW,
                     uintptr_t pos_rec, uintptr_t pos_thr) {
    xe_fix(stream_of(s), ptr<uint32_t>(E0), ptr<uint32_t>(E1), ptr<void>(X), x64, F, n, f_lo,
           F_loc, ptr<int64_t>(jobs), J, JW, ptr<int32_t>(pos_rec), ptr<double>(pos_thr));
  });
  m.def("xe_rank", [](uintptr_t s, uintptr_t pos_rec, uintptr_t pos_thr, int64_t P,
                      uintptr_t root_rows, uintptr_t rank_at, uintptr_t X, int x64, int F,
                      int64_t n, int f_lo, int F_loc, uintptr_t resolved, uintptr_t keys) {
    xe_rank(stream_of(s), ptr<int32_t>(pos_rec), ptr<double>(pos_thr), P, ptr<uint32_t>(root_rows),
            ptr<uint32_t>(rank_at), ptr<void>(X), x64, F, n, f_lo, F_loc, ptr<uint8_t>(resolved),
            ptr<uint32_t>(keys));
  }, py::arg("s"), py::arg("pos_rec"), py::arg("pos_thr"), py::arg("P"), py::arg("root_rows"),
     py::arg("rank_at"), py::arg("X"), py::arg("x64"), py::arg("F"), py::arg("n"),
     py::arg("f_lo"), py::arg("F_loc"), py::arg("resolved"), py::arg("keys") = 0);
  m.def("xe_resolved_pack", [](uintptr_t s, uintptr_t pos_rec, uintptr_t pos_thr, int64_t P,
                               uintptr_t rank, uintptr_t rows) {
    xe_resolved_pack(stream_of(s), ptr<int32_t>(pos_rec), ptr<double>(pos_thr), P,
                     ptr<int32_t>(rank), ptr<int64_t>(rows));
  });
  m.def("xe_resolved_scatter", [](uintptr_t s, uintptr_t rows, int64_t k, uintptr_t pos_rec,
                                  uintptr_t pos_thr) {
    xe_resolved_scatter(stream_of(s), ptr<int64_t>(rows), k, ptr<int32_t>(pos_rec),
                        ptr<double>(pos_thr));
  });
  m.def("xe_emit", [](uintptr_t s, uintptr_t keys, uintptr_t rows, int64_t n, int F_loc, int nc,
                      int chunk, uintptr_t cbase, uintptr_t ylab, uintptr_t yfix, uintptr_t E,
                      uintptr_t Y, uintptr_t rank_at) {
    xe_emit(stream_of(s), ptr<uint32_t>(keys), ptr<uint32_t>(rows), n, F_loc, nc, chunk,
            ptr<int32_t>(cbase), ptr<int32_t>(ylab), ptr<int64_t>(yfix), ptr<uint32_t>(E),
            ptr<int64_t>(Y), ptr<uint32_t>(rank_at));
  });
}

}  // namespace mt
