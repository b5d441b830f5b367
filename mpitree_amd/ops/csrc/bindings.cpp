// pybind11 entry points for the gfx950 kernels (module ``mpitree_amd._hip``).
//
// The Python side passes raw device pointers (``tensor.data_ptr()``) and the
// current HIP stream handle, so no PyTorch headers are compiled here: the
// extension builds in seconds with hipcc and calls cost one pybind hop.
#include <hip/hip_runtime.h>
#include <cstring>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include "common.h"
#include "grow.h"
#include "criterion.h"

namespace py = pybind11;

namespace mt {
int hist_feature_tile(int F_h, int B, int C, bool reg, int lds_budget);
int hist_class_tile(int F_h, int B, int C, bool reg, int lds_budget);
int64_t hist_slab_words(int F_h, int B, int C, bool reg);
void launch_hist(hipStream_t, const void*, int, int64_t, const uint32_t*, const void*, int,
                 const int64_t*, int, void*, void*, int, int, int, int, bool, int,
                 const int32_t*, const int64_t*, int, const int32_t*);
void launch_hist_reduce(hipStream_t, const int64_t*, int, int, const void*, void*, int, int, int,
                        bool, const int32_t*);
void launch_hist_derive(hipStream_t, const int64_t*, int, const void*, void*, int64_t, bool,
                        const int32_t*);
void launch_scan(hipStream_t, const void*, const int64_t*, int, const int32_t*, int, int, int,
                 int, int, int, double*, int32_t*, int64_t*, const double*, int,
                 const int32_t*, const int64_t*, const void*, const int32_t*, int32_t*,
                 int32_t*, const int32_t*);
bool scan_fused_select_ok(int B, int C, int crit);
void launch_partition(hipStream_t, const void*, int, int64_t, uint32_t*, uint32_t*, uint32_t,
                      const int64_t*, int, const int64_t*, int32_t*, const int32_t*, bool);
void launch_seg_stats(hipStream_t, const uint32_t*, const void*, int, bool, const int64_t*, int,
                      void*, int);
void launch_init_idx(hipStream_t, uint32_t*, const int32_t*, int, int64_t);
void launch_predict(hipStream_t, const void*, bool, int64_t, int, const void*, const double*,
                    int32_t*);
void launch_bin(hipStream_t, const void*, bool, int64_t, int, const void*, int, int,
                const int32_t*, const uint8_t*, void*, int, void*, int, int32_t*, int);
void launch_xlog2x(hipStream_t, double*, int64_t);
void launch_label_count(hipStream_t, const int64_t*, int64_t, int64_t, int, uint32_t*, bool,
                        int32_t*);
void launch_label_encode(hipStream_t, const int64_t*, int64_t, int64_t, const int64_t*, int32_t*);
void launch_finish(hipStream_t, const void*, int64_t, const void*, int, int64_t, uint32_t*,
                   uint32_t*, const int32_t*, int, const int64_t*, int, int32_t*, const int32_t*,
                   int, int, int, int, int, int64_t, int64_t, const double*, const float*, int,
                   int32_t*, int32_t*, int64_t*, int32_t*, int32_t, int, int, int, int64_t*, int,
                   int64_t*, int, int32_t*);
int finish_lds_bytes(int F, int B, int C);
void launch_hw_xlog2x(hipStream_t, float*, int);
int finish_feature_tile(int F, int B, int C);
int finish_job_rows_cap(int C);
int asm_tiles(int64_t P);
void launch_grow_plan(hipStream_t, const PlanArgs&);
size_t exact_setup_temp_bytes(int64_t, int);
void exact_setup_sort(hipStream_t, const float*, int64_t, int, uint32_t*, uint32_t*, uint32_t*,
                      uint32_t*, void*, size_t, int32_t*, int32_t*, int, int, const int32_t*);
void bind_exact2(pybind11::module_& m);
void bind_grow(pybind11::module_& m);
int exact_setup_chunk();
void launch_fp_combine(hipStream_t, const int64_t*, int, int, int, const int32_t*, int64_t*);
void launch_grow_dp_fixup(hipStream_t, const PlanArgs&);
void launch_grow_init(hipStream_t, const LevelLists&, int64_t, int64_t, int64_t, int, int,
                      const int64_t*,
                      int32_t*);
int finish_reg_lds_bytes(int B);
int finish_reg_blocks_per_cu(int B, int code_bytes);
int job_sort_max();
void launch_job_sort(hipStream_t, const int64_t*, int, int, int64_t*, int32_t*);
void launch_finish_reg(hipStream_t, const void*, int64_t, const void*, int, int64_t, uint32_t*,
                       uint32_t*, const int64_t*, const int64_t*, int, int32_t*, const int32_t*,
                       int, int, int, int64_t, int64_t, int32_t*, int64_t*, int, int, int64_t*,
                       int, int64_t*, int32_t*, int32_t, int, int32_t*);
void launch_seg_minmax(hipStream_t, const uint32_t*, const int64_t*, const int64_t*, int, int64_t*,
                       const int32_t*);
void launch_hist_reduce_tasks(hipStream_t, const int64_t*, int, const int64_t*, int, const void*,
                              void*, int, int, int, const int32_t*, const int32_t*, bool);
int edges_sample_rows(bool x64);
void launch_edges(hipStream_t, const void*, bool, int64_t, int, int, int, void*, int32_t*,
                  uint8_t*, double*, int);
void launch_asm_rank(hipStream_t, const int32_t*, int64_t, int32_t*, int64_t*, int32_t*,
                     const uint8_t*);
void launch_own_pack(hipStream_t, const int64_t*, int, uint8_t*, const int32_t*, const void*,
                     bool, int64_t, int, int32_t*, int64_t*, int32_t*, void*, int64_t);
void launch_own_scatter(hipStream_t, const void*, int64_t, int, int32_t*, void*, bool);
int64_t asm_node_bytes(int C, bool reg);
int small_fit_max_rows();
void launch_small_fit(hipStream_t, const void*, int, int64_t, int, int, const int32_t*, int, int,
                      int, int64_t, int64_t, const double*, int, uint16_t*, int32_t*, int32_t*,
                      int64_t);
void launch_asm_emit(hipStream_t, const int32_t*, const void*, bool, int64_t, int,
                     const int32_t*, const double*, int, const int64_t*, uint8_t*, bool, int, int,
                     const double*, int, const double*, const int64_t*, int, int, bool, int64_t);
void launch_dp_plan(hipStream_t, const int64_t*, int, int, int, const int64_t*, int, int,
                    int64_t*, int64_t*, int64_t*, int64_t*);
void launch_dp_gather(hipStream_t, const int64_t*, int, int, int, const uint32_t*,
                      const uint32_t*, uint32_t, const uint8_t*, int64_t, const void*, bool,
                      const int64_t*, uint8_t*, void*, int64_t);
void launch_dp_place(hipStream_t, const int64_t*, int64_t, const uint8_t*, const void*, bool,
                     int64_t, int64_t, int, int, uint8_t*, void*, void*);
void launch_targets(hipStream_t, const void*, bool, int64_t, int64_t*, int64_t*);
void launch_shm_seg_count(hipStream_t, const int64_t*, int, int, const int32_t*, int64_t,
                          const int64_t*, int64_t*);
int shm_max_segs();
void launch_shm_seg_prefix(hipStream_t, const int64_t*, int, int, const int64_t*, int, int,
                           int64_t*, int64_t*);
}  // namespace mt

template <typename T>
static T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

PYBIND11_MODULE(_hip, m) {
  m.doc() = "mpitree_amd gfx950 HIP kernels";
  m.def("hist_feature_tile", &mt::hist_feature_tile);
  m.def("hist_class_tile", &mt::hist_class_tile);
  m.def("hist_slab_words", &mt::hist_slab_words);
  m.def("hist", [](uintptr_t s, uintptr_t codes, int cb, int64_t rs, uintptr_t idx, uintptr_t y,
                   int lab_shift, uintptr_t items, int n_items, uintptr_t hist, uintptr_t slab,
                   int F_h, int f_lo, int B, int C, bool reg, int lds, uintptr_t dcount,
                   uintptr_t zred, int zred_bound, uintptr_t zcount) {
    mt::launch_hist(S(s), P<void>(codes), cb, rs, P<uint32_t>(idx), P<void>(y), lab_shift,
                    P<int64_t>(items), n_items, P<void>(hist), P<void>(slab), F_h, f_lo, B, C,
                    reg, lds, P<int32_t>(dcount), P<int64_t>(zred), zred_bound,
                    P<int32_t>(zcount));
  }, "", py::arg("s"), py::arg("codes"), py::arg("cb"), py::arg("rs"), py::arg("idx"),
     py::arg("y"), py::arg("lab_shift"), py::arg("items"), py::arg("n_items"), py::arg("hist"),
     py::arg("slab"), py::arg("F_h"), py::arg("f_lo"), py::arg("B"), py::arg("C"), py::arg("reg"),
     py::arg("lds"), py::arg("dcount") = 0, py::arg("zred") = 0, py::arg("zred_bound") = 0,
     py::arg("zcount") = 0);
  m.def("hist_reduce", [](uintptr_t s, uintptr_t red, int n, int max_k, uintptr_t slab,
                          uintptr_t hist, int F_h, int B, int C, bool reg, uintptr_t dcount) {
    mt::launch_hist_reduce(S(s), P<int64_t>(red), n, max_k, P<void>(slab), P<void>(hist), F_h, B,
                           C, reg, P<int32_t>(dcount));
  }, "", py::arg("s"), py::arg("red"), py::arg("n"), py::arg("max_k"), py::arg("slab"),
     py::arg("hist"), py::arg("F_h"), py::arg("B"), py::arg("C"), py::arg("reg"),
     py::arg("dcount") = 0);
  m.def("hist_derive", [](uintptr_t s, uintptr_t der, int n, uintptr_t prev, uintptr_t hist,
                          int64_t E, bool is64, uintptr_t dcount) {
    mt::launch_hist_derive(S(s), P<int64_t>(der), n, P<void>(prev), P<void>(hist), E, is64,
                           P<int32_t>(dcount));
  }, "", py::arg("s"), py::arg("der"), py::arg("n"), py::arg("prev"), py::arg("hist"),
     py::arg("E"), py::arg("is64"), py::arg("dcount") = 0);
  m.def("scan", [](uintptr_t s, uintptr_t hist, uintptr_t nodes, int k, uintptr_t nbins, int F_h,
                   int f_lo, int B, int C, int crit, int msl, uintptr_t cost, uintptr_t bins,
                   uintptr_t rec, uintptr_t xtab, int xtab_n, uintptr_t dcount, uintptr_t der,
                   uintptr_t prev, uintptr_t nbuilt, uintptr_t node_tot) {
    mt::launch_scan(S(s), P<void>(hist), P<int64_t>(nodes), k, P<int32_t>(nbins), F_h, f_lo, B, C,
                    crit, msl, P<double>(cost), P<int32_t>(bins), P<int64_t>(rec),
                    P<double>(xtab), xtab_n, P<int32_t>(dcount), P<int64_t>(der), P<void>(prev),
                    P<int32_t>(nbuilt), nullptr, nullptr, P<int32_t>(node_tot));
  }, "", py::arg("s"), py::arg("hist"), py::arg("nodes"), py::arg("k"), py::arg("nbins"),
     py::arg("F_h"), py::arg("f_lo"), py::arg("B"), py::arg("C"), py::arg("crit"), py::arg("msl"),
     py::arg("cost"), py::arg("bins"), py::arg("rec"), py::arg("xtab"), py::arg("xtab_n"),
     py::arg("dcount") = 0, py::arg("der") = 0, py::arg("prev") = 0, py::arg("nbuilt") = 0,
     py::arg("node_tot") = 0);
  m.def("partition", [](uintptr_t s, uintptr_t codes_fm, int cb, int64_t n_rows, uintptr_t idx,
                        uintptr_t tmp, uint32_t mask, uintptr_t items, int n_items,
                        uintptr_t split, uintptr_t cursors, uintptr_t dcount, bool copy_back) {
    mt::launch_partition(S(s), P<void>(codes_fm), cb, n_rows, P<uint32_t>(idx),
                         P<uint32_t>(tmp), mask, P<int64_t>(items), n_items, P<int64_t>(split),
                         P<int32_t>(cursors), P<int32_t>(dcount), copy_back);
  }, "", py::arg("s"), py::arg("codes_fm"), py::arg("cb"), py::arg("n_rows"), py::arg("idx"),
     py::arg("tmp"), py::arg("mask"), py::arg("items"), py::arg("n_items"), py::arg("split"),
     py::arg("cursors"), py::arg("dcount") = 0, py::arg("copy_back") = true);
  m.def("seg_stats", [](uintptr_t s, uintptr_t idx, uintptr_t y, int lab_shift, bool reg,
                        uintptr_t items, int n_items, uintptr_t out, int C) {
    mt::launch_seg_stats(S(s), P<uint32_t>(idx), P<void>(y), lab_shift, reg, P<int64_t>(items),
                         n_items, P<void>(out), C);
  });
  m.def("init_idx", [](uintptr_t s, uintptr_t idx, uintptr_t y, int lab_shift, int64_t n) {
    mt::launch_init_idx(S(s), P<uint32_t>(idx), P<int32_t>(y), lab_shift, n);
  });
  m.def("predict", [](uintptr_t s, uintptr_t X, bool x64, int64_t n, int F, uintptr_t nodes,
                      uintptr_t thr, uintptr_t leaf) {
    mt::launch_predict(S(s), P<void>(X), x64, n, F, P<void>(nodes), P<double>(thr),
                       P<int32_t>(leaf));
  });
  m.def(
      "bin",
      [](uintptr_t s, uintptr_t X, bool x64, int64_t n, int F, uintptr_t edges, int Bmax,
         uintptr_t nbins, uintptr_t exact, uintptr_t codes_rm, int row_elems, uintptr_t codes_fm,
         int cb, uintptr_t bad, int estride, bool skip_inexact) {
        mt::launch_bin(S(s), P<void>(X), x64, n, F, P<void>(edges), Bmax,
                       estride > 0 ? estride : Bmax, P<int32_t>(nbins), P<uint8_t>(exact),
                       P<void>(codes_rm), row_elems, P<void>(codes_fm), cb, P<int32_t>(bad),
                       skip_inexact ? 1 : 0);
      },
      py::arg("s"), py::arg("X"), py::arg("x64"), py::arg("n"), py::arg("F"), py::arg("edges"),
      py::arg("Bmax"), py::arg("nbins"), py::arg("exact"), py::arg("codes_rm"),
      py::arg("row_elems"), py::arg("codes_fm"), py::arg("cb"), py::arg("bad"),
      py::arg("estride") = 0, py::arg("skip_inexact") = false);
  m.def("finish_lds_bytes", &mt::finish_lds_bytes);
  m.def("finish_feature_tile", &mt::finish_feature_tile);
  m.def("finish_job_rows_cap", &mt::finish_job_rows_cap);
  m.def("finish", [](uintptr_t s, uintptr_t codes_rm, int64_t row_words, uintptr_t codes_fm,
                     int cb, int64_t n_rows, uintptr_t idx, uintptr_t tmp, uintptr_t y,
                     int lab_shift, uintptr_t jobs, int J, uintptr_t counter, uintptr_t nbins,
                     int F, int B, int C, int crit, int max_depth, int64_t mss, int64_t msl,
                     uintptr_t xtab, uintptr_t xtabf, int xtab_n, uintptr_t node_i32,
                     uintptr_t node_cnt, uintptr_t tasks, uintptr_t task_flag, int epoch,
                     int task_cap, int grid, int tiny_rows, uintptr_t tiny,
                     int tiny_grid, uintptr_t prof, int tiny_waves, uintptr_t tiny_order) {
    mt::launch_finish(S(s), P<void>(codes_rm), row_words, P<void>(codes_fm), cb, n_rows,
                      P<uint32_t>(idx), P<uint32_t>(tmp), P<int32_t>(y), lab_shift,
                      P<int64_t>(jobs), J, P<int32_t>(counter), P<int32_t>(nbins), F, B, C, crit,
                      max_depth, mss, msl, P<double>(xtab), P<float>(xtabf), xtab_n, P<int32_t>(node_i32),
                      P<int32_t>(node_cnt), P<int64_t>(tasks), P<int32_t>(task_flag), epoch,
                      task_cap, grid, tiny_rows,
                      P<int64_t>(tiny), tiny_grid, P<int64_t>(prof), tiny_waves,
                      P<int32_t>(tiny_order));
  }, py::arg("s"), py::arg("codes_rm"), py::arg("row_words"), py::arg("codes_fm"), py::arg("cb"),
     py::arg("n_rows"), py::arg("idx"), py::arg("tmp"), py::arg("y"), py::arg("lab_shift"),
     py::arg("jobs"), py::arg("J"), py::arg("counter"), py::arg("nbins"), py::arg("F"),
     py::arg("B"), py::arg("C"), py::arg("crit"), py::arg("max_depth"), py::arg("mss"),
     py::arg("msl"), py::arg("xtab"), py::arg("xtabf"), py::arg("xtab_n"), py::arg("node_i32"),
     py::arg("node_cnt"), py::arg("tasks"), py::arg("task_flag"), py::arg("epoch"),
     py::arg("task_cap"), py::arg("grid"), py::arg("tiny_rows"),
     py::arg("tiny"), py::arg("tiny_grid"), py::arg("prof"), py::arg("tiny_waves") = 0,
     py::arg("tiny_order") = 0);
  m.def("asm_tiles", &mt::asm_tiles);
  m.def("small_fit_max_rows", &mt::small_fit_max_rows);
  m.def("small_fit", [](uintptr_t s, uintptr_t codes_fm, int cb, int64_t n_stride, int n, int F,
                        uintptr_t y, int C, int crit, int max_depth, int64_t mss, int64_t msl,
                        uintptr_t xtab, int xtab_n, uintptr_t ord, uintptr_t node_i32,
                        uintptr_t node_cnt, int64_t npos) {
    mt::launch_small_fit(S(s), P<void>(codes_fm), cb, n_stride, n, F, P<int32_t>(y), C, crit,
                         max_depth, mss, msl, P<double>(xtab), xtab_n, P<uint16_t>(ord),
                         P<int32_t>(node_i32), P<int32_t>(node_cnt), npos);
  });
  m.def("finish_reg_lds_bytes", &mt::finish_reg_lds_bytes);
  m.def("finish_reg_blocks_per_cu", &mt::finish_reg_blocks_per_cu);
  m.def("finish_reg", [](uintptr_t s, uintptr_t codes_rm, int64_t row_words, uintptr_t codes_fm,
                         int cb, int64_t n_rows, uintptr_t buf0, uintptr_t buf1, uintptr_t y,
                         uintptr_t jobs, int J, uintptr_t counter, uintptr_t nbins, int F, int B,
                         int max_depth, int64_t mss, int64_t msl, uintptr_t node_i32,
                         uintptr_t node_st, int grid, int tiny_rows, uintptr_t tiny,
                         int tiny_grid, uintptr_t tasks, uintptr_t task_flag, int epoch,
                         int task_cap, uintptr_t tiny_order) {
    mt::launch_finish_reg(S(s), P<void>(codes_rm), row_words, P<void>(codes_fm), cb, n_rows,
                          P<uint32_t>(buf0), P<uint32_t>(buf1), P<int64_t>(y), P<int64_t>(jobs),
                          J, P<int32_t>(counter), P<int32_t>(nbins), F, B, max_depth, mss, msl,
                          P<int32_t>(node_i32), P<int64_t>(node_st), grid, tiny_rows,
                          P<int64_t>(tiny), tiny_grid, P<int64_t>(tasks), P<int32_t>(task_flag),
                          epoch, task_cap, P<int32_t>(tiny_order));
  }, py::arg("s"), py::arg("codes_rm"), py::arg("row_words"), py::arg("codes_fm"), py::arg("cb"),
     py::arg("n_rows"), py::arg("buf0"), py::arg("buf1"), py::arg("y"), py::arg("jobs"),
     py::arg("J"), py::arg("counter"), py::arg("nbins"), py::arg("F"), py::arg("B"),
     py::arg("max_depth"), py::arg("mss"), py::arg("msl"), py::arg("node_i32"),
     py::arg("node_st"), py::arg("grid"), py::arg("tiny_rows"), py::arg("tiny"),
     py::arg("tiny_grid"), py::arg("tasks"), py::arg("task_flag"), py::arg("epoch"),
     py::arg("task_cap"), py::arg("tiny_order") = 0);
  m.def("seg_minmax", [](uintptr_t s, uintptr_t idx, uintptr_t y, uintptr_t items, int n_items,
                         uintptr_t out, uintptr_t dcount) {
    mt::launch_seg_minmax(S(s), P<uint32_t>(idx), P<int64_t>(y), P<int64_t>(items), n_items,
                          P<int64_t>(out), P<int32_t>(dcount));
  });
  m.def("hist_reduce_tasks", [](uintptr_t s, uintptr_t red, int red_bound, uintptr_t tasks,
                                int task_bound, uintptr_t slab, uintptr_t hist, int F_h, int B,
                                int C, uintptr_t dred, uintptr_t dtasks, bool zero) {
    mt::launch_hist_reduce_tasks(S(s), P<int64_t>(red), red_bound, P<int64_t>(tasks), task_bound,
                                 P<void>(slab), P<void>(hist), F_h, B, C, P<int32_t>(dred),
                                 P<int32_t>(dtasks), zero);
  }, "", py::arg("s"), py::arg("red"), py::arg("red_bound"), py::arg("tasks"),
     py::arg("task_bound"), py::arg("slab"), py::arg("hist"), py::arg("F_h"), py::arg("B"),
     py::arg("C"), py::arg("dred"), py::arg("dtasks"), py::arg("zero") = true);
  m.def("job_sort_max", &mt::job_sort_max);
  m.def("fin_tiny_batch", []() { return mt::kFinTinyBatch; });
  m.def("scan_fused_select_ok", &mt::scan_fused_select_ok);
  m.def("job_sort", [](uintptr_t s, uintptr_t jobs, int J, int W, uintptr_t out,
                       uintptr_t counters) {
    mt::launch_job_sort(S(s), P<int64_t>(jobs), J, W, P<int64_t>(out), P<int32_t>(counters));
  });
  // level lists: dicts of device pointers {pos, start, cnt, depth, stats, items, red, der,
  // tasks, ctl, stats64, minmax, mitems, gcnt, src}
  auto lists = [](py::dict d) {
    auto g = [&](const char* k) { return d[k].cast<uintptr_t>(); };
    return mt::LevelLists{P<int64_t>(g("pos")),     P<int64_t>(g("start")), P<int32_t>(g("cnt")),
                          P<int32_t>(g("depth")),   P<int32_t>(g("stats")), P<int64_t>(g("items")),
                          P<int64_t>(g("red")),     P<int64_t>(g("der")),   P<int64_t>(g("tasks")),
                          P<int32_t>(g("ctl")),     P<int64_t>(g("stats64")),
                          P<int64_t>(g("minmax")),  P<int64_t>(g("mitems")),
                          P<int32_t>(g("gcnt")),    P<int32_t>(g("src"))};
  };
  m.def("grow_init", [lists](uintptr_t s, py::dict L, int64_t n, int64_t n_global, int64_t chunk,
                             int C, int reg, uintptr_t root, uintptr_t job_count) {
    mt::launch_grow_init(S(s), lists(L), n, n_global, chunk, C, reg, P<int64_t>(root),
                         P<int32_t>(job_count));
  });
  auto plan_args = [lists](py::dict cur, py::dict nxt, uintptr_t rec, uintptr_t split,
                           uintptr_t pitems, uintptr_t cursors, uintptr_t pctl, uintptr_t pos_rec,
                           uintptr_t pos_st, uintptr_t pos_st64, int reg, int out_buf,
                           uintptr_t jobs, uintptr_t job_count, int C, int max_depth, int n_cu,
                           int64_t mss, int64_t msl, int64_t fr, uintptr_t host_ctl, int host_tag,
                           int dp, py::dict own) {
    mt::OwnArgs o{0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0};
    if (own.size()) {
      auto g = [&](const char* k) { return own[k].cast<int64_t>(); };
      o = mt::OwnArgs{(int)g("P"), (int)g("rank"), (int)g("min_units"), (int)g("cap"),
                      P<int32_t>((uintptr_t)g("state")), P<int64_t>((uintptr_t)g("ranges")),
                      P<int32_t>((uintptr_t)g("node_owner")),
                      P<int32_t>((uintptr_t)g("job_owner")),
                      own.contains("jobs_at_switch") ? (int)g("jobs_at_switch") : 0,
                      own.contains("segs") ? P<int64_t>((uintptr_t)g("segs")) : nullptr,
                      own.contains("build_all") ? (int)g("build_all") : 0};
    }
    return mt::PlanArgs{lists(cur),          lists(nxt),         P<int64_t>(rec),
                        P<int64_t>(split),   P<int64_t>(pitems), P<int32_t>(cursors),
                        P<int32_t>(pctl),    P<int32_t>(pos_rec), P<int32_t>(pos_st),
                        P<int64_t>(pos_st64), reg, out_buf, P<int64_t>(jobs),
                        P<int32_t>(job_count), C, max_depth, n_cu, mss, msl, fr,
                        P<int32_t>(host_ctl), host_tag, dp, o};
  };
  m.def("grow_plan", [plan_args](uintptr_t s, py::dict cur, py::dict nxt, uintptr_t rec,
                                 uintptr_t split, uintptr_t pitems, uintptr_t cursors,
                                 uintptr_t pctl, uintptr_t pos_rec, uintptr_t pos_st,
                                 uintptr_t pos_st64, int reg, int out_buf, uintptr_t jobs,
                                 uintptr_t job_count, int C, int max_depth, int n_cu, int64_t mss,
                                 int64_t msl, int64_t fr, uintptr_t host_ctl, int host_tag,
                                 int dp, bool fixup, py::dict own, int derive_free) {
    mt::PlanArgs a = plan_args(cur, nxt, rec, split, pitems, cursors, pctl, pos_rec, pos_st,
                               pos_st64, reg, out_buf, jobs, job_count, C, max_depth, n_cu,
                               mss, msl, fr, host_ctl, host_tag, dp, own);
    a.derive_free = derive_free;
    if (fixup)
      mt::launch_grow_dp_fixup(S(s), a);
    else
      mt::launch_grow_plan(S(s), a);
  }, py::arg("s"), py::arg("cur"), py::arg("nxt"), py::arg("rec"), py::arg("split"),
     py::arg("pitems"), py::arg("cursors"), py::arg("pctl"), py::arg("pos_rec"),
     py::arg("pos_st"), py::arg("pos_st64"), py::arg("reg"), py::arg("out_buf"), py::arg("jobs"),
     py::arg("job_count"), py::arg("C"), py::arg("max_depth"), py::arg("n_cu"), py::arg("mss"),
     py::arg("msl"), py::arg("fr"), py::arg("host_ctl"), py::arg("host_tag"), py::arg("dp") = 0,
     py::arg("fixup") = false, py::arg("own") = py::dict(), py::arg("derive_free") = 0);
  m.def("exact_setup_temp_bytes", &mt::exact_setup_temp_bytes);
  m.def("exact_setup_chunk", &mt::exact_setup_chunk);
  m.def("exact_setup_sort", [](uintptr_t s, uintptr_t X, int64_t n, int F, uintptr_t k0,
                               uintptr_t k1, uintptr_t r0, uintptr_t r1, uintptr_t temp,
                               size_t temp_bytes, uintptr_t cnt, uintptr_t nuniq, int xs,
                               int f_lo, uintptr_t ylab) {
    mt::exact_setup_sort(S(s), P<float>(X), n, F, P<uint32_t>(k0), P<uint32_t>(k1),
                         P<uint32_t>(r0), P<uint32_t>(r1), P<void>(temp), temp_bytes,
                         P<int32_t>(cnt), P<int32_t>(nuniq), xs, f_lo, P<const int32_t>(ylab));
  }, py::arg("s"), py::arg("X"), py::arg("n"), py::arg("F"), py::arg("k0"), py::arg("k1"),
     py::arg("r0"), py::arg("r1"), py::arg("temp"), py::arg("temp_bytes"), py::arg("cnt"),
     py::arg("nuniq"), py::arg("xs") = 0, py::arg("f_lo") = 0, py::arg("ylab") = 0);
  m.def("fp_combine", [](uintptr_t s, uintptr_t g, int nranks, int KB, int R, uintptr_t dcount,
                         uintptr_t rec) {
    mt::launch_fp_combine(S(s), P<int64_t>(g), nranks, KB, R, P<int32_t>(dcount),
                          P<int64_t>(rec));
  });
  // Host-mapped, fine-grained (coherent) memory the kernels can store into
  // directly: the level loop's termination counters travel without a copy.
  // (coherent = false: coarse-grained, written through the L2 with full PCIe
  // write bursts -- what a kernel streaming a finished tree to the host wants;
  // tools/probes/zc_probe.hip)
  m.def("host_alloc", [](size_t nbytes, bool coherent) {
    void* p = nullptr;
    MT_HIP_CHECK(hipHostMalloc(&p, nbytes,
                               coherent ? (hipHostMallocMapped | hipHostMallocCoherent)
                                        : (hipHostMallocMapped | hipHostMallocNonCoherent)));
    std::memset(p, 0, nbytes);
    return reinterpret_cast<uintptr_t>(p);
  }, py::arg("nbytes"), py::arg("coherent") = true);
  m.def("host_device_ptr", [](uintptr_t p) {
    void* d = nullptr;
    MT_HIP_CHECK(hipHostGetDevicePointer(&d, reinterpret_cast<void*>(p), 0));
    return reinterpret_cast<uintptr_t>(d);
  });
  m.def("host_free", [](uintptr_t p) { MT_HIP_CHECK(hipHostFree(reinterpret_cast<void*>(p))); });
  // stream-ordered device -> pinned host copy (DMA)
  m.def("copy_d2h", [](uintptr_t s, uintptr_t dst, uintptr_t src, size_t nbytes) {
    if (nbytes)
      MT_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src),
                                  nbytes, hipMemcpyDeviceToHost, S(s)));
  });
  m.def("edges_sample_rows", &mt::edges_sample_rows);
  m.def(
      "edges",
      [](uintptr_t s, uintptr_t X, bool x64, int64_t n, int F, int rows, int limit,
         uintptr_t edges, uintptr_t nbins, uintptr_t exact, uintptr_t pack, bool probe) {
        mt::launch_edges(S(s), P<void>(X), x64, n, F, rows, limit, P<void>(edges),
                         P<int32_t>(nbins), P<uint8_t>(exact), P<double>(pack), probe ? 1 : 0);
      },
      py::arg("s"), py::arg("X"), py::arg("x64"), py::arg("n"), py::arg("F"), py::arg("rows"),
      py::arg("limit"), py::arg("edges"), py::arg("nbins"), py::arg("exact"),
      py::arg("pack") = 0, py::arg("probe") = false);
  m.def("asm_rank", [](uintptr_t s, uintptr_t rec, int64_t npos, uintptr_t tile, uintptr_t total,
                       uintptr_t rank, uintptr_t mask) {
    mt::launch_asm_rank(S(s), P<int32_t>(rec), npos, P<int32_t>(tile), P<int64_t>(total),
                        P<int32_t>(rank), P<uint8_t>(mask));
  }, py::arg("s"), py::arg("rec"), py::arg("npos"), py::arg("tile"), py::arg("total"),
     py::arg("rank"), py::arg("mask") = 0);
  m.def("own_pack", [](uintptr_t s, uintptr_t ranges, int cap, uintptr_t mask, uintptr_t rec,
                       uintptr_t st, bool st64, int64_t npos, int C, uintptr_t tile,
                       uintptr_t total, uintptr_t rank, uintptr_t rows, int64_t row_cap) {
    mt::launch_own_pack(S(s), P<int64_t>(ranges), cap, P<uint8_t>(mask), P<int32_t>(rec),
                        P<void>(st), st64, npos, C, P<int32_t>(tile), P<int64_t>(total),
                        P<int32_t>(rank), P<void>(rows), row_cap);
  }, py::arg("s"), py::arg("ranges"), py::arg("cap"), py::arg("mask"), py::arg("rec"),
     py::arg("st"), py::arg("st64"), py::arg("npos"), py::arg("C"), py::arg("tile"),
     py::arg("total"), py::arg("rank"), py::arg("rows"), py::arg("row_cap") = INT64_MAX);
  m.def("own_scatter", [](uintptr_t s, uintptr_t rows, int64_t k, int C, uintptr_t rec,
                          uintptr_t st, bool st64) {
    mt::launch_own_scatter(S(s), P<void>(rows), k, C, P<int32_t>(rec), P<void>(st), st64);
  });
  m.def("asm_node_bytes", &mt::asm_node_bytes);
  m.def("asm_emit", [](uintptr_t s, uintptr_t rec, uintptr_t st, bool st64, int64_t npos, int C,
                       uintptr_t rank, uintptr_t edges, int EB, uintptr_t total, uintptr_t base,
                       bool reg, int crit, int y_exp, uintptr_t xtab, int xtab_n,
                       uintptr_t thr_pos, uintptr_t tab, int n_tab, int me, bool emit_prefix,
                       int64_t cap_nodes) {
    mt::launch_asm_emit(S(s), P<int32_t>(rec), P<void>(st), st64, npos, C, P<int32_t>(rank),
                        P<double>(edges), EB, P<int64_t>(total), P<uint8_t>(base), reg, crit,
                        y_exp, P<double>(xtab), xtab_n, P<double>(thr_pos), P<int64_t>(tab),
                        n_tab, me, emit_prefix, cap_nodes);
  }, py::arg("s"), py::arg("rec"), py::arg("st"), py::arg("st64"), py::arg("npos"), py::arg("C"),
     py::arg("rank"), py::arg("edges"), py::arg("EB"), py::arg("total"), py::arg("base"),
     py::arg("reg"), py::arg("crit"), py::arg("y_exp"), py::arg("xtab"), py::arg("xtab_n"),
     py::arg("thr_pos") = 0, py::arg("tab") = 0, py::arg("n_tab") = 0, py::arg("me") = 0,
     py::arg("emit_prefix") = true, py::arg("cap_nodes") = 0);
  m.def("targets", [](uintptr_t s, uintptr_t y, bool y64, int64_t n, uintptr_t st, uintptr_t out) {
    mt::launch_targets(S(s), P<void>(y), y64, n, P<int64_t>(st), P<int64_t>(out));
  });
  // data-parallel subtree finishing (ops/device_grower.py _dp_finish)
  m.def("dp_plan", [](uintptr_t s, uintptr_t jobs, int J, int W, int C, uintptr_t allc, int P_,
                      int me, uintptr_t soff, uintptr_t hdr, uintptr_t jobs2, uintptr_t seg) {
    mt::launch_dp_plan(S(s), P<int64_t>(jobs), J, W, C, P<int64_t>(allc), P_, me,
                       P<int64_t>(soff), P<int64_t>(hdr), P<int64_t>(jobs2), P<int64_t>(seg));
  });
  m.def("dp_gather", [](uintptr_t s, uintptr_t jobs, int J, int W, int C, uintptr_t idx,
                        uintptr_t tmp, uint32_t row_mask, uintptr_t codes_rm, int64_t row_bytes,
                        uintptr_t y, bool y64, uintptr_t soff, uintptr_t out_codes,
                        uintptr_t out_y, int64_t max_rows) {
    // max_rows: a bound on every job's local rows (the grid's row-tile extent)
    mt::launch_dp_gather(S(s), P<int64_t>(jobs), J, W, C, P<uint32_t>(idx), P<uint32_t>(tmp),
                         row_mask, P<uint8_t>(codes_rm), row_bytes, P<void>(y), y64,
                         P<int64_t>(soff), P<uint8_t>(out_codes), P<void>(out_y), max_rows);
  });
  // received rows -> job-contiguous row-major and feature-major codes + targets
  m.def("dp_place", [](uintptr_t s, uintptr_t seg, int64_t nseg, uintptr_t in_codes,
                       uintptr_t in_y, bool y64, int64_t row_bytes, int64_t rows, int F, int cb,
                       uintptr_t out_rm, uintptr_t out_fm, uintptr_t out_y) {
    mt::launch_dp_place(S(s), P<int64_t>(seg), nseg, P<uint8_t>(in_codes), P<void>(in_y), y64,
                        row_bytes, rows, F, cb, P<uint8_t>(out_rm), P<void>(out_fm),
                        P<void>(out_y));
  });
  // node-local shared-host assembly (parallel/shared_tree.py)
  m.def("shm_seg_count", [](uintptr_t s, uintptr_t segs, int S_, int me, uintptr_t rank,
                            int64_t npos, uintptr_t total, uintptr_t gvec) {
    mt::launch_shm_seg_count(S(s), P<int64_t>(segs), S_, me, P<int32_t>(rank), npos,
                             P<int64_t>(total), P<int64_t>(gvec));
  });
  m.def("shm_max_segs", &mt::shm_max_segs);  // segments one shared assembly can sort
  m.def("shm_seg_prefix", [](uintptr_t s, uintptr_t gall, int nranks, int W, uintptr_t segs,
                             int S_, int me, uintptr_t total, uintptr_t tab) {
    mt::launch_shm_seg_prefix(S(s), P<int64_t>(gall), nranks, W, P<int64_t>(segs), S_, me,
                              P<int64_t>(total), P<int64_t>(tab));
  });
  // pin (and map for device access) host memory the process did not allocate
  // through HIP, e.g. a /dev/shm mapping several ranks share
  m.def("host_register", [](uintptr_t p, size_t nbytes) {
    MT_HIP_CHECK(hipHostRegister(reinterpret_cast<void*>(p), nbytes,
                                 hipHostRegisterMapped | hipHostRegisterPortable));
    void* d = nullptr;
    MT_HIP_CHECK(hipHostGetDevicePointer(&d, reinterpret_cast<void*>(p), 0));
    return reinterpret_cast<uintptr_t>(d);
  });
  m.def("host_unregister", [](uintptr_t p) {
    MT_HIP_CHECK(hipHostUnregister(reinterpret_cast<void*>(p)));
  });
  // enc (optional): also the labels' int32 codes y - lo (valid when they lie in range)
  m.def("label_count", [](uintptr_t s, uintptr_t y, int64_t n, int64_t lo, int R,
                          uintptr_t counts, bool checked, uintptr_t enc) {
    mt::launch_label_count(S(s), P<int64_t>(y), n, lo, R, P<uint32_t>(counts), checked,
                           P<int32_t>(enc));
  }, py::arg("s"), py::arg("y"), py::arg("n"), py::arg("lo"), py::arg("R"), py::arg("counts"),
     py::arg("checked") = false, py::arg("enc") = 0);
  m.def("label_encode", [](uintptr_t s, uintptr_t y, int64_t n, int64_t lo, uintptr_t lut,
                           uintptr_t out) {
    mt::launch_label_encode(S(s), P<int64_t>(y), n, lo, P<int64_t>(lut), P<int32_t>(out));
  });
  mt::bind_exact2(m);
  mt::bind_grow(m);
  m.def("xlog2x_device", [](uintptr_t s, uintptr_t out, int64_t n) {
    mt::launch_xlog2x(S(s), P<double>(out), n);
  });
  m.def("hw_xlog2x_device", [](uintptr_t s, uintptr_t out, int n) {
    mt::launch_hw_xlog2x(S(s), P<float>(out), n);
  });
  m.def("xlog2x_host", [](py::array_t<int64_t> x) {
    auto in = x.unchecked<1>();
    py::array_t<double> out(in.shape(0));
    auto o = out.mutable_unchecked<1>();
    for (py::ssize_t i = 0; i < in.shape(0); ++i) o(i) = mt::xlog2x((uint64_t)in(i));
    return out;
  });
}
