// Exact-threshold engine v2 (exact2.hip): device structures shared with the
// host bindings (exact2_bind.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mt {

// Per-level lists (one set per level parity).
// ctl: int32 {0: K frontier slots, 1: chunk items, 2: split nodes, 3: partition items,
//             4: jobs so far (copy), 5-15: -}
struct XeLists {
  int64_t* pos;     // [KMAX] pre-order position
  int64_t* start;   // [KMAX] segment start (every list)
  int32_t* cnt;     // [KMAX] rows
  int32_t* depth;   // [KMAX]
  int64_t* stats;   // [KMAX][Cs] class counts, or {count, target sum}
  int64_t* minmax;  // [KMAX][2] regression: target min / max (xe_carry)
  int64_t* items;   // [IMAX][4] {slot, segment start, chunk start, chunk count}
  int32_t* ifirst;  // [KMAX + 1] first item of each slot
  int32_t* ctl;     // [16]
};

// Everything a level needs besides the two list sets.
struct XeArgs {
  const uint32_t* E;   // current list buffer [F_loc][n]
  uint32_t* D;         // other list buffer
  const int64_t* Y;    // regression payload [F_loc][n] (current), or null
  int64_t* DY;         // regression payload (other), or null
  const uint32_t* rank_of;  // (unused by the level kernels)
  const void* X;       // features [n][F] (fp32 or fp64): threshold values
  int x64;
  int64_t n;
  int F, f_lo, F_loc;
  int C;               // classes (classification); 0 for regression
  // labels by row when C > 128 (xe_packed_classes): the list entries then carry
  // none and every label read gathers ylab[row]; null when the entries carry them
  const int32_t* ylab;
  int crit;
  int64_t msl;
  const double* xtab;
  int xtab_n;
  // level scratch
  int64_t* tot;        // [IMAX][F_loc][Cc] chunk totals (Cc = C, or 1 target sum)
  int64_t* carry;      // [IMAX][F_loc][Cc]
  int64_t* cmm;        // [IMAX][2] chunk target min / max (regression, local feature 0)
  uint64_t* cbest;     // [IMAX][F_loc][2] chunk best {cost key, position}
  uint32_t* cmin;      // [IMAX][F_loc] two-pass scan: chunk fp32 minimum (ordered bits)
  uint32_t* nmin;      // [KMAX][F_loc] two-pass scan: node fp32 minimum per feature
  float* gthr;         // [KMAX] two-pass scan: node candidate threshold
  int64_t* rec;        // [KMAX][R] split records, R = 6 + (C or 1) + 1
  // partition
  int64_t* split;      // [SMAX][4] {start, count, feature (global), n_left}
  int64_t* pitems;     // [PMAX][4] {split j, segment start, chunk start, chunk count}
  int32_t* pfirst;     // [SMAX + 1]
  uint32_t* flag;      // [(n + 31) / 32] row-direction bits (1: left)
  uint8_t* flagb;      // [(n + 31) / 32 * 32] row-direction bytes, packed into flag (or null)
  // single-pass scans (decoupled look-back): per (item, feature) status words
  // {tag : 30, state : 2 (1 aggregate, 2 inclusive prefix), value : 32}
  uint64_t* pstat;     // [PMAX][F_loc] left counts (partition)
  int32_t* tick;       // [4] {scan ticket, partition ticket, watchdog, -}
  uint32_t tag;        // this level's status tag (30 bits, nonzero)
  // two-class chunk totals counted by the partition (no xe_tot pass over the lists):
  // sitem [SMAX][2] = first next-level item of each split node's frontier child (-1:
  // leaf or finisher job), nctl = the next level's ctl, tot_ready = this level's
  // totals were counted by the previous level's partition; null / 0: xe_tot
  const int32_t* sitem;
  const int32_t* nctl;
  int tot_ready;
};

__host__ __device__ inline int xe_cc(int C) { return C > 0 ? C : 1; }
// record: {gain bits, feature, position, n_left, m, threshold rank, threshold row, left[Cc]}
__host__ __device__ inline int xe_rec_width(int C) { return 7 + xe_cc(C); }

// Planner (one workgroup): the split records of the level -> position space,
// finisher jobs, split list + partition items, the next frontier and its items.
// job row: {segment start, rows, depth, root position, list buffer, stats[Cs]}
struct XePlanArgs {
  XeLists cur, nxt;
  const int64_t* rec;
  int64_t* split;      // [SMAX][4]
  int64_t* pitems;     // [PMAX][4]
  int32_t* pfirst;     // [SMAX + 1]
  int32_t* pos_rec;    // [P][6]
  void* pos_st;        // [P][Cs] int32 class counts / int64 {count, sum}
  double* pos_thr;     // [P] threshold values
  const void* X;
  int x64;
  int F;
  int C;
  int out_buf;         // list buffer this level's partition writes
  int64_t* jobs;       // [JMAX][5 + Cs]
  int32_t* job_count;
  int max_depth;
  int64_t mss, msl, fr;
  int32_t* host_ctl;   // host-mapped {next frontier size, jobs so far, tag}
  int32_t host_tag;
  int32_t* tick;       // XeArgs::tick: the planner rearms both tickets
  int32_t* sitem;      // XeArgs::sitem, or null
};


// launchers (exact2.hip)
int xe_chunk();
int xe_part_units();  // partition wave units (status words) per chunk item
int xe_local_max();
int xe_max_classes();
int xe_packed_classes();
void xe_init(hipStream_t s, const XeLists& L, int64_t n, int Cs, const int64_t* root, int32_t* jc);
void xe_level_scan(hipStream_t s, const XeArgs& a, const XeLists& cur, int items_bound,
                   int slots_bound);
void xe_plan(hipStream_t s, const XePlanArgs& p);
void xe_flag(hipStream_t s, const XeArgs& a, const XeLists& cur, int pitems_bound, int write_right);
void xe_partition(hipStream_t s, const XeArgs& a, const XeLists& cur, int pitems_bound,
                  int splits_bound);
void xe_local_codes(hipStream_t s, const uint32_t* E0, const uint32_t* E1, const int64_t* Y0,
                    const int64_t* Y1, const void* X, int x64, int F, int fg_lo, int64_t n,
                    int F_loc, int f_lo, const int64_t* jobs, int J, int JW, uint8_t* codes_fm,
                    uint8_t* codes_rm, int row_bytes, uint32_t* ent, int64_t* yv,
                    const int32_t* ylab);
void xe_codes_rm(hipStream_t s, const uint8_t* codes_fm, int64_t n, int F, int row_bytes,
                 const int64_t* jobs, int J, int JW, uint8_t* codes_rm);
void xe_fix(hipStream_t s, const uint32_t* E0, const uint32_t* E1, const void* X, int x64, int F,
            int64_t n, int f_lo, int F_loc, const int64_t* jobs, int J, int JW, int32_t* pos_rec,
            double* pos_thr);
void xe_rank(hipStream_t s, int32_t* pos_rec, const double* pos_thr, int64_t P,
             const uint32_t* root_rows, const uint32_t* rank_at, const void* X, int x64, int F,
             int64_t n, int f_lo, int F_loc, uint8_t* resolved, const uint32_t* keys);
void xe_resolved_pack(hipStream_t s, const int32_t* pos_rec, const double* pos_thr, int64_t P,
                      const int32_t* rank, int64_t* rows);
void xe_resolved_scatter(hipStream_t s, const int64_t* rows, int64_t k, int32_t* pos_rec,
                         double* pos_thr);
void xe_emit(hipStream_t s, const uint32_t* keys, const uint32_t* rows, int64_t n, int F_loc,
             int nc, int chunk, const int32_t* cbase, const int32_t* ylab, const int64_t* yfix,
             uint32_t* E, int64_t* Y, uint32_t* rank_at);

}  // namespace mt
