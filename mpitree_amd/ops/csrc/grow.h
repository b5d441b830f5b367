// Level-loop work lists and planner arguments (grow.hip), shared with the
// host bindings.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mt {

// The finisher's int32 work counters; words that different workgroups update
// concurrently sit on separate 128-byte lines (see finish.hip).
// rows per partition work item (one workgroup): items of one node share its two
// cursor atomics, so fewer, larger items contend less on that cache line
constexpr int kPartChunk = 4096;
constexpr int kFinCounterWords = 128;
// job_counter words: the claim cursor (0), the tiny-subtree count / cursor, the
// {completed, handed off} queue word, the finished epoch and the watchdog, each
// on its own 128-B line (the regression finisher keeps its tiny words at 1, 2)
constexpr int kFinCtrTinyCount = 32;
// tiny-subtree records a block-finisher workgroup reserves per global atomic (a
// returning device-scope atomic costs ~1-3 us under load, on thread 0's serial
// path between two barriers); unused reserved records are left with m = 0 and
// the tiny kernels skip them. The tiny list holds J + rows / 2 + grid * this.
constexpr int kFinTinyBatch = 16;
constexpr int kFinCtrQueue = 64;
constexpr int kFinCtrFinished = 96;
constexpr int kFinCtrWatch = 100;


// Level work lists (one set per level parity). ctl: int32
// {0: K frontier nodes, 1: built nodes, 2: hist items, 3: slab reductions,
//  4: derive triples, 5: split nodes, 6: partition items, 7: reduction tasks,
//  8: min/max items (regression), 9-15: -}
struct LevelLists {
  int64_t* pos;     // [KMAX] pre-order position of each frontier slot
  int64_t* start;   // [KMAX] row segment start
  int32_t* cnt;     // [KMAX] rows
  int32_t* depth;   // [KMAX]
  int32_t* stats;   // [KMAX][C] class counts (classification)
  int64_t* items;   // [IMAX][4] {slot, start, count, dest slab or -1}
  int64_t* red;     // [KMAX][3] {slot, first slab, slabs}
  int64_t* der;     // [KMAX][3] {slot, parent slot (previous level), sibling slot}
  int64_t* tasks;   // [TMAX][3] {slot, first slab, <= 16 slabs} slab-reduction tasks
  int32_t* ctl;     // [16]
  int64_t* stats64; // [KMAX][2] {count, fixed-point target sum} (regression)
  int64_t* minmax;  // [KMAX][2] target min / max of the slot's rows (regression)
  int64_t* mitems;  // [MMAX][3] {slot, start, count} min/max work items (regression)
  // global row count of each slot (decisions, positions, job sizes). Row-replicated
  // fits alias it to cnt; row-sharded (data-parallel) fits keep this rank's local
  // segment in start / cnt, filled after the partition by grow_dp_fixup_kernel
  int32_t* gcnt;    // [KMAX]
  int32_t* src;     // [KMAX] 2 * (parent's split index) + side (data-parallel only)
};

// Subtree ownership (multi-GPU "subtree" / "auto" fits with replicated rows):
// the level loop runs replicated until the first level whose *units* -- split
// nodes with children that keep growing, plus finisher jobs created so far --
// number at least min_units (or the frontier ends); that level's planner
// assigns the units to ranks by greedy longest-processing-time on row counts
// (every rank computes the same assignment from the same replicated state) and
// from then on each rank grows only its own units. A unit's nodes occupy one
// contiguous pre-order position range, so the ranks' outputs are disjoint
// ranges of the position space.
struct OwnArgs {
  int P;             // ranks (>= 2: ownership on)
  int rank;
  int min_units;     // switch at the first level with at least this many units
  int cap;           // capacity of ranges / of the LPT (units beyond it: no switch)
  int32_t* state;    // [4] {switched (0/1), owned ranges, units at the switch, rows owned}
  int64_t* ranges;   // [cap][2] this rank's position ranges [lo, hi); unused rows {0, 0}
  int32_t* node_owner;  // [KMAX] scratch: owner of frontier node i at the switch
  int32_t* job_owner;   // [JMAX] scratch: owner of job j at the switch
  // > 0: at the switch level every owned child that would keep growing in the
  // level loop becomes a finisher job instead (when it has at most this many
  // rows): the rank's own work is its finisher jobs, no own levels
  int jobs_at_switch = 0;
  // (optional) [2 * cap][3] every unit's position segments {lo, hi, owner}, in unit
  // order: a node unit's left and right child subtrees, a job unit's subtree and an
  // empty {0, 0, -1}; the node-local shared-host assembly ranks its own nodes with
  // them (assemble.hip shm_*)
  int64_t* segs = nullptr;
  // 1: the levels before the switch were feature-parallel (each rank holds only
  // its feature block of the histograms), so at the switch every next-frontier
  // child is built from rows (no larger sibling is derived from a parent)
  int build_all = 0;
};

struct PlanArgs {
  LevelLists cur, nxt;
  const int64_t* rec;  // [KMAX][5 + 2C] split records of the current level
  int64_t* split;      // [KMAX][4] {start, count, feature, bin}
  int64_t* pitems;     // [PMAX][3] {split j, start, count}
  int32_t* cursors;    // [KMAX][2]
  int32_t* pctl;       // [2] {split nodes, partition items} (aliases cur.ctl + 5)
  int32_t* pos_rec;    // [P][6]
  int32_t* pos_st;     // [P][C] class counts (classification)
  int64_t* pos_st64;   // [P][2] {count, sum} (regression)
  int reg;
  int out_buf;         // row buffer (0 idx, 1 tmp) this level's partition writes
  int64_t* jobs;       // [JMAX][5 + C] finisher jobs
  int32_t* job_count;
  int C, max_depth, n_cu;
  int64_t mss, msl, fr;
  int32_t* host_ctl;   // [6] host-mapped {next frontier size, jobs so far, tag, switched,
                       //  units at the switch, rows owned}
  int32_t host_tag;    // written last: the host polls it to know the slot is complete
  int dp;              // rows sharded across ranks: local segments fixed up after partition
  OwnArgs own;         // subtree ownership (own.P < 2: off)
  // fused selection (two-class levels with no collective between scan and plan):
  // the planner builds each node's split record (``rec``) itself from the scan's
  // per-feature results -- cost / bin [K][F], left counts at the best bin
  // [K][F][2], node class totals and node term [K][4] = {t0, t1, term (f64)} --
  // and no select kernel runs
  const double* sel_cost = nullptr;
  const int32_t* sel_bins = nullptr;
  const int32_t* sel_left = nullptr;
  const int32_t* sel_tot = nullptr;
  int sel_F = 0;
  int crit = 0;
  // 1: every next-frontier child is built from rows, none derived (one histogram
  // buffer for both level parities: many-class fits whose two would not fit)
  int derive_free = 0;
};

// tiny-subtree records by rows descending (misc.hip): order[] for the tiny kernels
void launch_tiny_order(hipStream_t stream, const int64_t* tiny, const int32_t* count,
                       int32_t* scratch, int32_t* order, int grid);

}  // namespace mt
