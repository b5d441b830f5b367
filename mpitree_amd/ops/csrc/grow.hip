// Device-driven level loop: the per-level planner.
//
// The reference grows depth-first with one Python recursion per node
// (mpitree/tree/decision_tree.py:93-166). The level-wise engine batches a
// whole depth into a few kernels, but a host-driven loop still pays a device
// round trip and ~100 host numpy operations per level to turn the split
// records into the next level's work lists. Here that bookkeeping runs on the
// GPU: after scan/select, one workgroup (grow_plan_kernel) reads the level's
// split records and writes
//
//   * every decided node into the pre-order position space (see assemble.hip):
//     split nodes, and children that became leaves;
//   * finisher jobs for children with at most ``finisher_rows`` rows;
//   * the partition work list of this level's split nodes;
//   * the next frontier, slot-ordered built-then-derived (the smaller child of
//     a pair is built from rows, the larger derived as parent - sibling),
//     with its histogram items / slab reductions / derive triples and counts.
//
// Every kernel of a level reads its work count from device memory (grids are
// host-known upper bounds), so the host enqueues levels back to back with no
// synchronisation and learns only at the end -- from one lagged 32-byte read
// -- that the frontier is empty.
#include <climits>

#include "common.h"
#include "criterion.h"
#include "grow.h"

namespace mt {

#ifndef MT_PLAN_THREADS
#define MT_PLAN_THREADS 512
#endif
constexpr int kPlanThreads = MT_PLAN_THREADS;  // (variant builds: tools/build_variant.sh)
constexpr int kPlanWaves = kPlanThreads / kWave;

__device__ __forceinline__ int plan_scan_excl(int v, int* s_w, int& total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int incl = (int)wave_incl_scan_u32((uint32_t)v);
  if (lane == kWave - 1) s_w[w] = incl;
  __syncthreads();
  int off = 0, tot = 0;
  for (int k = 0; k < kPlanWaves; ++k) {
    const int x = s_w[k];
    off += k < w ? x : 0;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return off + incl - v;
}

// What happens to one frontier node and its children.
struct Decision {
  bool split;
  int feature, bin;
  int64_t nl, nr;
  int fate[2];  // 0 leaf, 1 finisher job, 2 next frontier
  int built;    // child index built from rows (-1 none), the other alive one is derived
};

__device__ __forceinline__ int plan_rec_width(const PlanArgs& a) {
  return a.reg ? 7 : 5 + 2 * a.C;
}

// finisher job row: {start, rows, depth, root position, buffer, stats[C]}; data-parallel
// fits append {local rows, 2 * split index + side} (start / local rows set after partition)
__device__ __forceinline__ int plan_job_width(const PlanArgs& a) {
  return 5 + a.C + (a.dp ? 2 : 0);
}

// Statistic k of child c (0 left, 1 right) of frontier node i: class counts,
// or {count, fixed-point sum} for regression (the record's left sum at r[5]).
__device__ __forceinline__ int64_t plan_child_stat(const PlanArgs& a, int i, const int64_t* r,
                                                   const int64_t nl, int c, int k) {
  if (a.reg) {
    const int64_t* st = a.cur.stats64 + (int64_t)i * 2;
    if (k == 0) return c == 0 ? nl : st[0] - nl;
    return c == 0 ? r[5] : st[1] - r[5];
  }
  const int64_t lc = r[5 + k];
  return c == 0 ? lc : (int64_t)a.cur.stats[(int64_t)i * a.C + k] - lc;
}

__device__ Decision plan_decide(const PlanArgs& a, int i) {
  const int C = a.C;
  const int R = plan_rec_width(a);
  const int64_t* r = a.rec + (int64_t)i * R;
  Decision d;
  const double gain = __longlong_as_double((long long)r[0]);
  d.split = gain > -__builtin_inf();
  // regression: a node whose targets are all equal is a leaf (purity is only
  // known once its rows are partitioned, so it is checked one level later)
  if (a.reg && a.cur.minmax[(int64_t)i * 2] == a.cur.minmax[(int64_t)i * 2 + 1]) d.split = false;
  d.feature = (int)r[1];
  d.bin = (int)r[2];
  const int64_t m = a.cur.gcnt[i];
  d.nl = r[3];
  d.nr = m - d.nl;
  d.fate[0] = d.fate[1] = 0;
  d.built = -1;
  if (!d.split) return d;
  const int cd = a.cur.depth[i] + 1;
  const bool depth_stop = a.max_depth >= 0 && cd >= a.max_depth;
  for (int c = 0; c < 2; ++c) {
    const int64_t cm = c == 0 ? d.nl : d.nr;
    int nz = 2;  // regression: purity is checked when the child is scanned
    if (!a.reg) {
      nz = 0;
      for (int k = 0; k < C; ++k) nz += plan_child_stat(a, i, r, d.nl, c, k) > 0;
    }
    const bool term = depth_stop || cm < a.mss || cm < 2 * a.msl || nz <= 1;
    d.fate[c] = term ? 0 : ((a.fr > 0 && cm <= a.fr) ? 1 : 2);
  }
  if (d.fate[0] == 2 && d.fate[1] == 2)
    d.built = d.nl <= d.nr ? 0 : 1;  // smaller child from rows (ties: left)
  else if (d.fate[0] == 2)
    d.built = 0;
  else if (d.fate[1] == 2)
    d.built = 1;
  return d;
}

// Workgroup-shared scratch of the planner and the data-parallel fixup kernel.
struct PlanShared {
  int w[kPlanWaves];
  int carry[4];
  long long rows;
  // cooperative expansion of per-node work items: node j of the current chunk
  // owns items [off[j], off[j + 1]); every thread writes items, found by a
  // binary search over the offsets, so one large node does not serialise a pass
  int off[kPlanThreads + 1];
  long long pa[kPlanThreads], pb[kPlanThreads];
  int pc[kPlanThreads];
};

template <typename Emit>
__device__ __forceinline__ void plan_expand(PlanShared& sh, int o_local, int total, Emit emit) {
  const int tid = threadIdx.x;
  sh.off[tid] = o_local;
  if (tid == 0) sh.off[kPlanThreads] = total;
  __syncthreads();
  for (int it = tid; it < total; it += kPlanThreads) {
    int lo = 0, hi = kPlanThreads;  // last j with off[j] <= it
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (sh.off[mid] <= it) lo = mid; else hi = mid;
    }
    emit(lo, it - sh.off[lo]);
  }
  __syncthreads();
}

// Histogram items of the next level's built slots [0, NB) (about 2 items per CU
// over the level's built rows), slab reductions and reduction tasks -> nxt.ctl.
__device__ void plan_hist_items(const PlanArgs& a, PlanShared& sh, int NB) {
  const int tid = threadIdx.x;
  long long built_rows = 0;
  for (int sl = tid; sl < NB; sl += kPlanThreads) built_rows += a.nxt.cnt[sl];
  if (tid == 0) sh.rows = 0;
  __syncthreads();
  {
    long long v = built_rows;
    for (int d = kWave / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
    if (lane_id() == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&sh.rows),
                                  (unsigned long long)v);
  }
  __syncthreads();
  const long long total = sh.rows;
  long long chunk = (total + 2LL * a.n_cu - 1) / (2LL * a.n_cu);
  chunk = chunk < 1024 ? 1024 : (chunk > 65535 ? 65535 : chunk);
  if (tid == 0) {
    sh.carry[0] = 0;  // items
    sh.carry[1] = 0;  // slabs
    sh.carry[2] = 0;  // reductions
    sh.carry[3] = 0;  // reduction tasks
  }
  __syncthreads();
  for (int b0 = 0; b0 < NB; b0 += kPlanThreads) {
    const int sl = b0 + tid;
    int64_t cnt = 0, kk = 0;
    if (sl < NB) {
      cnt = a.nxt.cnt[sl];
      kk = (cnt + chunk - 1) / chunk;
      if (kk < 1) kk = 1;
    }
    const int multi = kk > 1 ? 1 : 0;
    const int nt = multi ? (int)((kk + 15) / 16) : 0;
    // two packed scans: {items, slabs} and {reductions, tasks}. Per chunk the items
    // total <= level rows / chunk + kPlanThreads <= 2 n_cu + 1024 and tasks <= items,
    // so every 16-bit field holds its sum
    int tis, trt;
    const int ois = plan_scan_excl((int)kk | ((multi ? (int)kk : 0) << 16), sh.w, tis);
    const int ort = plan_scan_excl(multi | (nt << 16), sh.w, trt);
    const int ti = tis & 0xffff, tsl = tis >> 16, tr = trt & 0xffff, tt = trt >> 16;
    const int oi_l = ois & 0xffff;
    const int osl = (ois >> 16) + sh.carry[1];
    const int orr = (ort & 0xffff) + sh.carry[2];
    const int ot = (ort >> 16) + sh.carry[3];
    sh.pa[tid] = sl < NB ? a.nxt.start[sl] : 0;
    sh.pb[tid] = cnt;
    sh.pc[tid] = multi ? osl : -1;
    const int ibase = sh.carry[0];
    plan_expand(sh, oi_l, ti, [&](int j, int c) {
      int64_t* it = a.nxt.items + (int64_t)(ibase + sh.off[j] + c) * 4;
      const int64_t c0 = (int64_t)c * chunk;
      const int64_t cn = sh.pb[j] - c0;
      it[0] = b0 + j;
      it[1] = sh.pa[j] + c0;
      it[2] = cn < chunk ? cn : chunk;
      it[3] = sh.pc[j] >= 0 ? sh.pc[j] + c : -1;
    });
    if (sl < NB && multi) {
      int64_t* rr = a.nxt.red + (int64_t)orr * 3;
      rr[0] = sl;
      rr[1] = osl;
      rr[2] = kk;
      for (int t = 0; t < nt; ++t) {
        int64_t* tk = a.nxt.tasks + (int64_t)(ot + t) * 3;
        tk[0] = sl;
        tk[1] = osl + 16 * t;
        tk[2] = (kk - 16 * t) < 16 ? (kk - 16 * t) : 16;
      }
    }
    __syncthreads();
    if (tid == 0) {
      sh.carry[0] += ti;
      sh.carry[1] += tsl;
      sh.carry[2] += tr;
      sh.carry[3] += tt;
    }
    __syncthreads();
  }
  if (tid == 0) {
    a.nxt.ctl[2] = sh.carry[0];
    a.nxt.ctl[3] = sh.carry[2];
    a.nxt.ctl[7] = sh.carry[3];
  }
  __syncthreads();
}

// Regression: min/max work items (4096 rows) over every next-frontier slot -> nxt.ctl[8].
__device__ void plan_minmax_items(const PlanArgs& a, PlanShared& sh, int K2) {
  const int tid = threadIdx.x;
  __syncthreads();
  if (tid == 0) sh.carry[0] = 0;
  __syncthreads();
  for (int b0 = 0; b0 < K2; b0 += kPlanThreads) {
    const int sl = b0 + tid;
    int64_t cnt = 0, kk = 0;
    if (sl < K2) {
      cnt = a.nxt.cnt[sl];
      kk = (cnt + 4095) / 4096;
      if (kk < 1) kk = 1;
    }
    int tm;
    const int om_l = plan_scan_excl((int)kk, sh.w, tm);
    sh.pa[tid] = sl < K2 ? a.nxt.start[sl] : 0;
    sh.pb[tid] = cnt;
    const int mbase = sh.carry[0];
    plan_expand(sh, om_l, tm, [&](int j, int c) {
      int64_t* it = a.nxt.mitems + (int64_t)(mbase + sh.off[j] + c) * 3;
      const int64_t c0 = (int64_t)c * 4096;
      const int64_t cn = sh.pb[j] - c0;
      it[0] = b0 + j;
      it[1] = sh.pa[j] + c0;
      it[2] = cn < 4096 ? cn : 4096;
    });
    __syncthreads();
    if (tid == 0) sh.carry[0] += tm;
    __syncthreads();
  }
  if (tid == 0) a.nxt.ctl[8] = sh.carry[0];
  __syncthreads();
}


// ---- subtree ownership (see OwnArgs in grow.h) -------------------------------
constexpr int kOwnMax = 2048;                // units the switch level can sort in LDS
constexpr int32_t kOwnJob = 0x40000000;      // unit id flag: a finisher job (else a node)

struct OwnShared {
  uint64_t key[kOwnMax];  // {0x7FFFFFFF - rows : 32, root position : 32}: unique, total order
  int32_t unit[kOwnMax];  // frontier slot i, or kOwnJob | job index
  int n, any_next, jobs0, nr;
};

// Pass 0 of the switch level: collect the units (split nodes whose children keep
// growing, with their rows; finisher jobs so far), decide whether this level
// switches, and if so assign the units by greedy LPT (largest first, ties by
// position; each to the least-loaded rank, ties to the lowest), record this
// rank's position ranges and compact the job list to this rank's jobs.
// Returns true (block-uniform) when the level switched.
__device__ bool own_switch(const PlanArgs& a, OwnShared& os, PlanShared& sh, int K, int JW) {
  const int tid = threadIdx.x;
  const int P = a.own.P, me = a.own.rank;
  if (tid == 0) {
    os.n = 0;
    os.any_next = 0;
    os.jobs0 = atomicAdd(a.job_count, 0);
    os.nr = 0;
  }
  __syncthreads();
  const int J0 = os.jobs0;
  for (int i = tid; i < K; i += kPlanThreads) {
    a.own.node_owner[i] = -1;
    const Decision d = plan_decide(a, i);
    if (!d.split) continue;
    int64_t load = 0;
    for (int c = 0; c < 2; ++c) {
      if (d.fate[c] >= 1) load += c == 0 ? d.nl : d.nr;
      if (d.fate[c] == 2) os.any_next = 1;
    }
    if (load > 0) {
      const int u = atomicAdd(&os.n, 1);
      if (u < kOwnMax) {
        os.key[u] = ((uint64_t)(0x7FFFFFFFll - load) << 32) | (uint64_t)(a.cur.pos[i] & 0x7FFFFFFF);
        os.unit[u] = i;
      }
    }
  }
  for (int j = tid; j < J0; j += kPlanThreads) {
    const int64_t* J = a.jobs + (int64_t)j * JW;
    const int u = atomicAdd(&os.n, 1);
    if (u < kOwnMax) {
      os.key[u] = ((uint64_t)(0x7FFFFFFFll - J[1]) << 32) | (uint64_t)(J[3] & 0x7FFFFFFF);
      os.unit[u] = kOwnJob | j;
    }
  }
  __syncthreads();
  const int U = os.n;
  const bool sw = U > 0 && U <= kOwnMax && (U >= a.own.min_units || !os.any_next);
  if (!sw) return false;
  // bitonic sort of the unit keys (ascending: largest rows first)
  int N2 = 1;
  while (N2 < U) N2 <<= 1;
  for (int i = U + tid; i < N2; i += kPlanThreads) {
    os.key[i] = ~0ull;
    os.unit[i] = -1;
  }
  __syncthreads();
  for (int size = 2; size <= N2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < N2; i += kPlanThreads) {
        const int j = i ^ stride;
        if (j > i) {
          const uint64_t ka = os.key[i], kb = os.key[j];
          const bool up = (i & size) == 0;
          if ((ka > kb) == up) {
            os.key[i] = kb;
            os.key[j] = ka;
            const int32_t t = os.unit[i];
            os.unit[i] = os.unit[j];
            os.unit[j] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  // greedy LPT on one wave: lane r holds rank r's load
  if (tid < kWave) {
    const int lane = tid;
    uint64_t load = lane < P ? 0ull : ~0ull >> 9;
    for (int u = 0; u < U; ++u) {
      const uint64_t rows = 0x7FFFFFFFull - (os.key[u] >> 32);
      uint64_t v = (load << 8) | (uint64_t)lane;
      for (int d = kWave / 2; d > 0; d >>= 1) {
        const uint64_t o = (uint64_t)__shfl_xor((long long)v, d, kWave);
        v = o < v ? o : v;
      }
      const int r = (int)(v & 0xffu);
      if (lane == r) load += rows;
      if (lane == 0) {
        const int32_t id = os.unit[u];
        if (id & kOwnJob)
          a.own.job_owner[id & ~kOwnJob] = r;
        else
          a.own.node_owner[id] = r;
      }
    }
    if (lane == me) a.own.state[3] = (int32_t)load;
  }
  __threadfence_block();
  __syncthreads();
  // this rank's position ranges: a node's children subtrees [pos + 1, pos + 2m - 1),
  // a job's subtree [root, root + 2 rows - 1)
  for (int u = tid; u < U; u += kPlanThreads) {
    const int32_t id = os.unit[u];
    int64_t lo, hi;
    bool mine;
    if (id & kOwnJob) {
      const int64_t* J = a.jobs + (int64_t)(id & ~kOwnJob) * JW;
      mine = a.own.job_owner[id & ~kOwnJob] == me;
      lo = J[3];
      hi = J[3] + 2 * J[1] - 1;
    } else {
      mine = a.own.node_owner[id] == me;
      lo = a.cur.pos[id] + 1;
      hi = a.cur.pos[id] + 2 * (int64_t)a.cur.gcnt[id] - 1;
    }
    if (mine) {
      const int k = atomicAdd(&os.nr, 1);
      a.own.ranges[(int64_t)k * 2 + 0] = lo;
      a.own.ranges[(int64_t)k * 2 + 1] = hi;
    }
    if (a.own.segs) {  // every unit's child segments, with its owner (same on every rank)
      int64_t* sg = a.own.segs + (int64_t)u * 6;
      const int64_t owner = (id & kOwnJob) ? a.own.job_owner[id & ~kOwnJob] : a.own.node_owner[id];
      int64_t mid = hi, lo2 = 0, hi2 = 0, own2 = -1;
      if (!(id & kOwnJob)) {  // left child subtree [pos + 1, pos + 2 nl), right the rest
        mid = a.cur.pos[id] + 2 * plan_decide(a, id).nl;
        lo2 = mid;
        hi2 = hi;
        own2 = owner;
      }
      sg[0] = lo;
      sg[1] = mid;
      sg[2] = owner;
      sg[3] = lo2;
      sg[4] = hi2;
      sg[5] = own2;
    }
  }
  __syncthreads();
  const int NR = os.nr;
  for (int k = NR + tid; k < a.own.cap; k += kPlanThreads) {
    a.own.ranges[(int64_t)k * 2 + 0] = 0;
    a.own.ranges[(int64_t)k * 2 + 1] = 0;
  }
  // keep this rank's jobs (stable, in place: each column is read by every row
  // before any row of it is rewritten)
  if (tid == 0) sh.carry[0] = 0;
  __syncthreads();
  for (int b0 = 0; b0 < J0; b0 += kPlanThreads) {
    const int j = b0 + tid;
    const bool keep = j < J0 && a.own.job_owner[j] == me;
    int tot;
    const int o = plan_scan_excl(keep ? 1 : 0, sh.w, tot) + sh.carry[0];
    for (int k = 0; k < JW; ++k) {
      const int64_t v = keep ? a.jobs[(int64_t)j * JW + k] : 0;
      __syncthreads();
      if (keep) a.jobs[(int64_t)o * JW + k] = v;
      __syncthreads();
    }
    if (tid == 0) sh.carry[0] += tot;
    __syncthreads();
  }
  if (tid == 0) {
    *a.job_count = sh.carry[0];
    a.own.state[0] = 1;
    a.own.state[1] = NR;
    a.own.state[2] = U;
  }
  __threadfence_block();
  __syncthreads();
  return true;
}

// Fused selection: the split record of every frontier node from the scan's
// per-feature results (what select_kernel computes from the histograms): node
// term from the class totals (x log2 x evaluated, as the select kernel does),
// best gain over the features in ascending order with a strict > (ties to the
// lowest feature), the winning bin and its left counts. One thread per node.
__device__ void plan_fused_select(const PlanArgs& a, int K) {
  const int C = a.C;
  const int R = 5 + 2 * C;
  const int F = a.sel_F;
  int64_t* rec = const_cast<int64_t*>(a.rec);
  constexpr int kU = 32;  // cost loads in flight per thread
  for (int i = threadIdx.x; i < K; i += kPlanThreads) {
    int64_t tot[2];
    tot[0] = a.sel_tot[(int64_t)i * 4 + 0];
    tot[1] = C > 1 ? a.sel_tot[(int64_t)i * 4 + 1] : 0;
    const int64_t mm = tot[0] + tot[1];
    const double pterm = reinterpret_cast<const double*>(a.sel_tot)[(int64_t)i * 2 + 1];
    double g = -__builtin_inf();
    int bf = -1;
    for (int f0 = 0; f0 < F; f0 += kU) {
      double cv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) cv[u] = a.sel_cost[(int64_t)i * F + min(f0 + u, F - 1)];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (f0 + u < F && cv[u] < __builtin_inf()) {
          const double gf = pterm - cv[u];
          if (gf > g) {
            g = gf;
            bf = f0 + u;
          }
        }
      }
    }
    int64_t* out = rec + (int64_t)i * R;
    const bool ok = g > -__builtin_inf();
    out[0] = (int64_t)double_to_bits(g);
    out[1] = ok ? bf : -1;
    out[2] = ok ? a.sel_bins[(int64_t)i * F + bf] : -1;
    int64_t nl = 0;
    for (int c = 0; c < C; ++c) {
      const int64_t l = ok ? a.sel_left[((int64_t)i * F + bf) * 2 + c] : 0;
      out[5 + c] = l;
      out[5 + C + c] = tot[c];
      nl += l;
    }
    out[3] = nl;
    out[4] = mm;
  }
  __syncthreads();  // (records read by other threads below, e.g. the ownership pass)
}

// MT_PLAN_PROF (variant builds, bench/plan_prof.py): per-phase wall-clock ticks
// (100 MHz) summed over launches, read back with mt_plan_prof_read
#ifdef MT_PLAN_PROF
__device__ unsigned long long g_plan_prof[32];
#define PLAN_MARK(k)                                                   \
  do {                                                                 \
    if (threadIdx.x == 0) {                                            \
      const unsigned long long t_ = wall_clock64();                    \
      atomicAdd(&g_plan_prof[k], t_ - plan_t_prev_);                   \
      plan_t_prev_ = t_;                                               \
    }                                                                  \
  } while (0)
#else
#define PLAN_MARK(k)
#endif

__global__ __launch_bounds__(kPlanThreads) void grow_plan_kernel(PlanArgs a) {
  __shared__ PlanShared sh;
  const int tid = threadIdx.x;
#ifdef MT_PLAN_PROF
  unsigned long long plan_t_prev_ = wall_clock64();
  if (tid == 0) atomicAdd(&g_plan_prof[31], 1ull);
#endif
  const int C = a.C;
  const int JW = plan_job_width(a);
  const int K = a.cur.ctl[0];
  if (a.sel_left) plan_fused_select(a, K);
  PLAN_MARK(0);
  // ---- pass 0 (subtree ownership, before the switch): maybe switch this level
  __shared__ OwnShared own_sh;
  bool own_sw = false;
  if (a.own.P > 1 && !a.dp && a.own.state[0] == 0) own_sw = own_switch(a, own_sh, sh, K, JW);
  // a node this rank grows: every node, except at the switch level the units
  // other ranks own (nodes that are no unit -- leaves, splits into two leaves --
  // stay replicated)
  auto active = [&](int i) {
    return !own_sw || a.own.node_owner[i] < 0 || a.own.node_owner[i] == a.own.rank;
  };
  const bool build_all = a.derive_free || (own_sw && a.own.build_all);
  // decisions of this level; at the switch (jobs_at_switch) the children that
  // would keep growing become finisher jobs: the rank's own work is its jobs
  auto decide = [&](int i) {
    Decision d = plan_decide(a, i);
    if (own_sw && a.own.jobs_at_switch > 0 && d.split) {
      for (int c = 0; c < 2; ++c) {
        const int64_t cm = c == 0 ? d.nl : d.nr;
        if (d.fate[c] == 2 && cm <= a.own.jobs_at_switch) d.fate[c] = 1;
      }
      if (d.fate[0] == 2 && d.fate[1] == 2)
        d.built = d.nl <= d.nr ? 0 : 1;
      else if (d.fate[0] == 2)
        d.built = 0;
      else if (d.fate[1] == 2)
        d.built = 1;
      else
        d.built = -1;
    }
    return d;
  };
  PLAN_MARK(1);
  // ---- pass 1: totals (built / derived next-frontier children, split nodes);
  // a frontier of at most kPlanThreads nodes takes its total from pass 2's scan
  // (one decision per node instead of two)
  const bool one_chunk = K <= kPlanThreads;
  int nb_tot = 0;
  for (int b0 = 0; b0 < K && !one_chunk; b0 += kPlanThreads) {
    const int i = b0 + tid;
    int nb = 0;
    if (i < K && active(i)) {
      const Decision d = decide(i);
      nb = d.built < 0 ? 0 : (build_all && d.fate[0] == 2 && d.fate[1] == 2) ? 2 : 1;
    }
    int t;
    plan_scan_excl(nb, sh.w, t);
    nb_tot += t;
  }
  int NB = nb_tot;
  if (tid == 0) {
    sh.carry[0] = 0;  // built slots
    sh.carry[1] = 0;  // derived slots
    sh.carry[2] = 0;  // split nodes
    if (a.dp) a.nxt.ctl[10] = atomicAdd(a.job_count, 0);  // jobs before this level (dp fixup)
  }
  __syncthreads();
  PLAN_MARK(2);
  // ---- pass 2: write decided nodes, jobs, split list, next frontier, derive list
  for (int b0 = 0; b0 < K; b0 += kPlanThreads) {
    const int i = b0 + tid;
    Decision d;
    d.split = false;
    d.built = -1;
    d.fate[0] = d.fate[1] = 0;
    if (i < K) d = decide(i);
    const bool act = i < K && active(i);
    // (switch after feature-parallel levels: both children of a pair are built)
    const bool both = build_all && d.fate[0] == 2 && d.fate[1] == 2;
    const int nb = act && d.built >= 0 ? (both ? 2 : 1) : 0;
    const int nd = act && (d.fate[0] == 2 && d.fate[1] == 2) && !both ? 1 : 0;
    const int ns = act && d.split ? 1 : 0;
    // built / derived offsets share one scan (each field <= kPlanThreads < 2^16)
    int tbd, ts;
    const int obd = plan_scan_excl(nb | (nd << 16), sh.w, tbd);
    const int tb = tbd & 0xffff, td = tbd >> 16;
    if (one_chunk) NB = tb;  // (block-uniform: the scan's total)
    const int ob = (obd & 0xffff) + sh.carry[0];
    const int od = (obd >> 16) + sh.carry[1];
    const int os = plan_scan_excl(ns, sh.w, ts) + sh.carry[2];
    if (i < K) {
      const int64_t pos = a.cur.pos[i];
      const int64_t start = a.cur.start[i];
      const int64_t m = a.cur.gcnt[i];      // global rows (decisions, positions)
      const int64_t mloc = a.cur.cnt[i];    // this rank's segment (== m unless dp)
      const int depth = a.cur.depth[i];
      int32_t* P = a.pos_rec + pos * 6;
      const int64_t* r = a.rec + (int64_t)i * plan_rec_width(a);
      if (a.reg) {
        a.pos_st64[pos * 2 + 0] = a.cur.stats64[(int64_t)i * 2 + 0];
        a.pos_st64[pos * 2 + 1] = a.cur.stats64[(int64_t)i * 2 + 1];
      } else {
        for (int k = 0; k < C; ++k) a.pos_st[pos * C + k] = a.cur.stats[(int64_t)i * C + k];
      }
      P[4] = depth;
      P[5] = (int32_t)m;
      if (!d.split) {
        P[0] = -1;
        P[1] = -1;
        P[2] = -1;
        P[3] = -1;
      } else {
        const int64_t cpos[2] = {pos + 1, pos + 2 * d.nl};
        P[0] = d.feature;
        P[1] = d.bin;
        P[2] = (int32_t)cpos[0];
        P[3] = (int32_t)cpos[1];
      }
      if (d.split && act) {
        const int64_t cpos[2] = {pos + 1, pos + 2 * d.nl};
        // partition list (this rank's rows of the node)
        int64_t* S = a.split + (int64_t)os * 4;
        S[0] = start;
        S[1] = mloc;
        S[2] = d.feature;
        S[3] = d.bin;
        a.cursors[os * 2 + 0] = (int32_t)start;
        a.cursors[os * 2 + 1] = (int32_t)(start + mloc);
        const int cd = depth + 1;
        int slot[2] = {-1, -1};
        if (d.built >= 0) {
          slot[d.built] = ob;
          if (nd) slot[1 - d.built] = NB + od;
          if (both) slot[1 - d.built] = ob + 1;
        }
        for (int c = 0; c < 2; ++c) {
          const int64_t cm = c == 0 ? d.nl : d.nr;
          const int64_t cs = c == 0 ? start : start + d.nl;
          if (d.fate[c] == 0) {  // leaf: write it now
            int32_t* Q = a.pos_rec + cpos[c] * 6;
            Q[0] = -1;
            Q[1] = -1;
            Q[2] = -1;
            Q[3] = -1;
            Q[4] = cd;
            Q[5] = (int32_t)cm;
            if (a.reg) {
              a.pos_st64[cpos[c] * 2 + 0] = plan_child_stat(a, i, r, d.nl, c, 0);
              a.pos_st64[cpos[c] * 2 + 1] = plan_child_stat(a, i, r, d.nl, c, 1);
            } else {
              for (int k = 0; k < C; ++k)
                a.pos_st[cpos[c] * C + k] = (int32_t)plan_child_stat(a, i, r, d.nl, c, k);
            }
          } else if (d.fate[c] == 1) {  // finisher job
            const int j = atomicAdd(a.job_count, 1);
            int64_t* J = a.jobs + (int64_t)j * JW;
            J[0] = a.dp ? 0 : cs;
            J[1] = cm;
            J[2] = cd;
            J[3] = cpos[c];
            J[4] = a.out_buf;  // the child's rows live where this level partitions to
            for (int k = 0; k < C; ++k) J[5 + k] = plan_child_stat(a, i, r, d.nl, c, k);
            if (a.dp) {
              J[5 + C] = 0;
              J[6 + C] = 2 * os + c;
            }
          } else {  // next frontier
            const int sl = slot[c];
            a.nxt.pos[sl] = cpos[c];
            a.nxt.start[sl] = a.dp ? 0 : cs;
            a.nxt.cnt[sl] = (int32_t)(a.dp ? 0 : cm);
            a.nxt.gcnt[sl] = (int32_t)cm;
            a.nxt.src[sl] = 2 * os + c;
            a.nxt.depth[sl] = cd;
            if (a.reg) {
              a.nxt.stats64[(int64_t)sl * 2 + 0] = plan_child_stat(a, i, r, d.nl, c, 0);
              a.nxt.stats64[(int64_t)sl * 2 + 1] = plan_child_stat(a, i, r, d.nl, c, 1);
              a.nxt.minmax[(int64_t)sl * 2 + 0] = LLONG_MAX;
              a.nxt.minmax[(int64_t)sl * 2 + 1] = LLONG_MIN;
            } else {
              for (int k = 0; k < C; ++k)
                a.nxt.stats[(int64_t)sl * C + k] = (int32_t)plan_child_stat(a, i, r, d.nl, c, k);
            }
            if (c != d.built && !both) {  // derived: parent slot i, sibling built slot
              int64_t* D = a.nxt.der + (int64_t)(sl - NB) * 3;
              D[0] = sl;
              D[1] = i;
              D[2] = slot[d.built];
            }
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      sh.carry[0] += tb;
      sh.carry[1] += td;
      sh.carry[2] += ts;
    }
    __syncthreads();
  }
  const int ND = sh.carry[1];
  const int NS = sh.carry[2];
  const int K2 = NB + ND;
  __threadfence_block();  // nxt.start / cnt written above are read by other threads below
  __syncthreads();
  PLAN_MARK(3);
  // ---- pass 3: histogram items of the next level's built slots (dp: after the partition)
  if (!a.dp) plan_hist_items(a, sh, NB);
  PLAN_MARK(4);
  // ---- pass 4: partition items of this level's split nodes (kPartChunk rows each)
  __syncthreads();
  if (tid == 0) sh.carry[3] = 0;
  __syncthreads();
  for (int b0 = 0; b0 < NS; b0 += kPlanThreads) {
    const int j = b0 + tid;
    int64_t cnt = 0, kk = 0;
    if (j < NS) {
      cnt = a.split[(int64_t)j * 4 + 1];
      kk = (cnt + kPartChunk - 1) / kPartChunk;
      if (kk < 1) kk = 1;
    }
    int tp;
    const int op_l = plan_scan_excl((int)kk, sh.w, tp);
    sh.pa[tid] = j < NS ? a.split[(int64_t)j * 4 + 0] : 0;
    sh.pb[tid] = cnt;
    const int pbase = sh.carry[3];
    plan_expand(sh, op_l, tp, [&](int jj, int c) {
      int64_t* it = a.pitems + (int64_t)(pbase + sh.off[jj] + c) * 3;
      const int64_t c0 = (int64_t)c * kPartChunk;
      const int64_t cn = sh.pb[jj] - c0;
      it[0] = b0 + jj;
      it[1] = sh.pa[jj] + c0;
      it[2] = cn < kPartChunk ? cn : kPartChunk;
    });
    __syncthreads();
    if (tid == 0) sh.carry[3] += tp;
    __syncthreads();
  }
  const int n_pitems = sh.carry[3];
  PLAN_MARK(5);
  // ---- pass 5 (regression): min/max work items over every next-frontier slot
  if (a.reg && !a.dp) plan_minmax_items(a, sh, K2);
  if (tid == 0) {
    if (!a.reg) a.nxt.ctl[8] = 0;
    a.nxt.ctl[0] = K2;
    a.nxt.ctl[1] = NB;
    a.nxt.ctl[4] = ND;
    a.nxt.ctl[5] = 0;
    a.nxt.ctl[6] = 0;
    const int jobs_so_far = atomicAdd(a.job_count, 0);
    a.nxt.ctl[9] = jobs_so_far;  // finisher jobs so far
    a.pctl[0] = NS;
    a.pctl[1] = n_pitems;
    if (a.host_ctl) {  // the host's lagged termination read, stored straight to host memory
      if (a.own.P > 1) {  // {switched, units at the switch, rows owned}
        __hip_atomic_store(a.host_ctl + 3, a.own.state[0], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.host_ctl + 4, a.own.state[2], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.host_ctl + 5, a.own.state[3], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        __hip_atomic_store(a.host_ctl + 3, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __hip_atomic_store(a.host_ctl + 1, jobs_so_far, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.host_ctl, K2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
      __hip_atomic_store(a.host_ctl + 2, a.host_tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  PLAN_MARK(6);
}

#ifdef MT_PLAN_PROF
extern "C" void mt_plan_prof_read(unsigned long long* out) {
  MT_HIP_CHECK(hipDeviceSynchronize());
  MT_HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_plan_prof), sizeof(g_plan_prof)));
  const unsigned long long z[32] = {};
  MT_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_plan_prof), z, sizeof(z)));
}
#endif

// Data-parallel levels: after this rank's partition, every next-frontier slot
// and every job appended this level learns its local row segment from its
// parent's split cursors (left child: [start, cursor0), right: [cursor0, end)),
// then the next level's histogram (and regression min/max) work items are built
// from the local counts. One workgroup, like the planner.
__global__ __launch_bounds__(kPlanThreads) void grow_dp_fixup_kernel(PlanArgs a) {
  __shared__ PlanShared sh;
  const int tid = threadIdx.x;
  const int K2 = a.nxt.ctl[0];
  const int NB = a.nxt.ctl[1];
  const int j0 = a.nxt.ctl[10], j1 = a.nxt.ctl[9];
  const int C = a.C;
  const int JW = plan_job_width(a);
  auto seg = [&](int src, int64_t& st, int64_t& cn) {
    const int j = src >> 1, c = src & 1;
    const int64_t s0 = a.split[(int64_t)j * 4 + 0];
    const int64_t ml = a.split[(int64_t)j * 4 + 1];
    const int64_t nl = (int64_t)a.cursors[j * 2 + 0] - s0;
    st = c ? s0 + nl : s0;
    cn = c ? ml - nl : nl;
  };
  for (int sl = tid; sl < K2; sl += kPlanThreads) {
    int64_t st, cn;
    seg(a.nxt.src[sl], st, cn);
    a.nxt.start[sl] = st;
    a.nxt.cnt[sl] = (int32_t)cn;
  }
  for (int t = j0 + tid; t < j1; t += kPlanThreads) {
    int64_t* J = a.jobs + (int64_t)t * JW;
    int64_t st, cn;
    seg((int)J[6 + C], st, cn);
    J[0] = st;
    J[5 + C] = cn;
  }
  __threadfence_block();
  __syncthreads();
  plan_hist_items(a, sh, NB);
  if (a.reg) plan_minmax_items(a, sh, K2);
}

// Feature-parallel levels: every rank scanned its own feature block; the
// all-gathered records g[P][KB][R] are reduced per node to the best split
// (max gain; ties to the lowest rank = the lowest feature, as select_kernel
// breaks ties within a rank), written to rec[K][R].
__global__ __launch_bounds__(256) void fp_combine_kernel(const int64_t* __restrict__ g, int P,
                                                         int KB, int R,
                                                         const int32_t* __restrict__ dcount,
                                                         int64_t* __restrict__ rec) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *dcount || i >= KB) return;
  int best = 0;
  double bg = __longlong_as_double((long long)g[(int64_t)i * R]);
  for (int r = 1; r < P; ++r) {
    const double gr = __longlong_as_double((long long)g[((int64_t)r * KB + i) * R]);
    if (gr > bg) {
      bg = gr;
      best = r;
    }
  }
  const int64_t* src = g + ((int64_t)best * KB + i) * R;
  for (int k = 0; k < R; ++k) rec[(int64_t)i * R + k] = src[k];
}

void launch_fp_combine(hipStream_t stream, const int64_t* g, int P, int KB, int R,
                       const int32_t* dcount, int64_t* rec) {
  if (KB <= 0) return;
  hipLaunchKernelGGL(fp_combine_kernel, dim3((KB + 255) / 256), dim3(256), 0, stream, g, P, KB,
                     R, dcount, rec);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_grow_dp_fixup(hipStream_t stream, const PlanArgs& a) {
  hipLaunchKernelGGL(grow_dp_fixup_kernel, dim3(1), dim3(kPlanThreads), 0, stream, a);
  MT_HIP_CHECK(hipGetLastError());
}

// Level 0 (the root, built from rows) in one launch: root stats come from a
// small device array (classification: C counts; regression: count, sum, min, max).
__global__ __launch_bounds__(256) void grow_init_kernel(LevelLists L, int64_t n, int64_t n_global,
                                                        int64_t chunk, int C, int reg,
                                                        const int64_t* __restrict__ root,
                                                        int32_t* __restrict__ job_count) {
  const int64_t k = (n + chunk - 1) / chunk;
  const int64_t nt = k > 1 ? (k + 15) / 16 : 0;
  for (int64_t i = threadIdx.x; i < k; i += blockDim.x) {
    int64_t* it = L.items + i * 4;
    it[0] = 0;
    it[1] = i * chunk;
    it[2] = (n - i * chunk) < chunk ? (n - i * chunk) : chunk;
    it[3] = k > 1 ? i : -1;
  }
  for (int64_t t = threadIdx.x; t < nt; t += blockDim.x) {
    int64_t* tk = L.tasks + t * 3;
    tk[0] = 0;
    tk[1] = 16 * t;
    tk[2] = (k - 16 * t) < 16 ? (k - 16 * t) : 16;
  }
  if (threadIdx.x == 0) {
    *job_count = 0;
    L.pos[0] = 0;
    L.start[0] = 0;
    L.cnt[0] = (int32_t)n;  // this rank's rows (all of them unless row-sharded)
    L.gcnt[0] = (int32_t)n_global;
    L.src[0] = 0;
    L.depth[0] = 0;
    if (reg) {
      L.stats64[0] = root[0];
      L.stats64[1] = root[1];
      L.minmax[0] = root[2];
      L.minmax[1] = root[3];
    } else {
      for (int c = 0; c < C; ++c) L.stats[c] = (int32_t)root[c];
    }
    if (k > 1) {
      L.red[0] = 0;
      L.red[1] = 0;
      L.red[2] = k;
    }
    for (int i = 0; i < 16; ++i) L.ctl[i] = 0;
    L.ctl[0] = 1;
    L.ctl[1] = 1;
    L.ctl[2] = (int32_t)k;
    L.ctl[3] = k > 1 ? 1 : 0;
    L.ctl[7] = (int32_t)nt;
  }
}

void launch_grow_init(hipStream_t stream, const LevelLists& L, int64_t n, int64_t n_global,
                      int64_t chunk, int C, int reg, const int64_t* root, int32_t* job_count) {
  hipLaunchKernelGGL(grow_init_kernel, dim3(1), dim3(256), 0, stream, L, n, n_global, chunk, C,
                     reg, root, job_count);
  MT_HIP_CHECK(hipGetLastError());
}

// Finisher job order: largest subtree first, ties by root position -- a total
// order independent of the planner's (atomic, racy) append order, so every
// rank of a multi-GPU fit derives the same job list and job ownership. One
// workgroup bitonic-sorts 64-bit keys {0xFFFF - rows : 16, root position : 31,
// index : 13} in LDS and gathers the rows; it also zeroes the finisher's work
// counters.
constexpr int kSortMax = 8192;

__global__ __launch_bounds__(1024) void job_sort_kernel(const int64_t* __restrict__ jobs, int J,
                                                        int W, int64_t* __restrict__ out,
                                                        int32_t* __restrict__ counters) {
  extern __shared__ __align__(16) uint8_t smem[];
  uint64_t* key = reinterpret_cast<uint64_t*>(smem);  // [kSortMax]
  int N2 = 1;
  while (N2 < J) N2 <<= 1;
  for (int i = threadIdx.x; i < N2; i += 1024) {
    uint64_t k = ~0ull;
    if (i < J) {
      const int64_t c = jobs[(int64_t)i * W + 1];
      const uint64_t cc = c > 0xFFFF ? 0xFFFFull : (uint64_t)c;
      const uint64_t pos = (uint64_t)jobs[(int64_t)i * W + 3] & 0x7FFFFFFFull;
      k = ((0xFFFFull - cc) << 44) | (pos << 13) | (uint64_t)i;
    }
    key[i] = k;
  }
  if (threadIdx.x < kFinCounterWords) counters[threadIdx.x] = 0;
  __syncthreads();
  for (int size = 2; size <= N2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < N2; i += 1024) {
        const int j = i ^ stride;
        if (j > i) {
          const uint64_t a = key[i], b = key[j];
          const bool up = (i & size) == 0;
          if ((a > b) == up) {
            key[i] = b;
            key[j] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int e = threadIdx.x; e < J * W; e += 1024) {
    const int r = e / W, c = e - r * W;
    out[e] = jobs[(int64_t)(key[r] & 0x1FFFull) * W + c];
  }
}

int job_sort_max() { return kSortMax; }

void launch_job_sort(hipStream_t stream, const int64_t* jobs, int J, int W, int64_t* out,
                     int32_t* counters) {
  if (J > kSortMax) throw std::runtime_error("job_sort: too many jobs for one workgroup");
  int N2 = 1;
  while (N2 < J) N2 <<= 1;
  const int lds = N2 * (int)sizeof(uint64_t);
  MT_HIP_CHECK(mt_set_max_lds((const void*)job_sort_kernel, kSortMax * 8));
  hipLaunchKernelGGL(job_sort_kernel, dim3(1), dim3(1024), lds, stream, jobs, J, W, out, counters);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_grow_plan(hipStream_t stream, const PlanArgs& a) {
  hipLaunchKernelGGL(grow_plan_kernel, dim3(1), dim3(kPlanThreads), 0, stream, a);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
