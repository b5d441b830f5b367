// Subtree finisher: one workgroup grows an entire small subtree on gfx950.
//
// The reference recurses node by node to the leaves
// (mpitree/tree/decision_tree.py:150-164), and its parallel version hands
// whole subtrees to MPI sub-communicators (:446-477). Here, once a frontier
// node has at most ``finisher_rows`` rows, the level-wise engine stops
// launching per-level kernels for it and enqueues it as a *job*; a persistent
// grid of 256-thread workgroups (two per CU, so each CU overlaps two
// independent node pipelines) pulls jobs, largest first, from an atomic
// counter and grows each subtree depth-first with no further launches or
// host round trips:
//
//   per node: LDS histogram of all features (two 16-bit classes per word) ->
//   wave-per-feature prefix scan with the shared integer-form criterion and
//   an LDS-resident x*log2(x) table -> workgroup argmax (ties: lowest
//   feature) -> unstable partition of the node's rows from one row buffer
//   into the other (ping-pong, no copy-back) -> child records, terminal
//   checks, push the larger child first so the DFS stack stays O(log rows).
//
// Class counts travel on the DFS stack (known from the parent's split), so a
// node needs five workgroup barriers. Output is addressed by pre-order
// position: a subtree of r rows has at most 2r - 1 nodes, so a node at
// position p with n_left left rows puts its left child at p + 1 and its right
// child at p + 2 n_left. Every position is fixed by row counts alone -- no
// allocation counter, no renumbering -- and compacting the written positions
// (assemble.hip) yields the tree in exact pre-order, bitwise deterministic.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "criterion.h"
#include "tiny_sort.h"
#include "grow.h"

namespace mt {

// threads per finisher workgroup: 512 (two per CU). A 1024-thread variant where two
// 512-thread workgroups fit a CU and an in-kernel tiny-subtree queue were measured
// slower (profiles/kernel_experiments.md); 1024 threads run where only one fits.
constexpr int kFinThreadsSmall = 512;
constexpr int kFinThreadsWide = 1024;  // one workgroup per CU (F = 128 histograms)
// job_counter word layout: kFinCtr* in grow.h (int32 [kFinCounterWords], zeroed
// before each launch)
constexpr int kFinStack = 40;    // >= log2(max job rows) + 2
constexpr int kFinMaxC = 256;    // classes of the full-width histogram layout
// past kFinMaxC classes the jobs hold at most kFinClassJobRows rows, so every
// node has at most that many present classes and counts below 256: its
// compacted histogram (four 8-bit counts a word) is sized like one of
// kFinClassJobRows classes, whatever C is
constexpr int kFinClassJobRows = 255;
constexpr int kFinStackC = 16;   // C <= this: DFS-stack class counts in LDS, else global scratch
constexpr int kFinMaxB = 4096;   // bins (16-bit codes past 256: multi-pass scans, feature tiles)
constexpr int kTinyMaxC = 16;    // classes supported by the generic tiny kernel
constexpr int kFinTab = 1024;    // LDS x*log2(x) entries
// MT_FIN_UNROLL / MT_FIN_PAIR / MT_TINY_SMALL: compile-time overrides for variant
// builds (tools/build_variant.sh, measured in profiles/kernel_experiments.md)
#ifndef MT_FIN_HANDOFF  // hand off only children above this many tiny subtrees' rows
#define MT_FIN_HANDOFF 2
#endif
#ifndef MT_FIN_UNROLL
#define MT_FIN_UNROLL 4
#endif
#ifndef MT_FIN_PAIR
#define MT_FIN_PAIR 1
#endif
#ifndef MT_FIN_PF  // the hand-off check's loads issued before the partition (1) or in place
#define MT_FIN_PF 0
#endif
#ifndef MT_FIN_PRED  // fp32 first pass: look up the terms of non-candidate bins too (0) or
#define MT_FIN_PRED 0   // only those of candidate bins (exec-masked LDS reads: fewer conflicts)
#endif
#ifndef MT_FIN_VMASK  // fp32 first pass: terms {T(ml), T(l0), T(l1), T(mr), T(r0), T(r1)}
#define MT_FIN_VMASK 0  // computed on the VALU (bit set) instead of looked up in LDS
#endif
constexpr int kFinUnroll = MT_FIN_UNROLL;  // row gathers in flight per lane
constexpr int kFinMaxF = 256;    // features with LDS-cached bin counts (two-class path: all)
constexpr int kFinPair = MT_FIN_PAIR;  // features scanned together per wave (latency hiding)
constexpr int kFinChunk = 8;     // features per wave whose per-lane minima stay in registers
constexpr int kFinCG = 4;        // generic scan: classes whose loads / DPP scans overlap
// fp32 first pass: which of the six x*log2(x) terms per bin come from v_log_f32
// instead of the LDS table. The table lookups are random-address LDS reads (bank
// conflicts, shared by the CU's two workgroups); splitting the terms between the
// LDS and the VALU runs both pipes at once. Per-term error: see tfv.
constexpr int kFinVMask = MT_FIN_VMASK;

// x*log2(x) of an integer count in fp32 on the VALU (v_log_f32). Exhaustively
// measured over 0 <= x < 2^24 (tools/probes/vlog_probe.hip, profiles/r4/vlog_probe.log):
// relative error <= 2.90 * 2^-24, T(0) = T(1) = 0 exactly -- inside the first pass's
// per-term budget of 5 * 2^-24 (scan_c2_f). Measured slower than the table on the
// flagship (profiles/kernel_experiments.md), so the default mask is 0.
__device__ __forceinline__ float tfv(uint32_t x) {
  const float f = (float)x;
  return f * __builtin_amdgcn_logf(fmaxf(f, 1.0f));
}

// Histogram row stride in words: >= B*W + 1 (the odd word staggers features over
// LDS banks for the atomics), rounded to 4 so each feature row is 16-B aligned.
__host__ __device__ inline int fin_fstride(int B, int W) { return ((B * W + 1) + 3) & ~3; }
__host__ __device__ inline int fstride_of(int B, int C) { return fin_fstride(B, (C + 1) >> 1); }
// classes the LDS histogram tile is sized for
__host__ __device__ inline int fin_tile_classes(int C) { return C > kFinMaxC ? kFinClassJobRows : C; }

inline int getenv_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

struct FinRowLab {
  uint32_t mask;
  int shift;
};


// jobs: int64 [J][5 + C] = {start, count, depth, base, buffer, counts[C]}
// node_i32: [slots][6] = {feature, bin, left, right, depth, n}; node_cnt: [slots][C]

template <typename CodeT, bool kC2, int kFinThreads>
__global__ __launch_bounds__(kFinThreads) __attribute__((amdgpu_waves_per_eu(4))) void finish_cls_kernel(
    const uint32_t* __restrict__ codes_rm, int64_t row_words, const CodeT* __restrict__ codes_fm,
    int64_t n_rows, uint32_t* __restrict__ buf0, uint32_t* __restrict__ buf1,
    const int32_t* __restrict__ y, FinRowLab rl, const int64_t* __restrict__ jobs, int J,
    int32_t* __restrict__ job_counter, const int32_t* __restrict__ nbins, int F, int B, int C,
    int crit, int max_depth, int64_t mss, int64_t msl, const double* __restrict__ xtab,
    const float* __restrict__ xtabf, int xtab_n, int32_t* __restrict__ node_i32, int32_t* __restrict__ node_cnt,
    int64_t* __restrict__ tasks, int32_t* __restrict__ task_flag, int32_t epoch, int task_cap,
    int tiny_rows, int64_t* __restrict__ tiny, int32_t* __restrict__ tiny_count,
    int64_t* __restrict__ prof, int Ft, int32_t* __restrict__ gstk) {
  // Ft: features per LDS histogram tile. Ft == F is the single-pass layout; Ft < F
  // (many classes or many features: generic path only) builds and scans the
  // node's histogram one feature tile at a time, re-reading the node's rows per
  // tile, and counts the winning split's left classes during the partition.
  // gstk (C > kFinStackC): global scratch [grid][kFinStack + 2][C] for the DFS
  // stack's class counts and the node's / left class counts (no LDS for many
  // classes)
  // prof (optional): per workgroup {wall start, wall end, nodes, rows, cycles in
  // histogram, scan, partition, rest} -- the finisher's own phase profile
  constexpr int kFinWaves = kFinThreads / kWave;
  extern __shared__ __align__(16) uint32_t hist[];  // [F][B*W + 1] packed class pairs
  // x*log2(x) table: fp64 entries (generic path) or, for C <= 2, twice as many
  // fp32 entries that drive the approximate first pass of the split scan
  __shared__ double s_tab[kFinTab];
  // C <= 2 splits the same 8 KB: fp32 entries [0, kFinTab) in the first half,
  // fp64 entries [0, kFinTab / 4) in the second (exact rescoring, node terms)
  float* const s_tabf = reinterpret_cast<float*>(s_tab);
  double* const s_tabd = s_tab + kFinTab / 2;
  __shared__ int32_t s_nb[kFinMaxF];
  __shared__ float s_fmin[kFinMaxF];
  __shared__ float w_fmin[kFinWaves];
  __shared__ int s_job;
  __shared__ int64_t s_st_start[kFinStack];
  __shared__ int32_t s_st_count[kFinStack], s_st_depth[kFinStack], s_st_id[kFinStack];
  __shared__ int32_t s_st_buf[kFinStack];
  __shared__ int32_t s_st_cnt[kFinStack * kFinStackC];
  __shared__ int s_sp, s_root;
  __shared__ int64_t s_start;
  __shared__ int32_t s_count, s_depth, s_id, s_buf;
  // node / left class counts: LDS up to kFinStackC classes, else global scratch
  // (keeps the two-class kernel's static LDS small: two 512-thread workgroups
  // per CU with the 66 KB F = 64 histogram)
  __shared__ int32_t s_cnt_l[kFinStackC], s_left_l[kFinStackC];
  __shared__ double s_pterm;
  __shared__ double w_gain[kFinWaves];
  __shared__ int w_feat[kFinWaves], w_bin[kFinWaves];
  __shared__ int w_nc[kFinWaves];  // candidate features per wave; -1: one separated bin
  __shared__ int s_bf, s_bb;
  __shared__ int s_lc, s_rc;
  __shared__ int s_cand_total;
  __shared__ int s_tnext, s_tend;  // this workgroup's reserved tiny records (thread 0)
  if (threadIdx.x == 0) {
    s_cand_total = 0;
    s_tnext = s_tend = 0;
  }
  // a tiny-subtree record (thread 0 only): one device atomic per kFinTinyBatch
  auto tiny_slot = [&]() -> int64_t {
    if (s_tnext == s_tend) {
      const int t = atomicAdd(tiny_count, kFinTinyBatch);
      s_tnext = t;
      s_tend = t + kFinTinyBatch;
    }
    return (int64_t)(s_tnext++);
  };

  const int tid = threadIdx.x;
  // C > 2 (generic path): the node's present class ids + their count at [C],
  // then the class -> compacted slot map [C]
  int32_t* const cls_lds =
      (!kC2 && C > 2) ? reinterpret_cast<int32_t*>(hist + Ft * fstride_of(B, fin_tile_classes(C))) +
                            (B > 256 ? (kFinThreadsWide / kWave) * C : 0)
                      : nullptr;
  int32_t* const cmap = cls_lds ? cls_lds + C + 1 : nullptr;
  int32_t* const stc = gstk ? gstk + (int64_t)blockIdx.x * (kFinStack + 2) * C : s_st_cnt;
  const int stw = gstk ? C : kFinStackC;  // stack row stride
  // the node's / left class counts: static LDS up to kFinStackC classes, else
  // dynamic LDS after the class map (read per class in the scan's inner loop:
  // never from global scratch)
  int32_t* const s_cnt = (!kC2 && gstk && cmap) ? cmap + C : s_cnt_l;
  int32_t* const s_left = (!kC2 && gstk && cmap) ? cmap + 2 * C : s_left_l;
  const int wave = tid >> 6;
  const int lane = lane_id();
  const int W = (fin_tile_classes(C) + 1) >> 1;
  const int fstride = fin_fstride(B, W);
  constexpr int cpw = 4 / sizeof(CodeT);
  const int tn = min(kFinTab, xtab_n);
  const int tnd = min(kFinTab / 4, xtab_n);  // C <= 2: fp64 entries kept in LDS
  const int JW = 5 + C;

  // profile counters live in LDS (thread 0 only): no VGPRs on the hot path
  __shared__ int64_t s_pr[9];  // {wall0, nodes, rows, cycles[5], last clock}
  if (prof && tid == 0) {
    s_pr[0] = (int64_t)wall_clock64();
    for (int k = 1; k < 9; ++k) s_pr[k] = 0;
  }
  auto mark = [&](int k) {
    if (prof && tid == 0) {
      const int64_t t = (int64_t)clock64();
      s_pr[3 + k] += t - s_pr[8];
      s_pr[8] = t;
    }
  };
  if constexpr (kC2) {
    for (int i = tid; i < tn; i += kFinThreads) s_tabf[i] = xtabf[i];
    for (int i = tid; i < tnd; i += kFinThreads) s_tabd[i] = xtab[i];
  } else {
    for (int i = tid; i < tn; i += kFinThreads) s_tab[i] = xtab[i];
  }
  for (int f = tid; f < min(F, kFinMaxF); f += kFinThreads) s_nb[f] = min(B, nbins[f]);
  auto nbf = [&](int f) { return f < kFinMaxF ? s_nb[f] : min(B, nbins[f]); };
  const int hist_q = Ft * fstride / 4;  // uint4 words (fstride is a multiple of 4)
  uint4* hist4 = reinterpret_cast<uint4*>(hist);
  for (int e = tid; e < hist_q; e += kFinThreads) hist4[e] = make_uint4(0, 0, 0, 0);

  auto tl = [&](uint64_t x) -> double {
    if constexpr (kC2)
      return x < (uint64_t)tnd ? s_tabd[x]
                               : (x < (uint64_t)xtab_n ? __ldg(xtab + x) : xlog2x(x));
    return x < (uint64_t)tn ? s_tab[x] : (x < (uint64_t)xtab_n ? __ldg(xtab + x) : xlog2x(x));
  };

  // ---- C <= 2: both class counts of a bin packed in one 32-bit word (class 0
  // low half, class 1 high half). Lane l owns bins 4l..4l+3: one 16-B LDS read
  // and one packed DPP prefix sum give both classes' left counts.
  auto load_c2 = [&](const uint32_t* h, int nb, uint32_t (&v)[4], uint32_t& excl) {
    const int b0 = lane * 4;
    const uint4 hv = b0 < nb ? *reinterpret_cast<const uint4*>(h + b0) : make_uint4(0, 0, 0, 0);
    v[0] = hv.x;
    v[1] = hv.y;
    v[2] = hv.z;
    v[3] = hv.w;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (b0 + k >= nb) v[k] = 0u;
    excl = wave_incl_scan_dpp(v[0] + v[1] + v[2] + v[3]) - (v[0] + v[1] + v[2] + v[3]);
  };
  // Pass 1 (entropy): the minimum split cost of one feature in fp32 from the
  // fp32 table, branch-free. |fp32 - exact| <= 12 * 2^-24 * T(m) (six rounded
  // table values, six roundings of sums bounded by T(m), T superadditive), so
  // only features whose fp32 minimum lies within 2^-19 * T(m) of the node's
  // best can hold the exact optimum; pass 2 re-scores just those in fp64.
  // Processes kFinPair features per call with every table read issued before
  // the first wait: each feature is a dependent chain (LDS read -> DPP scan ->
  // lookups -> DPP min), so independent features are what hides the latency.
  // info[q] (for the exact-pass skip): bits 0-1 the lane's first minimum bin,
  // bit 2 set when every other bin of the lane costs more than
  // (min + T(m) 2^-19) + 2^-20 -- the candidate threshold's form with min >= the
  // node's best, so such a bin is never a candidate
  auto scan_c2_f = [&](auto big_tag, int f0, uint32_t t0, uint32_t t1, int m, float tmf,
                       float (&out)[kFinPair], uint32_t (&info)[kFinPair]) {
    constexpr bool kBig = decltype(big_tag)::value;
    auto lk = [&](uint32_t x) -> float {
      if constexpr (!kBig) {
        return s_tabf[x];
      } else {
        return x < (uint32_t)tn ? s_tabf[x] : __ldg(xtabf + x);
      }
    };
    uint32_t v[kFinPair][4], lp[kFinPair];
#pragma unroll
    for (int q = 0; q < kFinPair; ++q) {
      const int f = f0 + q * kFinWaves;
      if (f < F) {
        load_c2(hist + f * fstride, s_nb[f], v[q], lp[q]);
      } else {
        v[q][0] = v[q][1] = v[q][2] = v[q][3] = 0u;
        lp[q] = 0u;
      }
    }
    float tv[kFinPair][4][6];
    bool ok[kFinPair][4];
#pragma unroll
    for (int q = 0; q < kFinPair; ++q) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        lp[q] += v[q][k];
        const uint32_t l0 = lp[q] & 0xffffu, l1 = lp[q] >> 16;
        const uint32_t ml = l0 + l1, mr = (uint32_t)m - ml;
        ok[q][k] = v[q][k] != 0u && (int64_t)ml >= msl && (int64_t)mr >= msl;
        // every bin looks its terms up, empty ones included: redirecting empty
        // bins to one broadcast entry measured slower (the selects cost more VALU
        // than the bank conflicts they remove)
        const uint32_t xs[6] = {ml, l0, l1, mr, t0 - l0, t1 - l1};
        if (MT_FIN_PRED) {
#pragma unroll
          for (int e = 0; e < 6; ++e) tv[q][k][e] = 0.0f;
          if (ok[q][k]) {
#pragma unroll
            for (int e = 0; e < 6; ++e) tv[q][k][e] = lk(xs[e]);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 6; ++e) tv[q][k][e] = ((kFinVMask >> e) & 1) ? tfv(xs[e]) : lk(xs[e]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < kFinPair; ++q) {
      float c[4];
      float best = __builtin_inff();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float* t = tv[q][k];
        c[k] = ok[q][k] ? (t[0] - (t[1] + t[2])) + (t[3] - (t[4] + t[5])) : __builtin_inff();
        best = fminf(best, c[k]);
      }
      const int idx = c[0] == best ? 0 : (c[1] == best ? 1 : (c[2] == best ? 2 : 3));
      float s2 = __builtin_inff();
#pragma unroll
      for (int k = 0; k < 4; ++k) s2 = k == idx ? s2 : fminf(s2, c[k]);
      out[q] = best;
      info[q] = (uint32_t)idx | (s2 > (best + tmf * 0x1p-19f) + 0x1p-20f ? 4u : 0u);
    }
  };
  // Exact (fp64, global table) best split of one feature: (cost, lowest bin).
  auto scan_c2 = [&](const uint32_t* h, int nb, uint32_t t0, uint32_t t1, int m,
                     double& best_cost, int& best_bin) {
    const bool small = m < tnd;  // wave-uniform: every count of the node is in LDS
    auto lk = [&](uint32_t x) -> double { return small ? s_tabd[x] : __ldg(xtab + x); };
    uint32_t v[4], lp;
    load_c2(h, nb, v, lp);
    best_cost = __builtin_inf();
    best_bin = 0x7fffffff;
    const double tu = tie_unit(lk((uint32_t)m), (int64_t)m);
    const double tinv = 1.0 / tu;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      lp += v[k];
      const uint32_t l0 = lp & 0xffffu, l1 = lp >> 16;
      const uint32_t r0 = t0 - l0, r1 = t1 - l1;
      const int64_t ml = (int64_t)(l0 + l1);
      const int64_t mr = (int64_t)m - ml;
      if (v[k] != 0u && ml >= msl && mr >= msl) {
        double cost;
        if (crit == kEntropy) {
          const double sl = lk(l0) + lk(l1);
          const double sr = lk(r0) + lk(r1);
          cost = (lk((uint32_t)ml) - sl) + (lk((uint32_t)mr) - sr);
        } else {
          const int64_t ql = (int64_t)l0 * l0 + (int64_t)l1 * l1;
          const int64_t qr = (int64_t)r0 * r0 + (int64_t)r1 * r1;
          cost = gini_term(ml, ql) + gini_term(mr, qr);
        }
        cost = tie_round(cost, tinv, tu);
        if (cost < best_cost) {
          best_cost = cost;
          best_bin = lane * 4 + k;
        }
      }
    }
    wave_argmin_dpp(best_cost, best_bin);
  };

  // Work queue: the J sorted jobs, then subtrees that running workgroups hand
  // off while others idle (records in `tasks`, each published by an
  // epoch-tagged flag). A workgroup claims the next index; an index past the
  // published ones waits for its record or for the end of all work. One 64-bit
  // word counts {completed tasks : 32, handed off : 32}; the work is over when
  // completed == J + handed off (hand-offs only come from running tasks, so
  // that cannot hold early), which the last completion sees in its own atomic
  // and announces through q_finished. Waiters poll only their own flag and
  // q_finished: lines nobody else keeps writing.
  unsigned long long* const q_word =
      reinterpret_cast<unsigned long long*>(job_counter + kFinCtrQueue);
  int32_t* const q_finished = job_counter + kFinCtrFinished;
  for (;;) {
    if (tid == 0) {
      const int h = atomicAdd(job_counter, 1);
      int got = h;
      if (!kC2 || task_cap < 0) {  // the queue drives the two-class kernel only
        if (h >= J) got = -1;
      } else if (h >= J) {
        // Waiting is cheap and bounded: relaxed loads that bypass L1 (no cache
        // invalidation while co-resident workgroups work), one acquire fence
        // once the record is there, and a wall-clock watchdog that reports
        // through job_counter[6..7] instead of ever hanging the GPU.
        const uint64_t t_start = wall_clock64();
        for (uint32_t spins = 0;; ++spins) {
          if (h - J < task_cap &&
              __hip_atomic_load(task_flag + (h - J), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                  epoch) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            break;
          }
          if (__hip_atomic_load(q_finished, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) {
            got = -1;
            break;
          }
          if ((spins & 15u) == 15u && wall_clock64() - t_start > 500000000ull) {  // 5 s
            atomicExch(job_counter + kFinCtrWatch, 1);
            got = -1;
            break;
          }
          __builtin_amdgcn_s_sleep(32);
        }
      }
      s_job = got;
    }
    __syncthreads();
    const int job = s_job;
    if (job < 0) break;
    if (prof && tid == 0) s_pr[8] = (int64_t)clock64();
    const int64_t* jb =
        (!kC2 || job < J) ? jobs + (int64_t)job * JW : tasks + (int64_t)(job - J) * JW;
    int32_t* ni = node_i32;  // indexed by pre-order position (see launch_finish)
    int32_t* nc = node_cnt;
    if (tid == 0) {
      const int r = (int)jb[3];
      s_root = r;
      s_sp = 1;
      s_st_start[0] = jb[0];
      s_st_count[0] = (int32_t)jb[1];
      s_st_depth[0] = (int32_t)jb[2];
      s_st_id[0] = r;
      s_st_buf[0] = (int32_t)jb[4];
      int32_t* R = ni + (int64_t)r * 6;
      R[0] = -1;
      R[1] = -1;
      R[2] = -1;
      R[3] = -1;
      R[4] = (int32_t)jb[2];
      R[5] = (int32_t)jb[1];
      if (jb[1] <= tiny_rows) {  // the whole job is tiny: one wave finishes it
        const int64_t t = tiny_slot();
        int64_t* tr = tiny + t * 8;
        tr[0] = jb[0];
        tr[1] = jb[1];
        tr[2] = jb[2];
        tr[3] = jb[4];
        tr[4] = r;
        s_sp = 0;
      }
    }
    for (int c = tid; c < C; c += kFinThreads) stc[c] = (int32_t)jb[5 + c];
    __syncthreads();
    for (int c = tid; c < C; c += kFinThreads) nc[(int64_t)s_root * C + c] = (int32_t)jb[5 + c];
    while (s_sp > 0) {
      __syncthreads();  // everyone has read s_sp before thread 0 pops
      // ---- pop + node term (thread 0); the histogram is already zero
      if (tid == 0) {
        const int sp = --s_sp;
        s_start = s_st_start[sp];
        s_count = s_st_count[sp];
        s_depth = s_st_depth[sp];
        s_id = s_st_id[sp];
        s_buf = s_st_buf[sp];
        double acc = 0.0;
        int64_t mm = 0, sq = 0;
        for (int c = 0; c < C; ++c) {
          const int64_t t = stc[sp * stw + c];
          s_cnt[c] = (int32_t)t;
          s_left[c] = 0;  // tiled: counted during the partition
          mm += t;
          acc = acc + tl((uint64_t)t);
          sq += t * t;
        }
        s_pterm = crit == kEntropy ? tl((uint64_t)mm) - acc : gini_term(mm, sq);
        s_lc = 0;
        s_rc = 0;
      }
      __syncthreads();
      // ---- more than two classes: the node's present classes in ascending order
      // (dynamic LDS after the histogram and the carries). An absent class adds
      // T(0) = 0 (or 0 squared) to every left / right sum, so scanning the present
      // ones only leaves each sum bit-identical -- deep nodes hold few classes.
      int ncls = C;
      if constexpr (!kC2) {
        if (cls_lds) {
          if (wave == 0) {
            const unsigned long long lt = (1ull << lane) - 1ull;
            int off = 0;
            for (int c0 = 0; c0 < C; c0 += kWave) {
              const int c = c0 + lane;
              const bool pr = c < C && s_cnt[c] > 0;
              const unsigned long long mk = __ballot(pr);
              if (pr) cls_lds[off + __popcll(mk & lt)] = c;
              if (c < C) cmap[c] = pr ? off + __popcll(mk & lt) : 0;
              off += __popcll(mk);
            }
            if (lane == 0) cls_lds[C] = off;
          }
          __syncthreads();
          ncls = cls_lds[C];
        }
      }
      // the node's histogram layout: its present classes only, two 16-bit counts
      // per word -- or four 8-bit ones when the node has at most 255 rows -- so a
      // node holding few of many classes, or few rows, packs more features per LDS
      // tile: fewer tiles re-reading its rows, more waves scanning
      const bool pk8 = cls_lds != nullptr && s_count <= 255;
      const int psh = pk8 ? 2 : 1;                // log2(classes per word)
      const int fbits = pk8 ? 8 : 16;             // bits per count
      const uint32_t fmask = pk8 ? 0xffu : 0xffffu;
      int Wn = W, fstr = fstride, Ftn = Ft;
      if (cls_lds) {
        Wn = (ncls + (1 << psh) - 1) >> psh;
        fstr = fin_fstride(B, Wn);
        Ftn = min(min(F, kFinMaxF), (Ft * fstride) / fstr);
        if (Ftn >= 16 && Ftn < F) Ftn &= ~15;  // (16-B row loads at every tile start)
      }
      const bool tiled_n = Ftn < F;
      const int hq = Ftn * fstr / 4;  // uint4 words this node's tiles use
      const int64_t start = s_start;
      const int m = s_count;
      const int depth = s_depth;
      const int id = s_id;
      mark(3);
      if (prof && tid == 0) {
        s_pr[1] += 1;
        s_pr[2] += m;
      }
      uint32_t* __restrict__ src = s_buf ? buf1 : buf0;
      uint32_t* __restrict__ dst = s_buf ? buf0 : buf1;
      const double pterm = s_pterm;
      double bg = -__builtin_inf();
      int bfeat = 0x7fffffff, bbin = -1;
      int nc_report = 0x40000000;  // no exact-pass skip unless pass 1 proves one
      for (int ft0 = 0; ft0 < F; ft0 += Ftn) {
      const int ft1 = min(F, ft0 + Ftn);
      if (ft0 > 0) {  // next feature tile: clear the previous tile's counts
        __syncthreads();
        for (int e = tid; e < hq; e += kFinThreads) hist4[e] = make_uint4(0, 0, 0, 0);
        __syncthreads();
      }
      // ---- histogram of this node's rows (features [ft0, ft1)): VEC words per
      // lane, lanes_per_row lanes per row, kFinUnroll rows in flight per lane
      {
        const int w_lo = ft0 / cpw;
        const int words = (ft1 + cpw - 1) / cpw - w_lo;
        // 16-B row loads when the row stride and tile start allow it; lanes per
        // row = pow2 >= words/vec
        const int vec = (row_words % 4) == 0 && (w_lo % 4) == 0 ? 4 : 1;
        int lane_shift = 0;
        while ((1 << lane_shift) * vec < words && lane_shift < 6) ++lane_shift;
        const int L = 1 << lane_shift;
        const int sub = tid & (L - 1);
        const int rpp = kFinThreads >> lane_shift;
        const int my_w = w_lo + sub * vec;
        const bool active = sub * vec < words;
        for (int base_r = tid >> lane_shift; base_r < m; base_r += rpp * kFinUnroll) {
          // unconditional loads (an absent row re-reads the segment's first entry /
          // row 0): every gather of the unrolled rows is in flight before the
          // first use -- guarded loads compiled to one wait per row
          uint32_t ent[kFinUnroll];
          bool okr[kFinUnroll];
#pragma unroll
          for (int u = 0; u < kFinUnroll; ++u) {
            const int r = base_r + u * rpp;
            okr[u] = active && r < m;
            ent[u] = src[start + (okr[u] ? r : 0)];
          }
          uint32_t wv[kFinUnroll][4];
          int lab[kFinUnroll];
#pragma unroll
          for (int u = 0; u < kFinUnroll; ++u) {
            const uint32_t row = okr[u] ? (rl.shift ? (ent[u] & rl.mask) : ent[u]) : 0u;
            lab[u] = rl.shift ? (int)(ent[u] >> rl.shift) : y[row];
            if (vec == 4) {
              const uint4 v = *reinterpret_cast<const uint4*>(codes_rm + (int64_t)row * row_words + my_w);
              wv[u][0] = v.x;
              wv[u][1] = v.y;
              wv[u][2] = v.z;
              wv[u][3] = v.w;
            } else {
              wv[u][0] = codes_rm[(int64_t)row * row_words + my_w];
              wv[u][1] = wv[u][2] = wv[u][3] = 0u;
            }
            if (!okr[u]) ent[u] = 0xffffffffu;
          }
#pragma unroll
          for (int u = 0; u < kFinUnroll; ++u) {
            if (ent[u] == 0xffffffffu) continue;
            const int sl = cmap ? cmap[lab[u]] : lab[u];  // (compacted class slot)
            const uint32_t inc = 1u << ((sl & ((1 << psh) - 1)) * fbits);
            const int off = sl >> psh;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              if (v >= vec) break;
#pragma unroll
              for (int j = 0; j < cpw; ++j) {
                const int f = (my_w + v) * cpw + j;
                if (f >= ft0 && f < ft1) {
                  const uint32_t code = (wv[u][v] >> (j * 8 * sizeof(CodeT))) &
                                        ((sizeof(CodeT) == 1) ? 0xffu : 0xffffu);
                  atomicAdd(&hist[(f - ft0) * fstr + (int)code * Wn + off], inc);
                }
              }
            }
          }
        }
      }
      __syncthreads();
      mark(0);
      // ---- wave-per-feature scan (B <= 256: one 256-bin pass)
      if constexpr (kC2) {  // (single tile: Ft == F)
        const uint32_t t0 = (uint32_t)s_cnt[0], t1 = C > 1 ? (uint32_t)s_cnt[1] : 0u;
        bool cand_all = true, one_chunk = false;
        float thr = 0.0f;
        float lmin[kFinChunk];
        uint32_t linfo = 0u;  // scan_c2_f info of chunk feature i at bits 3i..3i+2
        uint32_t cand_mask = 0u;
        bool clean = false;
        if (crit == kEntropy) {
          // pass 1: per-lane fp32 minima over each feature's bins (no per-feature
          // wave reduction), one wave minimum, then the node-wide threshold.
          // Features f = wave + 4 i; chunks of kFinChunk keep the per-lane minima
          // in registers; past one chunk (F > 64) each feature is reduced to LDS.
          const bool big = m >= tn;  // wave-uniform: small nodes never leave LDS
          const int fpw = (F - wave + kFinWaves - 1) / kFinWaves;  // this wave's features
          one_chunk = F <= kFinWaves * kFinChunk;
          const float tmf = m < tn ? s_tabf[m] : __ldg(xtabf + m);
          float wl = __builtin_inff();
          for (int c0 = 0; c0 < fpw; c0 += kFinChunk) {
#pragma unroll
            for (int i = 0; i < kFinChunk; i += kFinPair) {
              float fm[kFinPair];
              uint32_t fi[kFinPair];
              if (c0 + i < fpw) {
                const int f = wave + (c0 + i) * kFinWaves;
                if (big)
                  scan_c2_f(std::true_type{}, f, t0, t1, m, tmf, fm, fi);
                else
                  scan_c2_f(std::false_type{}, f, t0, t1, m, tmf, fm, fi);
              }
#pragma unroll
              for (int q = 0; q < kFinPair; ++q) {
                lmin[i + q] = c0 + i + q < fpw ? fm[q] : __builtin_inff();
                if (c0 + i + q < fpw) linfo |= fi[q] << (3 * (i + q));
              }
            }
#pragma unroll
            for (int i = 0; i < kFinChunk; ++i) wl = fminf(wl, lmin[i]);
            if (!one_chunk) {
              for (int i = 0; i < kFinChunk && c0 + i < fpw; ++i) {
                const float fm = wave_min_f32_dpp(lmin[i]);
                if (lane == 0) s_fmin[wave + (c0 + i) * kFinWaves] = fm;
              }
            }
          }
          const float wmin = wave_min_f32_dpp(wl);
          if (lane == 0) w_fmin[wave] = wmin;
          __syncthreads();
          mark(4);
          float best = w_fmin[0];
          for (int w = 1; w < kFinWaves; ++w) best = fminf(best, w_fmin[w]);
          const float tm = m < tn ? s_tabf[m] : __ldg(xtabf + m);
          thr = best + tm * 0x1p-19f + 0x1p-20f;
          cand_all = false;
          if (one_chunk) {
#pragma unroll
            for (int i = 0; i < kFinChunk; ++i)
              if (__ballot(lmin[i] <= thr)) cand_mask |= 1u << i;
            // exact-pass skip: this wave's only candidate is one lane's one bin,
            // every other bin of that lane above the threshold. If it is also
            // the node's only candidate (checked after the barrier), its exact
            // cost is the unique minimum: every other bin's fp32 cost exceeds
            // best + T(m) 2^-19 + 2^-20 > best + 2 * 12 * 2^-24 T(m) (twice the
            // fp32 error bound), far more than the tie-rounding grid.
            nc_report = __popc(cand_mask);
            if (nc_report == 1) {
              const int i = __ffs((int)cand_mask) - 1;
              float li = lmin[0];
#pragma unroll
              for (int k = 1; k < kFinChunk; ++k) li = k == i ? lmin[k] : li;
              const unsigned long long lanes = __ballot(li <= thr);
              if (__popcll(lanes) == 1) {
                const int l = __ffsll((long long)lanes) - 1;
                const uint32_t inf = (uint32_t)__builtin_amdgcn_readlane((int)linfo, l) >> (3 * i);
                if (inf & 4u) {
                  clean = true;
                  nc_report = -1;
                  bfeat = wave + i * kFinWaves;
                  bbin = l * 4 + (int)(inf & 3u);
                }
              }
            }
          }
        }
        // pass 2: exact scores for candidate features only
        for (int i = 0, f = wave; f < F && !clean; ++i, f += kFinWaves) {
          if (!cand_all) {
            if (one_chunk ? !((cand_mask >> i) & 1u) : !(s_fmin[f] <= thr)) continue;
          }
          if (prof && lane == 0) atomicAdd(&s_cand_total, 1);
          double best_cost;
          int best_bin;
          scan_c2(hist + f * fstride, s_nb[f], t0, t1, m, best_cost, best_bin);
          if (best_cost < __builtin_inf()) {
            const double g = pterm - best_cost;
            if (g > bg) {  // features visited in increasing order: strict > keeps the lowest
              bg = g;
              bfeat = f;
              bbin = best_bin;
            }
          }
        }
      } else
      for (int f = ft0 + wave; f < ft1; f += kFinWaves) {
        const int nb = nbf(f);
        const uint32_t* h = hist + (f - ft0) * fstr;
        double best_cost = __builtin_inf();
        int best_bin = 0x7fffffff;
        const double tu = tie_unit(tl((uint64_t)m), (int64_t)m);
        const double tinv = 1.0 / tu;
        // B > 256 (16-bit codes): 256-bin passes, each class's left count carried
        // from pass to pass in this wave's LDS words (wave-uniform values)
        int32_t* const carry = reinterpret_cast<int32_t*>(hist + Ft * fstride) + wave * C;
        const bool multi = nb > kWave * 4;
        if (multi)
          for (int c = lane; c < C; c += kWave) carry[c] = 0;
        for (int bc = 0; bc < nb; bc += kWave * 4) {
        const int b0 = bc + lane * 4;
        uint32_t mL[4] = {0, 0, 0, 0}, ne[4] = {0, 0, 0, 0};
        double sL[4] = {0.0, 0.0, 0.0, 0.0}, sR[4] = {0.0, 0.0, 0.0, 0.0};
        int64_t qL[4] = {0, 0, 0, 0}, qR[4] = {0, 0, 0, 0};
        // classes in groups of kFinCG: a group's bin loads and DPP prefix sums are
        // independent chains issued together; the sums still add class by class in
        // ascending order (bit-identical to the sequential host sums)
        auto class_pass = [&](auto group_tag) {
        constexpr int kG = decltype(group_tag)::value;
        for (int j0 = 0; j0 < ncls; j0 += kG) {
          uint32_t vv[kG][4], p[kG][4], incl[kG];
          int cc[kG];
#pragma unroll
          for (int g = 0; g < kG; ++g) {
            const int j = j0 + g;  // compacted slot j holds class cls_lds[j]
            const int c = j < ncls ? (cls_lds ? cls_lds[j] : j) : -1;
            cc[g] = c;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int b = b0 + k;
              const uint32_t v = (c >= 0 && b < nb) ? h[b * Wn + (j >> psh)] : 0u;
              vv[g][k] = (v >> ((j & ((1 << psh) - 1)) * fbits)) & fmask;
            }
          }
#pragma unroll
          for (int g = 0; g < kG; ++g) {
            p[g][0] = vv[g][0];
            p[g][1] = p[g][0] + vv[g][1];
            p[g][2] = p[g][1] + vv[g][2];
            p[g][3] = p[g][2] + vv[g][3];
            incl[g] = wave_incl_scan_dpp(p[g][3]);
          }
#pragma unroll
          for (int g = 0; g < kG; ++g) {
            const int c = cc[g];
            if (c < 0) break;  // (wave-uniform: the group's tail)
            uint32_t excl = incl[g] - p[g][3];
            if (multi) {  // + the class's rows in the earlier passes
              const uint32_t cin = (uint32_t)carry[c];
              excl += cin;
              const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl[g], kWave - 1);
              if (lane == 0) carry[c] = (int32_t)(cin + tot);
            }
            const uint32_t tc = (uint32_t)s_cnt[c];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t L = excl + p[g][k];
              const uint32_t R = tc - L;
              mL[k] += L;
              ne[k] |= vv[g][k];
              if (crit == kEntropy) {
                sL[k] = sL[k] + tl(L);
                sR[k] = sR[k] + tl(R);
              } else {
                qL[k] += (int64_t)L * L;
                qR[k] += (int64_t)R * R;
              }
            }
          }
        }
        };
        if (ncls <= 2) {  // two classes share one word: one load, both halves
          uint32_t vlo[4], vhi[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int b = b0 + k;
            const uint32_t v = b < nb ? h[b * Wn] : 0u;
            vlo[k] = v & fmask;
            vhi[k] = (v >> fbits) & fmask;
          }
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            if (half >= ncls) break;
            const int c = cls_lds ? cls_lds[half] : half;  // (slot half's class)
            const uint32_t* vv = half ? vhi : vlo;
            uint32_t p[4];
            p[0] = vv[0];
            p[1] = p[0] + vv[1];
            p[2] = p[1] + vv[2];
            p[3] = p[2] + vv[3];
            const uint32_t incl = wave_incl_scan_dpp(p[3]);
            uint32_t excl = incl - p[3];
            if (multi) {  // + the class's rows in the earlier passes
              const uint32_t cin = (uint32_t)carry[c];
              excl += cin;
              const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
              if (lane == 0) carry[c] = (int32_t)(cin + tot);
            }
            const uint32_t tc = (uint32_t)s_cnt[c];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t L = excl + p[k];
              const uint32_t R = tc - L;
              mL[k] += L;
              ne[k] |= vv[k];
              if (crit == kEntropy) {
                sL[k] = sL[k] + tl(L);
                sR[k] = sR[k] + tl(R);
              } else {
                qL[k] += (int64_t)L * L;
                qR[k] += (int64_t)R * R;
              }
            }
          }
        } else {
          class_pass(std::integral_constant<int, kFinCG>{});
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int b = b0 + k;
          const int64_t ml = mL[k];
          const int64_t mr = (int64_t)m - ml;
          if (b < nb && ne[k] && ml >= msl && mr >= msl) {
            double cost;
            if (crit == kEntropy)
              cost = (tl((uint64_t)ml) - sL[k]) + (tl((uint64_t)mr) - sR[k]);
            else
              cost = gini_term(ml, qL[k]) + gini_term(mr, qR[k]);
            cost = tie_round(cost, tinv, tu);
            if (cost < best_cost) {
              best_cost = cost;
              best_bin = b;
            }
          }
        }
        }  // 256-bin passes
        if (multi)
          wave_argmin(best_cost, best_bin);  // (cost, bin): lanes' bins interleave across passes
        else
          wave_argmin_dpp(best_cost, best_bin);  // single 256-bin pass: lanes own ascending bins
        if (best_cost < __builtin_inf()) {
          const double g = pterm - best_cost;
          if (g > bg) {  // features visited in increasing order: strict > keeps the lowest
            bg = g;
            bfeat = f;
            bbin = best_bin;
          }
        }
      }
      }  // feature tiles
      if (lane == 0) {
        w_gain[wave] = bg;
        w_feat[wave] = bfeat;
        w_bin[wave] = bbin;
        w_nc[wave] = nc_report;
      }
      __syncthreads();
      mark(1);
      int bf = -1, bb = -1;
      int pf_head = 0, pf_pushed = 0;  // (thread 0: hand-off check, loaded early)
      bool decided = false;
      if constexpr (kC2) {
        int tot = 0, cw = -1;
        for (int w = 0; w < kFinWaves; ++w) {
          const int c = w_nc[w];
          tot += c < 0 ? 1 : min(c, 0x40000000 / kFinWaves);
          if (c < 0) cw = w;
        }
        if (cw >= 0 && tot == 1) {  // the node's only candidate: no exact pass
          bf = w_feat[cw];
          bb = w_bin[cw];
          decided = true;
        } else if (cw >= 0) {  // other candidates too: the skipped waves score theirs now
          if (w_nc[wave] < 0) {
            const uint32_t t0 = (uint32_t)s_cnt[0], t1 = C > 1 ? (uint32_t)s_cnt[1] : 0u;
            const int f = w_feat[wave];
            double best_cost;
            int best_bin;
            scan_c2(hist + f * fstride, s_nb[f], t0, t1, m, best_cost, best_bin);
            if (lane == 0) {
              w_gain[wave] = best_cost < __builtin_inf() ? pterm - best_cost : -__builtin_inf();
              w_bin[wave] = best_bin;
            }
          }
          __syncthreads();
        }
      }
      if (!decided) {
        double g = w_gain[0];
        bf = w_feat[0];
        bb = w_bin[0];
        for (int w = 1; w < kFinWaves; ++w) {
          if (w_gain[w] > g || (w_gain[w] == g && w_feat[w] < bf)) {
            g = w_gain[w];
            bf = w_feat[w];
            bb = w_bin[w];
          }
        }
        if (!(g > -__builtin_inf())) bf = -1;
      }
      if (bf >= 0) {
        // ---- left class counts of the winning split (tiled: counted below);
        // compacted slot j holds class cls_lds[j] (absent classes stay 0)
        for (int j = wave; j < ncls && !tiled_n; j += kFinWaves) {
          const int c = cls_lds ? cls_lds[j] : j;
          uint32_t s = 0;
          const uint32_t* h = hist + bf * fstr;
          for (int b = lane; b <= bb; b += kWave) {
            const uint32_t v = h[b * Wn + (j >> psh)];
            s += (v >> ((j & ((1 << psh) - 1)) * fbits)) & fmask;
          }
          s = wave_sum_u32(s);
          if (lane == 0) s_left[c] = (int32_t)s;
        }
        // the hand-off check's two device-scope loads (thread 0, children below),
        // issued before the partition so their latency overlaps it
        if (MT_FIN_PF && kC2 && tid == 0) {
          pf_head = __hip_atomic_load(job_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          pf_pushed = (int)(__hip_atomic_load(q_word, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) >> 32);
        }
        // ---- partition rows src -> dst (unstable; left from the front, right from the back)
        const CodeT* col = codes_fm + (int64_t)bf * n_rows;
        const unsigned long long lt = (1ull << lane) - 1ull;
        for (int r0 = 0; r0 < m; r0 += kFinThreads * kFinUnroll) {
          uint32_t ent[kFinUnroll];
          uint32_t cv[kFinUnroll];
#pragma unroll
          for (int u = 0; u < kFinUnroll; ++u) {  // (unconditional: see the histogram)
            const int r = r0 + u * kFinThreads + tid;
            ent[u] = src[start + (r < m ? r : 0)];
          }
#pragma unroll
          for (int u = 0; u < kFinUnroll; ++u) cv[u] = (uint32_t)col[ent[u] & rl.mask];
#pragma unroll
          for (int u = 0; u < kFinUnroll; ++u) {
            const int r = r0 + u * kFinThreads + tid;
            const bool valid = r < m;
            const bool go = valid && cv[u] <= (uint32_t)bb;
            const unsigned long long bl = __ballot(go);
            const unsigned long long br = __ballot(valid && !go);
            int basel = 0, baser = 0;
            if (lane == 0) {
              const int nl = __popcll(bl), nr = __popcll(br);
              basel = nl ? atomicAdd(&s_lc, nl) : 0;
              baser = nr ? atomicAdd(&s_rc, nr) : 0;
            }
            basel = __builtin_amdgcn_readfirstlane(basel);
            baser = __builtin_amdgcn_readfirstlane(baser);
            if (valid) {
              if (tiled_n && go) {
                const uint32_t e = ent[u];
                atomicAdd(&s_left[rl.shift ? (int)(e >> rl.shift) : y[e & rl.mask]], 1);
              }
              if (go)
                dst[start + basel + __popcll(bl & lt)] = ent[u];
              else
                dst[start + m - 1 - (baser + __popcll(br & lt))] = ent[u];
            }
          }
        }
      }
      __syncthreads();
      mark(2);
      // ---- clear the histogram for the next node (all scan reads are done)
      for (int e = tid; e < hq; e += kFinThreads) hist4[e] = make_uint4(0, 0, 0, 0);
      // ---- children
      if (tid == 0 && bf >= 0) {
        const int nl = s_lc;
        const int nr = m - nl;
        const int lid = id + 1, rid = id + 2 * nl;  // left subtree owns 2 nl - 1 positions
        ni[(int64_t)id * 6 + 0] = bf;
        ni[(int64_t)id * 6 + 1] = bb;
        ni[(int64_t)id * 6 + 2] = lid;
        ni[(int64_t)id * 6 + 3] = rid;
        int nzl = 0, nzr = 0;
        for (int c = 0; c < C; ++c) {
          const int32_t lc = s_left[c], rc = s_cnt[c] - s_left[c];
          nc[(int64_t)lid * C + c] = lc;
          nc[(int64_t)rid * C + c] = rc;
          nzl += lc > 0;
          nzr += rc > 0;
        }
        const int cd = depth + 1;
        const bool depth_stop = max_depth >= 0 && cd >= max_depth;
        const bool tlf = depth_stop || nl < mss || nl < 2 * msl || nzl <= 1;
        const bool trf = depth_stop || nr < mss || nr < 2 * msl || nzr <= 1;
        int32_t* L = ni + (int64_t)lid * 6;
        int32_t* Rr = ni + (int64_t)rid * 6;
        L[0] = -1; L[1] = -1; L[2] = -1; L[3] = -1; L[4] = cd; L[5] = nl;
        Rr[0] = -1; Rr[1] = -1; Rr[2] = -1; Rr[3] = -1; Rr[4] = cd; Rr[5] = nr;
        // push the larger child first so the smaller one is processed next --
        // or hand the larger one to an idle workgroup (claims past the
        // published work) when it is worth a workgroup
        const bool left_small = nl <= nr;
        for (int pass = 0; pass < 2; ++pass) {
          const bool is_left = (pass == 0) ? !left_small : left_small;
          if (is_left ? tlf : trf) continue;
          const int cm_rows = is_left ? nl : nr;
          if (kC2 && pass == 0 && cm_rows > MT_FIN_HANDOFF * tiny_rows) {
            // (values from before the partition: a stale one only changes whether
            // this child is handed off, never the tree)
            const int head = MT_FIN_PF ? pf_head
                                       : __hip_atomic_load(job_counter, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
            const int pushed = MT_FIN_PF ? pf_pushed
                                         : (int)(__hip_atomic_load(q_word, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT) >> 32);
            if (head > J + pushed && pushed < task_cap) {
              const int k = (int)(__hip_atomic_fetch_add(q_word, 1ull << 32, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) >> 32);
              if (k < task_cap) {
                int64_t* T = tasks + (int64_t)k * JW;
                T[0] = is_left ? start : start + nl;
                T[1] = cm_rows;
                T[2] = cd;
                T[3] = is_left ? lid : rid;
                T[4] = s_buf ^ 1;
                for (int c = 0; c < C; ++c) T[5 + c] = is_left ? s_left[c] : s_cnt[c] - s_left[c];
                // the child's rows (this workgroup's partition) and record are
                // visible chip-wide before the flag (agent-scope release)
                __threadfence();
                __hip_atomic_store(task_flag + k, epoch, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
                continue;
              }
              // (over capacity: the counter overshoot is undone below)
              __hip_atomic_fetch_add(q_word, ~0ull << 32, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          if (cm_rows <= tiny_rows) {  // hand the tiny subtree to a wavefront
            const int64_t t = tiny_slot();
            int64_t* tr = tiny + t * 8;
            tr[0] = is_left ? start : start + nl;
            tr[1] = cm_rows;
            tr[2] = cd;
            tr[3] = s_buf ^ 1;
            tr[4] = is_left ? lid : rid;
            continue;
          }
          const int sp = s_sp++;
          s_st_start[sp] = is_left ? start : start + nl;
          s_st_count[sp] = is_left ? nl : nr;
          s_st_depth[sp] = cd;
          s_st_id[sp] = is_left ? lid : rid;
          s_st_buf[sp] = s_buf ^ 1;
          for (int c = 0; c < C; ++c)
            stc[sp * stw + c] = is_left ? s_left[c] : s_cnt[c] - s_left[c];
        }
      }
      __syncthreads();
    }
    mark(3);
    if (kC2 && tid == 0) {
      // the completion that brings {completed, handed off} to completed == J +
      // handed off is the last one (no task runs, so none can be handed off):
      // it releases the waiting workgroups
      const unsigned long long q =
          __hip_atomic_fetch_add(q_word, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(uint32_t)q + 1 == J + (int)(q >> 32))
        __hip_atomic_store(q_finished, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tid == 0)  // reserved records left unused: empty (m = 0), skipped by the tiny kernels
    for (int k = s_tnext; k < s_tend; ++k) tiny[(int64_t)k * 8 + 1] = 0;
  if (prof && tid == 0) {
    int64_t* P = prof + (int64_t)blockIdx.x * 10;
    P[0] = s_pr[0];
    P[1] = (int64_t)wall_clock64();
    P[2] = s_pr[1];
    P[3] = s_pr[2];
    for (int k = 0; k < 5; ++k) P[4 + k] = s_pr[3 + k];
    P[9] = s_cand_total;
  }
}

// ---------------------------------------------------------------------------
// Tiny subtrees (<= 64 rows): one wavefront per subtree, one row per lane.
//
// A node is a 64-bit mask of the wave's lanes, so partitioning is a mask AND
// and never moves data. Per feature, each lane finds the set of lanes whose
// code is <= its own with 8 ballots (an MSB-first radix rank over the code
// bits); class counts of that left set are popcounts against per-class lane
// masks; the split cost uses the same integer-form criterion (table lookups
// for counts <= 64) and the wave picks (min cost, then min code) with DPP
// reductions. No LDS histogram, no workgroup barriers: four independent
// subtrees per 256-thread workgroup, dozens per CU.
//
// tiny: int64 [K][8] = {start, m, depth, buffer, root_slot, -, -, -}; child
// slots come from the global node counter, two per split.
//
// Measured alternative (not kept): the block finisher running its own job's
// tiny subtrees in a tail (5 waves in the reused histogram LDS, no second
// launch) took 1.98 ms on the flagship fit vs 1.66 ms for block + tiny kernel;
// each tail serialises behind its job and the chip runs <= 10 tail waves per
// CU, where this kernel keeps ~12 waves per CU busy on any pending subtree.
constexpr int kTinyRows = 64;
constexpr int kTinyWaves = 4;

__device__ __forceinline__ uint32_t wave_min_u32_dpp(uint32_t v) {
  v = min(v, dpp_u32<kDppRowShr + 1>(v, v));
  v = min(v, dpp_u32<kDppRowShr + 2>(v, v));
  v = min(v, dpp_u32<kDppRowShr + 4>(v, v));
  v = min(v, dpp_u32<kDppRowShr + 8>(v, v));
  v = min(v, dpp_u32<kDppRowBcast15, 0xa>(v, v));
  v = min(v, dpp_u32<kDppRowBcast31, 0xc>(v, v));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

constexpr int kTinyMaxF = 128;
constexpr int kTinyStride = kTinyMaxF / 4 + 1;  // words per staged row (+1: bank spread)

// kMany (C > kTinyMaxC, up to 256 classes): the subtree's classes present in
// its <= 64 rows -- at most 64 -- are compacted in ascending class order at the
// subtree root (their lane masks and counts live in LDS), and every class sum
// runs over them only. Absent classes add T(0) = 0 / 0 to the host builder's
// sequential sums, so the fp64 results are bit-identical.
template <bool kMany>
__global__ __launch_bounds__(256) void finish_tiny_kernel(
    const uint32_t* __restrict__ codes_rm, int64_t row_words, const uint32_t* __restrict__ buf0,
    const uint32_t* __restrict__ buf1, const int32_t* __restrict__ y, FinRowLab rl,
    const int64_t* __restrict__ tiny, const int32_t* __restrict__ tiny_count,
    int32_t* __restrict__ tiny_counter, int F, int C, int crit, int max_depth, int64_t mss,
    int64_t msl, const double* __restrict__ xtab, int32_t* __restrict__ node_i32,
    int32_t* __restrict__ node_cnt, const int32_t* __restrict__ order) {
  constexpr int kMC = kMany ? kTinyRows : kTinyMaxC;  // class slots per wave
  __shared__ double s_tab[kTinyRows + 1];
  __shared__ uint32_t s_codes[kTinyWaves][kTinyRows * kTinyStride];
  __shared__ unsigned long long s_mask[kTinyWaves][16];
  __shared__ int32_t s_dep[kTinyWaves][16], s_slot[kTinyWaves][16];
  // kMany: compacted classes {lane mask, class id} and the node's counts per wave
  __shared__ unsigned long long s_cm[kMany ? kTinyWaves : 1][kMany ? kTinyRows : 1];
  __shared__ int32_t s_cid[kMany ? kTinyWaves : 1][kMany ? kTinyRows : 1];
  __shared__ int32_t s_mc[kMany ? kTinyWaves : 1][kMany ? kTinyRows : 1];
  // kMany: the node's present classes (ascending): their row masks in the node and
  // counts -- the feature loop sums over these only (deep nodes hold few classes)
  __shared__ unsigned long long s_nm[kMany ? kTinyWaves : 1][kMany ? kTinyRows : 1];
  __shared__ int32_t s_nmc[kMany ? kTinyWaves : 1][kMany ? kTinyRows : 1];
  const int lane = lane_id();
  const int wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i <= kTinyRows; i += blockDim.x) s_tab[i] = xtab[i];
  __syncthreads();
  const int K = *tiny_count;
  const int nw = (int)min<int64_t>(row_words, kTinyMaxF / 4);
  uint32_t* my_codes = &s_codes[wave][lane * kTinyStride];
  const uint8_t* my_bytes = reinterpret_cast<const uint8_t*>(my_codes);
  WaveClaim claim;
  const int claim_batch = wave_claim_batch(K);
  for (;;) {
    const int k = wave_claim_next(claim, tiny_counter, K, claim_batch);
    if (k >= K) break;
    // order (optional): the records by rows descending (launch_tiny_order)
    const int64_t* rec = tiny + (int64_t)(order ? order[k] : k) * 8;
    const int64_t start = rec[0];
    const int m = (int)rec[1];
    if (m < 2) continue;  // (an unused reserved record)
    const int depth0 = (int)rec[2];
    const uint32_t* src = rec[3] ? buf1 : buf0;
    const int64_t root_slot = rec[4];
    const bool act = lane < m;
    int lab = 0;
    if (act) {
      const uint32_t ent = src[start + lane];
      const uint32_t row = rl.shift ? (ent & rl.mask) : ent;
      lab = rl.shift ? (int)(ent >> rl.shift) : y[row];
      for (int i = 0; i < nw; ++i) my_codes[i] = codes_rm[(int64_t)row * row_words + i];
    }
    unsigned long long cm[kMany ? 1 : kTinyMaxC];
    int nc = C;  // class slots in use
    if constexpr (kMany) {
      // ascending distinct labels of the subtree: repeated wave minimum
      unsigned long long left = __ballot(act);
      nc = 0;
      while (left) {
        const uint32_t cur = wave_min_u32_dpp(((left >> lane) & 1ull) ? (uint32_t)lab : 0xffffffffu);
        const unsigned long long mk = __ballot(((left >> lane) & 1ull) && (uint32_t)lab == cur);
        if (lane == 0) {
          s_cm[wave][nc] = mk;
          s_cid[wave][nc] = (int)cur;
        }
        left &= ~mk;
        ++nc;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    } else {
#pragma unroll
      for (int c = 0; c < kTinyMaxC; ++c) cm[c] = c < C ? __ballot(act && lab == c) : 0ull;
    }
    auto cmask = [&](int c) -> unsigned long long {
      if constexpr (kMany) return s_cm[wave][c];
      else return cm[c];
    };
    if (lane == 0) {
      s_mask[wave][0] = m == 64 ? ~0ull : ((1ull << m) - 1ull);
      s_dep[wave][0] = depth0;
      s_slot[wave][0] = (int32_t)root_slot;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int sp = 1;
    while (sp > 0) {
      --sp;
      const unsigned long long M = s_mask[wave][sp];
      const int d = s_dep[wave][sp];
      const int64_t slot = s_slot[wave][sp];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int mm = __popcll(M);
      int mc[kMany ? 1 : kTinyMaxC];
      double acc = 0.0;
      int64_t sq = 0;
      int ncn = 0;  // kMany: classes present in this node
      if constexpr (kMany) {
        for (int c = 0; c < nc; ++c) {
          const unsigned long long nm = M & s_cm[wave][c];
          const int v = __popcll(nm);
          if (lane == 0) {
            s_mc[wave][c] = v;
            if (v > 0) {
              s_nm[wave][ncn] = nm;
              s_nmc[wave][ncn] = v;
            }
          }
          ncn += v > 0;
          acc = acc + s_tab[v];
          sq += (int64_t)v * v;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      } else {
#pragma unroll
        for (int c = 0; c < kTinyMaxC; ++c) {
          mc[c] = c < C ? __popcll(M & cm[c]) : 0;
          if (c < C) {
            acc = acc + s_tab[mc[c]];
            sq += (int64_t)mc[c] * mc[c];
          }
        }
      }
      auto ccount = [&](int c) -> int {
        if constexpr (kMany) return s_mc[wave][c];
        else return mc[c];
      };
      const double pterm = crit == kEntropy ? s_tab[mm] - acc : gini_term(mm, sq);
      const double tu = tie_unit(s_tab[mm], (int64_t)mm);
      const double tinv = 1.0 / tu;
      const bool inm = (M >> lane) & 1ull;
      double bg = -__builtin_inf(), bc = __builtin_inf();
      int bf = 0x7fffffff;
      uint32_t bb = 0xffffffffu;
      for (int f = 0; f < F; ++f) {
        const uint32_t code = my_bytes[f];
        // lanes of M whose code is greater than / equal to mine (radix rank, MSB first)
        unsigned long long eq = M, gt = 0ull;
#pragma unroll
        for (int b = 7; b >= 0; --b) {
          const unsigned long long bm = __ballot((code >> b) & 1u) & M;
          if ((code >> b) & 1u) {
            eq &= bm;
          } else {
            gt |= eq & bm;
            eq &= ~bm;
          }
        }
        const unsigned long long le = M & ~gt;
        const int ml = __popcll(le);
        const int mr = mm - ml;
        double cost = __builtin_inf();
        if (inm && ml >= msl && mr >= msl) {
          // absent classes add T(0) = 0 (or 0 squared) to both sums: the node's
          // present classes in ascending order give bit-identical sums
          if constexpr (kMany) {
            if (crit == kEntropy) {
              double sl = 0.0, sr = 0.0;
              for (int i = 0; i < ncn; ++i) {
                const int lc = __popcll(le & s_nm[wave][i]);
                sl = sl + s_tab[lc];
                sr = sr + s_tab[s_nmc[wave][i] - lc];
              }
              cost = (s_tab[ml] - sl) + (s_tab[mr] - sr);
            } else {
              int64_t ql = 0, qr = 0;
              for (int i = 0; i < ncn; ++i) {
                const int64_t lc = __popcll(le & s_nm[wave][i]);
                const int64_t rc = s_nmc[wave][i] - lc;
                ql += lc * lc;
                qr += rc * rc;
              }
              cost = gini_term(ml, ql) + gini_term(mr, qr);
            }
          } else if (crit == kEntropy) {
            double sl = 0.0, sr = 0.0;
#pragma unroll
            for (int c = 0; c < kMC; ++c) {
              if (c < nc) {
                const int lc = __popcll(le & cmask(c));
                sl = sl + s_tab[lc];
                sr = sr + s_tab[ccount(c) - lc];
              }
            }
            cost = (s_tab[ml] - sl) + (s_tab[mr] - sr);
          } else {
            int64_t ql = 0, qr = 0;
#pragma unroll
            for (int c = 0; c < kMC; ++c) {
              if (c < nc) {
                const int64_t lc = __popcll(le & cmask(c));
                const int64_t rc = ccount(c) - lc;
                ql += lc * lc;
                qr += rc * rc;
              }
            }
            cost = gini_term(ml, ql) + gini_term(mr, qr);
          }
          cost = tie_round(cost, tinv, tu);
        }
        // per-lane running best; features ascend, so strict > keeps the lowest
        const double g = pterm - cost;
        if (g > bg) {
          bg = g;
          bf = f;
          bc = cost;
          bb = code;
        }
      }
      // one wave reduction per node: max gain, then lowest feature, then lowest
      // cost, then lowest code -- the same choice as reducing every feature
      // separately (min cost, min code) and keeping the first strictly better gain
#pragma unroll
      for (int d = kWave / 2; d > 0; d >>= 1) {
        const double og = __shfl_xor(bg, d, kWave);
        const int of = __shfl_xor(bf, d, kWave);
        const double oc = __shfl_xor(bc, d, kWave);
        const uint32_t ob = (uint32_t)__shfl_xor((int)bb, d, kWave);
        const bool take =
            og > bg ||
            (og == bg && (of < bf || (of == bf && (oc < bc || (oc == bc && ob < bb)))));
        if (take) {
          bg = og;
          bf = of;
          bc = oc;
          bb = ob;
        }
      }
      bf = __builtin_amdgcn_readfirstlane(bf);
      bb = (uint32_t)__builtin_amdgcn_readfirstlane((int)bb);
      if (!(bg > -__builtin_inf()) || bf < 0) continue;  // leaf: the creation record stands
      const unsigned long long LM = M & __ballot((uint32_t)my_bytes[bf] <= bb);
      const unsigned long long RM = M & ~LM;
      const int nl = __popcll(LM), nr = __popcll(RM);
      // a split always leaves rows on both sides; anything else is a kernel bug --
      // stop here instead of re-splitting into positions outside the subtree
      if (nl == 0 || nr == 0) continue;
      const int64_t ls = slot + 1, rs = slot + 2 * nl;  // pre-order position ranges
      int nzl = 0, nzr = 0;
      if constexpr (kMany) {
        // every class of both children: absent ones 0, the subtree's from its masks
        for (int c = lane; c < C; c += kWave) {
          node_cnt[ls * C + c] = 0;
          node_cnt[rs * C + c] = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int c = 0; c < nc; ++c) {
          const int lc = __popcll(LM & s_cm[wave][c]);
          const int rc = s_mc[wave][c] - lc;
          nzl += lc > 0;
          nzr += rc > 0;
          if (lane == 0) {
            node_cnt[ls * C + s_cid[wave][c]] = lc;
            node_cnt[rs * C + s_cid[wave][c]] = rc;
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < kTinyMaxC; ++c) {
          if (c < C) {
            const int lc = __popcll(LM & cm[c]);
            const int rc = mc[c] - lc;
            nzl += lc > 0;
            nzr += rc > 0;
            if (lane == c) {
              node_cnt[ls * C + c] = lc;
              node_cnt[rs * C + c] = rc;
            }
          }
        }
      }
      const int cd = d + 1;
      if (lane == 0) {
        int32_t* P = node_i32 + slot * 6;
        P[0] = bf;
        P[1] = (int32_t)bb;
        P[2] = (int32_t)ls;
        P[3] = (int32_t)rs;
        int32_t* L = node_i32 + ls * 6;
        int32_t* R = node_i32 + rs * 6;
        L[0] = -1; L[1] = -1; L[2] = -1; L[3] = -1; L[4] = cd; L[5] = nl;
        R[0] = -1; R[1] = -1; R[2] = -1; R[3] = -1; R[4] = cd; R[5] = nr;
      }
      const bool depth_stop = max_depth >= 0 && cd >= max_depth;
      const bool tlf = depth_stop || nl < mss || nl < 2 * msl || nzl <= 1;
      const bool trf = depth_stop || nr < mss || nr < 2 * msl || nzr <= 1;
      const bool left_small = nl <= nr;
      for (int pass = 0; pass < 2; ++pass) {
        const bool is_left = (pass == 0) ? !left_small : left_small;
        if (is_left ? tlf : trf) continue;
        if (lane == 0) {
          s_mask[wave][sp] = is_left ? LM : RM;
          s_dep[wave][sp] = cd;
          s_slot[wave][sp] = (int32_t)(is_left ? ls : rs);
        }
        ++sp;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// ---------------------------------------------------------------------------
// Tiny subtrees, C <= 2: presorted per-feature lane orders.
//
// A child's rows are a subset of its parent's, so the order of the subtree's
// rows by each feature's code is computed once per tiny subtree (an 8-ballot
// MSB-first radix rank, stable by lane) and stored in LDS as 16-bit entries
// srt[f][k] = {code : 8, run end : 1, -, lane : 6} for sorted position k.
// At every node of the subtree lane k reads srt[f][k] (64 consecutive
// halfwords: conflict-free); one packed DPP prefix sum of {in node, in node and
// class 1} along the sorted order gives both left counts of the split "code <=
// code at k". Splits are scored at the ends of equal-code runs of the subtree
// order: a run holding node rows yields exactly the reference candidate (the
// last node row of that code); a run without node rows repeats the previous
// partition with a larger code and never wins the (gain, feature, cost, code)
// order. Costs come from a per-launch table H[a][b] = T(a) - (T(a-b) + T(b))
// (entropy) or gini_term(a, (a-b)^2 + b^2), a <= 64 -- two lookups and one add
// per candidate, bitwise equal to the six-lookup form. Two features are scanned
// per iteration (independent DPP chains); the wave reduces once per node.
//
// LDS per wave: srt [F][64] halfwords + 64 flag bytes (tiny_wave_bytes); per
// workgroup: the H table (tiny_h_entries doubles).
#ifndef MT_TINY_SMALL
#define MT_TINY_SMALL 16
#endif
constexpr int kTinySmallNode = MT_TINY_SMALL;  // nodes of 3..16 rows: one lane per feature
constexpr int kTinyH = (kTinyRows + 1) * (kTinyRows + 2) / 2;  // triangular a <= 64, b <= a
__device__ __forceinline__ int tiny_h_idx(int a, int b) { return ((a * (a + 1)) >> 1) + b; }

// H table for one criterion (entropy from the shared x*log2(x) values).
__device__ __forceinline__ void tiny_fill_h(double* __restrict__ H, const double* __restrict__ xtab,
                                            int crit) {
  for (int i = threadIdx.x; i < kTinyH; i += blockDim.x) {
    int a = 0;
    while (tiny_h_idx(a + 1, 0) <= i) ++a;
    const int b = i - tiny_h_idx(a, 0);
    H[i] = crit == kEntropy ? xtab[a] - (xtab[a - b] + xtab[b])
                            : gini_term(a, (int64_t)(a - b) * (a - b) + (int64_t)b * b);
  }
}

// code_bytes 1: 16-bit sorted entries {code : 8, run end : 1, -, lane : 6};
// 2 (more than 256 bins): 32-bit entries {code : 16, run end : 1, -, lane : 6}
__host__ __device__ inline int tiny_wave_bytes(int F, int code_bytes = 1) {
  return F * kWave * 2 * code_bytes + kWave;
}

struct TinyOut {
  int32_t* node_i32;
  int32_t* node_cnt;
};

template <typename CodeT>
__device__ __forceinline__ void tiny_sorted_subtree(
    const uint32_t* __restrict__ codes_rm, int64_t row_words, const uint32_t* __restrict__ src,
    const int32_t* __restrict__ y, FinRowLab rl, int64_t start, int m, int depth0,
    int64_t root_slot, int F, int C, int crit, int max_depth, int64_t mss, int64_t msl,
    const double* __restrict__ H, const uint32_t* __restrict__ Hrow,
    std::conditional_t<sizeof(CodeT) == 1, uint16_t, uint32_t>* __restrict__ srt,
    uint8_t* __restrict__ flag,
    unsigned long long* __restrict__ st_mask, int32_t* __restrict__ st_dep,
    int32_t* __restrict__ st_slot, TinyOut out, bool coherent = false) {
  const int lane = lane_id();
  const unsigned long long below = (1ull << lane) - 1ull;
  const bool act = lane < m;
  uint32_t row = 0;
  int lab = 0;
  if (act) {
    // coherent: the rows were written by another workgroup of this kernel
    const uint32_t ent =
        coherent ? __hip_atomic_load(const_cast<uint32_t*>(src) + start + lane, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT)
                 : src[start + lane];
    row = rl.shift ? (ent & rl.mask) : ent;
    lab = rl.shift ? (int)(ent >> rl.shift) : y[row];
  }
  const unsigned long long R = m == 64 ? ~0ull : ((1ull << m) - 1ull);
  const unsigned long long cm1 = C > 1 ? __ballot(act && lab == 1) : 0ull;
  const int mslw = (int)(msl < 65 ? msl : 65);
  // ---- presort: srt[f][position] = {code, run end, lane}. Keys {code : 8,
  // lane : 8} are unique, so a bitonic network over the wave sorts them stably;
  // two features share a 32-bit register (packed 16-bit min / max). 16-bit
  // codes: keys {code : 16, lane : 8}, one feature per register.
  constexpr int kCpw = 4 / (int)sizeof(CodeT);         // codes per 32-bit word
  constexpr uint32_t kCodeMask = sizeof(CodeT) == 1 ? 0xffu : 0xffffu;
  const uint32_t* rowp = codes_rm + (int64_t)row * row_words;
  const int nwords = (F + kCpw - 1) / kCpw;
  // subtrees of at most kTinySmallNode rows never scan (every node takes the
  // lane-per-feature path below), so they skip the presort
  if (m > kTinySmallNode && sizeof(CodeT) == 2) {
    int lg = 1;  // sort network size 2^lg >= m (m >= 2)
    while ((1 << lg) < m) ++lg;
    for (int w = 0; w < nwords; ++w) {
      const uint32_t word = act ? rowp[w] : 0u;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int f = w * 2 + h;
        if (f >= F) break;
        uint32_t v = act ? ((word >> (16 * h)) & 0xffffu) << 8 | (uint32_t)lane : 0xffffffffu;
        v = bitonic64_u32(v, lane, lg);
        const uint32_t nv = (uint32_t)__shfl_down((int)v, 1, kWave);
        const bool endl = lane == m - 1;
        const uint32_t ea = (endl || (nv >> 8) != (v >> 8)) ? 0x80u : 0u;
        srt[f * kWave + lane] = act ? (v | ea) : 0xffffff3fu;
      }
    }
  } else if (m > kTinySmallNode) {
    int lg = 1;  // sort network size 2^lg >= m (m >= 2)
    while ((1 << lg) < m) ++lg;
    for (int w = 0; w < nwords; ++w) {
      const uint32_t word = act ? rowp[w] : 0u;
  #pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int f = w * 4 + 2 * h;
        if (f >= F) break;
        const uint32_t ka = ((word >> (16 * h)) & 0xffu) << 8 | (uint32_t)lane;
        const uint32_t kb = ((word >> (16 * h + 8)) & 0xffu) << 8 | (uint32_t)lane;
        uint32_t v = act ? (ka | (kb << 16)) : 0xffffffffu;
        v = bitonic64_pk_u16(v, lane, lg);
        const uint32_t nv = (uint32_t)__shfl_down((int)v, 1, kWave);
        const bool endl = lane == m - 1;
        const uint32_t ea = (endl || ((nv >> 8) & 0xffu) != ((v >> 8) & 0xffu)) ? 0x80u : 0u;
        const uint32_t eb = (endl || (nv >> 24) != (v >> 24)) ? 0x80u : 0u;
        // positions past the subtree: lane 63 (never a row there, so no node
        // bits), no run end -- the scan loop needs no activity test
        srt[f * kWave + lane] = act ? (uint16_t)((v & 0xffffu) | ea) : (uint16_t)0xff3fu;
        if (f + 1 < F) srt[(f + 1) * kWave + lane] = act ? (uint16_t)((v >> 16) | eb) : (uint16_t)0xff3fu;
      }
    }
  }
  if (lane == 0) {
    st_mask[0] = R;
    st_dep[0] = depth0;
    st_slot[0] = (int32_t)root_slot;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  int sp = 1;
  while (sp > 0) {
    --sp;
    const unsigned long long M = st_mask[sp];
    const int d = st_dep[sp];
    const int64_t slot = st_slot[sp];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int mm = __popcll(M);
    const int mc1 = __popcll(M & cm1);
    const double pterm = H[tiny_h_idx(mm, mc1)];
    const double tu = tie_unit(xlog2x((uint64_t)mm), (int64_t)mm);
    const double tinv = 1.0 / tu;
    const char* Hb = reinterpret_cast<const char*>(H);
    // H[tri(a) + b] by byte offset; Hrow[a] = 8 tri(a) (an LDS lookup is cheaper
    // than the multiply on the VALU-bound path)
    auto hval = [&](int a, int b) -> double {
      return *reinterpret_cast<const double*>(Hb + Hrow[a] + ((uint32_t)b << 3));
    };
    int bf = -1;
    uint32_t bb = 0xffffffffu;
    unsigned long long LM = 0ull;
    if (mm == 2) {
      // Two rows of different classes (pure nodes are never pushed): the only
      // partition is {a} | {b}, which costs 0 (entropy and gini) for every
      // feature whose codes differ, so the lowest such feature wins at the
      // smaller code -- no scans.
      const int a = __ffsll((long long)M) - 1, b = 63 - __clzll((long long)M);
      if (mslw <= 1) {
        const uint32_t ra = (uint32_t)__builtin_amdgcn_readlane((int)row, a);
        const uint32_t rb = (uint32_t)__builtin_amdgcn_readlane((int)row, b);
        for (int w0 = 0; w0 < nwords; w0 += kWave) {
          const int w = w0 + lane;
          uint32_t x = 0u, wa = 0u;
          if (w < nwords) {
            wa = codes_rm[(int64_t)ra * row_words + w];
            x = wa ^ codes_rm[(int64_t)rb * row_words + w];
          }
          const unsigned long long nz = __ballot(x != 0u);
          if (nz) {
            const int wl = __ffsll((long long)nz) - 1;
            const uint32_t xw = (uint32_t)__builtin_amdgcn_readlane((int)x, wl);
            const uint32_t aw = (uint32_t)__builtin_amdgcn_readlane((int)wa, wl);
            constexpr int kBits = 8 * (int)sizeof(CodeT);
            const int byte = (__ffs((int)xw) - 1) / kBits;  // (the code's index in the word)
            const int f = (w0 + wl) * kCpw + byte;
            if (f < F) {  // (codes past F are row padding)
              const uint32_t ca = (aw >> (kBits * byte)) & kCodeMask;
              const uint32_t cb = ca ^ ((xw >> (kBits * byte)) & kCodeMask);
              bf = f;
              bb = ca < cb ? ca : cb;
              LM = ca < cb ? (1ull << a) : (1ull << b);
            }
            break;
          }
        }
      }
      if (bf < 0) continue;  // identical rows (or min_samples_leaf > 1): leaf
    } else if (mm <= kTinySmallNode) {
      // Small node: one lane per feature. Lane f reads the node rows' codes of
      // feature f (coalesced bytes of each row, L2-resident) and scores every
      // distinct code as a threshold from the left counts {rows, class-1 rows}
      // -- mm^2 integer steps and mm table costs per lane instead of a wave
      // scan per feature pair; same tie-rounded costs and the same
      // (gain, feature, cost, code) order as the scan below.
      uint32_t rj[kTinySmallNode], lj[kTinySmallNode];
      unsigned long long rest = M;
#pragma unroll
      for (int t = 0; t < kTinySmallNode; ++t) {
        const int j = rest ? __ffsll((long long)rest) - 1 : 0;
        rest &= rest - 1ull;
        rj[t] = (uint32_t)__builtin_amdgcn_readlane((int)row, j);
        lj[t] = 1u | ((uint32_t)((cm1 >> j) & 1ull) << 16);  // {row, class-1 row}
      }
      double bg = -__builtin_inf(), bc = __builtin_inf();
      bf = 0x7fffffff;
      const CodeT* cb8 = reinterpret_cast<const CodeT*>(codes_rm);
      const int64_t rbytes = row_words * kCpw;  // (codes per row)
      uint32_t code[kTinySmallNode];
      for (int f0 = 0; f0 < F; f0 += kWave) {
        const int f = f0 + lane;
#pragma unroll
        for (int t = 0; t < kTinySmallNode; ++t)
          code[t] = (t < mm && f < F) ? (uint32_t)cb8[(int64_t)rj[t] * rbytes + f] : 0xffffu;
        if (f < F) {
#pragma unroll
          for (int i = 0; i < kTinySmallNode; ++i) {
            if (i >= mm) break;
            const uint32_t c = code[i];
            uint32_t acc = 0u;
#pragma unroll
            for (int t = 0; t < kTinySmallNode; ++t) acc += code[t] <= c ? lj[t] : 0u;
            const int ml = (int)(acc & 0xffffu), l1 = (int)(acc >> 16);
            const int mr = mm - ml, r1 = mc1 - l1;
            if (ml >= mslw && mr >= mslw) {
              const double cost = tie_round(hval(ml, l1) + hval(mr, r1), tinv, tu);
              const double g = pterm - cost;
              if (g > bg || (g == bg && (f < bf || (f == bf && (cost < bc ||
                                                             (cost == bc && c < bb)))))) {
                bg = g;
                bf = f;
                bc = cost;
                bb = c;
              }
            }
          }
        }
      }
#pragma unroll
      for (int dd = kWave / 2; dd > 0; dd >>= 1) {
        const double og = __shfl_xor(bg, dd, kWave);
        const int of = __shfl_xor(bf, dd, kWave);
        const double oc = __shfl_xor(bc, dd, kWave);
        const uint32_t ob = (uint32_t)__shfl_xor((int)bb, dd, kWave);
        const bool tk =
            og > bg || (og == bg && (of < bf || (of == bf && (oc < bc || (oc == bc && ob < bb)))));
        if (tk) {
          bg = og;
          bf = of;
          bc = oc;
          bb = ob;
        }
      }
      bf = __builtin_amdgcn_readfirstlane(bf);
      bb = (uint32_t)__builtin_amdgcn_readfirstlane((int)bb);
      if (!(bg > -__builtin_inf()) || bf < 0 || bf >= F) continue;
      // left rows from lane bf's codes of the node rows
      const int f0w = bf & ~(kWave - 1);
      if (F > kWave) {  // code[] holds the last chunk: reload the winning one
#pragma unroll
        for (int t = 0; t < kTinySmallNode; ++t)
          code[t] = (t < mm && f0w + lane < F) ? (uint32_t)cb8[(int64_t)rj[t] * rbytes + f0w + lane]
                                              : 0xffffu;
      }
      rest = M;
#pragma unroll
      for (int t = 0; t < kTinySmallNode; ++t) {
        if (t >= mm) break;
        const int j = __ffsll((long long)rest) - 1;
        rest &= rest - 1ull;
        const uint32_t ct = (uint32_t)__builtin_amdgcn_readlane((int)code[t], bf - f0w);
        if (ct <= bb) LM |= 1ull << j;
      }
    } else {
      // candidates compare by their tie-rounding grid index q = rint(cost / tu):
      // the gain pterm - q tu orders exactly as -q (tu >> the fp64 error of the
      // product and the difference), so (max gain, min cost) is (min q) -- the
      // grid product and the subtraction are never computed per candidate
      double bq = __builtin_inf();
      bf = 0x7fffffff;
      // this lane's row in the node: {in : 8, in and class 1 : 8}, fetched per
      // feature at sorted position k with one ds_bpermute from lane srt[f][k]
      const bool lin = act && ((M >> lane) & 1ull);
      const int nodebits = lin ? (1 | ((((cm1 >> lane) & 1ull) != 0ull) ? 0x100 : 0)) : 0;
      // split cost at this lane's sorted position from the left counts (ml, l1)
      auto cost_of = [&](uint32_t v, int ml, int l1) -> double {
        const int mr = mm - ml, r1 = mc1 - l1;
        const bool ok = (v & 0x80u) && ml >= mslw && mr >= mslw;
        const double q = __builtin_rint((hval(ml, l1) + hval(mr, r1)) * tinv);
        return ok ? q : __builtin_inf();
      };
      auto take = [&](int f, double q, uint32_t v) {
        const bool better = q < bq;  // features ascend: strict < keeps the lowest
        bq = better ? q : bq;
        bf = better ? f : bf;
        bb = better ? (v >> 8) : bb;
      };
      // two features per DPP scan: {in, class 1} counts of feature a in the low
      // 16 bits, of feature b in the high 16 (every field <= 64)
      for (int f = 0; f < F; f += 2) {
        const bool two = f + 1 < F;
        const uint32_t va = srt[f * kWave + lane];
        const uint32_t vb = two ? (uint32_t)srt[(f + 1) * kWave + lane] : 0u;
        const uint32_t xa = (uint32_t)__shfl(nodebits, (int)(va & 0x3fu), kWave);
        const uint32_t xb = (uint32_t)__shfl(nodebits, (int)(vb & 0x3fu), kWave);
        const uint32_t incl = wave_incl_scan_dpp(xa | (xb << 16));
        const double ca = cost_of(va, (int)(incl & 0xffu), (int)((incl >> 8) & 0xffu));
        const double cb = cost_of(vb, (int)((incl >> 16) & 0xffu), (int)(incl >> 24));
        take(f, ca, va);
        if (two) take(f + 1, cb, vb);
      }
#pragma unroll
      for (int dd = kWave / 2; dd > 0; dd >>= 1) {
        const double oq = __shfl_xor(bq, dd, kWave);
        const int of = __shfl_xor(bf, dd, kWave);
        const uint32_t ob = (uint32_t)__shfl_xor((int)bb, dd, kWave);
        const bool tk = oq < bq || (oq == bq && (of < bf || (of == bf && ob < bb)));
        if (tk) {
          bq = oq;
          bf = of;
          bb = ob;
        }
      }
      bf = __builtin_amdgcn_readfirstlane(bf);
      bb = (uint32_t)__builtin_amdgcn_readfirstlane((int)bb);
      if (!(bq < __builtin_inf()) || bf < 0) continue;  // leaf: the creation record stands
      // left rows: sorted positions of feature bf with code <= bb, scattered back to lanes
      {
        const uint32_t v = srt[bf * kWave + lane];
        if (act) flag[v & 0x3fu] = (uint8_t)((v >> 8) <= bb);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      LM = M & __ballot(act && flag[lane]);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    const unsigned long long RM = M & ~LM;
    const int nl = __popcll(LM), nr = __popcll(RM);
    // a split always leaves rows on both sides; anything else is a kernel bug --
    // stop here instead of re-splitting into positions outside the subtree
    if (nl == 0 || nr == 0) continue;
    const int64_t ls = slot + 1, rs = slot + 2 * nl;  // pre-order position ranges
    const int lc1 = __popcll(LM & cm1), rc1 = (int)mc1 - lc1;
    const int lc0 = nl - lc1, rc0 = nr - rc1;
    const int nzl = (lc0 > 0) + (lc1 > 0), nzr = (rc0 > 0) + (rc1 > 0);
    const int cd = d + 1;
    if (lane == 0) {
      int32_t* P = out.node_i32 + slot * 6;
      P[0] = bf;
      P[1] = (int32_t)bb;
      P[2] = (int32_t)ls;
      P[3] = (int32_t)rs;
      int32_t* L = out.node_i32 + ls * 6;
      int32_t* Rr = out.node_i32 + rs * 6;
      L[0] = -1; L[1] = -1; L[2] = -1; L[3] = -1; L[4] = cd; L[5] = nl;
      Rr[0] = -1; Rr[1] = -1; Rr[2] = -1; Rr[3] = -1; Rr[4] = cd; Rr[5] = nr;
      out.node_cnt[ls * C + 0] = lc0;
      out.node_cnt[rs * C + 0] = rc0;
      if (C > 1) {
        out.node_cnt[ls * C + 1] = lc1;
        out.node_cnt[rs * C + 1] = rc1;
      }
    }
    const bool depth_stop = max_depth >= 0 && cd >= max_depth;
    const bool tlf = depth_stop || nl < mss || nl < 2 * msl || nzl <= 1;
    const bool trf = depth_stop || nr < mss || nr < 2 * msl || nzr <= 1;
    const bool left_small = nl <= nr;
    for (int pass = 0; pass < 2; ++pass) {
      const bool is_left = (pass == 0) ? !left_small : left_small;
      if (is_left ? tlf : trf) continue;
      if (lane == 0) {
        st_mask[sp] = is_left ? LM : RM;
        st_dep[sp] = cd;
        st_slot[sp] = (int32_t)(is_left ? ls : rs);
      }
      ++sp;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// kW waves per workgroup share one H table; the launcher picks kW so the most
// waves fit a CU's LDS (F = 64: 16 waves in one 1024-thread workgroup instead of
// 3 x 4; F = 128: 8 instead of 4), see tiny_sorted_waves.
template <int kW, typename CodeT>
__global__ __launch_bounds__(kW * kWave) void finish_tiny_sorted_kernel(
    const uint32_t* __restrict__ codes_rm, int64_t row_words, const uint32_t* __restrict__ buf0,
    const uint32_t* __restrict__ buf1, const int32_t* __restrict__ y, FinRowLab rl,
    const int64_t* __restrict__ tiny, const int32_t* __restrict__ tiny_count,
    int32_t* __restrict__ tiny_counter, int F, int C, int crit, int max_depth, int64_t mss,
    int64_t msl, const double* __restrict__ xtab, int32_t* __restrict__ node_i32,
    int32_t* __restrict__ node_cnt, const int32_t* __restrict__ order) {
  extern __shared__ __align__(16) uint32_t dyn[];
  __shared__ double s_h[kTinyH];
  __shared__ uint32_t s_hrow[kTinyRows + 1];
  __shared__ unsigned long long s_mask[kW][16];
  __shared__ int32_t s_dep[kW][16], s_slot[kW][16];
  const int lane = lane_id();
  const int wave = threadIdx.x >> 6;
  using SrtT = std::conditional_t<sizeof(CodeT) == 1, uint16_t, uint32_t>;
  uint8_t* wbase = reinterpret_cast<uint8_t*>(dyn) + (size_t)wave * tiny_wave_bytes(F, sizeof(CodeT));
  SrtT* srt = reinterpret_cast<SrtT*>(wbase);
  uint8_t* flag = wbase + F * kWave * sizeof(SrtT);
  tiny_fill_h(s_h, xtab, crit);
  for (int a = threadIdx.x; a <= kTinyRows; a += blockDim.x) s_hrow[a] = 8u * (uint32_t)tiny_h_idx(a, 0);
  __syncthreads();
  const int K = *tiny_count;
  WaveClaim claim;
  const int claim_batch = wave_claim_batch(K);
  for (;;) {
    const int k = wave_claim_next(claim, tiny_counter, K, claim_batch);
    if (k >= K) break;
    // order (optional): the records by rows descending (launch_tiny_order)
    const int64_t* rec = tiny + (int64_t)(order ? order[k] : k) * 8;
    if (rec[1] < 2) continue;  // (an unused reserved record)
    tiny_sorted_subtree<CodeT>(codes_rm, row_words, rec[3] ? buf1 : buf0, y, rl, rec[0], (int)rec[1],
                        (int)rec[2], rec[4], F, C, crit, max_depth, mss, msl, s_h, s_hrow, srt, flag,
                        s_mask[wave], s_dep[wave], s_slot[wave], TinyOut{node_i32, node_cnt});
  }
}

// Waves per workgroup of the sorted tiny kernel: the most resident waves per CU
// under the LDS budget and the VGPR cap (<= 128 VGPRs: 4 waves per SIMD), fewer
// waves per workgroup on ties.
static int tiny_sorted_lds(int F, int w, int cb = 1) {  // static + dynamic LDS of one workgroup
  return kTinyH * 8 + (kTinyRows + 1) * 4 + w * 16 * 16 + w * tiny_wave_bytes(F, cb);
}

static int tiny_sorted_waves(int F, int cb = 1) {
  constexpr int kLdsPerCu = 160 * 1024, kWavesPerCu = 16;
  int best_w = 1, best = 0;
  for (int w : {1, 2, 4, 8, 16}) {
    const int bytes = tiny_sorted_lds(F, w, cb);
    if (bytes > kLdsPerCu) continue;
    const int waves = std::min(kLdsPerCu / bytes, kWavesPerCu / w) * w;
    if (waves > best) best = waves, best_w = w;
  }
  return best_w;
}

// Features per LDS histogram tile of the block finisher; 0: unsupported shape.
// The whole node histogram in one pass when it fits (<= 150 KB, F <= 256);
// else tiles sized for two 512-thread workgroups per CU (<= 62 KB), or -- when
// that leaves fewer than 4 features per tile (many classes) -- for one
// 1024-thread workgroup per CU (<= 140 KB).
static int finish_feature_tile_of(int F, int B, int Ct) {
  const int per_f = fin_fstride(B, (Ct + 1) / 2) * 4;
  if (F <= kFinMaxF && F * per_f <= 150 * 1024) return F;
  int ft = 62 * 1024 / per_f;
  if (ft < 4) ft = 140 * 1024 / per_f;
  if (ft <= 0) return 0;
  // <= 256: a tile's row words (one byte per code) fit one wave's 64 lanes
  ft = std::min(ft, kFinMaxF);
  if (ft >= 16) ft &= ~15;  // 16-B row loads stay aligned at every tile start
  return std::min(ft, F);
}
static int finish_lds_bytes_of(int F, int B, int C, int ft) {
  // + per-wave class carries of the multi-pass (B > 256) scan, + the node's
  // present-class list (C > 2)
  return ft * fin_fstride(B, (fin_tile_classes(C) + 1) / 2) * 4 +
         (B > 256 ? (kFinThreadsWide / kWave) * C * 4 : 0) + (C > 2 ? (2 * C + 1) * 4 : 0) +
         (C > kFinStackC ? 2 * C * 4 : 0);
}
int finish_feature_tile(int F, int B, int C) {
  if (F <= 0 || C <= 0 || B <= 0 || B > kFinMaxB) return 0;
  if (C > kFinMaxC && B > 256) return 0;  // (many classes: one 256-bin pass only)
  const int ft = finish_feature_tile_of(F, B, fin_tile_classes(C));
  // the class arrays grow with C: past what one CU's LDS holds, no finisher
  if (ft <= 0 || finish_lds_bytes_of(F, B, C, ft) > 150 * 1024) return 0;
  return ft;
}
int finish_lds_bytes(int F, int B, int C) {
  return finish_lds_bytes_of(F, B, C, finish_feature_tile(F, B, C));
}
int finish_max_classes() { return kFinMaxC; }
// Largest finisher job (rows) for C classes (the x log2 x table bound otherwise).
int finish_job_rows_cap(int C) { return C > kFinMaxC ? kFinClassJobRows : (1 << 16) - 1; }

// Global scratch for the DFS stack's class counts and the node's / left class
// counts (C > kFinStackC): [grid][kFinStack + 2][C], grow-only, one buffer per
// device (finisher launches of a device share one stream).
static int32_t* fin_stack_scratch(int grid, int C) {
  static int32_t* buf[64] = {};
  static size_t cap[64] = {};
  int dev = 0;
  MT_HIP_CHECK(hipGetDevice(&dev));
  const size_t need = (size_t)grid * (kFinStack + 2) * C * sizeof(int32_t);
  if (dev < 0 || dev >= 64) throw std::runtime_error("finisher: device index out of range");
  if (need > cap[dev]) {
    if (buf[dev]) MT_HIP_CHECK(hipFree(buf[dev]));
    MT_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&buf[dev]), need));
    cap[dev] = need;
  }
  return buf[dev];
}

void launch_finish(hipStream_t stream, const void* codes_rm, int64_t row_words,
                   const void* codes_fm, int code_bytes, int64_t n_rows, uint32_t* buf0,
                   uint32_t* buf1, const int32_t* y, int lab_shift, const int64_t* jobs, int J,
                   int32_t* counter, const int32_t* nbins, int F, int B, int C, int crit,
                   int max_depth, int64_t mss, int64_t msl, const double* xtab,
                   const float* xtabf, int xtab_n,
                   int32_t* node_i32, int32_t* node_cnt, int64_t* tasks, int32_t* task_flag,
                   int32_t epoch, int task_cap, int grid, int tiny_rows, int64_t* tiny,
                   int tiny_grid, int64_t* prof, int tiny_waves, int32_t* tiny_order) {
  // counter: int32 [8] = {job cursor, tiny count, tiny cursor, -...}, zeroed by the
  // host. node_i32 / node_cnt are indexed by pre-order position (jobs[j][3] is
  // job j's root position); rows a fit never writes keep n = 0 (host memset).
  if (J <= 0) return;
  const int Ft = finish_feature_tile(F, B, C);
  if (Ft <= 0) throw std::runtime_error("finisher: unsupported shape (class arrays or bins "
                                        "past the LDS budget)");
  // the two-class kernel (fp32 prefilter, hand-off queue) needs the single-pass
  // layout (Ft == F <= kFinMaxF: per-feature LDS arrays)
  const bool c2 = C <= 2 && Ft == F && F <= kFinMaxF && B <= 256;
  const bool tiny_sorted = C <= 2 && getenv_int("MPITREE_TINY_SORTED", 1) != 0;
  // (16-bit codes: the sorted tiny kernel only, 32-bit sorted entries)
  if (tiny == nullptr || (code_bytes != 1 && !tiny_sorted)) tiny_rows = 0;
  if (!tiny_sorted && F > kTinyMaxF) tiny_rows = 0;
  if (tiny_sorted && tiny_sorted_lds(F, 1, code_bytes) > 160 * 1024) tiny_rows = 0;  // > ~1100 features
  tiny_rows = std::min(tiny_rows, kTinyRows);
  FinRowLab rl{lab_shift ? ((1u << lab_shift) - 1u) : 0xffffffffu, lab_shift};
  const size_t lds = (size_t)finish_lds_bytes(F, B, C);
  int32_t* gstk = nullptr;
#define MT_FIN_NT(CT, C2, NT)                                                                 \
  MT_HIP_CHECK(mt_set_max_lds((const void*)finish_cls_kernel<CT, C2, NT>,                \
                                   (int)lds));    \
  hipLaunchKernelGGL((finish_cls_kernel<CT, C2, NT>), dim3(grid), dim3(NT), lds, stream,      \
                     (const uint32_t*)codes_rm, row_words, (const CT*)codes_fm, n_rows, buf0, \
                     buf1, y, rl, jobs, J, counter, nbins, F, B, C, crit, max_depth, mss,     \
                     msl, xtab, xtabf, xtab_n, node_i32, node_cnt, tasks, task_flag, epoch,   \
                     task_cap, tiny_rows,                                                     \
                     tiny, counter + kFinCtrTinyCount, prof, Ft, gstk);
  // When the histogram leaves room for only one 512-thread workgroup per CU
  // (F = 128: 133 KB), run 1024 threads per workgroup instead: same LDS, twice
  // the waves to hide the gather and LDS latency. The persistent grid shrinks
  // to match (one workgroup per CU where there were two).
  bool wide = false;
  if (getenv_int("MPITREE_FIN_WIDE", 1) != 0) {
    int per_cu = 0;
    const void* k512 = code_bytes == 1 ? (c2 ? (const void*)finish_cls_kernel<uint8_t, true, kFinThreadsSmall>
                                             : (const void*)finish_cls_kernel<uint8_t, false, kFinThreadsSmall>)
                                       : (c2 ? (const void*)finish_cls_kernel<uint16_t, true, kFinThreadsSmall>
                                             : (const void*)finish_cls_kernel<uint16_t, false, kFinThreadsSmall>);
    MT_HIP_CHECK(mt_set_max_lds(k512, (int)lds));
    MT_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k512, kFinThreadsSmall, lds));
    wide = per_cu == 1;
  }
  if (wide) {
    int dev = 0, n_cu = 0;
    MT_HIP_CHECK(hipGetDevice(&dev));
    MT_HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    grid = std::max(1, std::min(grid, n_cu));
  }
  if (C > kFinStackC) gstk = fin_stack_scratch(grid, C);
#define MT_FIN(CT, C2)                       \
  if (wide) {                                \
    MT_FIN_NT(CT, C2, kFinThreadsWide)       \
  } else {                                   \
    MT_FIN_NT(CT, C2, kFinThreadsSmall)      \
  }
  if (code_bytes == 1) {
    if (c2) {
      MT_FIN(uint8_t, true)
    } else {
      MT_FIN(uint8_t, false)
    }
  } else {
    if (c2) {
      MT_FIN(uint16_t, true)
    } else {
      MT_FIN(uint16_t, false)
    }
  }
#undef MT_FIN
#undef MT_FIN_NT
  MT_HIP_CHECK(hipGetLastError());
  if (tiny_rows > 0) {
    // (tiny_order: [2 * 65] scratch, then the order; null keeps discovery order)
    int32_t* order = nullptr;
    if (tiny_order) {
      order = tiny_order + 2 * 65;
      launch_tiny_order(stream, tiny, counter + kFinCtrTinyCount, tiny_order, order, 128);
    }
    if (tiny_sorted) {
      const int cb = code_bytes;
      // waves per workgroup: the most that fit a CU (many subtrees: occupancy), or
      // the caller's request (few subtrees -- a subtree-owning rank -- spread over
      // more CUs); MPITREE_TINY_WAVES overrides both
      int w = getenv_int("MPITREE_TINY_WAVES",
                         tiny_waves > 0 ? tiny_waves : tiny_sorted_waves(F, cb));
      for (int cand : {16, 8, 4, 2, 1}) {  // the largest allowed width <= the request
        if (cand <= w && tiny_sorted_lds(F, cand, cb) <= 160 * 1024) {
          w = cand;
          break;
        }
      }
      // tiny_grid counts 4-wave workgroups: keep the total wave count
      const int g = std::max(1, tiny_grid * kTinyWaves / w);
      const size_t lds = (size_t)w * tiny_wave_bytes(F, cb);
#define MT_TS(W, CT)                                                                         \
  MT_HIP_CHECK(mt_set_max_lds((const void*)finish_tiny_sorted_kernel<W, CT>,            \
                                   (int)lds));   \
  hipLaunchKernelGGL((finish_tiny_sorted_kernel<W, CT>), dim3(g), dim3(W * kWave), lds,      \
                     stream, (const uint32_t*)codes_rm, row_words, buf0, buf1, y, rl, tiny,  \
                     counter + kFinCtrTinyCount, counter + kFinCtrTinyCount + 1, F, C, crit, \
                     max_depth, mss, msl, xtab, node_i32, node_cnt, order);
#define MT_TSW(CT)   \
  if (w == 16) {     \
    MT_TS(16, CT)    \
  } else if (w == 8) { \
    MT_TS(8, CT)     \
  } else if (w == 4) { \
    MT_TS(4, CT)     \
  } else if (w == 2) { \
    MT_TS(2, CT)     \
  } else {           \
    MT_TS(1, CT)     \
  }
      if (cb == 1) {
        MT_TSW(uint8_t)
      } else {
        MT_TSW(uint16_t)
      }
#undef MT_TSW
#undef MT_TS
    } else {
#define MT_TG(MANY)                                                                          \
  hipLaunchKernelGGL(finish_tiny_kernel<MANY>, dim3(tiny_grid), dim3(kTinyWaves * kWave), 0,  \
                     stream, (const uint32_t*)codes_rm, row_words, buf0, buf1, y, rl, tiny,   \
                     counter + kFinCtrTinyCount, counter + kFinCtrTinyCount + 1, F, C, crit, \
                     max_depth, mss, msl, xtab, node_i32, node_cnt, order);
      if (C > kTinyMaxC) {
        MT_TG(true)
      } else {
        MT_TG(false)
      }
#undef MT_TG
    }
    MT_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace mt
