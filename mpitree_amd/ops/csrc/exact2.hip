// Exact split search on presorted per-feature lists, driven from the device.
//
// The reference takes every unique value of a feature as a candidate
// threshold (mpitree/tree/decision_tree.py:73-90). Histogram engines are exact
// only while a feature has at most 256 values; with continuous data a feature
// has up to n. This engine keeps, for each of this rank's features (a
// contiguous block [f_lo, f_hi) -- the whole range on one GPU, F/P features
// per rank when feature-parallel), the rows sorted by value and grouped by
// frontier node, in 4-byte entries
//
//   E[f][p] = row | dup << 24 | label << 25          (rows < 2^24, labels < 128)
//
// (more than 128 classes: E[f][p] = row | dup << 24 and labels are gathered from
// the row-indexed label array -- any class count, one gather per label read)
//
// (dup: the value occurs more than once in the column; only then do two
// neighbours' values need comparing, from X itself) plus, for regression, the
// fixed-point target Y[f][p] moved alongside. Split thresholds are data values
// X[row][f]; their value ranks (the threshold bins) are resolved once at the
// end by a binary search in the setup's sorted order (xe_rank_kernel). Node i owns positions [start_i, start_i + m_i) of
// every list. A level is a fixed chain of launches whose work counts are read
// from device memory, with a one-workgroup planner -- the host never waits:
//
//   xe_tot       per (chunk, feature): class-1 count / class counts / target sum
//                (+ min / max of the targets for feature 0: regression purity)
//   xe_carry     per (node, feature): exclusive prefix of the chunk totals
//   xe_scan      per (chunk, feature): class prefix (or target prefix sum) at
//                every position, the shared integer-form cost (criterion.h) at
//                every value boundary, the chunk's best (cost, position)
//   xe_select    per node: best feature (max gain, ties to the lowest feature),
//                the split's left statistics, threshold row and value rank
//   [feature-parallel: all-gather of the records + fp_combine_kernel]
//   xe_plan      one workgroup: decisions -> position space, finisher jobs, split
//                list, next frontier, the next level's chunk items
//   xe_flag      rows of split nodes: left iff their position in the split
//                feature's segment is < n_left (the feature's owner writes them;
//                feature-parallel ranks sum the flags with one all-reduce)
//   xe_pcount / xe_pcarry / xe_pscatter
//                stable partition of every feature's split segments into the
//                other list buffer (left rows first, both halves stay sorted)
//
// Every quantity is an integer or the shared fp64 criterion, so trees equal the
// host builders' bit for bit. Segments of at most 256 rows leave as finisher
// jobs (the histogram finishers on subtree-local 8-bit codes, xe_local_codes).
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "common.h"
#include "criterion.h"
#include "grow.h"
#include "exact2.h"

namespace mt {

constexpr int kXeThreads = 256;
constexpr int kXePer = 8;                       // entries per thread
constexpr int kXeChunk = kXeThreads * kXePer;   // entries per chunk item
constexpr int kXeWaves = kXeThreads / kWave;
constexpr int kXeMaxC = 128;                    // labels live in 7 bits of an entry
constexpr int kXeMaxClasses = 1 << 20;          // labels by row (XeArgs::ylab) past kXeMaxC
constexpr int kXePlanThreads = 512;
constexpr int kXePlanWaves = kXePlanThreads / kWave;
constexpr int kXeLocalMax = 256;                // finisher jobs: local codes fit a byte

__device__ __forceinline__ uint32_t xe_row(uint32_t e) { return e & 0xFFFFFFu; }
__device__ __forceinline__ bool xe_dup(uint32_t e) { return (e >> 24) & 1u; }
__device__ __forceinline__ int xe_lab(uint32_t e) { return (int)(e >> 25); }
// the label of an entry: packed in the entry, or (C > kXeMaxC) gathered by row
__device__ __forceinline__ int xe_label(const XeArgs& a, uint32_t e) {
  return a.ylab ? a.ylab[xe_row(e)] : xe_lab(e);
}

__device__ __forceinline__ double xe_tl(int64_t x, const double* __restrict__ tab, int tn) {
  return x < (int64_t)tn ? tab[x] : xlog2x((uint64_t)x);
}

// Monotone uint64 image of a double (total order of non-NaN values).
__device__ __forceinline__ uint64_t xe_dkey(double d) {
  const uint64_t b = (uint64_t)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double xe_dval(uint64_t k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}

// ---------------------------------------------------------------------------
// Decoupled look-back: single-pass segmented prefix sums over chunk items.
//
// Work is claimed through an atomic ticket t -> (item t / F_loc, feature
// t % F_loc), so an item's predecessors in its segment hold smaller tickets:
// running (or finished) workgroups, which publish their chunk's aggregate
// before they look back themselves. The smallest unfinished ticket never
// waits, so the grid always drains. Status words are relaxed agent-scope
// atomics -- the value travels inside the word, nothing else needs ordering --
// tagged per level, so they are never cleared.
constexpr uint64_t kXeAgg = 1, kXeIncl = 2;


__device__ __forceinline__ void xe_publish(uint64_t* w, uint32_t tag, uint64_t state, uint32_t v) {
  __hip_atomic_store(w, ((uint64_t)tag << 34) | (state << 32) | (uint64_t)v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of chunk q >= 1 of a segment whose status words are
// st[-stride], ..., st[-q stride] (nearest first). Called by one whole wave:
// each round reads 64 predecessors at once (lane l: st[-(d0 + l) stride]) and
// ends at the nearest inclusive prefix once every status up to it has been
// published, adding the aggregates before it; a window of 64 aggregates moves
// the next one back. Every decision is a wave-uniform ballot and the loop is
// bounded by q, so it always ends; a wait beyond 2 s (a bug, never a schedule)
// sets *watch and returns instead of hanging the GPU. Every lane returns the
// prefix.
__device__ __forceinline__ int64_t xe_lookback(const uint64_t* st, int64_t stride, int q,
                                               uint32_t tag, int32_t* watch) {
  const int lane = lane_id();
  q = __builtin_amdgcn_readfirstlane(q);
  int64_t acc = 0;
  const uint64_t t0 = wall_clock64();
  int d0 = 1;
  uint32_t spins = 0;
  while (d0 <= q) {
    const int d = d0 + lane;
    const bool in = d <= q;
    const uint64_t s =
        in ? __hip_atomic_load(st - (int64_t)d * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
           : 0ull;
    const bool ready = in && (uint32_t)(s >> 34) == tag;
    const unsigned long long nr = __ballot(in && !ready);
    const unsigned long long bi = __ballot(ready && ((s >> 32) & 3ull) == kXeIncl);
    const int fi = bi ? __ffsll((long long)bi) - 1 : kWave;  // nearest inclusive prefix
    const int fn = nr ? __ffsll((long long)nr) - 1 : kWave;  // nearest unpublished
    if (fi < kWave ? fn > fi : nr == 0ull) {
      acc += (int64_t)wave_sum_u32((in && lane <= fi) ? (uint32_t)s : 0u);
      if (fi < kWave) break;
      d0 += kWave;  // 64 aggregates (the segment's first chunk is inclusive)
      continue;
    }
    if ((++spins & 63u) == 0u && wall_clock64() - t0 > 200000000ull) {
      if (lane == 0) atomicExch(watch, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return acc;
}

// ---------------------------------------------------------------------------
// xe_tot: grid (items bound, F_loc); block (it, f) exits past the device count.
__device__ __forceinline__ void xe_tot_item(const XeArgs& a, const XeLists& L, int64_t it, int f,
                            uint32_t* s_c, int64_t (*s_w)[3]);

// Items are visited grid-stride (the grid is a bounded slice of the host's
// item bound): a level with few items costs few empty workgroups.
__global__ __launch_bounds__(kXeThreads) void xe_tot_kernel(XeArgs a, XeLists L) {
  __shared__ uint32_t s_c[kXeMaxC];
  __shared__ int64_t s_w[kXeWaves][3];
  const int NI = L.ctl[1];
  for (int64_t it = blockIdx.x; it < NI; it += gridDim.x) {
    xe_tot_item(a, L, it, blockIdx.y, s_c, s_w);
    __syncthreads();
  }
}

__device__ __forceinline__ void xe_tot_item(const XeArgs& a, const XeLists& L, int64_t it, int f,
                            uint32_t* s_c, int64_t (*s_w)[3]) {
  const int64_t c0 = L.items[it * 4 + 2], cn = L.items[it * 4 + 3];
  const uint32_t* E = a.E + (int64_t)f * a.n + c0;
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int Cc = xe_cc(a.C);
  int64_t* out = a.tot + (it * a.F_loc + f) * Cc;
  if (a.C == 0) {  // regression: target sum (+ min / max on the first local feature)
    const int64_t* Yp = a.Y + (int64_t)f * a.n + c0;
    int64_t s = 0, mn = LLONG_MAX, mx = LLONG_MIN;
    for (int64_t i = tid; i < cn; i += kXeThreads) {
      const int64_t v = Yp[i];
      s += v;
      mn = v < mn ? v : mn;
      mx = v > mx ? v : mx;
    }
    for (int d = kWave / 2; d > 0; d >>= 1) {
      s += __shfl_xor(s, d, kWave);
      const int64_t o1 = __shfl_xor(mn, d, kWave), o2 = __shfl_xor(mx, d, kWave);
      mn = o1 < mn ? o1 : mn;
      mx = o2 > mx ? o2 : mx;
    }
    if (lane == 0) {
      s_w[w][0] = s;
      s_w[w][1] = mn;
      s_w[w][2] = mx;
    }
    __syncthreads();
    if (tid == 0) {
      int64_t t = 0, a1 = LLONG_MAX, a2 = LLONG_MIN;
      for (int q = 0; q < kXeWaves; ++q) {
        t += s_w[q][0];
        a1 = s_w[q][1] < a1 ? s_w[q][1] : a1;
        a2 = s_w[q][2] > a2 ? s_w[q][2] : a2;
      }
      out[0] = t;
      if (f == 0) {
        a.cmm[it * 2 + 0] = a1;
        a.cmm[it * 2 + 1] = a2;
      }
    }
    return;
  }
  if (a.C <= 2) {  // class-1 entries by wave sums
    uint32_t e[kXePer];
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      const int64_t i = (int64_t)k * kXeThreads + tid;
      e[k] = i < cn ? E[i] : 0u;
    }
    uint32_t ones = 0;
#pragma unroll
    for (int k = 0; k < kXePer; ++k)
      ones += ((int64_t)k * kXeThreads + tid < cn && xe_lab(e[k]) == 1) ? 1u : 0u;
    ones = wave_sum_u32(ones);
    if (lane == 0) s_w[w][0] = ones;
    __syncthreads();
    if (tid == 0) {
      int64_t t = 0;
      for (int q = 0; q < kXeWaves; ++q) t += s_w[q][0];
      out[0] = cn - t;
      if (a.C == 2) out[1] = t;
    }
    return;
  }
  if (a.C > kXeMaxC) {  // many classes: count straight into the chunk's totals
    for (int c = tid; c < a.C; c += kXeThreads) out[c] = 0;
    __threadfence_block();
    __syncthreads();
    for (int64_t i = tid; i < cn; i += kXeThreads)
      atomicAdd(reinterpret_cast<unsigned long long*>(out + xe_label(a, E[i])), 1ull);
    return;
  }
  for (int c = tid; c < a.C; c += kXeThreads) s_c[c] = 0;
  __syncthreads();
  for (int64_t i = tid; i < cn; i += kXeThreads) atomicAdd(&s_c[xe_label(a, E[i])], 1u);
  __syncthreads();
  for (int c = tid; c < a.C; c += kXeThreads) out[c] = s_c[c];
}

// xe_carry: one thread per (slot, local feature, stat): exclusive prefix of the
// chunk totals over the slot's items; regression slot min / max (f = 0, k = 0).
__global__ __launch_bounds__(kXeThreads) void xe_carry_kernel(XeArgs a, XeLists L) {
  const int K = L.ctl[0];
  const int Cc = xe_cc(a.C);
  const int64_t g = (int64_t)blockIdx.x * kXeThreads + threadIdx.x;
  if (g >= (int64_t)K * a.F_loc * Cc) return;
  const int k = (int)(g % Cc);
  const int f = (int)((g / Cc) % a.F_loc);
  const int64_t slot = g / ((int64_t)Cc * a.F_loc);
  const int i0 = L.ifirst[slot], i1 = L.ifirst[slot + 1];
  if (k == 0 && a.nmin) a.nmin[slot * a.F_loc + f] = 0xffffffffu;  // (two-pass scan)
  int64_t acc = 0;
  for (int it = i0; it < i1; it += 8) {  // 8 totals in flight per round trip
    int64_t v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      v[q] = it + q < i1 ? a.tot[((int64_t)(it + q) * a.F_loc + f) * Cc + k] : 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (it + q < i1) a.carry[((int64_t)(it + q) * a.F_loc + f) * Cc + k] = acc;
      acc += v[q];
    }
  }
  if (a.C == 0 && f == 0 && k == 0) {
    int64_t mn = LLONG_MAX, mx = LLONG_MIN;
    for (int it = i0; it < i1; ++it) {
      mn = a.cmm[it * 2 + 0] < mn ? a.cmm[it * 2 + 0] : mn;
      mx = a.cmm[it * 2 + 1] > mx ? a.cmm[it * 2 + 1] : mx;
    }
    L.minmax[slot * 2 + 0] = mn;
    L.minmax[slot * 2 + 1] = mx;
  }
}

// The same with one wave per (slot, feature, class): 64 totals per round trip and a
// wave prefix sum (integer sums: any order is exact). For levels with few slots, each
// holding hundreds of chunks (level 0: ~500 chunks, 50 us serially per thread).
__global__ __launch_bounds__(kXeThreads) void xe_carry_wave_kernel(XeArgs a, XeLists L) {
  const int K = L.ctl[0];
  const int Cc = xe_cc(a.C);
  const int lane = lane_id();
  const int64_t g = ((int64_t)blockIdx.x * kXeThreads + threadIdx.x) >> 6;  // wave
  if (g >= (int64_t)K * a.F_loc * Cc) return;
  const int k = (int)(g % Cc);
  const int f = (int)((g / Cc) % a.F_loc);
  const int64_t slot = g / ((int64_t)Cc * a.F_loc);
  const int i0 = L.ifirst[slot], i1 = L.ifirst[slot + 1];
  if (lane == 0 && k == 0 && a.nmin) a.nmin[slot * a.F_loc + f] = 0xffffffffu;
  int64_t acc = 0;
  for (int it0 = i0; it0 < i1; it0 += kWave) {
    const int it = it0 + lane;
    const int64_t v = it < i1 ? a.tot[((int64_t)it * a.F_loc + f) * Cc + k] : 0;
    const int64_t incl = wave_incl_scan_i64(v);
    if (it < i1) a.carry[((int64_t)it * a.F_loc + f) * Cc + k] = acc + incl - v;
    acc += __shfl(incl, kWave - 1, kWave);
  }
  if (a.C == 0 && f == 0 && k == 0) {
    int64_t mn = LLONG_MAX, mx = LLONG_MIN;
    for (int it = i0 + lane; it < i1; it += kWave) {
      mn = a.cmm[it * 2 + 0] < mn ? a.cmm[it * 2 + 0] : mn;
      mx = a.cmm[it * 2 + 1] > mx ? a.cmm[it * 2 + 1] : mx;
    }
    for (int d = kWave / 2; d > 0; d >>= 1) {
      const int64_t o1 = __shfl_xor(mn, d, kWave), o2 = __shfl_xor(mx, d, kWave);
      mn = o1 < mn ? o1 : mn;
      mx = o2 > mx ? o2 : mx;
    }
    if (lane == 0) {
      L.minmax[slot * 2 + 0] = mn;
      L.minmax[slot * 2 + 1] = mx;
    }
  }
}

// Feature value of a row (the input matrix, fp32 or fp64, row-major [n][F]).
__device__ __forceinline__ double xe_x(const void* X, int x64, int F, uint32_t row, int fg) {
  const int64_t o = (int64_t)row * F + fg;
  return x64 ? reinterpret_cast<const double*>(X)[o]
             : (double)reinterpret_cast<const float*>(X)[o];
}

// Value boundary between consecutive entries of a segment: equal values need
// both entries flagged dup (a value that occurs more than once in the column)
// and equal values (-0.0 == 0.0, as np.unique).
__device__ __forceinline__ bool xe_boundary(uint32_t e, uint32_t nx, const XeArgs& a, int fg) {
  if (nx == 0xFFFFFFFFu || !xe_dup(e) || !xe_dup(nx)) return true;
  return xe_x(a.X, a.x64, a.F, xe_row(e), fg) != xe_x(a.X, a.x64, a.F, xe_row(nx), fg);
}

// xe_scan: per (chunk, feature): the chunk's best {cost key, position}.
// Classification keys are tie-rounded costs (criterion.h tie_round units) so
// ties compare equal and the lowest position (smallest threshold) wins;
// regression keys are the exact fp64 costs (the host builder's strict <).
struct XeScanShared {
  uint32_t cnt[kXePer * kXeWaves];
  int64_t sum[kXePer * kXeWaves];
  uint64_t min[kXeWaves][2];
  float fmin[kXeWaves];
  uint32_t e[kXeThreads * kXePer + 1];
};

// kKind: the problem kind compiled into the item (0 regression, 2 more than
// two classes; two classes run xe_scan_c2_kernel) -- each kernel carries one path only, which keeps the
// scan's register (and scalar-register) footprint to what that path needs.
template <int kKind>
__device__ __forceinline__ void xe_scan_item(const XeArgs& a, const XeLists& L, int64_t it, int f,
                                             XeScanShared& sh);

template <int kKind>
__global__ __launch_bounds__(kXeThreads) void xe_scan_kernel(XeArgs a, XeLists L) {
  __shared__ XeScanShared sh;
  const int NI = L.ctl[1];
  for (int64_t it = blockIdx.x; it < NI; it += gridDim.x) {
    xe_scan_item<kKind>(a, L, it, blockIdx.y, sh);
    __syncthreads();
  }
}

template <int kKind>
__device__ __forceinline__ void xe_scan_item(const XeArgs& a, const XeLists& L, int64_t it, int f,
                                             XeScanShared& sh) {
  uint32_t* s_cnt = sh.cnt;
  int64_t* s_sum = sh.sum;
  uint64_t (*s_min)[2] = sh.min;
  uint32_t* s_e = sh.e;
  const int64_t slot = L.items[it * 4 + 0], sstart = L.items[it * 4 + 1];
  const int64_t c0 = L.items[it * 4 + 2], cn = L.items[it * 4 + 3];
  const int64_t m = L.cnt[slot];
  const uint32_t* Ef = a.E + (int64_t)f * a.n;
  const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int Cc = xe_cc(a.C);
  // entry i = k * 256 + tid of the chunk (coalesced), staged in LDS so every
  // thread sees its successor; the entry after the chunk (if the segment goes on)
  uint32_t e[kXePer];
#pragma unroll
  for (int k = 0; k < kXePer; ++k) {
    const int64_t i = (int64_t)k * kXeThreads + tid;
    e[k] = i < cn ? Ef[c0 + i] : 0xFFFFFFFFu;
    s_e[i] = e[k];
  }
  if (tid == 0) s_e[kXeChunk] = (c0 + cn - sstart) < m ? Ef[c0 + cn] : 0xFFFFFFFFu;
  __syncthreads();
  bool valid[kXePer];
#pragma unroll
  for (int k = 0; k < kXePer; ++k) {
    const int64_t i = (int64_t)k * kXeThreads + tid;
    const int64_t pos = c0 + i - sstart;
    const int64_t ml = pos + 1, mr = m - ml;
    bool v = i < cn && mr > 0 && ml >= a.msl && mr >= a.msl;
    if (v) v = xe_boundary(e[k], s_e[i + 1], a, a.f_lo + f);
    valid[k] = v;
  }
  unsigned long long mine = ~0ull;
  uint64_t mine_pos = ~0ull;
  if constexpr (kKind == 0) {
    // ---- regression: prefix sums of the targets, exact fp64 costs
    const int64_t* Yp = a.Y + (int64_t)f * a.n;
    int64_t y[kXePer];
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      const int64_t i = (int64_t)k * kXeThreads + tid;
      y[k] = i < cn ? Yp[c0 + i] : 0;
    }
    // (step, wave) sums -> exclusive scan over the 32 steps; lanes within a wave
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      const int64_t incl = wave_incl_scan_i64(y[k]);
      if (lane == kWave - 1) s_sum[k * kXeWaves + wave] = incl;
      y[k] = incl;  // inclusive within the wave
    }
    __syncthreads();
    if (tid < kWave) {
      const int64_t v = tid < kXePer * kXeWaves ? s_sum[tid] : 0;
      const int64_t incl = wave_incl_scan_i64(v);
      if (tid < kXePer * kXeWaves) s_sum[tid] = incl - v;
    }
    __syncthreads();
    const int64_t base = a.carry[(it * a.F_loc + f) * Cc];
    const int64_t S = L.stats[slot * 2 + 1];
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      if (!valid[k]) continue;
      const int64_t i = (int64_t)k * kXeThreads + tid;
      const int64_t pos = c0 + i - sstart;
      const int64_t ml = pos + 1, mr = m - ml;
      const int64_t sl = base + s_sum[k * kXeWaves + wave] + y[k];
      const double cost = mse_term(ml, sl) + mse_term(mr, S - sl);
      const uint64_t key = xe_dkey(cost);
      if (key < mine || (key == mine && (uint64_t)pos < mine_pos)) {
        mine = key;
        mine_pos = (uint64_t)pos;
      }
    }
  } else {
    // ---- C > 2: per class, one block scan of the class indicator
    const double tm = xe_tl(m, a.xtab, a.xtab_n);
    const double tu = tie_unit(tm, m);
    const double tinv = 1.0 / tu;
    double sL[kXePer], sR[kXePer];
    int64_t qL[kXePer], qR[kXePer];
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      sL[k] = sR[k] = 0.0;
      qL[k] = qR[k] = 0;
    }
    int lab[kXePer];
#pragma unroll
    for (int k = 0; k < kXePer; ++k)
      lab[k] = (int64_t)k * kXeThreads + tid < cn ? xe_label(a, e[k]) : -1;
    for (int c = 0; c < a.C; ++c) {
      // a class absent from the node adds T(0) = 0 (or 0 squared) on both sides:
      // skipping it leaves every sum bit-identical (block-uniform: one slot per item)
      if (L.stats[slot * Cc + c] == 0) continue;
      unsigned long long bal[kXePer];
#pragma unroll
      for (int k = 0; k < kXePer; ++k) {
        bal[k] = __ballot(lab[k] == c);
        if (lane == 0) s_cnt[k * kXeWaves + wave] = (uint32_t)__popcll(bal[k]);
      }
      __syncthreads();
      if (tid < kWave) {
        const uint32_t v = tid < kXePer * kXeWaves ? s_cnt[tid] : 0u;
        const uint32_t incl = wave_incl_scan_dpp(v);
        if (tid < kXePer * kXeWaves) s_cnt[tid] = incl - v;
      }
      __syncthreads();
      const int64_t basec = a.carry[(it * a.F_loc + f) * Cc + c];
      const int64_t tc = L.stats[slot * Cc + c];
#pragma unroll
      for (int k = 0; k < kXePer; ++k) {
        const int64_t Lc = basec + s_cnt[k * kXeWaves + wave] + __popcll(bal[k] & lt) +
                           ((bal[k] >> lane) & 1ull);
        const int64_t Rc = tc - Lc;
        if (a.crit == kEntropy) {
          sL[k] = sL[k] + xe_tl(Lc, a.xtab, a.xtab_n);
          sR[k] = sR[k] + xe_tl(Rc, a.xtab, a.xtab_n);
        } else {
          qL[k] += Lc * Lc;
          qR[k] += Rc * Rc;
        }
      }
      __syncthreads();  // s_cnt reuse
    }
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      if (!valid[k]) continue;
      const int64_t pos = c0 + (int64_t)k * kXeThreads + tid - sstart;
      const int64_t ml = pos + 1, mr = m - ml;
      double cost;
      if (a.crit == kEntropy)
        cost = (xe_tl(ml, a.xtab, a.xtab_n) - sL[k]) + (xe_tl(mr, a.xtab, a.xtab_n) - sR[k]);
      else
        cost = gini_term(ml, qL[k]) + gini_term(mr, qR[k]);
      double q = __builtin_rint(cost * tinv);
      const unsigned long long key = (unsigned long long)(q < 0.0 ? 0.0 : q);
      if (key < mine || (key == mine && (uint64_t)pos < mine_pos)) {
        mine = key;
        mine_pos = (uint64_t)pos;
      }
    }
  }
  // block lexicographic min of {key, position}
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const unsigned long long ok = __shfl_xor(mine, d, kWave);
    const unsigned long long op = __shfl_xor(mine_pos, d, kWave);
    if (ok < mine || (ok == mine && op < mine_pos)) {
      mine = ok;
      mine_pos = op;
    }
  }
  if (lane == 0) {
    s_min[wave][0] = mine;
    s_min[wave][1] = mine_pos;
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t bk = s_min[0][0], bp = s_min[0][1];
    for (int w = 1; w < kXeWaves; ++w)
      if (s_min[w][0] < bk || (s_min[w][0] == bk && s_min[w][1] < bp)) {
        bk = s_min[w][0];
        bp = s_min[w][1];
      }
    uint64_t* o = a.cbest + (it * a.F_loc + f) * 2;
    o[0] = bk;
    o[1] = bp;
  }
}

// Two-class scan, one wave per (chunk item, feature) and no workgroup barriers:
// the wave walks its 2048-entry chunk in four 512-entry rounds (8 entries per
// lane, round-robin so loads coalesce), carrying the class-1 count from round to
// round; a position's successor comes from the next lane (lane 63: the next row
// of the round, or memory past it). Per round: one ballot per row gives every
// left count, fp32 costs from the hardware log2 pick the candidates, their exact
// tie-rounded keys, and a running (key, position) minimum. Same outputs (cbest
// per item) and carries as the block scan; waves of a workgroup take different
// (item, feature) pairs. Per-position arithmetic is 32-bit (rows < 2^24).
//
// kPass 0 (gini; or entropy with MT_XE_TWO_PASS=0): candidates within the pad of
//   the ROUND's fp32 minimum -- near a flat optimum a round's costs all lie
//   within the pad, so nearly every position pays an exact key.
// kPass 1 (entropy): fp32 costs only; the chunk's minimum over valid positions
//   -> cmin[item][f], and an atomic minimum per (node, feature) -> nmin.
// kPass 2 (entropy): G = the node's fp32 minimum over this rank's features.
//   The node's exact best b satisfies c32(b) <= exact(b) + err <= exact(p) + err
//   <= c32(p) + 2 err for the valid position p attaining G, so only chunks with
//   cmin <= G + pad (pad >= 2 err) can hold it: every other chunk writes an
//   empty record without reading its entries, and a candidate chunk keys only
//   positions with c32 <= G + pad.
#ifndef MT_XE_HWLOG
#define MT_XE_HWLOG 1
#endif
#ifndef MT_XE_PAD  // candidate pad exponent: >= 2 x the fp32 error bound (35 * 2^-24)
#define MT_XE_PAD -17
#endif
#ifndef MT_XE_TWO_PASS
#define MT_XE_TWO_PASS 1
#endif
#ifndef MT_XE_P2_GRID  // workgroups of the second pass
#define MT_XE_P2_GRID 1024
#endif
// IEEE order as unsigned order (-0.0 folded into +0.0), and back
__device__ __forceinline__ uint32_t xe_fkey(float v) {
  const uint32_t b = __float_as_uint(v + 0.0f);
  return (b >> 31) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float xe_fval(uint32_t k) {
  return __uint_as_float((k >> 31) ? (k & 0x7fffffffu) : ~k);
}

template <int kPass>
__device__ __forceinline__ void xe_scan_wave_c2(const XeArgs& a, const XeLists& L, int64_t it,
                                                int f, float gthr = 0.0f) {
  const int lane = lane_id();
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int64_t slot = L.items[it * 4 + 0], sstart = L.items[it * 4 + 1];
  const int64_t c0 = L.items[it * 4 + 2];
  const int cn = (int)L.items[it * 4 + 3];
  const int m = L.cnt[slot];
  const int Cc = xe_cc(a.C);
  const uint32_t* Ef = a.E + (int64_t)f * a.n;
  const int t0 = (int)L.stats[slot * Cc + 0], t1 = a.C == 2 ? (int)L.stats[slot * Cc + 1] : 0;
  int run1 = a.C == 2 ? (int)a.carry[(it * a.F_loc + f) * Cc + 1] : 0;  // class-1 rows before
  const int msl = (int)(a.msl < (int64_t)m ? a.msl : (int64_t)m);
  const int p0 = (int)(c0 - sstart);  // the chunk's first position in its segment
  const double tm = xe_tl(m, a.xtab, a.xtab_n);
  const double tu = tie_unit(tm, m);
  const double tinv = 1.0 / tu;
  const bool entropy = a.crit == kEntropy;
  // candidates: within 2^MT_XE_PAD T(m) of the reference fp32 minimum (the
  // terms' error is <= 35 * 2^-24 T(m), so any pad >= 2^-17 = 128 * 2^-24 is safe)
  const float thr_pad = (float)tm * __builtin_ldexpf(1.0f, MT_XE_PAD);
  const int fg = a.f_lo + f;
  auto t32 = [](int x) -> float {
    const float v = (float)x;  // counts < 2^24: exact
#if MT_XE_HWLOG
    // hardware log2 (v_log_f32, |error| <= 4 * 2^-24 * x log2 x, checked for
    // x < 2^22 by tests/test_gpu_kernels.py::test_hw_log_terms_error_bound)
    return x > 1 ? v * __builtin_amdgcn_logf(v) : 0.0f;
#else
    return x > 1 ? v * log2f(v) : 0.0f;
#endif
  };
  unsigned long long mine = ~0ull;
  uint64_t mine_pos = ~0ull;
  // kPass 2: gthr = the node-wide candidate threshold (xe_gthr_kernel); the
  // caller only runs chunks whose fp32 minimum is within it
  float wmin = __builtin_inff();  // kPass 1: the chunk's fp32 minimum
  constexpr int kRound = kWave * kXePer;  // 512
  constexpr int kRounds = kXeChunk / kRound;  // an item holds at most kXeChunk entries
  // pass 1 (every chunk, the hot pass): every round's entries and the entry after
  // the item in flight at once -- unconditional loads clamped into the item (the
  // rounds used to load, wait and compute one after another); the other passes
  // keep one round in registers (pass 2 runs on few chunks, at its register budget)
  // (holding every round for pass 1 measured slower: 102 -> 116 us a level at 126
  // VGPRs, half the waves; MT_XE_HOLD_ROUNDS=1 builds it)
#ifndef MT_XE_HOLD_ROUNDS
#define MT_XE_HOLD_ROUNDS 0
#endif
  constexpr bool kAll = MT_XE_HOLD_ROUNDS && kPass == 1;
  constexpr int kHeld = kAll ? kRounds : 1;
  uint32_t ea[kHeld][kXePer];
  auto load_round = [&](int r, uint32_t (&dst)[kXePer]) {
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      const int i = r * kRound + k * kWave + lane;
      dst[k] = Ef[c0 + (i < cn ? i : cn - 1)];
    }
  };
  uint32_t tail = 0xFFFFFFFFu;
  if constexpr (kAll) {
#pragma unroll
    for (int r = 0; r < kRounds; ++r) load_round(r, ea[r]);
    tail = Ef[c0 + (p0 + cn < m ? cn : cn - 1)];  // the next item's first entry
  }
  // one round of the item: its entries e[] (past the item: all ones) and the
  // entry after the round (the next round's first, or the next item's first)
  auto round = [&](const int r0, uint32_t (&e)[kXePer], const uint32_t after) {
    unsigned long long bal[kXePer];
    int l1[kXePer];
    bool valid[kXePer];
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      const int i = r0 + k * kWave + lane;
      bal[k] = __ballot(i < cn && xe_lab(e[k]) == 1);
      l1[k] = run1 + __popcll(bal[k] & lt) + (int)((bal[k] >> lane) & 1ull);
      run1 += __popcll(bal[k]);
      // successor: next lane, or (lane 63) the next row's lane 0 / the entry after
      uint32_t nx = (uint32_t)__shfl_down((int)e[k], 1, kWave);
      const uint32_t row_next = k + 1 < kXePer
                                    ? (uint32_t)__builtin_amdgcn_readlane((int)e[k + 1 < kXePer ? k + 1 : k], 0)
                                    : after;
      if (lane == kWave - 1) nx = (k + 1 < kXePer && i + 1 < cn) ? row_next : after;
      const int ml = p0 + i + 1, mr = m - ml;
      bool v = i < cn && mr > 0 && ml >= msl && mr >= msl;
      if (v) v = xe_boundary(e[k], nx, a, fg);
      valid[k] = v;
    }
    auto exact_key = [&](int k) -> unsigned long long {
      const int64_t ml = p0 + r0 + k * kWave + lane + 1, mr = m - ml;
      const int64_t L1 = l1[k], L0 = ml - L1, R1 = t1 - L1, R0 = t0 - L0;
      double cost;
      if (entropy) {
        const double sl = xe_tl(L0, a.xtab, a.xtab_n) + xe_tl(L1, a.xtab, a.xtab_n);
        const double sr = xe_tl(R0, a.xtab, a.xtab_n) + xe_tl(R1, a.xtab, a.xtab_n);
        cost = (xe_tl(ml, a.xtab, a.xtab_n) - sl) + (xe_tl(mr, a.xtab, a.xtab_n) - sr);
      } else {
        cost = gini_term(ml, L0 * L0 + L1 * L1) + gini_term(mr, R0 * R0 + R1 * R1);
      }
      const double q = __builtin_rint(cost * tinv);
      return (unsigned long long)(q < 0.0 ? 0.0 : q);
    };
    float c32[kXePer];
    float fm = __builtin_inff();
    if (entropy) {
#pragma unroll
      for (int k = 0; k < kXePer; ++k) {
        c32[k] = __builtin_inff();
        if (!valid[k]) continue;
        const int ml = p0 + r0 + k * kWave + lane + 1, mr = m - ml;
        const int L1 = l1[k], L0 = ml - L1, R1 = t1 - L1, R0 = t0 - L0;
        c32[k] = (t32(ml) - (t32(L0) + t32(L1))) + (t32(mr) - (t32(R0) + t32(R1)));
        fm = fminf(fm, c32[k]);
      }
      if constexpr (kPass == 0) fm = wave_min_f32_dpp(fm);
    }
    if constexpr (kPass == 1) {
      wmin = fminf(wmin, fm);
      return;
    }
    const float thr = kPass == 2 ? gthr : fm + thr_pad;
#pragma unroll
    for (int k = 0; k < kXePer; ++k) {
      if (!valid[k] || (entropy && !(c32[k] <= thr))) continue;
      const unsigned long long key = exact_key(k);
      const uint64_t pos = (uint64_t)(p0 + r0 + k * kWave + lane);
      if (key < mine || (key == mine && pos < mine_pos)) {
        mine = key;
        mine_pos = pos;
      }
    }
    };
  if constexpr (kAll) {
#pragma unroll
    for (int rr = 0; rr < kRounds; ++rr) {
      const int r0 = rr * kRound;
      if (r0 >= cn) break;
      uint32_t e[kXePer];
#pragma unroll
      for (int k = 0; k < kXePer; ++k)
        e[k] = r0 + k * kWave + lane < cn ? ea[rr][k] : 0xFFFFFFFFu;
      uint32_t after = 0xFFFFFFFFu;
      if (r0 + kRound < cn)
        after = (uint32_t)__builtin_amdgcn_readlane((int)ea[rr + 1 < kRounds ? rr + 1 : rr][0], 0);
      else if (p0 + cn < m)
        after = tail;
      round(r0, e, after);
    }
  } else {
    for (int r0 = 0; r0 < cn; r0 += kRound) {
      uint32_t e[kXePer];
#pragma unroll
      for (int k = 0; k < kXePer; ++k) {
        const int i = r0 + k * kWave + lane;
        e[k] = i < cn ? Ef[c0 + i] : 0xFFFFFFFFu;
      }
      // entries past the round: lane 63 of the last row reads its successor
      const int iend = r0 + kRound;  // first index of the next round
      uint32_t after = 0xFFFFFFFFu;
      if (lane == kWave - 1) {
        if (iend < cn) after = Ef[c0 + iend];
        else if (p0 + cn < m) after = Ef[c0 + cn];
      }
      round(r0, e, after);
    }
  }
  if constexpr (kPass == 1) {
    wmin = wave_min_f32_dpp(wmin);
    if (lane == 0) {
      const uint32_t k = wmin < __builtin_inff() ? xe_fkey(wmin) : 0xffffffffu;
      a.cmin[it * a.F_loc + f] = k;
      if (k != 0xffffffffu) atomicMin(a.nmin + slot * a.F_loc + f, k);
    }
    return;
  }
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const unsigned long long ok = __shfl_xor(mine, d, kWave);
    const unsigned long long op = __shfl_xor(mine_pos, d, kWave);
    if (ok < mine || (ok == mine && op < mine_pos)) {
      mine = ok;
      mine_pos = op;
    }
  }
  if (lane == 0) {
    uint64_t* o = a.cbest + (it * a.F_loc + f) * 2;
    o[0] = mine;
    o[1] = mine_pos;
  }
}

// Pass-2 pairs per wave step: one chunk item's features (at most a wave)
__host__ __device__ inline int xe_p2_pairs(int F_loc) { return F_loc < kWave ? F_loc : kWave; }

// One wave per (chunk item, feature) pair, grid-stride over the level's pairs.
template <int kPass>
__global__ __launch_bounds__(kXeThreads) void xe_scan_c2_kernel(XeArgs a, XeLists L) {
  const int64_t total = (int64_t)L.ctl[1] * a.F_loc;
  const int64_t waves = (int64_t)gridDim.x * kXeWaves;
  if constexpr (kPass == 2) {
    // xe_p2_pairs(F_loc) pairs per wave step: each lane checks one chunk's fp32
    // minimum against its node's threshold (lane-parallel empty records for the
    // rest), then the wave scans the few candidate chunks one by one. Fewer than
    // 64 pairs when a chunk item has fewer features (feature-parallel ranks):
    // 64 pairs would span several consecutive chunks of one node -- the chunks
    // around its best threshold, candidates together -- and serialise them.
    const int lane = lane_id();
    const int pw = xe_p2_pairs(a.F_loc);
    for (int64_t b = ((int64_t)blockIdx.x * kXeWaves + (threadIdx.x >> 6)) * pw; b < total;
         b += waves * pw) {
      const int64_t w = b + lane;
      bool cand = false;
      float th = 0.0f;
      if (lane < pw && w < total) {
        const int64_t it = w / a.F_loc;
        th = a.gthr[L.items[it * 4 + 0]];
        cand = xe_fval(a.cmin[w]) <= th;  // (an empty chunk's key decodes to NaN)
        if (!cand) {
          uint64_t* o = a.cbest + w * 2;
          o[0] = ~0ull;
          o[1] = ~0ull;
        }
      }
      unsigned long long cm = __ballot(cand);
      while (cm) {
        const int l = __ffsll((long long)cm) - 1;
        cm &= cm - 1ull;
        const int64_t wu = b + l;
        const float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(th), l));
        xe_scan_wave_c2<2>(a, L, wu / a.F_loc, (int)(wu % a.F_loc), t);
      }
    }
    return;
  }
  for (int64_t w = (int64_t)blockIdx.x * kXeWaves + (threadIdx.x >> 6); w < total; w += waves) {
    const int64_t wu = __builtin_amdgcn_readfirstlane((int)w);
    xe_scan_wave_c2<kPass>(a, L, wu / a.F_loc, (int)(wu % a.F_loc));
  }
}

// Per slot: the node's fp32 minimum over this rank's features (pass 1's atomic
// minima) -> the pass-2 candidate threshold min + 2^MT_XE_PAD T(m) (-inf: no
// valid position, every chunk writes an empty record). One wave per slot.
__global__ __launch_bounds__(kXeThreads) void xe_gthr_kernel(XeArgs a, XeLists L) {
  const int64_t slot = (int64_t)blockIdx.x * kXeWaves + (threadIdx.x >> 6);
  if (slot >= L.ctl[0]) return;
  const int lane = lane_id();
  uint32_t nk = 0xffffffffu;
  for (int q = lane; q < a.F_loc; q += kWave) {
    const uint32_t v = a.nmin[slot * a.F_loc + q];
    nk = v < nk ? v : nk;
  }
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)nk, d, kWave);
    nk = o < nk ? o : nk;
  }
  if (lane == 0) {
    const int m = L.cnt[slot];
    const float pad = (float)xe_tl(m, a.xtab, a.xtab_n) * __builtin_ldexpf(1.0f, MT_XE_PAD);
    a.gthr[slot] = nk == 0xffffffffu ? -__builtin_inff() : xe_fval(nk) + pad;
  }
}

// xe_select: per slot, the best split over this rank's features.
// rec [K][R] = {gain bits, feature (global, -1 none), position, n_left, m,
//               threshold value rank, threshold row, left[Cc]}
// kXeSelThreads: 1024 while a level has few slots (a level-0 slot's 64 features x ~500
// chunk records per wave-feature loop were a 52 us chain of dependent loads with 4
// waves), 256 past that (many slots of few records)
template <int kXeSelThreads>
__global__ __launch_bounds__(kXeSelThreads) void xe_select_kernel(XeArgs a, XeLists L) {
  constexpr int kXeSelWaves = kXeSelThreads / kWave;
  __shared__ double s_gain[kXeSelWaves];
  __shared__ int s_feat[kXeSelWaves];
  __shared__ int64_t s_pos[kXeSelWaves];
  __shared__ double s_pterm;
  __shared__ uint32_t s_c[kXeMaxC];
  __shared__ int64_t s_sum[kXeSelWaves];
  const int64_t slot = blockIdx.x;
  if (slot >= L.ctl[0]) return;
  const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const int Cc = xe_cc(a.C);
  const int R = xe_rec_width(a.C);
  const int64_t start = L.start[slot], m = L.cnt[slot];
  const int64_t* st = L.stats + slot * Cc;
  int64_t* out = a.rec + slot * R;
  if (tid == 0) {  // sequential over classes, matching every other engine
    if (a.C == 0) {
      s_pterm = mse_term(m, L.stats[slot * 2 + 1]);
    } else {
      double acc = 0.0;
      int64_t sq = 0;
      for (int c = 0; c < a.C; ++c) {
        acc = acc + xlog2x((uint64_t)st[c]);
        sq += st[c] * st[c];
      }
      s_pterm = a.crit == kEntropy ? xlog2x((uint64_t)m) - acc : gini_term(m, sq);
    }
  }
  for (int c = tid; c < a.C && c < kXeMaxC; c += kXeSelThreads) s_c[c] = 0;
  __syncthreads();
  const double pterm = s_pterm;
  const double tu = a.C ? tie_unit(xe_tl(m, a.xtab, a.xtab_n), m) : 0.0;
  const int i0 = L.ifirst[slot], i1 = L.ifirst[slot + 1];
  double g = -__builtin_inf();
  int bf = 0x7fffffff;
  int64_t bp = -1;
  // one wave per feature, lanes over the slot's chunks: (key, position) minimum
  // (a level-0 slot holds n / 2048 chunks per feature)
  for (int f = wave; f < a.F_loc; f += kXeSelWaves) {
    uint64_t bk = ~0ull, bpos = ~0ull;
    for (int it = i0 + lane; it < i1; it += kWave) {
      const uint64_t* c = a.cbest + ((int64_t)it * a.F_loc + f) * 2;
      const uint64_t k = c[0], q = c[1];
      if (k < bk || (k == bk && q < bpos)) {
        bk = k;
        bpos = q;
      }
    }
#pragma unroll
    for (int d = kWave / 2; d > 0; d >>= 1) {
      const uint64_t ok = (uint64_t)__shfl_xor((unsigned long long)bk, d, kWave);
      const uint64_t oq = (uint64_t)__shfl_xor((unsigned long long)bpos, d, kWave);
      if (ok < bk || (ok == bk && oq < bpos)) {
        bk = ok;
        bpos = oq;
      }
    }
    if (bk == ~0ull) continue;  // (wave-uniform after the reduction)
    const double cost = a.C ? (double)bk * tu : xe_dval(bk);
    const double gf = pterm - cost;
    if (gf > g) {  // features ascend per wave: strict > keeps the lowest
      g = gf;
      bf = a.f_lo + f;
      bp = (int64_t)bpos;
    }
  }
  // (gain desc, feature asc) over the block
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const double og = __shfl_xor(g, d, kWave);
    const int of = __shfl_xor(bf, d, kWave);
    const int64_t op = __shfl_xor(bp, d, kWave);
    if (og > g || (og == g && of < bf)) {
      g = og;
      bf = of;
      bp = op;
    }
  }
  if (lane == 0) {
    s_gain[wave] = g;
    s_feat[wave] = bf;
    s_pos[wave] = bp;
  }
  __syncthreads();
  g = s_gain[0];
  bf = s_feat[0];
  bp = s_pos[0];
  for (int w = 1; w < kXeSelWaves; ++w)
    if (s_gain[w] > g || (s_gain[w] == g && s_feat[w] < bf)) {
      g = s_gain[w];
      bf = s_feat[w];
      bp = s_pos[w];
    }
  if (!(g > -__builtin_inf())) {
    if (tid == 0) {
      out[0] = (int64_t)double_to_bits(-__builtin_inf());
      out[1] = -1;
      out[2] = -1;
      out[3] = 0;
      out[4] = m;
      out[5] = -1;
      out[6] = -1;
    }
    for (int c = tid; c < Cc; c += kXeSelThreads) out[7 + c] = 0;
    return;
  }
  // left statistics: the carry of the chunk holding bp + the chunk's entries up to it
  const int fl = bf - a.f_lo;
  const uint32_t* Ef = a.E + (int64_t)fl * a.n;
  const int64_t ci = i0 + bp / kXeChunk;
  const int64_t cfirst = start + (bp / kXeChunk) * kXeChunk;
  const int64_t* car = a.carry + (ci * a.F_loc + fl) * Cc;
  if (a.C == 0) {
    const int64_t* Yp = a.Y + (int64_t)fl * a.n;
    int64_t s = 0;
    for (int64_t p = cfirst + tid; p <= start + bp; p += kXeSelThreads) s += Yp[p];
    s = wave_sum_i64(s);
    if (lane == 0) s_sum[wave] = s;
    __syncthreads();
    if (tid == 0) {
      int64_t t = car[0];
      for (int w = 0; w < kXeSelWaves; ++w) t += s_sum[w];
      out[7] = t;
    }
  } else if (a.C <= 2) {  // class-1 entries counted, class 0 the rest
    uint32_t ones = 0;
    for (int64_t p = cfirst + tid; p <= start + bp; p += kXeSelThreads)
      ones += xe_lab(Ef[p]) == 1 ? 1u : 0u;
    ones = wave_sum_u32(ones);
    if (lane == 0) s_sum[wave] = ones;
    __syncthreads();
    if (tid == 0) {
      int64_t t = 0;
      for (int w = 0; w < kXeSelWaves; ++w) t += s_sum[w];
      const int64_t nrows = bp - (cfirst - start) + 1;
      out[7] = car[0] + (nrows - t);
      if (a.C == 2) out[8] = car[1] + t;
    }
  } else if (a.C > kXeMaxC) {  // many classes: the chunk carry, then count into the record
    for (int c = tid; c < a.C; c += kXeSelThreads) out[7 + c] = car[c];
    __threadfence_block();
    __syncthreads();
    for (int64_t p = cfirst + tid; p <= start + bp; p += kXeSelThreads)
      atomicAdd(reinterpret_cast<unsigned long long*>(out + 7 + xe_label(a, Ef[p])), 1ull);
  } else {
    for (int64_t p = cfirst + tid; p <= start + bp; p += kXeSelThreads)
      atomicAdd(&s_c[xe_label(a, Ef[p])], 1u);
    __syncthreads();
    for (int c = tid; c < a.C; c += kXeSelThreads) out[7 + c] = car[c] + (int64_t)s_c[c];
  }
  if (tid == 0) {
    const uint32_t row = xe_row(Ef[start + bp]);
    out[0] = (int64_t)double_to_bits(g);
    out[1] = bf;
    out[2] = bp;
    out[3] = bp + 1;
    out[4] = m;
    out[5] = -1;  // value rank: resolved after growth (xe_rank_kernel)
    out[6] = (int64_t)row;
  }
}

// ---------------------------------------------------------------------------
// Planner (one workgroup): see XePlanArgs in exact2.h.
// Chunk-item runs of more than kXePlanDefer items (a big node's partition items or a big
// child's next-level items) are written by the whole workgroup after the node pass
// instead of by the node's thread (level 0: ~1000 items by one thread, 79 us).
constexpr int kXePlanDefer = 16;
constexpr int kXePlanBig = 64;
struct XePlanRun {
  int64_t* base;  // the run's first item
  int64_t s0, m;  // segment start and length
  int tag, cnt;   // item tag (split or slot index), items
};
struct XePlanShared {
  int w[kXePlanWaves];
  int carry[4];
  int nbig;
  XePlanRun big[kXePlanBig];
};

// Items q of a segment [s0, s0 + m): {tag, s0, s0 + q chunk, min(chunk, m - q chunk)}.
__device__ __forceinline__ void xe_plan_item(int64_t* it, int tag, int64_t s0, int64_t m, int q) {
  it[0] = tag;
  it[1] = s0;
  it[2] = s0 + (int64_t)q * kXeChunk;
  const int64_t rem = m - (int64_t)q * kXeChunk;
  it[3] = rem < kXeChunk ? rem : kXeChunk;
}

// A run of cnt items: deferred to the workgroup when long and a record is free.
__device__ __forceinline__ void xe_plan_run(XePlanShared& sh, int64_t* base, int tag, int64_t s0,
                                            int64_t m, int cnt) {
  if (cnt > kXePlanDefer) {
    const int b = atomicAdd(&sh.nbig, 1);
    if (b < kXePlanBig) {
      sh.big[b] = XePlanRun{base, s0, m, tag, cnt};
      return;
    }
  }
  for (int q = 0; q < cnt; ++q) xe_plan_item(base + (int64_t)q * 4, tag, s0, m, q);
}

__device__ __forceinline__ int xe_scan_excl(int v, int* s_w, int& total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int incl = (int)wave_incl_scan_u32((uint32_t)v);
  if (lane == kWave - 1) s_w[w] = incl;
  __syncthreads();
  int off = 0, tot = 0;
  for (int k = 0; k < kXePlanWaves; ++k) {
    const int x = s_w[k];
    off += k < w ? x : 0;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return off + incl - v;
}

__global__ __launch_bounds__(kXePlanThreads) void xe_plan_kernel(XePlanArgs a) {
  __shared__ XePlanShared sh;
  const int tid = threadIdx.x;
  const int K = a.cur.ctl[0];
  const int C = a.C, Cs = C > 0 ? C : 2;
  const bool reg = C == 0;
  const int R = xe_rec_width(C);
  const int JW = 5 + Cs;
  if (tid == 0) {
    sh.carry[0] = 0;  // next frontier slots
    sh.carry[1] = 0;  // split nodes
    sh.carry[2] = 0;  // next chunk items
    sh.carry[3] = 0;  // partition items
    sh.nbig = 0;
  }
  __syncthreads();
  for (int b0 = 0; b0 < K; b0 += kXePlanThreads) {
    const int i = b0 + tid;
    bool split = false;
    int fate[2] = {0, 0};
    int64_t nl = 0, m = 0, cs[2][2] = {{0, 0}, {0, 0}};  // regression child {count, sum}
    const int64_t* r = a.rec + (int64_t)(i < K ? i : 0) * R;
    int depth = 0;
    if (i < K) {
      m = a.cur.cnt[i];
      depth = a.cur.depth[i];
      const double gain = __longlong_as_double((long long)r[0]);
      split = gain > -__builtin_inf() && r[1] >= 0;
      if (reg && a.cur.minmax[(int64_t)i * 2] == a.cur.minmax[(int64_t)i * 2 + 1]) split = false;
      if (split) {
        nl = r[3];
        const int cd = depth + 1;
        const bool depth_stop = a.max_depth >= 0 && cd >= a.max_depth;
        for (int c = 0; c < 2; ++c) {
          const int64_t cm = c == 0 ? nl : m - nl;
          int nz = 2;
          if (!reg) {
            nz = 0;
            for (int k = 0; k < C; ++k) {
              const int64_t lc = r[7 + k];
              const int64_t v = c == 0 ? lc : a.cur.stats[(int64_t)i * C + k] - lc;
              nz += v > 0;
            }
          } else {
            cs[c][0] = cm;
            cs[c][1] = c == 0 ? r[7] : a.cur.stats[(int64_t)i * 2 + 1] - r[7];
          }
          const bool term = depth_stop || cm < a.mss || cm < 2 * a.msl || nz <= 1;
          fate[c] = term ? 0 : ((a.fr > 0 && cm <= a.fr) ? 1 : 2);
        }
      }
    }
    const int nn = (fate[0] == 2) + (fate[1] == 2);
    const int ns = split ? 1 : 0;
    // next-level chunk items of this node's frontier children
    int ni = 0;
    for (int c = 0; c < 2; ++c)
      if (fate[c] == 2) {
        const int64_t cm = c == 0 ? nl : m - nl;
        ni += (int)((cm + kXeChunk - 1) / kXeChunk);
      }
    const int np = split ? (int)((m + kXeChunk - 1) / kXeChunk) : 0;
    int t_nn, t_ns, t_ni, t_np;
    const int o_nn = xe_scan_excl(nn, sh.w, t_nn) + sh.carry[0];
    const int o_ns = xe_scan_excl(ns, sh.w, t_ns) + sh.carry[1];
    const int o_ni = xe_scan_excl(ni, sh.w, t_ni) + sh.carry[2];
    const int o_np = xe_scan_excl(np, sh.w, t_np) + sh.carry[3];
    if (i < K) {
      const int64_t pos = a.cur.pos[i];
      const int64_t start = a.cur.start[i];
      int32_t* P = a.pos_rec + pos * 6;
      if (reg) {
        int64_t* ps = reinterpret_cast<int64_t*>(a.pos_st) + pos * 2;
        ps[0] = a.cur.stats[(int64_t)i * 2 + 0];
        ps[1] = a.cur.stats[(int64_t)i * 2 + 1];
      } else {
        int32_t* ps = reinterpret_cast<int32_t*>(a.pos_st) + pos * C;
        for (int k = 0; k < C; ++k) ps[k] = (int32_t)a.cur.stats[(int64_t)i * C + k];
      }
      P[4] = depth;
      P[5] = (int32_t)m;
      if (!split) {
        P[0] = P[1] = P[2] = P[3] = -1;
      } else {
        const int feat = (int)r[1];
        const int64_t row = r[6];
        const int64_t cpos[2] = {pos + 1, pos + 2 * nl};
        P[0] = feat;
        P[1] = -2;  // threshold value rank: resolved after growth (xe_rank_kernel)
        P[2] = (int32_t)cpos[0];
        P[3] = (int32_t)cpos[1];
        // (+ 0.0: a -0.0 threshold prints as 0.0, as np.unique's representative)
        a.pos_thr[pos] = (a.x64 ? reinterpret_cast<const double*>(a.X)[row * a.F + feat]
                                : (double)reinterpret_cast<const float*>(a.X)[row * a.F + feat]) +
                         0.0;
        int64_t* S = a.split + (int64_t)o_ns * 4;
        S[0] = start;
        S[1] = m;
        S[2] = feat;
        S[3] = nl;
        if (a.sitem) {  // (the partition counts the frontier children's chunk totals)
          a.sitem[o_ns * 2 + 0] = -1;
          a.sitem[o_ns * 2 + 1] = -1;
        }
        // partition items of this split node
        xe_plan_run(sh, a.pitems + (int64_t)o_np * 4, o_ns, start, m, np);
        a.pfirst[o_ns] = o_np;
        const int cd = depth + 1;
        int sl = o_nn, io = o_ni;
        for (int c = 0; c < 2; ++c) {
          const int64_t cm = c == 0 ? nl : m - nl;
          const int64_t cst = c == 0 ? start : start + nl;
          auto child_stat = [&](int k) -> int64_t {
            if (reg) return cs[c][k];
            const int64_t lc = r[7 + k];
            return c == 0 ? lc : a.cur.stats[(int64_t)i * C + k] - lc;
          };
          if (fate[c] == 0) {
            int32_t* Q = a.pos_rec + cpos[c] * 6;
            Q[0] = Q[1] = Q[2] = Q[3] = -1;
            Q[4] = cd;
            Q[5] = (int32_t)cm;
            if (reg) {
              int64_t* ps = reinterpret_cast<int64_t*>(a.pos_st) + cpos[c] * 2;
              ps[0] = child_stat(0);
              ps[1] = child_stat(1);
            } else {
              int32_t* ps = reinterpret_cast<int32_t*>(a.pos_st) + cpos[c] * C;
              for (int k = 0; k < C; ++k) ps[k] = (int32_t)child_stat(k);
            }
          } else if (fate[c] == 1) {
            const int j = atomicAdd(a.job_count, 1);
            int64_t* J = a.jobs + (int64_t)j * JW;
            J[0] = cst;
            J[1] = cm;
            J[2] = cd;
            J[3] = cpos[c];
            J[4] = a.out_buf;
            for (int k = 0; k < Cs; ++k) J[5 + k] = child_stat(k);
          } else {
            a.nxt.pos[sl] = cpos[c];
            a.nxt.start[sl] = cst;
            a.nxt.cnt[sl] = (int32_t)cm;
            a.nxt.depth[sl] = cd;
            for (int k = 0; k < Cs; ++k) a.nxt.stats[(int64_t)sl * Cs + k] = child_stat(k);
            a.nxt.ifirst[sl] = io;
            if (a.sitem) a.sitem[o_ns * 2 + c] = io;
            const int64_t nck = (cm + kXeChunk - 1) / kXeChunk;
            xe_plan_run(sh, a.nxt.items + (int64_t)io * 4, sl, cst, cm, (int)nck);
            io += (int)nck;
            ++sl;
          }
        }
      }
    }
    __syncthreads();
    {  // the deferred long item runs, by the whole workgroup
      const int nb = min(sh.nbig, kXePlanBig);
      for (int b = 0; b < nb; ++b) {
        const XePlanRun e = sh.big[b];
        for (int q = tid; q < e.cnt; q += kXePlanThreads)
          xe_plan_item(e.base + (int64_t)q * 4, e.tag, e.s0, e.m, q);
      }
    }
    __syncthreads();
    if (tid == 0) {
      sh.carry[0] += t_nn;
      sh.carry[1] += t_ns;
      sh.carry[2] += t_ni;
      sh.carry[3] += t_np;
      sh.nbig = 0;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const int K2 = sh.carry[0], NS = sh.carry[1], NI = sh.carry[2], NP = sh.carry[3];
    a.nxt.ifirst[K2] = NI;
    a.pfirst[NS] = NP;
    for (int q = 0; q < 16; ++q) a.nxt.ctl[q] = 0;
    a.nxt.ctl[0] = K2;
    a.nxt.ctl[1] = NI;
    a.cur.ctl[2] = NS;
    a.cur.ctl[3] = NP;
    const int jobs_so_far = atomicAdd(a.job_count, 0);
    a.nxt.ctl[4] = jobs_so_far;
    a.tick[0] = 0;  // the next level's scan and this level's partition claim from 0
    a.tick[1] = 0;
    if (a.host_ctl) {
      __hip_atomic_store(a.host_ctl + 1, jobs_so_far, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.host_ctl, K2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
      __hip_atomic_store(a.host_ctl + 2, a.host_tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------
// Partition of the level's split segments.
// xe_flag: grid (partition items bound); rows of split j in the split feature's
// list: bit 1 for the first n_left positions. Only the feature's owner (f in
// [f_lo, f_lo + F_loc)) writes; with write_right every entry of a split segment
// sets or clears its bit (one GPU: no clearing needed), else only the left rows
// set theirs (the words were zeroed; the ranks' bits are disjoint -- one owner
// per row -- so an integer-sum all-reduce ORs them). One bit per row keeps the
// partition's random gathers in a 128 KB (n = 1M) array: L2-resident per XCD.
__global__ __launch_bounds__(kXeThreads) void xe_flag_kernel(XeArgs a, XeLists cur, int write_right) {
  const int NP = cur.ctl[3];
  for (int64_t it = blockIdx.x; it < NP; it += gridDim.x) {
    const int64_t j = a.pitems[it * 4 + 0], s0 = a.pitems[it * 4 + 1];
    const int64_t c0 = a.pitems[it * 4 + 2], cn = a.pitems[it * 4 + 3];
    const int f = (int)a.split[j * 4 + 2] - a.f_lo;
    if (f < 0 || f >= a.F_loc) continue;
    const int64_t nl = a.split[j * 4 + 3];
    const uint32_t* Ef = a.E + (int64_t)f * a.n;
    for (int64_t i = threadIdx.x; i < cn; i += kXeThreads) {
      const int64_t p = c0 + i;
      const bool left = (p - s0) < nl;
      const uint32_t r = xe_row(Ef[p]);
      if (a.flagb) {  // plain byte stores; xe_flag_pack_kernel packs them
        if (left || write_right) a.flagb[r] = left ? 1 : 0;
      } else if (left) {
        atomicOr(a.flag + (r >> 5), 1u << (r & 31));
      } else if (write_right) {
        atomicAnd(a.flag + (r >> 5), ~(1u << (r & 31)));
      }
    }
  }
}

// flag[w] = the 32 row-direction bytes of rows 32w .. 32w + 31 as bits. (Device-wide
// bit atomics are performed past the XCDs' non-coherent L2s: 1M of them took 41 us
// per level; byte stores + this pass take a fraction of that.)
__global__ __launch_bounds__(256) void xe_flag_pack_kernel(const uint8_t* __restrict__ flagb,
                                                           uint32_t* __restrict__ flag,
                                                           int64_t nw) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= nw) return;
  const uint4* src = reinterpret_cast<const uint4*>(flagb + w * 32);
  uint32_t bits = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint4 v = src[h];
    const uint32_t q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        bits |= (((q[k] >> (8 * b)) & 0xffu) != 0u ? 1u : 0u) << (h * 16 + k * 4 + b);
  }
  flag[w] = bits;
}

// xe_part: stable partition of every split segment of every feature list into
// the other list buffer: left rows to the segment's front, right rows after
// the split's n_left, both in list order.
//
// Work unit: one wave and 512 entries (a quarter of a planner chunk item), no
// workgroup barriers. A wave claims a ticket t -> (feature t % F_loc, sub-chunk
// t / F_loc), gathers its rows' direction bits -- from an LDS copy of the
// n-bit flag array when it fits (n <= kXePartLdsRows: every workgroup copies it
// once, then all gathers are LDS reads), else from global memory -- counts its
// left rows, publishes that aggregate, takes the exclusive prefix over the
// segment's earlier sub-chunks by look-back (xe_lookback) and scatters.
constexpr int kXePartWaves = 16;                       // waves per workgroup
constexpr int kXePartPer = 16;                         // entries per lane and unit
constexpr int kXeSub = kWave * kXePartPer;             // entries per wave unit (1024)
constexpr int kXeSubPerChunk = kXeChunk / kXeSub;      // wave units per chunk item (2)
constexpr int kXePartLdsWords = 36 * 1024;             // 144 KB of flag words in LDS
constexpr int64_t kXePartLdsRows = (int64_t)kXePartLdsWords * 32;
#ifndef MT_XE_PART_BATCH  // (4 / 8 / 32 / 64 measured slower: profiles/kernel_experiments.md)
#define MT_XE_PART_BATCH 16
#endif
constexpr int kXePartBatch = MT_XE_PART_BATCH;         // tickets per claim (at most)

// Tickets per claim for F_loc lists: a ticket depends on the one F_loc earlier
// (same feature, previous sub-chunk), so a batch must not be longer than F_loc
// and should divide it -- then batch b's tickets wait only on batch b - F_loc /
// batch in the same order and consecutive waves lag by one ticket. A longer
// batch serialises the waves (feature-parallel ranks with F_loc = 8 spent
// 1.7 ms per partition with 16-ticket claims: profiles/r3/session3/).
__device__ __forceinline__ int xe_part_batch(int F_loc) {
  if (F_loc <= kXePartBatch) return F_loc;
  for (int d = kXePartBatch; d >= 4; --d)
    if (F_loc % d == 0) return d;
  // no divisor: tickets run over F_loc rounded up to a multiple of the batch (the
  // padding tickets are skipped) -- a batch that straddles sub-chunks shifts each
  // ticket's dependency to another position of an earlier batch, which chains the
  // waves (a 15-ticket batch over 64 lists ran 200x slower)
  return kXePartBatch;
}

// The n-bit row-direction flags -> this workgroup's LDS (every thread returns
// after the barrier)
__device__ __forceinline__ void xe_flags_to_lds(const XeArgs& a, uint32_t* s_flag) {
  const int nw = (int)((a.n + 31) >> 5);
  // 16-byte loads, kU in flight per lane before the LDS stores: the copy is one
  // round of L2 latency instead of one per 4 KB
  constexpr int kU = 8;
  const int nq = nw >> 2;
  const uint4* src = reinterpret_cast<const uint4*>(a.flag);
  uint4* dst = reinterpret_cast<uint4*>(s_flag);
  // full rounds without guards (guarded loads / stores were issued one at a
  // time: a load, its wait, its LDS store), then the remainder
  const int bd = (int)blockDim.x;
  int i0 = threadIdx.x;
  for (; i0 + (kU - 1) * bd < nq; i0 += bd * kU) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = src[i0 + u * bd];
#pragma unroll
    for (int u = 0; u < kU; ++u) dst[i0 + u * bd] = v[u];
  }
  for (int i = i0; i < nq; i += bd) dst[i] = src[i];
  for (int i = (nq << 2) + threadIdx.x; i < nw; i += blockDim.x) s_flag[i] = a.flag[i];
  __syncthreads();
}

// Counted partition, pass 1 (the default; MPITREE_EXACT_PART_COUNTED=0 keeps the
// single-pass look-back partition): every wave unit's left rows -> pstat[u][f].
// The single-pass kernel claimed its units through one ticket counter (a device
// atomic per 1-16 units, serialised on one address) and waited in look-back
// chains as long at 8 lists as at 64 (n / 1024 units per list at the root): a
// feature-parallel rank with 8 lists spent 114 us a level on 8M entries
// (profiles/r5/exact_p8_rank_kernels.txt). Counting first reads the entries
// twice but leaves no wait and no shared counter anywhere.
template <bool kLdsFlags>
__global__ __launch_bounds__(kXePartWaves * kWave) void xe_part_count_kernel(XeArgs a, XeLists cur) {
  extern __shared__ uint32_t s_flag[];
  if (a.sitem && a.nctl) {  // (xe_tot_zero_kernel's work: the next level's chunk totals,
    // which the scatter adds into -- this level's scan has read them already)
    const int64_t tz = (int64_t)a.nctl[1] * a.F_loc * xe_cc(a.C);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tz;
         i += (int64_t)gridDim.x * blockDim.x)
      a.tot[i] = 0;
  }
  if constexpr (kLdsFlags) xe_flags_to_lds(a, s_flag);
  const uint32_t* fl = kLdsFlags ? s_flag : a.flag;
  const int lane = lane_id();
  const int64_t total = (int64_t)cur.ctl[3] * kXeSubPerChunk * a.F_loc;
  for (int64_t w = (int64_t)blockIdx.x * kXePartWaves + (threadIdx.x >> 6); w < total;
       w += (int64_t)gridDim.x * kXePartWaves) {
    const int f = (int)(w % a.F_loc);
    const int64_t u = w / a.F_loc;
    const int64_t it = u / kXeSubPerChunk, k = u % kXeSubPerChunk;
    const int64_t c0 = a.pitems[it * 4 + 2] + k * kXeSub;
    const int64_t cn = a.pitems[it * 4 + 3] - k * kXeSub;  // may be <= 0
    const uint32_t* Ef = a.E + (int64_t)f * a.n;
    uint32_t e[kXePartPer];
#pragma unroll
    for (int q = 0; q < kXePartPer; ++q) {
      const int64_t i = (int64_t)q * kWave + lane;
      e[q] = i < cn ? Ef[c0 + i] : 0xFFFFFFFFu;
    }
    uint32_t T = 0;
#pragma unroll
    for (int q = 0; q < kXePartPer; ++q) {
      const int64_t i = (int64_t)q * kWave + lane;
      const uint32_t r = xe_row(e[q]);
      T += (uint32_t)__popcll(__ballot(i < cn && ((fl[r >> 5] >> (r & 31)) & 1u)));
    }
    if (lane == 0) a.pstat[w] = T;
  }
}

// Counted partition, pass 2: per list, the exclusive prefix of the units' left
// rows within each split segment (a unit whose chunk starts its segment resets
// the sum), in place. One 1024-thread workgroup per list, 1024 units a round.
__global__ __launch_bounds__(1024) void xe_part_prefix_kernel(XeArgs a, XeLists cur) {
  __shared__ uint64_t s_tail[1024 / kWave];
  __shared__ int s_head[1024 / kWave];
  __shared__ uint64_t s_carry;
  const int f = blockIdx.x;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int64_t U = (int64_t)cur.ctl[3] * kXeSubPerChunk;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < U; b0 += 1024) {
    const int64_t u = b0 + tid;
    uint64_t v = 0;
    int h = 0;
    if (u < U) {
      const int64_t it = u / kXeSubPerChunk, k = u % kXeSubPerChunk;
      h = k == 0 && a.pitems[it * 4 + 2] == a.pitems[it * 4 + 1];  // (chunk start == segment start)
      v = a.pstat[u * a.F_loc + f];
    }
    // segmented inclusive scan in the wave: (h1, v1) . (h2, v2) = (h1 | h2, h2 ? v2 : v1 + v2)
    uint64_t x = v;
    int hx = h;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint64_t y = __shfl_up(x, d, kWave);
      const int hy = __shfl_up(hx, d, kWave);
      if (lane >= d) {
        if (!hx) x += y;
        hx |= hy;
      }
    }
    if (lane == kWave - 1) {
      s_tail[wv] = x;
      s_head[wv] = hx;
    }
    __syncthreads();
    // the prefix entering this lane's run: earlier waves (back to the nearest head)
    // and the carry of the earlier rounds
    if (!hx) {
      uint64_t add = 0;
      int w = wv - 1;
      for (; w >= 0; --w) {
        add += s_tail[w];
        if (s_head[w]) break;
      }
      if (w < 0) add += s_carry;
      x += add;
    }
    if (u < U) a.pstat[u * a.F_loc + f] = x - v;  // exclusive
    __syncthreads();
    if (tid == 1023) s_carry = x;  // (the round's last unit: inclusive, carried on)
    __syncthreads();
  }
}

template <bool kLdsFlags, bool kReg, bool kPre>
__global__ __launch_bounds__(kXePartWaves * kWave) void xe_part_kernel(XeArgs a, XeLists cur) {
  extern __shared__ uint32_t s_flag[];
  if constexpr (kLdsFlags) xe_flags_to_lds(a, s_flag);
  const uint32_t* fl = kLdsFlags ? s_flag : a.flag;
  const int lane = lane_id();
  const unsigned long long lt = (1ull << lane) - 1ull;
  // tickets per sub-chunk: F_loc rounded up to a multiple of the batch
  const int B0 = xe_part_batch(a.F_loc);
#ifndef MT_XE_PART_NOPAD  // (A/B build: the unpadded ticket order)
  const int Fp = (a.F_loc + B0 - 1) / B0 * B0;
#else
  const int Fp = a.F_loc;
#endif
  const int64_t total = (int64_t)cur.ctl[3] * kXeSubPerChunk * Fp;
  // tickets are claimed kXePartBatch at a time (one counter serialises its
  // atomics: ~10 ns each) and run in order, so the wave holding the smallest
  // unfinished ticket still never waits
  // a level with under 4 tickets per wave (the deep levels: a few long segments)
  // claims smaller batches -- still divisors of F_loc -- so its tickets spread over
  // the waves; a 16-ticket batch ran them one after another (~130 us for 8 items).
  // (A batch that does not divide F_loc, e.g. 15 of 64, stalled the top levels 200x.)
  const int64_t per_wave = total / ((int64_t)gridDim.x * kXePartWaves);
  int batch = B0;
  if (per_wave < 4) {
    batch = 1;
    for (int d = (int)std::max<int64_t>(per_wave, 1); d >= 1; --d)
      if (Fp % d == 0) {
        batch = d;
        break;
      }
  }
  // counted partition: no unit waits on another, so a static grid-stride slice
  // replaces the ticket counter (one device atomic per claim, serialised on one
  // address: ~90 us a level at 8 lists with 1- and 2-ticket batches)
  const int gw = (int)blockIdx.x * kXePartWaves + (int)(threadIdx.x >> 6);
  const int nwv = (int)gridDim.x * kXePartWaves;
  for (int t = 0, tb = 0, nclaim = 0;; ++t) {
    if (t == tb) {
      if constexpr (kPre) {
        t = gw + nclaim++ * nwv;
        tb = t + 1;
      } else {
        // a wave whose last batch reached the end claims nothing more (a relaxed
        // load of the counter before each claim measured slower: 14.9 -> 16.6 ms)
        if (tb >= total && tb > 0) break;
        int c = 0;
        if (lane == 0) c = atomicAdd(a.tick + 1, batch);
        t = __builtin_amdgcn_readfirstlane(c);
        tb = t + batch;
      }
    }
    if (t >= total) break;
    const int f = t % Fp;
    const int u = t / Fp;  // sub-chunk index over the level's partition items
    if (f >= a.F_loc) continue;  // (padding ticket)
    const int it = u / kXeSubPerChunk, k = u % kXeSubPerChunk;
    const int64_t j = a.pitems[(int64_t)it * 4 + 0], s0 = a.pitems[(int64_t)it * 4 + 1];
    const int64_t c0 = a.pitems[(int64_t)it * 4 + 2] + (int64_t)k * kXeSub;
    const int64_t cn = a.pitems[(int64_t)it * 4 + 3] - (int64_t)k * kXeSub;  // may be <= 0
    if (cn <= 0) continue;  // past its segment's end: no successor reads its status
    const uint32_t* Ef = a.E + (int64_t)f * a.n;
    uint32_t* O = a.D + (int64_t)f * a.n;
    uint32_t e[kXePartPer];
    int64_t y[kReg ? kXePartPer : 1];
#pragma unroll
    for (int q = 0; q < kXePartPer; ++q) {
      const int64_t i = (int64_t)q * kWave + lane;
      e[q] = i < cn ? Ef[c0 + i] : 0xFFFFFFFFu;
      if constexpr (kReg) y[q] = i < cn ? a.Y[(int64_t)f * a.n + c0 + i] : 0;
    }
    unsigned long long bal[kXePartPer];
    uint32_t T = 0;
#pragma unroll
    for (int q = 0; q < kXePartPer; ++q) {
      const int64_t i = (int64_t)q * kWave + lane;
      const uint32_t r = xe_row(e[q]);
      bal[q] = __ballot(i < cn && ((fl[r >> 5] >> (r & 31)) & 1u));
      T += (uint32_t)__popcll(bal[q]);
    }
    // sub-chunk index within the split's segment; its status word, and the
    // exclusive prefix of left rows over the segment's earlier sub-chunks
    const int qs = (int)((c0 - s0) / kXeSub);
    uint64_t* st = a.pstat + (int64_t)u * a.F_loc + f;
    int64_t lb = 0;
    if constexpr (kPre) {  // (counted partition: the prefix is already there)
      lb = (int64_t)st[0];
    } else {
      if (lane == 0) xe_publish(st, a.tag, qs == 0 ? kXeIncl : kXeAgg, T);
      if (qs > 0) {
        lb = xe_lookback(st, a.F_loc, qs, a.tag, a.tick + 2);
        if (lane == 0) xe_publish(st, a.tag, kXeIncl, (uint32_t)(lb + T));
      }
    }
    const int64_t nlj = a.split[j * 4 + 3];
    if (!kReg && a.sitem) {
      // the next level's two-class chunk totals: this unit's left rows land at
      // [lb, lb + T) of the left child, its right rows at [(c0 - s0) - lb, ...) of
      // the right child -- each a run of <= 1024 positions, so at most two
      // 2048-entry chunks per side; count {class 0, class 1} per chunk
      const int64_t pl0 = lb, pr0 = (c0 - s0) - lb;
      const int64_t ql0 = pl0 / kXeChunk, qr0 = pr0 / kXeChunk;
      uint32_t acc[2] = {0u, 0u};  // [side]: {chunk 0 class 0, chunk 0 class 1, chunk 1 c0, c1} bytes
      uint32_t acc2[2] = {0u, 0u};
      int lrun = 0, rrun = 0;
#pragma unroll
      for (int q = 0; q < kXePartPer; ++q) {
        const int64_t i = (int64_t)q * kWave + lane;
        const unsigned long long vm = __ballot(i < cn);
        const unsigned long long rm = vm & ~bal[q];
        const bool go = (bal[q] >> lane) & 1ull;
        if (i < cn) {
          const int lab = xe_lab(e[q]) & 1;
          const int64_t pos = go ? pl0 + lrun + __popcll(bal[q] & lt)
                                 : pr0 + rrun + __popcll(rm & lt);
          const int k = (int)(pos / kXeChunk - (go ? ql0 : qr0));  // 0 or 1
          const uint32_t one = 1u << (16 * lab);
          if (k == 0) acc[go ? 0 : 1] += one;
          else acc2[go ? 0 : 1] += one;
        }
        lrun += __popcll(bal[q]);
        rrun += __popcll(rm);
      }
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) {
        const uint32_t t0 = wave_sum_u32(acc[sd]), t1 = wave_sum_u32(acc2[sd]);
        const int32_t it0 = a.sitem[j * 2 + sd];
        if (lane == 0 && it0 >= 0) {
          const int64_t qb = sd == 0 ? ql0 : qr0;
          const int Cc = xe_cc(a.C);
          for (int k = 0; k < 2; ++k) {
            const uint32_t t = k == 0 ? t0 : t1;
            if (t == 0u) continue;
            unsigned long long* o = reinterpret_cast<unsigned long long*>(
                a.tot + ((int64_t)(it0 + qb + k) * a.F_loc + f) * Cc);
            atomicAdd(o, (unsigned long long)(t & 0xffffu));
            if (Cc > 1) atomicAdd(o + 1, (unsigned long long)(t >> 16));
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < kXePartPer; ++q) {
      const int64_t i = (int64_t)q * kWave + lane;
      const int64_t l = lb + __popcll(bal[q] & lt);
      lb += __popcll(bal[q]);
      if (i < cn) {
        const int64_t dst = ((bal[q] >> lane) & 1ull) ? s0 + l : s0 + nlj + (c0 + i - s0) - l;
        O[dst] = e[q];
        if constexpr (kReg) a.DY[(int64_t)f * a.n + dst] = y[q];
      }
    }
  }
}

// Zero the next level's chunk totals (the partition adds into them): grid-stride
// over the device count of next-level items.
__global__ __launch_bounds__(256) void xe_tot_zero_kernel(int64_t* __restrict__ tot,
                                                          const int32_t* __restrict__ nctl,
                                                          int64_t per_item) {
  const int64_t total = (int64_t)nctl[1] * per_item;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256)
    tot[i] = 0;
}

// ---------------------------------------------------------------------------
// Root lists (level 0): one slot over all n rows.
__global__ void xe_init_kernel(XeLists L, int64_t n, int Cs, const int64_t* __restrict__ root,
                               int32_t* __restrict__ job_count) {
  const int64_t k = (n + kXeChunk - 1) / kXeChunk;
  for (int64_t q = threadIdx.x; q < k; q += blockDim.x) {
    int64_t* it = L.items + q * 4;
    it[0] = 0;
    it[1] = 0;
    it[2] = q * kXeChunk;
    const int64_t rem = n - q * kXeChunk;
    it[3] = rem < kXeChunk ? rem : kXeChunk;
  }
  if (threadIdx.x == 0) {
    *job_count = 0;
    L.pos[0] = 0;
    L.start[0] = 0;
    L.cnt[0] = (int32_t)n;
    L.depth[0] = 0;
    for (int c = 0; c < Cs; ++c) L.stats[c] = root[c];
    L.ifirst[0] = 0;
    L.ifirst[1] = (int32_t)k;
    for (int q = 0; q < 16; ++q) L.ctl[q] = 0;
    L.ctl[0] = 1;
    L.ctl[1] = (int32_t)k;
  }
}

// ---------------------------------------------------------------------------
// Finisher jobs (segments of <= 256 rows) on subtree-local 8-bit codes: a row's
// code in feature f is the offset of the first entry of its value in the
// segment of f's list, so the finisher's "code <= b" is the split "x <= value
// at offset b" with the list engine's candidates, costs and ties. Virtual rows
// of segment [s, s + m): s + (the row's order among the segment's row ids) --
// the same on every rank whatever its feature block. Outputs for this rank's
// features: codes_fm[f_lo + f][v]; the label-packed entries ent[v] (classes)
// (classification) or the row ids ent[v] = v and targets yv[v] (regression).
// jobs: int64 [J][W] = {start, rows, depth, position, list buffer, ...}
template <typename XT>
__global__ __launch_bounds__(kXeLocalMax) void xe_local_codes_kernel(
    const uint32_t* __restrict__ E0, const uint32_t* __restrict__ E1,
    const int64_t* __restrict__ Y0, const int64_t* __restrict__ Y1, const XT* __restrict__ X,
    int F, int fg_lo, int64_t n, int F_loc, int f_lo,
    const int64_t* __restrict__ jobs, int JW, uint8_t* __restrict__ codes_fm,
    uint8_t* __restrict__ codes_rm, int row_bytes,
    uint32_t* __restrict__ ent, int64_t* __restrict__ yv, const int32_t* __restrict__ ylab) {
  // kFt features per pass: the codes of the pass in LDS (both output layouts are
  // written from there); values are read from X only where two adjacent entries
  // are both duplicated values (rare on continuous data)
  constexpr int kFt = 32;
  __shared__ uint8_t cb[kFt * kXeLocalMax];  // [kFt][kXeLocalMax] codes by virtual row
  __shared__ uint32_t s_row[kXeLocalMax];
  const int64_t* J = jobs + (int64_t)blockIdx.x * JW;
  const int64_t s = J[0];
  const int m = (int)J[1];
  const bool b1 = J[4] != 0;
  const uint32_t* E = b1 ? E1 : E0;
  const int t = threadIdx.x, lane = lane_id(), w = t >> 6;
  // virtual row order: rank of the row id among the segment's rows (bitonic sort)
  const uint32_t e0 = t < m ? E[s + t] : 0xFFFFFFFFu;
  s_row[t] = t < m ? xe_row(e0) : 0xFFFFFFFFu;
  __syncthreads();
  for (int size = 2; size <= kXeLocalMax; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int j = t ^ stride;
      if (j > t) {
        const uint32_t x = s_row[t], y = s_row[j];
        const bool up = (t & size) == 0;
        if ((x > y) == up) {
          s_row[t] = y;
          s_row[j] = x;
        }
      }
      __syncthreads();
    }
  }
  // virtual index of a row: binary search in s_row[0, m) -- a fixed 8 steps, so the
  // searches of a wave's entries unroll and overlap
  auto vidx = [&](uint32_t row) -> int {
    int lo = 0;
#pragma unroll
    for (int step = kXeLocalMax / 2; step > 0; step >>= 1) {
      const int mid = lo + step;
      if (mid < m && s_row[mid] <= row) lo = mid;
    }
    return lo;
  };
  if (t < m) {  // labels / targets by virtual row (from the first local list)
    const int v = vidx(xe_row(e0));
    if (yv) {  // regression: plain virtual row ids + the targets
      ent[s + v] = (uint32_t)(s + v);
      yv[s + v] = (b1 ? Y1 : Y0)[s + t];
    } else {
      const uint32_t lab = ylab ? (uint32_t)ylab[xe_row(e0)] : (uint32_t)xe_lab(e0);
      ent[s + v] = (lab << 24) | (uint32_t)(s + v);  // (finisher jobs: <= 256 classes)
    }
  }
  for (int f0 = 0; f0 < F_loc; f0 += kFt) {
    const int nf = min(kFt, F_loc - f0);
    // one wave per feature, 4 consecutive entries per lane: the offset of the first
    // entry of each value is an inclusive max-scan of the run starts. The wave's
    // kFw features load their entries and virtual rows first (independent chains).
    constexpr int kFw = kFt / (kXeLocalMax / kWave);
    constexpr int kPer = kXeLocalMax / kWave;  // entries per lane (4)
    uint32_t e[kFw][kPer];
    int vv[kFw][kPer];
#pragma unroll
    for (int r = 0; r < kFw; ++r) {
      const int k = w + r * (kXeLocalMax / kWave);
      const uint32_t* Ef = E + (int64_t)(f0 + k) * n + s;
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int i = lane * kPer + q;
        e[r][q] = (k < nf && i < m) ? Ef[i] : 0xFFFFFFFFu;
      }
    }
#pragma unroll
    for (int r = 0; r < kFw; ++r)
#pragma unroll
      for (int q = 0; q < kPer; ++q)
        vv[r][q] = e[r][q] != 0xFFFFFFFFu ? vidx(xe_row(e[r][q])) : 0;
#pragma unroll
    for (int r = 0; r < kFw; ++r) {
      const int k = w + r * (kXeLocalMax / kWave);
      if (k >= nf) break;  // (wave-uniform)
      const XT* xk = X + fg_lo + f0 + k;
      const uint32_t pe = __shfl_up(e[r][kPer - 1], 1, kWave);
      uint32_t b = 0;
      uint32_t bq[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int i = lane * kPer + q;
        const uint32_t ep = q == 0 ? pe : e[r][q - 1];
        const bool start =
            i == 0 || (i < m && (!(xe_dup(e[r][q]) && xe_dup(ep)) ||
                                 xk[(int64_t)xe_row(e[r][q]) * F] != xk[(int64_t)xe_row(ep) * F]));
        if (i < m && start) b = (uint32_t)i;
        bq[q] = b;  // (max so far: starts ascend within the lane)
      }
      // exclusive max over the lower lanes
      uint32_t x = b;
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t o = __shfl_up(x, d, kWave);
        if (lane >= d) x = max(x, o);
      }
      uint32_t ex = __shfl_up(x, 1, kWave);
      if (lane == 0) ex = 0;
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int i = lane * kPer + q;
        if (i < m) cb[k * kXeLocalMax + vv[r][q]] = (uint8_t)max(ex, bq[q]);
      }
    }
    __syncthreads();
    for (int i = t; i < nf * m; i += kXeLocalMax) {
      const int k = i / m, v = i - k * m;
      codes_fm[(int64_t)(f_lo + f0 + k) * n + s + v] = cb[k * kXeLocalMax + v];
    }
    if (codes_rm) {  // one-rank fits: the row-major codes too (4 features a word)
      const int wpr = (nf + 3) >> 2;
      for (int i = t; i < m * wpr; i += kXeLocalMax) {
        const int v = i / wpr, q = i - v * wpr;
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (4 * q + b < nf) word |= (uint32_t)cb[(4 * q + b) * kXeLocalMax + v] << (8 * b);
        *reinterpret_cast<uint32_t*>(codes_rm + (s + v) * row_bytes + f0 + 4 * q) = word;
      }
      if (f0 + kFt >= F_loc)  // zero padding bytes past the last feature
        for (int i = t; i < m * (row_bytes - F_loc); i += kXeLocalMax) {
          const int pw = row_bytes - F_loc;
          const int v = i / pw, c = i - v * pw;
          codes_rm[(s + v) * row_bytes + F_loc + c] = 0;
        }
    }
    __syncthreads();
  }
}

// Row-major copy of the finisher codes: codes_rm[v][f] for every virtual row of
// every job (the finisher reads both layouts; feature-parallel fits, after the
// codes all-gather -- one-rank fits write it from xe_local_codes_kernel).
__global__ __launch_bounds__(256) void xe_codes_rm_kernel(const uint8_t* __restrict__ codes_fm,
                                                          int64_t n, int F, int row_bytes,
                                                          const int64_t* __restrict__ jobs,
                                                          int JW, uint8_t* __restrict__ codes_rm) {
  const int64_t* J = jobs + (int64_t)blockIdx.x * JW;
  const int64_t s = J[0];
  const int m = (int)J[1];
  for (int e = threadIdx.x; e < m * row_bytes; e += 256) {
    const int v = e / row_bytes, f = e - v * row_bytes;
    codes_rm[(s + v) * row_bytes + f] = f < F ? codes_fm[(int64_t)f * n + s + v] : (uint8_t)0;
  }
}

// Finished job j owns positions [pos, pos + 2m - 1) of the position space; its
// split nodes hold {feature, local code}. For this rank's features: code ->
// the threshold row (the first entry of the value at that offset of the
// feature's segment) -> value rank and threshold value. The feature-parallel
// exchange packs what this rank resolved (resolved[p] = 1).
__global__ __launch_bounds__(256) void xe_fix_kernel(
    const uint32_t* __restrict__ E0, const uint32_t* __restrict__ E1,
    const void* __restrict__ X, int x64, int F, int64_t n,
    int f_lo, int F_loc, const int64_t* __restrict__ jobs, int JW, int32_t* __restrict__ pos_rec,
    double* __restrict__ pos_thr) {
  const int64_t* J = jobs + (int64_t)blockIdx.x * JW;
  const int64_t s = J[0], m = J[1], pos = J[3];
  const uint32_t* E = J[4] ? E1 : E0;
  for (int64_t p = pos + threadIdx.x; p < pos + 2 * m - 1; p += blockDim.x) {
    int32_t* R = pos_rec + p * 6;
    if (R[5] <= 0 || R[0] < 0) continue;
    const int f = R[0] - f_lo;
    if (f < 0 || f >= F_loc) continue;
    const uint32_t row = xe_row(E[(int64_t)f * n + s + R[1]]);
    R[1] = -2;  // value rank: xe_rank_kernel
    pos_thr[p] = xe_x(X, x64, F, row, R[0]) + 0.0;
  }
}

// Threshold bins of every split node whose feature is this rank's: the value
// rank of the threshold = the rank at the first position of the feature's
// setup-sorted order whose value is >= the threshold (binary search; rows and
// ranks by sorted position were kept from the setup). resolved[p] = 1 marks
// what this rank resolved (the feature-parallel exchange packs those).
__global__ __launch_bounds__(256) void xe_rank_kernel(
    int32_t* __restrict__ pos_rec, const double* __restrict__ pos_thr, int64_t P,
    const uint32_t* __restrict__ root_rows, const uint32_t* __restrict__ rank_at,
    const void* __restrict__ X, int x64, int F, int64_t n, int f_lo, int F_loc,
    uint8_t* __restrict__ resolved, const uint32_t* __restrict__ keys) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  int32_t* R = pos_rec + p * 6;
  if (R[5] <= 0 || R[0] < 0) return;
  const int f = R[0] - f_lo;
  if (f < 0 || f >= F_loc) return;
  const double thr = pos_thr[p];
  const uint32_t* rows = root_rows + (int64_t)f * n;
  int64_t lo = 0, hi = n;  // first sorted position with value >= thr
  if (keys) {  // fp32 input: the setup's sorted order-preserving keys, one read a step
    const uint32_t* kf = keys + (int64_t)f * n;
    const uint32_t b = __float_as_uint((float)thr + 0.0f);
    const uint32_t tk = (b >> 31) ? ~b : (b | 0x80000000u);
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (kf[mid] < tk) lo = mid + 1; else hi = mid;
    }
  } else {
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (xe_x(X, x64, F, xe_row(rows[mid]), R[0]) < thr) lo = mid + 1; else hi = mid;
    }
  }
  R[1] = (int32_t)rank_at[(int64_t)f * n + lo];
  if (resolved) resolved[p] = 1;
}

// Pack / scatter {position, bin, threshold bits} of the positions a rank resolved
// (feature-parallel finisher nodes), in position order via asm_rank (mask).
__global__ __launch_bounds__(256) void xe_resolved_pack_kernel(const int32_t* __restrict__ pos_rec,
                                                               const double* __restrict__ pos_thr,
                                                               int64_t P, const int32_t* __restrict__ rank,
                                                               int64_t* __restrict__ rows) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const int j = rank[p];
  if (j < 0) return;
  rows[(int64_t)j * 3 + 0] = p;
  rows[(int64_t)j * 3 + 1] = pos_rec[p * 6 + 1];
  rows[(int64_t)j * 3 + 2] = (int64_t)__double_as_longlong(pos_thr[p]);
}

__global__ __launch_bounds__(256) void xe_resolved_scatter_kernel(const int64_t* __restrict__ rows,
                                                                  int64_t k, int32_t* __restrict__ pos_rec,
                                                                  double* __restrict__ pos_thr) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= k) return;
  const int64_t p = rows[i * 3 + 0];
  pos_rec[p * 6 + 1] = (int32_t)rows[i * 3 + 1];
  pos_thr[p] = __longlong_as_double((long long)rows[i * 3 + 2]);
}

// ---------------------------------------------------------------------------
// Setup: each feature's sorted 32-bit value keys with row ids (exact_setup.hip
// sort; with packed labels the sort already carries them in bits 25..31 of the row
// value) -> entries, value ranks by sorted position, duplicate flags. cbase: per-
// (feature, chunk) first rank (exact_setup's count / scan of value changes).
// One workgroup per (4096-entry chunk, feature): entry k * 256 + t of the chunk is
// thread t's k-th; neighbours come from adjacent lanes, the ranks from 16 wave scans
// and one workgroup barrier.
constexpr int kXeEmitK = 16;  // entries per thread (chunk = 16 x 256)
__global__ __launch_bounds__(256) void xe_emit_kernel(const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ rows, int64_t n,
                                                      int nc, const int32_t* __restrict__ cbase,
                                                      const int32_t* __restrict__ ylab,
                                                      const int64_t* __restrict__ yfix,
                                                      uint32_t* __restrict__ E,
                                                      int64_t* __restrict__ Y,
                                                      uint32_t* __restrict__ rank_at) {
  const int f = blockIdx.y, c = blockIdx.x;
  const int64_t base = (int64_t)f * n;
  const int64_t p0 = (int64_t)c * (kXeEmitK * 256);
  __shared__ uint32_t s_w[kXeEmitK][256 / kWave];
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  uint32_t incl[kXeEmitK];
  uint32_t dupm = 0;  // bit k: entry k is a duplicate value
#pragma unroll
  for (int k = 0; k < kXeEmitK; ++k) {
    const int64_t p = p0 + k * 256 + tid;
    const bool in = p < n;
    const uint32_t key = in ? keys[base + p] : 0u;
    uint32_t prev = __shfl_up(key, 1, kWave);
    uint32_t next = __shfl_down(key, 1, kWave);
    if (lane == 0 && in && p > 0) prev = keys[base + p - 1];
    if (lane == kWave - 1 && p + 1 < n) next = keys[base + p + 1];
    const bool nwv = in && (p == 0 || prev != key);
    const bool dn = in && p + 1 < n && next == key;
    if (in && (!nwv || dn)) dupm |= 1u << k;
    incl[k] = wave_incl_scan_dpp(nwv ? 1u : 0u);
    if (lane == kWave - 1) s_w[k][w] = incl[k];
  }
  __syncthreads();
  int32_t run = cbase[(int64_t)f * nc + c];
#pragma unroll
  for (int k = 0; k < kXeEmitK; ++k) {
    int32_t off = run;
    int32_t tot = 0;
#pragma unroll
    for (int q = 0; q < 256 / kWave; ++q) {
      const int32_t v = (int32_t)s_w[k][q];
      off += q < w ? v : 0;
      tot += v;
    }
    run += tot;
    const int64_t p = p0 + k * 256 + tid;
    if (p < n) {
      const uint32_t rv = rows[base + p];
      const uint32_t row = rv & 0xFFFFFFu;
      const uint32_t lab = ylab ? (uint32_t)ylab[row] << 25 : 0u;
      E[base + p] = rv | (((dupm >> k) & 1u) << 24) | lab;
      if (Y) Y[base + p] = yfix[row];
      rank_at[base + p] = (uint32_t)(off + (int32_t)incl[k] - 1);
    }
  }
}

// --------------------------------------------------------------- launchers
int xe_chunk() { return kXeChunk; }
int xe_part_units() { return kXeSubPerChunk; }
int xe_local_max() { return kXeLocalMax; }
int xe_max_classes() { return kXeMaxClasses; }
int xe_packed_classes() { return kXeMaxC; }

void xe_init(hipStream_t s, const XeLists& L, int64_t n, int Cs, const int64_t* root, int32_t* jc) {
  hipLaunchKernelGGL(xe_init_kernel, dim3(1), dim3(256), 0, s, L, n, Cs, root, jc);
  MT_HIP_CHECK(hipGetLastError());
}

// the scan / select half of a level (grids are host bounds; blocks past the
// device counts exit)
// x extent of the (items, features) grids: items are visited grid-stride, so a
// level's grid is a bounded slice (~16k workgroups) whatever its item bound
static int xe_gx(int items_bound, int F_loc) {
  const int cap = std::max(4, 16384 / std::max(1, F_loc));
  return std::max(1, std::min(items_bound, cap));
}

void xe_level_scan(hipStream_t s, const XeArgs& a, const XeLists& cur, int items_bound,
                   int slots_bound) {
  if (items_bound <= 0 || slots_bound <= 0) return;
  const int Cc = xe_cc(a.C);
  // chunk totals (unless the previous partition counted them), carries, then the scan
  const int gx = xe_gx(items_bound, a.F_loc);
  if (!a.tot_ready)
    hipLaunchKernelGGL(xe_tot_kernel, dim3(gx, a.F_loc), dim3(kXeThreads), 0, s, a, cur);
  const int64_t nc = (int64_t)slots_bound * a.F_loc * Cc;
  if (slots_bound <= 64)  // few slots of many chunks: a wave each
    hipLaunchKernelGGL(xe_carry_wave_kernel,
                       dim3((unsigned)((nc * kWave + kXeThreads - 1) / kXeThreads)),
                       dim3(kXeThreads), 0, s, a, cur);
  else
    hipLaunchKernelGGL(xe_carry_kernel, dim3((unsigned)((nc + kXeThreads - 1) / kXeThreads)),
                       dim3(kXeThreads), 0, s, a, cur);
  if (a.C == 0)
    hipLaunchKernelGGL(xe_scan_kernel<0>, dim3(gx, a.F_loc), dim3(kXeThreads), 0, s, a, cur);
  else if (a.C <= 2) {  // one wave per (item, feature): no workgroup barriers
    const dim3 g((unsigned)std::min<int64_t>(
        ((int64_t)items_bound * a.F_loc + kXeWaves - 1) / kXeWaves, 8192));
    if (MT_XE_TWO_PASS && a.crit == kEntropy && a.nmin && a.cmin && a.gthr) {
      hipLaunchKernelGGL(xe_scan_c2_kernel<1>, g, dim3(kXeThreads), 0, s, a, cur);
      hipLaunchKernelGGL(xe_gthr_kernel, dim3((unsigned)((slots_bound + kXeWaves - 1) / kXeWaves)),
                         dim3(kXeThreads), 0, s, a, cur);
      // pass 2: 64 chunk checks per wave step, entries read only near the minimum
      const int64_t pw = (int64_t)xe_p2_pairs(a.F_loc) * kXeWaves;  // pairs per workgroup step
      hipLaunchKernelGGL(xe_scan_c2_kernel<2>,
                         dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(
                             ((int64_t)items_bound * a.F_loc + pw - 1) / pw, MT_XE_P2_GRID))),
                         dim3(kXeThreads), 0, s, a, cur);
    } else {
      hipLaunchKernelGGL(xe_scan_c2_kernel<0>, g, dim3(kXeThreads), 0, s, a, cur);
    }
  }
  else
    hipLaunchKernelGGL(xe_scan_kernel<2>, dim3(gx, a.F_loc), dim3(kXeThreads), 0, s, a, cur);
  if (slots_bound <= 512)
    hipLaunchKernelGGL(xe_select_kernel<1024>, dim3(slots_bound), dim3(1024), 0, s, a, cur);
  else
    hipLaunchKernelGGL(xe_select_kernel<kXeThreads>, dim3(slots_bound), dim3(kXeThreads), 0, s, a,
                       cur);
  MT_HIP_CHECK(hipGetLastError());
}

void xe_plan(hipStream_t s, const XePlanArgs& p) {
  hipLaunchKernelGGL(xe_plan_kernel, dim3(1), dim3(kXePlanThreads), 0, s, p);
  MT_HIP_CHECK(hipGetLastError());
}

void xe_flag(hipStream_t s, const XeArgs& a, const XeLists& cur, int pitems_bound, int write_right) {
  if (pitems_bound <= 0) return;
  hipLaunchKernelGGL(xe_flag_kernel, dim3(std::min(pitems_bound, 4096)), dim3(kXeThreads), 0, s, a,
                     cur, write_right);
  MT_HIP_CHECK(hipGetLastError());
  if (a.flagb) {
    const int64_t nw = (a.n + 31) / 32;
    hipLaunchKernelGGL(xe_flag_pack_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s,
                       a.flagb, a.flag, nw);
    MT_HIP_CHECK(hipGetLastError());
  }
}

void xe_partition(hipStream_t s, const XeArgs& a, const XeLists& cur, int pitems_bound,
                  int splits_bound) {
  if (pitems_bound <= 0 || splits_bound <= 0) return;
  const char* cv = std::getenv("MPITREE_EXACT_PART_COUNTED");
  const bool counted = !(cv && cv[0] == '0');
  if (a.sitem && a.nctl && !counted)  // (the counted partition's count kernel zeroes them)
    hipLaunchKernelGGL(xe_tot_zero_kernel, dim3(1024), dim3(256), 0, s, a.tot, a.nctl,
                       (int64_t)a.F_loc * xe_cc(a.C));
  int dev = 0, n_cu = 0;
  MT_HIP_CHECK(hipGetDevice(&dev));
  MT_HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  // one workgroup of 16 wave workers per CU (the LDS flag copy is per workgroup)
  const int64_t units = (int64_t)pitems_bound * kXeSubPerChunk * a.F_loc;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(n_cu, (units + kXePartWaves - 1) /
                                                                          kXePartWaves));
  static const bool lds_off = [] {  // (MPITREE_EXACT_PART_LDS=0: global flags, tests)
    const char* v = std::getenv("MPITREE_EXACT_PART_LDS");
    return v && v[0] == '0';
  }();
  // counted partition (count, per-segment prefix, scatter: no look-back waits,
  // no ticket counter) -- faster at every list count measured: 8 lists 114 ->
  // ~15 us a level, the 64-list continuous fit 14.27 -> 13.46 ms
  // (profiles/r5/ab_exact_counted.log); MPITREE_EXACT_PART_COUNTED=0: the
  // single-pass look-back partition (read per launch: tests switch it)
  const bool in_lds = a.n <= kXePartLdsRows && !lds_off;
  const size_t lds = in_lds ? (size_t)((a.n + 31) / 32) * 4 : 0;
  const int g = in_lds ? grid : grid * 2;
  if (counted) {
    if (in_lds) {
      MT_HIP_CHECK(mt_set_max_lds((const void*)xe_part_count_kernel<true>, (int)lds));
      hipLaunchKernelGGL(xe_part_count_kernel<true>, dim3(g), dim3(kXePartWaves * kWave), lds, s,
                         a, cur);
    } else {
      hipLaunchKernelGGL(xe_part_count_kernel<false>, dim3(g), dim3(kXePartWaves * kWave), 0, s,
                         a, cur);
    }
    hipLaunchKernelGGL(xe_part_prefix_kernel, dim3(a.F_loc), dim3(1024), 0, s, a, cur);
  }
#define MT_XP(LDS, REG, PRE)                                                                    \
  do {                                                                                          \
    if (LDS) MT_HIP_CHECK(mt_set_max_lds((const void*)xe_part_kernel<LDS, REG, PRE>, (int)lds)); \
    hipLaunchKernelGGL((xe_part_kernel<LDS, REG, PRE>), dim3(g), dim3(kXePartWaves * kWave),    \
                       lds, s, a, cur);                                                         \
  } while (0)
#define MT_XP2(LDS, REG) \
  do {                   \
    if (counted)         \
      MT_XP(LDS, REG, true); \
    else                 \
      MT_XP(LDS, REG, false); \
  } while (0)
  if (in_lds) {
    if (a.C == 0) MT_XP2(true, true);
    else MT_XP2(true, false);
  } else {
    if (a.C == 0) MT_XP2(false, true);
    else MT_XP2(false, false);
  }
#undef MT_XP2
#undef MT_XP
  MT_HIP_CHECK(hipGetLastError());
}

void xe_local_codes(hipStream_t s, const uint32_t* E0, const uint32_t* E1, const int64_t* Y0,
                    const int64_t* Y1, const void* X, int x64, int F, int fg_lo, int64_t n,
                    int F_loc, int f_lo, const int64_t* jobs, int J, int JW, uint8_t* codes_fm,
                    uint8_t* codes_rm, int row_bytes, uint32_t* ent, int64_t* yv,
                    const int32_t* ylab) {
  if (J <= 0) return;
  if (codes_rm && (f_lo != 0 || (row_bytes & 3) || row_bytes < F_loc))
    throw std::runtime_error("xe_local_codes: row-major codes need f_lo = 0, 4-byte rows");
  if (x64) {
    hipLaunchKernelGGL(xe_local_codes_kernel<double>, dim3(J), dim3(kXeLocalMax), 0, s, E0, E1,
                       Y0, Y1, (const double*)X, F, fg_lo, n, F_loc, f_lo, jobs, JW, codes_fm,
                       codes_rm, row_bytes, ent, yv, ylab);
  } else {
    hipLaunchKernelGGL(xe_local_codes_kernel<float>, dim3(J), dim3(kXeLocalMax), 0, s, E0, E1,
                       Y0, Y1, (const float*)X, F, fg_lo, n, F_loc, f_lo, jobs, JW, codes_fm,
                       codes_rm, row_bytes, ent, yv, ylab);
  }
  MT_HIP_CHECK(hipGetLastError());
}

void xe_codes_rm(hipStream_t s, const uint8_t* codes_fm, int64_t n, int F, int row_bytes,
                 const int64_t* jobs, int J, int JW, uint8_t* codes_rm) {
  if (J <= 0) return;
  hipLaunchKernelGGL(xe_codes_rm_kernel, dim3(J), dim3(256), 0, s, codes_fm, n, F, row_bytes,
                     jobs, JW, codes_rm);
  MT_HIP_CHECK(hipGetLastError());
}

void xe_fix(hipStream_t s, const uint32_t* E0, const uint32_t* E1, const void* X, int x64, int F,
            int64_t n, int f_lo, int F_loc, const int64_t* jobs, int J, int JW, int32_t* pos_rec,
            double* pos_thr) {
  if (J <= 0) return;
  hipLaunchKernelGGL(xe_fix_kernel, dim3(J), dim3(256), 0, s, E0, E1, X, x64, F, n, f_lo, F_loc,
                     jobs, JW, pos_rec, pos_thr);
  MT_HIP_CHECK(hipGetLastError());
}

void xe_rank(hipStream_t s, int32_t* pos_rec, const double* pos_thr, int64_t P,
             const uint32_t* root_rows, const uint32_t* rank_at, const void* X, int x64, int F,
             int64_t n, int f_lo, int F_loc, uint8_t* resolved, const uint32_t* keys) {
  const int64_t b = (P + 255) / 256;
  if (b == 0) return;
  hipLaunchKernelGGL(xe_rank_kernel, dim3((unsigned)b), dim3(256), 0, s, pos_rec, pos_thr, P,
                     root_rows, rank_at, X, x64, F, n, f_lo, F_loc, resolved, keys);
  MT_HIP_CHECK(hipGetLastError());
}

void xe_resolved_pack(hipStream_t s, const int32_t* pos_rec, const double* pos_thr, int64_t P,
                      const int32_t* rank, int64_t* rows) {
  const int64_t b = (P + 255) / 256;
  if (b == 0) return;
  hipLaunchKernelGGL(xe_resolved_pack_kernel, dim3((unsigned)b), dim3(256), 0, s, pos_rec, pos_thr,
                     P, rank, rows);
  MT_HIP_CHECK(hipGetLastError());
}

void xe_resolved_scatter(hipStream_t s, const int64_t* rows, int64_t k, int32_t* pos_rec,
                         double* pos_thr) {
  if (k <= 0) return;
  hipLaunchKernelGGL(xe_resolved_scatter_kernel, dim3((unsigned)((k + 255) / 256)), dim3(256), 0,
                     s, rows, k, pos_rec, pos_thr);
  MT_HIP_CHECK(hipGetLastError());
}

void xe_emit(hipStream_t s, const uint32_t* keys, const uint32_t* rows, int64_t n, int F_loc,
             int nc, int chunk, const int32_t* cbase, const int32_t* ylab, const int64_t* yfix,
             uint32_t* E, int64_t* Y, uint32_t* rank_at) {
  if (n <= 0 || F_loc <= 0) return;
  if (chunk != kXeEmitK * 256) throw std::runtime_error("xe_emit: chunk must be 4096");
  hipLaunchKernelGGL(xe_emit_kernel, dim3(nc, F_loc), dim3(256), 0, s, keys, rows, n, nc,
                     cbase, ylab, yfix, E, Y, rank_at);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
