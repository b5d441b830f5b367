// Exact split search on presorted per-feature lists (continuous features).
//
// The reference takes every unique value of a feature as a candidate
// threshold (mpitree/tree/decision_tree.py:73-90). Histogram kernels do the
// same only while a feature has at most 256 values (one LDS bin per value);
// with continuous data a feature can have n of them. This engine keeps, per
// feature, the rows sorted by value and partitioned by frontier node:
//
//   E[f][p] = value rank << 32 | label << 24 | row      (uint64, rows < 2^24)
//
// so node i owns positions [start_i, start_i + m_i) of every feature's list,
// sorted by value inside. A level then needs no histogram at all:
//
//   ex_tot      per (chunk, feature): class totals of a <= 2048-entry chunk
//   ex_carry    per (node, feature, class): exclusive prefix over the node's chunks
//   ex_scan     per (chunk, feature): class prefix at every position, the
//               integer-form cost at every value boundary, tie-rounded
//               (criterion.h) and packed as (cost units << 24 | position) --
//               one 64-bit atomicMin per chunk keeps the lowest cost, then the
//               lowest position, i.e. the smallest threshold (np.argmin)
//   ex_select   per node: best feature (max gain, ties to the lowest feature)
//               and the winning split's left class counts -> split record
//   ex_flag / ex_pcount / ex_pcarry / ex_pscatter
//               rows of split nodes go left iff their rank in the split
//               feature is <= the threshold rank; every feature's segment is
//               stably partitioned (left rows first, both halves stay sorted)
//               into the other list buffer
//
// Every quantity is an integer or the shared fp64 criterion, so the tree is
// bit-identical to the host builders on the same exact thresholds.
#include "common.h"
#include "criterion.h"

namespace mt {

constexpr int kExThreads = 256;
constexpr int kExPer = 8;                      // entries per thread
constexpr int kExChunk = kExThreads * kExPer;  // entries per chunk item
constexpr int kExMaxC = 256;

__device__ __forceinline__ uint32_t ex_row(uint64_t e) { return (uint32_t)e & 0xFFFFFFu; }
__device__ __forceinline__ int ex_lab(uint64_t e) { return (int)((e >> 24) & 0xFFu); }
__device__ __forceinline__ uint32_t ex_rank(uint64_t e) { return (uint32_t)(e >> 32); }

__device__ __forceinline__ double ex_tlog(uint64_t x, const double* __restrict__ tab, int tn) {
  return x < (uint64_t)tn ? __ldg(tab + x) : xlog2x(x);
}

// Block-wide exclusive prefix of one uint32 per thread (4 waves); returns the
// block total through `total`.
__device__ __forceinline__ uint32_t ex_block_excl(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan_dpp(v);
  if (lane == kWave - 1) s_w[w] = incl;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kExThreads / kWave; ++k) {
    const uint32_t x = s_w[k];
    off += k < w ? x : 0u;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return off + incl - v;
}

// items: int64 [NI][4] = {slot, segment start, chunk start, chunk count}
__global__ __launch_bounds__(kExThreads) void ex_tot_kernel(const uint64_t* __restrict__ E,
                                                            int64_t n, const int64_t* __restrict__ items,
                                                            int F, int C, int32_t* __restrict__ tot) {
  __shared__ uint32_t cnt[kExMaxC];
  const int64_t it = blockIdx.x;
  const int f = blockIdx.y;
  const int64_t c0 = items[it * 4 + 2], cn = items[it * 4 + 3];
  if (C <= 2) {  // class-1 count by wave sums (LDS atomics on two words serialise)
    const uint64_t* L = E + (int64_t)f * n + c0;
    uint32_t ones = 0;
    uint64_t e[kExPer];
#pragma unroll
    for (int k = 0; k < kExPer; ++k) {  // all loads in flight before the first use
      const int64_t i = (int64_t)k * kExThreads + threadIdx.x;
      e[k] = i < cn ? L[i] : 0ull;
    }
#pragma unroll
    for (int k = 0; k < kExPer; ++k) ones += ex_lab(e[k]) == 1 ? 1u : 0u;
    ones = wave_sum_u32(ones);
    if (lane_id() == 0) cnt[threadIdx.x >> 6] = ones;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < kExThreads / kWave; ++w) t += cnt[w];
      tot[(it * F + f) * C + 0] = (int32_t)(cn - t);
      if (C == 2) tot[(it * F + f) * C + 1] = (int32_t)t;
    }
    return;
  }
  for (int c = threadIdx.x; c < C; c += kExThreads) cnt[c] = 0;
  __syncthreads();
  const uint64_t* L = E + (int64_t)f * n + c0;
  for (int64_t i = threadIdx.x; i < cn; i += kExThreads) atomicAdd(&cnt[ex_lab(L[i])], 1u);
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kExThreads)
    tot[(it * F + f) * C + c] = (int32_t)cnt[c];
}

// One thread per (slot, feature, class): exclusive prefix of the chunk totals
// over the slot's chunks [ifirst[slot], ifirst[slot + 1]); slot totals (f == 0).
__global__ __launch_bounds__(kExThreads) void ex_carry_kernel(
    const int32_t* __restrict__ tot, const int64_t* __restrict__ ifirst, int K, int F, int C,
    int32_t* __restrict__ carry, int32_t* __restrict__ slot_tot) {
  const int64_t g = (int64_t)blockIdx.x * kExThreads + threadIdx.x;
  if (g >= (int64_t)K * F * C) return;
  const int c = (int)(g % C);
  const int f = (int)((g / C) % F);
  const int64_t slot = g / ((int64_t)C * F);
  int32_t acc = 0;
  for (int64_t it = ifirst[slot]; it < ifirst[slot + 1]; ++it) {
    const int64_t o = (it * F + f) * C + c;
    carry[o] = acc;
    acc += tot[o];
  }
  if (f == 0) slot_tot[slot * C + c] = acc;
}

// Best (cost, position) of every chunk of every (slot, feature) segment.
// seg: int64 [K][2] = {start, count}; best: uint64 [K][F], preset to ~0.
__global__ __launch_bounds__(kExThreads) void ex_scan_kernel(
    const uint64_t* __restrict__ E, int64_t n, const int64_t* __restrict__ items,
    const int64_t* __restrict__ seg, const int32_t* __restrict__ carry,
    const int32_t* __restrict__ slot_tot, int F, int C, int crit, int64_t msl,
    const double* __restrict__ xtab, int xtab_n, unsigned long long* __restrict__ best) {
  __shared__ uint32_t s_w[kExThreads / kWave];
  __shared__ uint32_t s_first[kExThreads];
  __shared__ unsigned long long s_min[kExThreads / kWave];
  const int64_t it = blockIdx.x;
  const int f = blockIdx.y;
  const int64_t slot = items[it * 4 + 0], sstart = items[it * 4 + 1];
  const int64_t c0 = items[it * 4 + 2], cn = items[it * 4 + 3];
  const int64_t m = seg[slot * 2 + 1];
  const uint64_t* L = E + (int64_t)f * n;
  const int tid = threadIdx.x;
  const int64_t p0 = c0 + (int64_t)tid * kExPer;  // first absolute position of this thread
  uint64_t e[kExPer];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    const int64_t p = p0 + k;
    e[k] = (p - c0) < cn ? L[p] : ~0ull;
  }
  // the rank right after this thread's last entry (next thread, or the next chunk)
  s_first[tid] = ex_rank(e[0]);
  __syncthreads();
  uint32_t next_rank;
  {
    const int64_t pn = p0 + kExPer;
    if (tid + 1 < kExThreads) {
      next_rank = s_first[tid + 1];
    } else {
      next_rank = (pn - sstart) < m ? ex_rank(L[pn]) : 0xFFFFFFFFu;
    }
    if ((pn - c0) >= cn && (pn - sstart) < m) next_rank = ex_rank(L[pn]);
  }
  double sL[kExPer], sR[kExPer];
  int64_t qL[kExPer], qR[kExPer];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    sL[k] = 0.0;
    sR[k] = 0.0;
    qL[k] = 0;
    qR[k] = 0;
  }
  const int32_t* car = carry + (it * F + f) * C;
  const int32_t* st = slot_tot + slot * C;
  for (int c = 0; c < C; ++c) {
    uint32_t pre[kExPer];
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < kExPer; ++k) {
      run += (e[k] != ~0ull && ex_lab(e[k]) == c) ? 1u : 0u;
      pre[k] = run;
    }
    uint32_t total;
    const uint32_t excl = ex_block_excl(run, s_w, total);
    const uint32_t base = (uint32_t)car[c] + excl;
    const uint32_t tc = (uint32_t)st[c];
#pragma unroll
    for (int k = 0; k < kExPer; ++k) {
      const uint32_t Lc = base + pre[k];
      const uint32_t Rc = tc - Lc;
      if (crit == kEntropy) {
        sL[k] = sL[k] + ex_tlog(Lc, xtab, xtab_n);
        sR[k] = sR[k] + ex_tlog(Rc, xtab, xtab_n);
      } else {
        qL[k] += (int64_t)Lc * Lc;
        qR[k] += (int64_t)Rc * Rc;
      }
    }
  }
  const double tu = tie_unit(ex_tlog((uint64_t)m, xtab, xtab_n), m);
  const double tinv = 1.0 / tu;
  unsigned long long mine = ~0ull;
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    const int64_t pos = p0 + k - sstart;  // position inside the segment
    const int64_t ml = pos + 1, mr = m - ml;
    if ((p0 + k - c0) >= cn || mr <= 0) continue;
    const uint32_t nr = k + 1 < kExPer ? ex_rank(e[k + 1]) : next_rank;
    if (nr == ex_rank(e[k])) continue;  // not a value boundary
    if (ml < msl || mr < msl) continue;
    double cost;
    if (crit == kEntropy)
      cost = (ex_tlog((uint64_t)ml, xtab, xtab_n) - sL[k]) +
             (ex_tlog((uint64_t)mr, xtab, xtab_n) - sR[k]);
    else
      cost = gini_term(ml, qL[k]) + gini_term(mr, qR[k]);
    double q = __builtin_rint(cost * tinv);  // the grid of tie_round (criterion.h)
    q = q < 0.0 ? 0.0 : q;
    const unsigned long long key = ((unsigned long long)q << 24) | (unsigned long long)pos;
    mine = key < mine ? key : mine;
  }
  // block min -> one atomic per chunk
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const unsigned long long o = __shfl_xor(mine, d, kWave);
    mine = o < mine ? o : mine;
  }
  if (lane_id() == 0) s_min[tid >> 6] = mine;
  __syncthreads();
  if (tid == 0) {
    unsigned long long b = s_min[0];
    for (int w = 1; w < kExThreads / kWave; ++w) b = s_min[w] < b ? s_min[w] : b;
    if (b != ~0ull) atomicMin(best + slot * F + f, b);
  }
}

// Two classes (the common case): one block scan of the class-1 prefix gives
// every position's four side counts. Entropy costs are first scored in fp32
// (hardware log2) -- |fp32 - exact| <= 2^-17.5 T(m) over the six terms and
// their sums -- and only positions within 2^-16 (T(m) + m) of the chunk's fp32
// minimum (twice that error plus one tie-rounding unit) are re-scored exactly
// in fp64 with the shared xlog2x: the chunk's exact (tie-rounded) best is among
// them. Gini is exact integer arithmetic plus two divisions: scored directly.
__device__ __forceinline__ float ex_t32(uint32_t x) {
  const float xf = (float)x;
  return x <= 1u ? 0.0f : xf * __log2f(xf);
}

template <int CRIT>
__global__ __launch_bounds__(kExThreads) void ex_scan_c2_kernel(
    const uint64_t* __restrict__ E, int64_t n, const int64_t* __restrict__ items,
    const int64_t* __restrict__ seg, const int32_t* __restrict__ carry,
    const int32_t* __restrict__ slot_tot, int F, int64_t msl,
    unsigned long long* __restrict__ best, const double* __restrict__ xtab, int xtab_n) {
  constexpr int kWaves = kExThreads / kWave;
  __shared__ uint32_t s_cnt[kExPer * kWaves];    // class-1 entries of each (step, wave)
  __shared__ uint32_t s_first[kExPer * kWaves];  // rank of each (step, wave)'s lane 0
  __shared__ unsigned long long s_min[kWaves];
  __shared__ float s_fmin[kWaves];
  const int64_t it = blockIdx.x;
  const int f = blockIdx.y;
  const int64_t slot = items[it * 4 + 0], sstart = items[it * 4 + 1];
  const int64_t c0 = items[it * 4 + 2], cn = items[it * 4 + 3];
  const int64_t m = seg[slot * 2 + 1];
  const uint64_t* L = E + (int64_t)f * n;
  const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  // entry i = k * 256 + tid of the chunk (coalesced loads)
  uint64_t e[kExPer];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    const int64_t i = (int64_t)k * kExThreads + tid;
    e[k] = i < cn ? L[c0 + i] : ~0ull;
  }
  unsigned long long bal[kExPer];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    bal[k] = __ballot(e[k] != ~0ull && ex_lab(e[k]) == 1);
    if (lane == 0) {
      s_cnt[k * kWaves + wave] = (uint32_t)__popcll(bal[k]);
      s_first[k * kWaves + wave] = ex_rank(e[k]);
    }
  }
  __syncthreads();
  if (tid < kWave) {  // exclusive scan of the 32 step counts
    const uint32_t v = tid < kExPer * kWaves ? s_cnt[tid] : 0u;
    const uint32_t incl = wave_incl_scan_dpp(v);
    if (tid < kExPer * kWaves) s_cnt[tid] = incl - v;
  }
  __syncthreads();
  const int32_t* car = carry + (it * F + f) * 2;
  const uint32_t base1 = (uint32_t)car[1];
  const int64_t t0 = slot_tot[slot * 2 + 0], t1 = slot_tot[slot * 2 + 1];
  bool valid[kExPer];
  int64_t l1[kExPer];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    const int64_t i = (int64_t)k * kExThreads + tid;
    const uint32_t r = ex_rank(e[k]);
    // rank of the next position: the next lane, the next (step, wave)'s lane 0,
    // or past the chunk the list itself (none past the segment)
    uint32_t nr = __shfl_down(r, 1, kWave);
    if (lane == kWave - 1) {
      const int q = k * kWaves + wave + 1;
      nr = q < kExPer * kWaves ? s_first[q] : 0xFFFFFFFFu;
    }
    if (i + 1 >= cn) nr = (c0 + i + 1 - sstart) < m ? ex_rank(L[c0 + i + 1]) : 0xFFFFFFFFu;
    const int64_t pos = c0 + i - sstart;
    const int64_t ml = pos + 1, mr = m - ml;
    valid[k] = i < cn && mr > 0 && nr != r && ml >= msl && mr >= msl;
    l1[k] = (int64_t)(base1 + s_cnt[k * kWaves + wave] + (uint32_t)__popcll(bal[k] & lt) +
                      (uint32_t)((bal[k] >> lane) & 1ull));
  }
  // x*log2(x) from the shared table (built by the same xlog2x: identical bits)
  // below xtab_n, the atanh series above it
  auto tl = [&](int64_t x) -> double {
    return x < (int64_t)xtab_n ? __ldg(xtab + x) : xlog2x((uint64_t)x);
  };
  const double tm = tl(m);
  const double tu = tie_unit(tm, m);
  const double tinv = 1.0 / tu;
  auto exact_key = [&](int k) -> unsigned long long {
    const int64_t pos = c0 + (int64_t)k * kExThreads + tid - sstart;
    const int64_t ml = pos + 1, mr = m - ml;
    const int64_t L1 = l1[k], L0 = ml - L1, R1 = t1 - L1, R0 = t0 - L0;
    double cost;
    if (CRIT == kEntropy) {
      const double sl = tl(L0) + tl(L1);
      const double sr = tl(R0) + tl(R1);
      cost = (tl(ml) - sl) + (tl(mr) - sr);
    } else {
      cost = gini_term(ml, L0 * L0 + L1 * L1) + gini_term(mr, R0 * R0 + R1 * R1);
    }
    double q = __builtin_rint(cost * tinv);
    q = q < 0.0 ? 0.0 : q;
    return ((unsigned long long)q << 24) | (unsigned long long)pos;
  };
  unsigned long long mine = ~0ull;
  if (CRIT == kEntropy) {
    float c32[kExPer];
    float lmin = __builtin_inff();
#pragma unroll
    for (int k = 0; k < kExPer; ++k) {
      const uint32_t ml = (uint32_t)(c0 + (int64_t)k * kExThreads + tid - sstart + 1),
                     mr = (uint32_t)(m - ml);
      const uint32_t L1 = (uint32_t)l1[k], L0 = ml - L1;
      const uint32_t R1 = (uint32_t)t1 - L1, R0 = (uint32_t)t0 - L0;
      const float c = (ex_t32(ml) - (ex_t32(L0) + ex_t32(L1))) +
                      (ex_t32(mr) - (ex_t32(R0) + ex_t32(R1)));
      c32[k] = valid[k] ? c : __builtin_inff();
      lmin = fminf(lmin, c32[k]);
    }
    lmin = wave_min_f32_dpp(lmin);
    if (lane == 0) s_fmin[wave] = lmin;
    __syncthreads();
    float bmin = s_fmin[0];
#pragma unroll
    for (int w = 1; w < kExThreads / kWave; ++w) bmin = fminf(bmin, s_fmin[w]);
    const float thr = bmin + (float)((tm + (double)m) * 0x1p-16);
#pragma unroll
    for (int k = 0; k < kExPer; ++k) {
      if (valid[k] && c32[k] <= thr) {  // (thr is +inf when the chunk has no candidate)
        const unsigned long long key = exact_key(k);
        mine = key < mine ? key : mine;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kExPer; ++k) {
      if (valid[k]) {
        const unsigned long long key = exact_key(k);
        mine = key < mine ? key : mine;
      }
    }
  }
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const unsigned long long o = __shfl_xor(mine, d, kWave);
    mine = o < mine ? o : mine;
  }
  if (lane == 0) s_min[wave] = mine;
  __syncthreads();
  if (tid == 0) {
    unsigned long long b = s_min[0];
    for (int w = 1; w < kExThreads / kWave; ++w) b = s_min[w] < b ? s_min[w] : b;
    if (b != ~0ull) atomicMin(best + slot * F + f, b);
  }
}

// Per slot: best feature and the winning split's record
// rec: int64 [K][5 + 2C] = {gain bits, feature, threshold rank, n_left, m, left[C], total[C]}.
__global__ __launch_bounds__(kExThreads) void ex_select_kernel(
    const uint64_t* __restrict__ E, int64_t n, const int64_t* __restrict__ seg,
    const int64_t* __restrict__ ifirst, const int32_t* __restrict__ carry,
    const int32_t* __restrict__ slot_tot, const unsigned long long* __restrict__ best, int F,
    int C, int crit, const double* __restrict__ xtab, int xtab_n, int64_t* __restrict__ rec) {
  __shared__ double s_gain[kExThreads / kWave];
  __shared__ int s_feat[kExThreads / kWave], s_pos[kExThreads / kWave];
  __shared__ double s_pterm;
  __shared__ uint32_t cnt[kExMaxC];
  const int64_t slot = blockIdx.x;
  const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const int64_t start = seg[slot * 2 + 0], m = seg[slot * 2 + 1];
  const int32_t* st = slot_tot + slot * C;
  const int R = 5 + 2 * C;
  int64_t* out = rec + slot * R;
  if (tid == 0) {  // sequential over classes, matching every other engine
    double acc = 0.0;
    int64_t mm = 0, sq = 0;
    for (int c = 0; c < C; ++c) {
      const int64_t t = st[c];
      mm += t;
      acc = acc + xlog2x((uint64_t)t);
      sq += t * t;
    }
    s_pterm = crit == kEntropy ? xlog2x((uint64_t)mm) - acc : gini_term(mm, sq);
    out[4] = mm;
  }
  for (int c = tid; c < C; c += kExThreads) {
    out[5 + C + c] = st[c];
    cnt[c] = 0;
  }
  __syncthreads();
  const double pterm = s_pterm;
  const double tu = tie_unit(ex_tlog((uint64_t)m, xtab, xtab_n), m);
  double g = -__builtin_inf();
  int bf = 0x7fffffff, bp = -1;
  for (int f = tid; f < F; f += kExThreads) {
    const unsigned long long key = best[slot * F + f];
    if (key != ~0ull) {
      const double cost = (double)(key >> 24) * tu;
      const double gf = pterm - cost;
      if (gf > g) {  // features ascend per thread: strict > keeps the lowest
        g = gf;
        bf = f;
        bp = (int)(key & 0xFFFFFFull);
      }
    }
  }
  wave_argmax(g, bf, bp);
  if (lane == 0) {
    s_gain[wave] = g;
    s_feat[wave] = bf;
    s_pos[wave] = bp;
  }
  __syncthreads();
  g = s_gain[0];
  bf = s_feat[0];
  bp = s_pos[0];
  for (int w = 1; w < kExThreads / kWave; ++w) {
    if (s_gain[w] > g || (s_gain[w] == g && s_feat[w] < bf)) {
      g = s_gain[w];
      bf = s_feat[w];
      bp = s_pos[w];
    }
  }
  const bool ok = g > -__builtin_inf();
  if (!ok) {
    if (tid == 0) {
      out[0] = (int64_t)double_to_bits(g);
      out[1] = -1;
      out[2] = -1;
      out[3] = 0;
    }
    for (int c = tid; c < C; c += kExThreads) out[5 + c] = 0;
    return;
  }
  // left counts: the carry of the chunk holding position bp + classes up to it
  const uint64_t* L = E + (int64_t)bf * n;
  const int64_t chunk = ifirst[slot] + bp / kExChunk;
  const int64_t cfirst = start + (int64_t)(bp / kExChunk) * kExChunk;
  for (int64_t p = cfirst + tid; p <= start + bp; p += kExThreads) atomicAdd(&cnt[ex_lab(L[p])], 1u);
  __syncthreads();
  const int32_t* car = carry + (chunk * F + bf) * C;
  for (int c = tid; c < C; c += kExThreads) out[5 + c] = (int64_t)car[c] + cnt[c];
  if (tid == 0) {
    out[0] = (int64_t)double_to_bits(g);
    out[1] = bf;
    out[2] = (int64_t)ex_rank(L[start + bp]);
    out[3] = (int64_t)bp + 1;
  }
}

// Partition. pitems: int64 [NP][4] = {split j, segment start, chunk start, chunk count};
// split: int64 [S][4] = {start, count, feature, threshold rank}.
__global__ __launch_bounds__(kExThreads) void ex_flag_kernel(const uint64_t* __restrict__ E,
                                                             int64_t n, const int64_t* __restrict__ pitems,
                                                             const int64_t* __restrict__ split,
                                                             uint8_t* __restrict__ flag) {
  const int64_t it = blockIdx.x;
  const int64_t j = pitems[it * 4 + 0], c0 = pitems[it * 4 + 2], cn = pitems[it * 4 + 3];
  const int64_t f = split[j * 4 + 2];
  const uint32_t thr = (uint32_t)split[j * 4 + 3];
  const uint64_t* L = E + f * n + c0;
  for (int64_t i = threadIdx.x; i < cn; i += kExThreads) {
    const uint64_t e = L[i];
    flag[ex_row(e)] = ex_rank(e) <= thr ? 1 : 0;
  }
}

// Left entries of every (chunk, feature): the row flags are gathered once here
// and kept as one 64-bit ballot per (step, wave) in ``bits`` [NP][F][kExPer][4],
// so the scatter streams them instead of gathering every flag again.
__global__ __launch_bounds__(kExThreads) void ex_pcount_kernel(const uint64_t* __restrict__ E,
                                                               int64_t n, const int64_t* __restrict__ pitems,
                                                               const uint8_t* __restrict__ flag, int F,
                                                               int32_t* __restrict__ lc,
                                                               unsigned long long* __restrict__ bits) {
  constexpr int kWaves = kExThreads / kWave;
  __shared__ uint32_t s_w[kWaves];
  const int64_t it = blockIdx.x;
  const int f = blockIdx.y;
  const int64_t c0 = pitems[it * 4 + 2], cn = pitems[it * 4 + 3];
  const uint64_t* L = E + (int64_t)f * n + c0;
  const int lane = lane_id(), w = threadIdx.x >> 6;
  uint64_t e[kExPer];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {  // all loads, then all flag gathers, in flight
    const int64_t i = (int64_t)k * kExThreads + threadIdx.x;
    e[k] = i < cn ? L[i] : ~0ull;
  }
  uint32_t v = 0;
  unsigned long long* B = bits + (it * F + f) * (int64_t)(kExPer * kWaves);
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    const unsigned long long b = __ballot(e[k] != ~0ull && flag[ex_row(e[k])] != 0);
    if (lane == 0) {
      B[k * kWaves + w] = b;
      v += (uint32_t)__popcll(b);
    }
  }
  if (lane == 0) s_w[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t total = 0;
    for (int q = 0; q < kWaves; ++q) total += s_w[q];
    lc[it * F + f] = (int32_t)total;
  }
}

// One thread per (split, feature): exclusive prefix of the chunk left counts
// over the split's chunks [pfirst[j], pfirst[j + 1]); left total per split.
__global__ __launch_bounds__(kExThreads) void ex_pcarry_kernel(
    const int32_t* __restrict__ lc, const int64_t* __restrict__ pfirst, int S, int F,
    int32_t* __restrict__ lcar, int32_t* __restrict__ nl) {
  const int64_t g = (int64_t)blockIdx.x * kExThreads + threadIdx.x;
  if (g >= (int64_t)S * F) return;
  const int f = (int)(g % F);
  const int64_t j = g / F;
  int32_t acc = 0;
  for (int64_t it = pfirst[j]; it < pfirst[j + 1]; ++it) {
    lcar[it * F + f] = acc;
    acc += lc[it * F + f];
  }
  if (f == 0) nl[j] = acc;
}

// Stable partition of one chunk: entry c0 + k * 256 + tid (coalesced loads);
// its rank among the chunk's left entries is the earlier (k, wave) steps' left
// counts (one LDS scan over 8 x 4 ballot popcounts) + the lower lanes' bits.
__global__ __launch_bounds__(kExThreads) void ex_pscatter_kernel(
    const uint64_t* __restrict__ E, uint64_t* __restrict__ D, int64_t n,
    const int64_t* __restrict__ pitems, const int32_t* __restrict__ lcar,
    const int32_t* __restrict__ nl, const unsigned long long* __restrict__ bits, int F) {
  constexpr int kWaves = kExThreads / kWave;
  __shared__ uint32_t s_cnt[kExPer * kWaves];
  const int64_t it = blockIdx.x;
  const int f = blockIdx.y;
  const int64_t j = pitems[it * 4 + 0], s0 = pitems[it * 4 + 1];
  const int64_t c0 = pitems[it * 4 + 2], cn = pitems[it * 4 + 3];
  const uint64_t* L = E + (int64_t)f * n;
  uint64_t* O = D + (int64_t)f * n;
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  uint64_t e[kExPer];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    const int64_t i = (int64_t)k * kExThreads + threadIdx.x;
    e[k] = i < cn ? L[c0 + i] : ~0ull;
  }
  const unsigned long long* Bt = bits + (it * F + f) * (int64_t)(kExPer * kWaves);
  unsigned long long bal[kExPer];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    bal[k] = Bt[k * kWaves + w];  // (wave-uniform: one scalar load)
    if (lane == 0) s_cnt[k * kWaves + w] = (uint32_t)__popcll(bal[k]);
  }
  __syncthreads();
  if (threadIdx.x < kWave) {  // exclusive scan of the 32 step counts
    const uint32_t v = threadIdx.x < kExPer * kWaves ? s_cnt[threadIdx.x] : 0u;
    const uint32_t incl = wave_incl_scan_dpp(v);
    if (threadIdx.x < kExPer * kWaves) s_cnt[threadIdx.x] = incl - v;
  }
  __syncthreads();
  const int64_t lb = (int64_t)lcar[it * F + f];  // left entries of the segment before c0
  const int64_t nlj = nl[j];
#pragma unroll
  for (int k = 0; k < kExPer; ++k) {
    const int64_t i = (int64_t)k * kExThreads + threadIdx.x;
    if (i >= cn) break;
    const int64_t l = lb + s_cnt[k * kWaves + w] + __popcll(bal[k] & lt);  // left before
    if ((bal[k] >> lane) & 1ull)
      O[s0 + l] = e[k];
    else
      O[s0 + nlj + (c0 + i - s0) - l] = e[k];
  }
}

// ---------------------------------------------------------------------------
// Small subtrees leave the list engine for the histogram finisher (finish.hip)
// on subtree-local 8-bit codes. For a deferred segment [s, s + m) (m <= 256)
// a row's code in feature f is the offset of the first entry of its value in
// the segment of f's sorted list: codes ascend with the value, equal values
// share a code, and the finisher's split "code <= b" is the split "x <= value
// at s + b", so its candidates, costs and ties are the list engine's. Virtual
// rows are positions of feature 0's list (v = s + offset there), giving the
// finisher row-major codes codes_rm[v][.], feature-major codes_fm[f][v] and
// packed entries ent[v] = label << 24 | v. ex_local_fix_kernel turns the
// finished nodes' codes back into value ranks.
// seg: int64 [J][3] = {start, count, list buffer}
constexpr int kExLocalMax = 256;

__global__ __launch_bounds__(kExLocalMax) void ex_local_codes_kernel(
    const uint64_t* __restrict__ E0, const uint64_t* __restrict__ E1, int64_t n,
    const int64_t* __restrict__ seg, int F, int row_bytes, uint8_t* __restrict__ codes_rm,
    uint8_t* __restrict__ codes_fm, uint32_t* __restrict__ ent, uint32_t* __restrict__ inv) {
  extern __shared__ __align__(16) uint8_t s_code[];  // [m][row_bytes]
  __shared__ uint32_t s_rank[kExLocalMax];
  __shared__ uint32_t s_w[kExLocalMax / kWave];
  const int64_t s = seg[blockIdx.x * 3 + 0];
  const int m = (int)seg[blockIdx.x * 3 + 1];
  const uint64_t* __restrict__ E = seg[blockIdx.x * 3 + 2] ? E1 : E0;
  const int t = threadIdx.x, lane = lane_id(), w = t >> 6;
  const int words = m * row_bytes / 4;
  for (int i = t; i < words; i += kExLocalMax) reinterpret_cast<uint32_t*>(s_code)[i] = 0u;
  if (t < m) {
    const uint64_t e = E[s + t];
    inv[ex_row(e)] = (uint32_t)t;
    ent[s + t] = ((uint32_t)ex_lab(e) << 24) | (uint32_t)(s + t);
  }
  __threadfence_block();
  __syncthreads();
  for (int f = 0; f < F; ++f) {
    uint32_t rank = 0xFFFFFFFFu, v = 0;
    if (t < m) {
      const uint64_t e = E[(int64_t)f * n + s + t];
      rank = ex_rank(e);
      v = inv[ex_row(e)];
    }
    s_rank[t] = rank;
    __syncthreads();
    // offset of the first entry of this value: inclusive max-scan of run starts
    uint32_t b = (t < m && (t == 0 || s_rank[t - 1] != rank)) ? (uint32_t)t : 0u;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t o = __shfl_up(b, d, kWave);
      if (lane >= d) b = max(b, o);
    }
    if (lane == kWave - 1) s_w[w] = b;
    __syncthreads();
    for (int k = 0; k < w; ++k) b = max(b, s_w[k]);
    if (t < m) {
      s_code[v * row_bytes + f] = (uint8_t)b;
      codes_fm[(int64_t)f * n + s + v] = (uint8_t)b;
    }
    __syncthreads();  // s_rank / s_w reuse
  }
  uint32_t* out = reinterpret_cast<uint32_t*>(codes_rm + s * row_bytes);
  for (int i = t; i < words; i += kExLocalMax) out[i] = reinterpret_cast<const uint32_t*>(s_code)[i];
}

// Finished subtree j owns positions [pos, pos + 2m - 1) of node_i32 ({feature,
// bin, left, right, depth, n}; n = 0 marks an unused position): split codes ->
// value ranks of the list the segment lives in.
// jobs: int64 [J][4] = {root position, m, segment start, list buffer}
__global__ __launch_bounds__(256) void ex_local_fix_kernel(const uint64_t* __restrict__ E0,
                                                          const uint64_t* __restrict__ E1,
                                                          int64_t n, const int64_t* __restrict__ jobs,
                                                          int32_t* __restrict__ node_i32) {
  const int64_t pos = jobs[blockIdx.x * 4 + 0], m = jobs[blockIdx.x * 4 + 1];
  const int64_t s = jobs[blockIdx.x * 4 + 2];
  const uint64_t* __restrict__ E = jobs[blockIdx.x * 4 + 3] ? E1 : E0;
  for (int64_t p = pos + threadIdx.x; p < pos + 2 * m - 1; p += blockDim.x) {
    int32_t* R = node_i32 + p * 6;
    if (R[5] > 0 && R[0] >= 0) R[1] = (int32_t)ex_rank(E[(int64_t)R[0] * n + s + R[1]]);
  }
}

// --------------------------------------------------------------- launchers
void ex_scan_level(hipStream_t stream, const uint64_t* E, int64_t n, const int64_t* items, int NI,
                   const int64_t* ifirst, const int64_t* seg, int K, int F, int C, int crit,
                   int64_t msl, const double* xtab, int xtab_n, int32_t* tot, int32_t* carry,
                   int32_t* slot_tot, unsigned long long* best, int64_t* rec) {
  if (K <= 0 || NI <= 0) return;
  if (C > kExMaxC) throw std::runtime_error("exact engine: at most 256 classes");
  hipLaunchKernelGGL(ex_tot_kernel, dim3(NI, F), dim3(kExThreads), 0, stream, E, n, items, F, C,
                     tot);
  MT_HIP_CHECK(hipGetLastError());
  const int64_t nc = (int64_t)K * F * C;
  hipLaunchKernelGGL(ex_carry_kernel, dim3((unsigned)((nc + kExThreads - 1) / kExThreads)),
                     dim3(kExThreads), 0, stream, tot, ifirst, K, F, C, carry, slot_tot);
  MT_HIP_CHECK(hipGetLastError());
  MT_HIP_CHECK(hipMemsetAsync(best, 0xFF, (size_t)K * F * sizeof(unsigned long long), stream));
  if (C == 2 && crit == kEntropy)
    hipLaunchKernelGGL(ex_scan_c2_kernel<kEntropy>, dim3(NI, F), dim3(kExThreads), 0, stream, E,
                       n, items, seg, carry, slot_tot, F, msl, best, xtab, xtab_n);
  else if (C == 2)
    hipLaunchKernelGGL(ex_scan_c2_kernel<kGini>, dim3(NI, F), dim3(kExThreads), 0, stream, E, n,
                       items, seg, carry, slot_tot, F, msl, best, xtab, xtab_n);
  else
    hipLaunchKernelGGL(ex_scan_kernel, dim3(NI, F), dim3(kExThreads), 0, stream, E, n, items,
                       seg, carry, slot_tot, F, C, crit, msl, xtab, xtab_n, best);
  MT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(ex_select_kernel, dim3(K), dim3(kExThreads), 0, stream, E, n, seg, ifirst,
                     carry, slot_tot, best, F, C, crit, xtab, xtab_n, rec);
  MT_HIP_CHECK(hipGetLastError());
}

void ex_partition_level(hipStream_t stream, const uint64_t* E, uint64_t* D, int64_t n,
                        const int64_t* pitems, int NP, const int64_t* pfirst, const int64_t* split,
                        int S, int F, uint8_t* flag, int32_t* lc, int32_t* lcar, int32_t* nl,
                        unsigned long long* bits) {
  if (S <= 0 || NP <= 0) return;
  hipLaunchKernelGGL(ex_flag_kernel, dim3(NP), dim3(kExThreads), 0, stream, E, n, pitems, split,
                     flag);
  MT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(ex_pcount_kernel, dim3(NP, F), dim3(kExThreads), 0, stream, E, n, pitems,
                     flag, F, lc, bits);
  MT_HIP_CHECK(hipGetLastError());
  const int64_t ns = (int64_t)S * F;
  hipLaunchKernelGGL(ex_pcarry_kernel, dim3((unsigned)((ns + kExThreads - 1) / kExThreads)),
                     dim3(kExThreads), 0, stream, lc, pfirst, S, F, lcar, nl);
  MT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(ex_pscatter_kernel, dim3(NP, F), dim3(kExThreads), 0, stream, E, D, n,
                     pitems, lcar, nl, bits, F);
  MT_HIP_CHECK(hipGetLastError());
}

int ex_chunk() { return kExChunk; }
int ex_part_bits_words() { return kExPer * (kExThreads / kWave); }  // per (chunk, feature)

void ex_local_codes(hipStream_t stream, const uint64_t* E0, const uint64_t* E1, int64_t n,
                    const int64_t* seg, int J, int F, int row_bytes, uint8_t* codes_rm,
                    uint8_t* codes_fm, uint32_t* ent, uint32_t* inv) {
  if (J <= 0) return;
  if (row_bytes % 4 != 0 || row_bytes < F) throw std::runtime_error("ex_local_codes: row_bytes");
  const size_t lds = (size_t)kExLocalMax * row_bytes;
  MT_HIP_CHECK(hipFuncSetAttribute((const void*)ex_local_codes_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(ex_local_codes_kernel, dim3(J), dim3(kExLocalMax), lds, stream, E0, E1, n,
                     seg, F, row_bytes, codes_rm, codes_fm, ent, inv);
  MT_HIP_CHECK(hipGetLastError());
}

void ex_local_fix(hipStream_t stream, const uint64_t* E0, const uint64_t* E1, int64_t n,
                  const int64_t* jobs, int J, int32_t* node_i32) {
  if (J <= 0) return;
  hipLaunchKernelGGL(ex_local_fix_kernel, dim3(J), dim3(256), 0, stream, E0, E1, n, jobs,
                     node_i32);
  MT_HIP_CHECK(hipGetLastError());
}

int ex_local_max() { return kExLocalMax; }


}  // namespace mt
