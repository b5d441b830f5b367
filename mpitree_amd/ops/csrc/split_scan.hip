// Split search over node histograms on gfx950.
//
// Replaces the reference's per-threshold cost loop and its argmin/argmax
// (mpitree/tree/decision_tree.py:76-91 and :130-140): one wavefront scans one
// (node, feature) histogram. Each lane owns 4 consecutive bins; per class the
// wave does a 64-lane prefix sum (with a carry across 256-bin chunks), and the
// per-bin split cost is accumulated in fp64 from the integer left/right class
// counts with the shared integer-form criterion (criterion.h), so the result
// is bit-identical to the host builders. A wave argmin over (cost, bin) picks
// the first minimum; ``select_kernel`` then reduces (gain, feature) per node
// with ties to the lowest feature and gathers the winning split's left counts.
#include <type_traits>

#include "common.h"
#include "criterion.h"

namespace mt {

constexpr int kBinsPerLane = 4;
constexpr int kChunk = kWave * kBinsPerLane;  // 256 bins per wave pass
constexpr int kScanCG = 4;                     // classes whose scans overlap (C > 2)

// T(x) = x*log2(x) from a device table built by the same function (so the
// values are identical) for small counts, evaluated otherwise. The scan is
// fp64-VALU bound without it at deep levels.
__device__ __forceinline__ double tlog(uint64_t x, const double* __restrict__ tab, int tn) {
  return x < (uint64_t)tn ? __ldg(tab + x) : xlog2x(x);
}

// N table values with every load in flight before the first use: unconditional
// loads (clamped index), the evaluated form only for counts past the table. The
// per-value form above compiled to a guarded load and a wait per lookup -- 24
// dependent L2 round trips per bin group of a two-class scan.
template <int N>
__device__ __forceinline__ void tlog_batch(const uint32_t (&x)[N], double (&out)[N],
                                           const double* __restrict__ tab, int tn) {
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = __ldg(tab + min(x[i], (uint32_t)(tn - 1)));
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (x[i] >= (uint32_t)tn) out[i] = xlog2x(x[i]);
}

// hist: uint32 [slots][F_h][B][C]; nodes: int64 [k] slot ids
// out_cost: f64 [k][F_h]; out_bin: i32 [k][F_h]
// Fused sibling derivation (device level loop): with ``der``, slots >= *nbuilt
// are derived, der[slot - nbuilt] = {slot, parent slot in ``prev``, built
// sibling slot}; the wave writes its feature's parent - sibling histogram into
// ``hist`` (the select kernel and the next level read it) and scans the copy it
// keeps in LDS -- one launch per level less than a separate derive kernel.
__global__ __launch_bounds__(256) void scan_cls_kernel(
    uint32_t* __restrict__ hist, const int64_t* __restrict__ nodes,
    const int32_t* __restrict__ nbins, int F_h, int f_lo, int B, int C, int crit, int msl,
    double* __restrict__ out_cost, int32_t* __restrict__ out_bin,
    const double* __restrict__ xtab, int xtab_n, const int32_t* __restrict__ dcount,
    const int64_t* __restrict__ der, const uint32_t* __restrict__ prev,
    const int32_t* __restrict__ nbuilt, int der_lds, int32_t* __restrict__ sel_left,
    int32_t* __restrict__ sel_tot, const int32_t* __restrict__ node_tot) {
  // sel_left / sel_tot (fused selection, two-class fast path): the left class
  // counts at this feature's best bin [node][F_h][2] and, from feature 0's wave,
  // the node's class totals and node term [node][4] = {t0, t1, term (f64)}, for
  // the planner to build the split record
  // der_lds: the derived histogram (B*C words per wave) fits in LDS; else the
  // scan reads parent - sibling from global memory on the fly (many classes)
  if (dcount && (int)blockIdx.x >= *dcount) return;  // device-side node count
  // per wave: C class totals + C carries [+ B*C derived]. (Staging the first 1024
  // x*log2(x) values in LDS for many classes was measured slower: 1.77 -> 2.02 ms
  // per level at C = 64, profiles/kernel_experiments.md.)
  extern __shared__ uint32_t sm[];
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int f = blockIdx.y * 4 + wave;
  auto tl = [&](uint64_t x) -> double { return tlog(x, xtab, xtab_n); };
  if (f >= F_h) return;
  const int64_t node = blockIdx.x;
  const int64_t slot = nodes[node];
  const int64_t E = (int64_t)B * C;
  const uint32_t* h = hist + (slot * F_h + f) * E;
  uint32_t* tot = sm + wave * 2 * C;
  uint32_t* carry = tot + C;
  const int nb = min(B, nbins[f_lo + f]);
  const uint32_t* gp = nullptr;  // on-the-fly derivation: parent and sibling
  const uint32_t* gs = nullptr;
  if (der != nullptr) {
    const int NB = *nbuilt;
    if (slot >= NB) {
      const int64_t* d = der + (slot - NB) * 3;
      const uint32_t* pp = prev + (d[1] * F_h + f) * E;
      const uint32_t* sp = hist + (d[2] * F_h + f) * E;
      uint32_t* out = hist + (slot * F_h + f) * E;
      uint32_t* loc = der_lds ? sm + 4 * 2 * C + wave * E : nullptr;
      // kDU loads of each operand in flight per lane (a rolled loop waited for
      // every element pair in turn: 8 round trips for a 256-bin two-class feature)
      constexpr int kDU = 8;
      for (int64_t e0 = lane; e0 < E; e0 += (int64_t)kWave * kDU) {
        uint32_t a[kDU], bq[kDU];
#pragma unroll
        for (int u = 0; u < kDU; ++u) {
          const int64_t e = e0 + (int64_t)u * kWave;
          const int64_t es = e < E ? e : 0;
          a[u] = pp[es];
          bq[u] = sp[es];
        }
#pragma unroll
        for (int u = 0; u < kDU; ++u) {
          const int64_t e = e0 + (int64_t)u * kWave;
          if (e < E) {
            const uint32_t v = a[u] - bq[u];
            if (der_lds) loc[e] = v;
            out[e] = v;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (der_lds) {
        h = loc;
      } else {
        gp = pp;
        gs = sp;
      }
    }
  }
  auto hv = [&](int64_t i) -> uint32_t { return gp ? gp[i] - gs[i] : h[i]; };

  // ---- <= 2 classes, <= 256 bins (the common shape): one load of the lane's 4
  // bins x 2 classes (unconditional, clamped), totals from the prefix scans, and
  // every x*log2(x) lookup issued in two batches -- no separate totals pass, no
  // per-lookup round trip
  if (C <= 2 && nb <= kChunk && gp == nullptr) {
    const int b0 = lane * kBinsPerLane;
    uint32_t v[2][kBinsPerLane], p[2][kBinsPerLane], incl[2], tc[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int cc = c < C ? c : C - 1;
#pragma unroll
      for (int k = 0; k < kBinsPerLane; ++k) {
        const int b = b0 + k;
        const uint32_t raw = h[(int64_t)(b < nb ? b : nb - 1) * C + cc];
        v[c][k] = (b < nb && c < C) ? raw : 0u;
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      p[c][0] = v[c][0];
#pragma unroll
      for (int k = 1; k < kBinsPerLane; ++k) p[c][k] = p[c][k - 1] + v[c][k];
      incl[c] = wave_incl_scan_dpp(p[c][kBinsPerLane - 1]);
      tc[c] = (uint32_t)__builtin_amdgcn_readlane((int)incl[c], kWave - 1);
    }
    const uint32_t m2 = tc[0] + tc[1];
    const double tu2 = tie_unit(tlog((uint64_t)m2, xtab, xtab_n), (int64_t)m2);
    const double tinv2 = 1.0 / tu2;
    uint32_t L[2][kBinsPerLane], ml[kBinsPerLane];
#pragma unroll
    for (int k = 0; k < kBinsPerLane; ++k) ml[k] = 0u;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < kBinsPerLane; ++k) {
        L[c][k] = incl[c] - p[c][kBinsPerLane - 1] + p[c][k];
        ml[k] += L[c][k];
      }
    double cost[kBinsPerLane];
    if (crit == kEntropy) {
      // class 0 then class 1, left then right: the host's summation order
      uint32_t xs[4 * kBinsPerLane];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int k = 0; k < kBinsPerLane; ++k) {
          xs[(2 * c) * kBinsPerLane + k] = L[c][k];
          xs[(2 * c + 1) * kBinsPerLane + k] = tc[c] - L[c][k];
        }
      double tv[4 * kBinsPerLane];
      tlog_batch(xs, tv, xtab, xtab_n);
      uint32_t xm[2 * kBinsPerLane];
#pragma unroll
      for (int k = 0; k < kBinsPerLane; ++k) {
        xm[k] = ml[k];
        xm[kBinsPerLane + k] = m2 - ml[k];
      }
      double tm2[2 * kBinsPerLane];
      tlog_batch(xm, tm2, xtab, xtab_n);
#pragma unroll
      for (int k = 0; k < kBinsPerLane; ++k) {
        double sl = 0.0, sr = 0.0;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          if (tc[c] == 0u) continue;  // (absent class: the generic pass skips it too)
          sl = sl + tv[(2 * c) * kBinsPerLane + k];
          sr = sr + tv[(2 * c + 1) * kBinsPerLane + k];
        }
        cost[k] = (tm2[k] - sl) + (tm2[kBinsPerLane + k] - sr);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kBinsPerLane; ++k) {
        int64_t ql = 0, qr = 0;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int64_t a = L[c][k], r = (int64_t)tc[c] - a;
          ql += a * a;
          qr += r * r;
        }
        cost[k] = gini_term(ml[k], ql) + gini_term((int64_t)m2 - ml[k], qr);
      }
    }
    double bc = __builtin_inf();
    int bb = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < kBinsPerLane; ++k) {
      const int b = b0 + k;
      const int64_t mlk = ml[k];
      const int64_t mrk = (int64_t)m2 - mlk;
      if (b < nb && (v[0][k] | v[1][k]) && mlk >= msl && mrk >= msl) {
        const double cr = tie_round(cost[k], tinv2, tu2);
        if (cr < bc) {
          bc = cr;
          bb = b;
        }
      }
    }
    wave_argmin_dpp(bc, bb);  // one pass: lanes own ascending bins
    const bool found = bc < __builtin_inf();
    if (lane == 0) {
      out_cost[node * F_h + f] = bc;
      out_bin[node * F_h + f] = found ? bb : -1;
    }
    if (sel_left) {
      // the winning bin's left counts live in lane bb / 4, register bb % 4
      const int src = found ? (bb >> 2) : 0, kk = found ? (bb & 3) : 0;
      uint32_t lsel[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        uint32_t x = L[c][0];
#pragma unroll
        for (int k = 1; k < kBinsPerLane; ++k) x = kk == k ? L[c][k] : x;
        lsel[c] = (uint32_t)__builtin_amdgcn_readlane((int)x, src);
      }
      if (lane == 0) {
        sel_left[(node * F_h + f) * 2 + 0] = found ? (int32_t)lsel[0] : 0;
        sel_left[(node * F_h + f) * 2 + 1] = found ? (int32_t)lsel[1] : 0;
        if (f == 0) {
          sel_tot[node * 4 + 0] = (int32_t)tc[0];
          sel_tot[node * 4 + 1] = (int32_t)tc[1];
          // the node term as select_kernel computes it (classes in order; the
          // table holds x log2 x bit for bit)
          double acc = 0.0;
          int64_t sq = 0;
          for (int c = 0; c < C; ++c) {
            acc = acc + tlog((uint64_t)tc[c], xtab, xtab_n);
            sq += (int64_t)tc[c] * tc[c];
          }
          const double pt = crit == kEntropy ? tlog((uint64_t)m2, xtab, xtab_n) - acc
                                             : gini_term((int64_t)m2, sq);
          reinterpret_cast<double*>(sel_tot)[node * 2 + 1] = pt;
        }
      }
    }
    return;
  }

  // pass 1: per-class totals -- the node's class counts when the caller has them
  // (the device level loop: int32 [node][C]; every feature's bins sum to them),
  // else kScanCG classes at a time over the bins (independent reductions)
  uint32_t m = 0;
  if (node_tot != nullptr) {
    const int32_t* nt = node_tot + node * C;
    uint32_t part = 0;
    for (int c = lane; c < C; c += kWave) {
      const uint32_t t = (uint32_t)nt[c];
      tot[c] = t;
      carry[c] = 0;
      part += t;
    }
    m = wave_sum_u32(part);
  }
  for (int c0 = 0; c0 < C && node_tot == nullptr; c0 += kScanCG) {
    uint32_t s[kScanCG];
#pragma unroll
    for (int g = 0; g < kScanCG; ++g) s[g] = 0;
    for (int b = lane; b < nb; b += kWave) {
#pragma unroll
      for (int g = 0; g < kScanCG; ++g)
        if (c0 + g < C) s[g] += hv((int64_t)b * C + c0 + g);
    }
#pragma unroll
    for (int g = 0; g < kScanCG; ++g) {
      if (c0 + g >= C) break;
      const uint32_t t = wave_sum_u32(s[g]);
      if (lane == 0) {
        tot[c0 + g] = t;
        carry[c0 + g] = 0;
      }
      m += t;
    }
  }
  // tot/carry are private to this wave: order lane 0's LDS writes before the
  // other lanes' reads without a workgroup barrier (waves may have exited).
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();

  double best_cost = __builtin_inf();
  int best_bin = 0x7fffffff;
  const double tu = tie_unit(tlog((uint64_t)m, xtab, xtab_n), (int64_t)m);
  const double tinv = 1.0 / tu;
  for (int base = 0; base < nb; base += kChunk) {
    const int b0 = base + lane * kBinsPerLane;
    uint32_t mL[kBinsPerLane];
    uint32_t nonempty[kBinsPerLane];
    double sL[kBinsPerLane], sR[kBinsPerLane];
    int64_t qL[kBinsPerLane], qR[kBinsPerLane];
#pragma unroll
    for (int k = 0; k < kBinsPerLane; ++k) {
      mL[k] = 0;
      nonempty[k] = 0;
      sL[k] = 0.0;
      sR[k] = 0.0;
      qL[k] = 0;
      qR[k] = 0;
    }
    // classes in groups of kScanCG: a group's loads and DPP prefix sums are
    // independent chains issued together; classes absent from the node (total 0)
    // add exact zeros and are skipped; the sums still add class by class in
    // ascending order (bit-identical to the sequential host sums)
    // (two classes: one class per group, the register footprint of the scalar loop)
    auto class_pass = [&](auto group_tag) {
    constexpr int kG = decltype(group_tag)::value;
    for (int c0 = 0; c0 < C; c0 += kG) {
      uint32_t v[kG][kBinsPerLane], p[kG][kBinsPerLane], incl[kG];
      bool live[kG];
#pragma unroll
      for (int g = 0; g < kG; ++g) {
        const int c = c0 + g;
        live[g] = c < C && tot[c] != 0u;  // (wave-uniform)
#pragma unroll
        for (int k = 0; k < kBinsPerLane; ++k) {
          const int b = b0 + k;
          v[g][k] = (live[g] && b < nb) ? hv((int64_t)b * C + c) : 0u;
        }
      }
#pragma unroll
      for (int g = 0; g < kG; ++g) {
        p[g][0] = v[g][0];
#pragma unroll
        for (int k = 1; k < kBinsPerLane; ++k) p[g][k] = p[g][k - 1] + v[g][k];
        incl[g] = live[g] ? wave_incl_scan_dpp(p[g][kBinsPerLane - 1]) : 0u;
      }
#pragma unroll
      for (int g = 0; g < kG; ++g) {
        if (!live[g]) continue;
        const int c = c0 + g;
        const uint32_t excl = incl[g] - p[g][kBinsPerLane - 1] + carry[c];
        const uint32_t tc = tot[c];
        uint32_t xs[2 * kBinsPerLane];
#pragma unroll
        for (int k = 0; k < kBinsPerLane; ++k) {
          const uint32_t L = excl + p[g][k];
          const uint32_t R = tc - L;
          xs[2 * k] = L;
          xs[2 * k + 1] = R;
          mL[k] += L;
          nonempty[k] |= v[g][k];
          if (crit != kEntropy) {
            qL[k] += (int64_t)L * L;
            qR[k] += (int64_t)R * R;
          }
        }
        if (crit == kEntropy) {
          double tv[2 * kBinsPerLane];
          tlog_batch(xs, tv, xtab, xtab_n);
#pragma unroll
          for (int k = 0; k < kBinsPerLane; ++k) {
            sL[k] = sL[k] + tv[2 * k];
            sR[k] = sR[k] + tv[2 * k + 1];
          }
        }
        const uint32_t chunk_total = __shfl(incl[g], kWave - 1, kWave);
        if (lane == 0) carry[c] += chunk_total;
      }
    }
    };
    if (C <= 2)
      class_pass(std::integral_constant<int, 1>{});
    else
      class_pass(std::integral_constant<int, kScanCG>{});
    double tm[2 * kBinsPerLane];
    if (crit == kEntropy) {
      uint32_t xm[2 * kBinsPerLane];
#pragma unroll
      for (int k = 0; k < kBinsPerLane; ++k) {
        xm[2 * k] = mL[k];
        xm[2 * k + 1] = m - mL[k];
      }
      tlog_batch(xm, tm, xtab, xtab_n);
    }
#pragma unroll
    for (int k = 0; k < kBinsPerLane; ++k) {
      const int b = b0 + k;
      const int64_t ml = mL[k];
      const int64_t mr = (int64_t)m - ml;
      if (b < nb && nonempty[k] && ml >= msl && mr >= msl) {
        double cost;
        if (crit == kEntropy)
          cost = (tm[2 * k] - sL[k]) + (tm[2 * k + 1] - sR[k]);
        else
          cost = gini_term(ml, qL[k]) + gini_term(mr, qR[k]);
        cost = tie_round(cost, tinv, tu);
        if (cost < best_cost) {
          best_cost = cost;
          best_bin = b;
        }
      }
    }
  }
  if (nb <= kChunk)
    wave_argmin_dpp(best_cost, best_bin);  // one pass: lanes own ascending bins
  else
    wave_argmin(best_cost, best_bin);  // several passes: exact (cost, bin) order
  if (lane == 0) {
    out_cost[node * F_h + f] = best_cost;
    out_bin[node * F_h + f] = best_cost < __builtin_inf() ? best_bin : -1;
  }
}

// hist: int64 [slots][F_h][B][2] = {count, fixed sum}
__global__ __launch_bounds__(256) void scan_reg_kernel(
    const int64_t* __restrict__ hist, const int64_t* __restrict__ nodes,
    const int32_t* __restrict__ nbins, int F_h, int f_lo, int B, int msl,
    double* __restrict__ out_cost, int32_t* __restrict__ out_bin,
    const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.x >= *dcount) return;
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int f = blockIdx.y * 4 + wave;
  if (f >= F_h) return;
  const int64_t node = blockIdx.x;
  const int64_t slot = nodes[node];
  const int64_t* h = hist + (slot * F_h + f) * (int64_t)B * 2;
  const int nb = min(B, nbins[f_lo + f]);
  int64_t m = 0, S = 0;
  for (int b = lane; b < nb; b += kWave) {
    m += h[2 * b];
    S += h[2 * b + 1];
  }
  m = wave_sum_i64(m);
  S = wave_sum_i64(S);
  double best_cost = __builtin_inf();
  int best_bin = 0x7fffffff;
  int64_t carry_n = 0, carry_s = 0;
  for (int base = 0; base < nb; base += kChunk) {
    const int b0 = base + lane * kBinsPerLane;
    int64_t cn[kBinsPerLane], cs[kBinsPerLane];
#pragma unroll
    for (int k = 0; k < kBinsPerLane; ++k) {
      const int b = b0 + k;
      cn[k] = b < nb ? h[2 * b] : 0;
      cs[k] = b < nb ? h[2 * b + 1] : 0;
    }
    int64_t pn[kBinsPerLane], ps[kBinsPerLane];
    pn[0] = cn[0];
    ps[0] = cs[0];
#pragma unroll
    for (int k = 1; k < kBinsPerLane; ++k) {
      pn[k] = pn[k - 1] + cn[k];
      ps[k] = ps[k - 1] + cs[k];
    }
    const int64_t in_n = wave_incl_scan_i64(pn[kBinsPerLane - 1]);
    const int64_t in_s = wave_incl_scan_i64(ps[kBinsPerLane - 1]);
    const int64_t ex_n = in_n - pn[kBinsPerLane - 1] + carry_n;
    const int64_t ex_s = in_s - ps[kBinsPerLane - 1] + carry_s;
#pragma unroll
    for (int k = 0; k < kBinsPerLane; ++k) {
      const int b = b0 + k;
      const int64_t ml = ex_n + pn[k];
      const int64_t sl = ex_s + ps[k];
      const int64_t mr = m - ml;
      if (b < nb && cn[k] > 0 && ml >= msl && mr >= msl) {
        const double cost = mse_term(ml, sl) + mse_term(mr, S - sl);
        if (cost < best_cost) {
          best_cost = cost;
          best_bin = b;
        }
      }
    }
    carry_n += __shfl(in_n, kWave - 1, kWave);
    carry_s += __shfl(in_s, kWave - 1, kWave);
  }
  wave_argmin(best_cost, best_bin);
  if (lane == 0) {
    out_cost[node * F_h + f] = best_cost;
    out_bin[node * F_h + f] = best_cost < __builtin_inf() ? best_bin : -1;
  }
}

// One workgroup per node: best feature and the winning split's statistics.
// rec: int64 [k][R]: {gain bits, feature(global), bin, n_left, m,
//                     left[C], total[C]}             (classification, R = 5 + 2C)
//                    {gain bits, feature, bin, n_left, m, left_sum, total_sum}
//                                                     (regression, R = 7)
__global__ __launch_bounds__(256) void select_kernel(
    const void* __restrict__ hist_v, const int64_t* __restrict__ nodes,
    const double* __restrict__ cost, const int32_t* __restrict__ bins, int F_h, int f_lo, int B,
    int C, int crit, int64_t* __restrict__ rec, const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.x >= *dcount) return;
  extern __shared__ int64_t cls[];  // [C] totals, then [C] left counts
  __shared__ double s_gain[4];
  __shared__ int s_feat[4], s_bin[4];
  __shared__ int64_t s_a[4], s_b[4];
  __shared__ double s_pterm;
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t node = blockIdx.x;
  const int64_t slot = nodes[node];
  const bool reg = crit == kSquaredError;
  const int R = reg ? 7 : 5 + 2 * C;
  int64_t* out = rec + node * R;

  // node statistics from feature 0 of the histogram (every feature sums the same)
  if (reg) {
    const int64_t* h = (const int64_t*)hist_v + (slot * F_h) * (int64_t)B * 2;
    int64_t a = 0, s = 0;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
      a += h[2 * b];
      s += h[2 * b + 1];
    }
    a = wave_sum_i64(a);
    s = wave_sum_i64(s);
    if (lane == 0) {
      s_a[wave] = a;
      s_b[wave] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const int64_t m = s_a[0] + s_a[1] + s_a[2] + s_a[3];
      const int64_t S = s_b[0] + s_b[1] + s_b[2] + s_b[3];
      s_pterm = mse_term(m, S);
      out[4] = m;
      out[6] = S;
    }
  } else {
    const uint32_t* h = (const uint32_t*)hist_v + (slot * F_h) * (int64_t)B * C;
    for (int c = wave; c < C; c += 4) {
      uint32_t s = 0;
      for (int b0 = lane; b0 < B; b0 += 4 * kWave) {  // 4 bins per lane in flight
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int b = b0 + u * kWave;
          v[u] = h[(int64_t)(b < B ? b : 0) * C + c];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) s += (b0 + u * kWave < B) ? v[u] : 0u;
      }
      s = wave_sum_u32(s);
      if (lane == 0) cls[c] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // sequential over classes, matching the host order
      double acc = 0.0;
      int64_t mm = 0, sq = 0;
      for (int c = 0; c < C; ++c) {
        const int64_t t = cls[c];
        mm += t;
        acc = acc + xlog2x((uint64_t)t);
        sq += t * t;
      }
      s_pterm = crit == kEntropy ? xlog2x((uint64_t)mm) - acc : gini_term(mm, sq);
      out[4] = mm;
    }
    for (int c = threadIdx.x; c < C; c += blockDim.x) out[5 + C + c] = cls[c];
  }
  __syncthreads();
  const double pterm = s_pterm;

  // best feature: argmax gain, ties -> lowest feature
  double g = -__builtin_inf();
  int bf = 0x7fffffff, bb = -1;
  for (int f = threadIdx.x; f < F_h; f += blockDim.x) {
    const double c = cost[node * F_h + f];
    if (c < __builtin_inf()) {
      const double gf = pterm - c;
      if (gf > g) {
        g = gf;
        bf = f;
        bb = bins[node * F_h + f];
      }
    }
  }
  wave_argmax(g, bf, bb);
  if (lane == 0) {
    s_gain[wave] = g;
    s_feat[wave] = bf;
    s_bin[wave] = bb;
  }
  __syncthreads();
  g = s_gain[0];
  bf = s_feat[0];
  bb = s_bin[0];
  for (int w = 1; w < 4; ++w) {
    if (s_gain[w] > g || (s_gain[w] == g && s_feat[w] < bf)) {
      g = s_gain[w];
      bf = s_feat[w];
      bb = s_bin[w];
    }
  }
  const bool ok = g > -__builtin_inf();
  if (threadIdx.x == 0) {
    out[0] = (int64_t)double_to_bits(g);
    out[1] = ok ? f_lo + bf : -1;
    out[2] = ok ? bb : -1;
  }
  if (!ok) {
    if (threadIdx.x == 0) {
      out[3] = 0;
      if (reg) out[5] = 0;
    }
    if (!reg)
      for (int c = threadIdx.x; c < C; c += blockDim.x) out[5 + c] = 0;
    return;
  }
  // winning split's left statistics
  if (reg) {
    const int64_t* h = (const int64_t*)hist_v + (slot * F_h + bf) * (int64_t)B * 2;
    int64_t a = 0, s = 0;
    for (int b = threadIdx.x; b <= bb; b += blockDim.x) {
      a += h[2 * b];
      s += h[2 * b + 1];
    }
    a = wave_sum_i64(a);
    s = wave_sum_i64(s);
    __syncthreads();
    if (lane == 0) {
      s_a[wave] = a;
      s_b[wave] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      out[3] = s_a[0] + s_a[1] + s_a[2] + s_a[3];
      out[5] = s_b[0] + s_b[1] + s_b[2] + s_b[3];
    }
  } else {
    const uint32_t* h = (const uint32_t*)hist_v + (slot * F_h + bf) * (int64_t)B * C;
    int64_t* left = cls + C;
    for (int c = wave; c < C; c += 4) {
      uint32_t s = 0;
      for (int b0 = lane; b0 <= bb; b0 += 4 * kWave) {  // 4 bins per lane in flight
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int b = b0 + u * kWave;
          v[u] = h[(int64_t)(b <= bb ? b : 0) * C + c];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) s += (b0 + u * kWave <= bb) ? v[u] : 0u;
      }
      s = wave_sum_u32(s);
      if (lane == 0) left[c] = s;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) out[5 + c] = left[c];
    if (threadIdx.x == 0) {
      int64_t nl = 0;
      for (int c = 0; c < C; ++c) nl += left[c];
      out[3] = nl;
    }
  }
}

// The select stays a launch of its own. Fusing it into scan_cls_kernel (the
// last of a node's feature-group workgroups runs it, behind an agent-scope
// release / acquire on a per-node counter) was measured on the 1M x 64
// flagship: the scan went from ~19 to ~82 us per level -- every workgroup's
// agent-scope release writes back its XCD's L2 -- against the ~6 us launch
// it saves.
bool scan_fused_select_ok(int B, int C, int crit) {
  return C <= 2 && B <= kChunk && crit != kSquaredError;
}

void launch_scan(hipStream_t stream, const void* hist, const int64_t* nodes, int k,
                 const int32_t* nbins, int F_h, int f_lo, int B, int C, int crit, int msl,
                 double* cost, int32_t* bins, int64_t* rec, const double* xtab, int xtab_n,
                 const int32_t* dcount, const int64_t* der, const void* prev,
                 const int32_t* nbuilt, int32_t* sel_left, int32_t* sel_tot,
                 const int32_t* node_tot) {
  // sel_left (fused selection): the planner builds the records, no select launch
  if (k <= 0) return;
  if (sel_left && !scan_fused_select_ok(B, C, crit))
    throw std::runtime_error("scan: fused selection needs <= 2 classes and <= 256 bins");
  dim3 grid(k, (F_h + 3) / 4);
  if (crit == kSquaredError) {
    hipLaunchKernelGGL(scan_reg_kernel, grid, dim3(256), 0, stream, (const int64_t*)hist, nodes,
                       nbins, F_h, f_lo, B, msl, cost, bins, dcount);
  } else {
    // derived histograms stay in LDS up to 4096 bins x classes (64 KB for the
    // four waves); past that the scan derives each count from global memory
    const int der_lds = der != nullptr && (int64_t)B * C <= 4096;
    size_t lds = (size_t)4 * 2 * C * sizeof(uint32_t) +
                 (der_lds ? (size_t)4 * B * C * sizeof(uint32_t) : 0);
    MT_HIP_CHECK(mt_set_max_lds((const void*)scan_cls_kernel, (int)lds));
    hipLaunchKernelGGL(scan_cls_kernel, grid, dim3(256), lds, stream, (uint32_t*)hist,
                       nodes, nbins, F_h, f_lo, B, C, crit, msl, cost, bins, xtab, xtab_n,
                       dcount, der, (const uint32_t*)prev, nbuilt, der_lds, sel_left, sel_tot,
                       node_tot);
  }
  MT_HIP_CHECK(hipGetLastError());
  if (sel_left) return;
  const size_t sel_lds = crit == kSquaredError ? 16 : (size_t)2 * C * sizeof(int64_t);
  MT_HIP_CHECK(mt_set_max_lds((const void*)select_kernel, (int)sel_lds));
  hipLaunchKernelGGL(select_kernel, dim3(k), dim3(256), sel_lds, stream, hist, nodes, cost, bins,
                     F_h, f_lo, B, C, crit, rec, dcount);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
