// Whole-tree fit of a small classification problem in ONE workgroup (gfx950).
//
// The reference's published benchmark is its worst case for a GPU: n <= 241
// rows, one feature and n classes (mpitree experiments.ipynb:198-209: every
// row its own class). Histograms of B x C counts per node do not fit in LDS
// for C ~ B ~ 256, and a level-wise engine pays ~8 launches per level for a
// tree of a few hundred nodes. Here one 1024-thread workgroup grows the whole
// tree level by level with no launch and no host round trip in between:
//
//   presort  per feature, the rows sorted by code (LDS bitonic network), and
//            once more by label; global scratch ord[2][F + 1][n] (u16 rows)
//   level    every frontier node owns the same position segment [s, s + m)
//            of all F + 1 orders (a stable partition keeps each order sorted
//            inside every segment)
//     node pass     thread per node: class counts from its label-order
//                   segment (runs), node term, stopping rules, output record
//     feature f     thread per position p: rank[row] = p, code; a candidate
//                   is the end of an equal-code run inside a segment; its
//                   left / right class counts come from one walk over the
//                   node's label-order segment (rows with rank <= p go left),
//                   summed per class in ascending class order -- the exact
//                   integer-form criterion and tie rounding of every other
//                   engine (criterion.h), so the tree is theirs bit for bit;
//                   (cost units << 24 | position) min per node (LDS atomic),
//                   then the best feature by gain (ties: lowest feature)
//     split pass    children positions (pre-order: p + 1, p + 2 n_left), the
//                   next frontier (block scan), rows' go-left flags
//     partition     every order stably split into left | right per segment
//
// Work per level is O(F * sum m^2) for the candidate walks -- 58k steps at the
// root of the n = 241 benchmark -- and ~6 F workgroup barriers. Limits: n <=
// 1024 rows (one position per thread), labels < 65536, codes < 65536.

#include <climits>

#include "common.h"
#include "criterion.h"

namespace mt {

constexpr int kSfThreads = 1024;
constexpr int kSfWaves = kSfThreads / kWave;
constexpr int kSfMaxRows = 1024;

// exclusive block prefix of one int per thread; total via *tot
__device__ __forceinline__ int sf_scan_excl(int v, int* s_w, int* tot) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int incl = (int)wave_incl_scan_u32((uint32_t)v);
  if (lane == kWave - 1) s_w[w] = incl;
  __syncthreads();
  int off = 0, t = 0;
#pragma unroll
  for (int k = 0; k < kSfWaves; ++k) {
    const int x = s_w[k];
    off += k < w ? x : 0;
    t += x;
  }
  __syncthreads();
  *tot = t;
  return off + incl - v;
}

// ascending bitonic sort of kSfThreads u32 keys in LDS (one key per thread)
__device__ __forceinline__ void sf_sort(uint32_t* key) {
  const int t = threadIdx.x;
  for (int k = 2; k <= kSfThreads; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int o = t ^ j;
      if (o > t) {
        const uint32_t a = key[t], b = key[o];
        const bool up = (t & k) == 0;
        if ((a > b) == up) {
          key[t] = b;
          key[o] = a;
        }
      }
      __syncthreads();
    }
  }
}

template <typename CodeT>
__global__ __launch_bounds__(kSfThreads) void small_fit_kernel(
    const CodeT* __restrict__ codes_fm, int64_t n_stride, int n, int F,
    const int32_t* __restrict__ y, int C, int crit, int max_depth, int64_t mss, int64_t msl,
    const double* __restrict__ xtab, int xtab_n, uint16_t* __restrict__ ord,
    int32_t* __restrict__ node_i32, int32_t* __restrict__ node_cnt, int64_t P) {
  __shared__ double s_tab[kSfMaxRows + 1];
  __shared__ uint32_t s_key[kSfThreads];
  __shared__ int16_t s_lab[kSfMaxRows];
  __shared__ int16_t s_seg[kSfMaxRows];   // frontier slot of position p (-1: none)
  __shared__ uint16_t s_rank[kSfMaxRows];
  __shared__ uint16_t s_code[kSfMaxRows];
  __shared__ uint8_t s_gol[kSfMaxRows];   // row goes left at this level's split
  // frontier (at most n nodes of >= 1 row)
  __shared__ int16_t f_start[kSfMaxRows], f_cnt[kSfMaxRows], f_depth[kSfMaxRows];
  __shared__ int32_t f_pos[kSfMaxRows];
  __shared__ int16_t n_start[kSfMaxRows], n_cnt[kSfMaxRows], n_depth[kSfMaxRows];
  __shared__ int32_t n_pos[kSfMaxRows];
  __shared__ double f_pterm[kSfMaxRows], f_tu[kSfMaxRows], f_gain[kSfMaxRows];
  __shared__ unsigned long long f_key[kSfMaxRows];
  __shared__ int16_t f_bf[kSfMaxRows], f_nl[kSfMaxRows];
  __shared__ uint16_t f_thr[kSfMaxRows];
  __shared__ uint8_t f_term[kSfMaxRows];
  __shared__ int s_w[kSfWaves];
  __shared__ int s_K;

  const int tid = threadIdx.x;
  const int NA = F + 1;  // orders: F features, then the label order
  uint16_t* ord_cur = ord;
  uint16_t* ord_nxt = ord + (int64_t)NA * n;
  auto T = [&](int64_t x) -> double {
    return x <= kSfMaxRows ? s_tab[x] : (x < xtab_n ? xtab[x] : xlog2x((uint64_t)x));
  };
  auto codeof = [&](int f, int r) -> uint32_t {
    return (uint32_t)codes_fm[(int64_t)f * n_stride + r];
  };
  for (int i = tid; i <= kSfMaxRows; i += kSfThreads) s_tab[i] = i < xtab_n ? xtab[i] : xlog2x(i);
  if (tid < n) s_lab[tid] = (int16_t)y[tid];
  // counts of every position start at zero (positions are written sparsely)
  for (int64_t i = tid; i < P * C; i += kSfThreads) node_cnt[i] = 0;
  __syncthreads();
  // ---- presort every feature by code, then the rows by label (stable by row)
  for (int a = 0; a < NA; ++a) {
    s_key[tid] = tid < n ? ((a < F ? codeof(a, tid) : (uint32_t)(uint16_t)s_lab[tid]) << 16 |
                            (uint32_t)tid)
                         : 0xffffffffu;
    __syncthreads();
    sf_sort(s_key);
    if (tid < n) ord_cur[(int64_t)a * n + tid] = (uint16_t)(s_key[tid] & 0xffffu);
    __syncthreads();
  }
  if (tid == 0) {
    s_K = 1;
    f_start[0] = 0;
    f_cnt[0] = (int16_t)n;
    f_depth[0] = 0;
    f_pos[0] = 0;
  }
  if (tid < n) s_seg[tid] = 0;
  __syncthreads();
  for (int level = 0; level <= kSfMaxRows; ++level) {
    const int K = s_K;
    if (K == 0) break;
    // ---- node pass: counts (label-order runs), record, stopping rules
    for (int j = tid; j < K; j += kSfThreads) {
      const int s = f_start[j], m = f_cnt[j], d = f_depth[j];
      const int64_t pos = f_pos[j];
      const uint16_t* lo = ord_cur + (int64_t)F * n + s;
      double acc = 0.0;
      int64_t sq = 0;
      int nz = 0, run = 0, prev = -1;
      for (int q = 0; q <= m; ++q) {
        const int lab = q < m ? s_lab[lo[q]] : -2;
        if (lab != prev && run > 0) {
          node_cnt[pos * C + prev] = run;
          acc = acc + T(run);
          sq += (int64_t)run * run;
          ++nz;
          run = 0;
        }
        prev = lab;
        ++run;
      }
      int32_t* R = node_i32 + pos * 6;
      R[0] = -1;
      R[1] = -1;
      R[2] = -1;
      R[3] = -1;
      R[4] = d;
      R[5] = m;
      f_pterm[j] = crit == kEntropy ? T(m) - acc : gini_term(m, sq);
      f_tu[j] = tie_unit(T(m), (int64_t)m);
      const bool depth_stop = max_depth >= 0 && d >= max_depth;
      f_term[j] = (depth_stop || m < mss || m < 2 * msl || nz <= 1) ? 1 : 0;
      f_gain[j] = -__builtin_inf();
      f_bf[j] = -1;
      f_key[j] = ~0ull;
    }
    __syncthreads();
    // ---- split search, one feature at a time
    for (int f = 0; f < F; ++f) {
      int r = 0;
      if (tid < n) {
        r = ord_cur[(int64_t)f * n + tid];
        s_rank[r] = (uint16_t)tid;
        s_code[tid] = (uint16_t)codeof(f, r);
      }
      __syncthreads();
      if (tid < n) {
        const int j = s_seg[tid];
        if (j >= 0 && !f_term[j]) {
          const int s = f_start[j], m = f_cnt[j];
          const int e = s + m;
          const int ml = tid - s + 1, mr = m - ml;
          if (tid + 1 < e && s_code[tid + 1] != s_code[tid] && ml >= msl && mr >= msl) {
            const uint16_t* lo = ord_cur + (int64_t)F * n + s;
            double sl = 0.0, sr = 0.0;
            int64_t ql = 0, qr = 0;
            int cl = 0, ct = 0, prev = -1;
            for (int q = 0; q <= m; ++q) {
              int lab = -2, rr = 0;
              if (q < m) {
                rr = lo[q];
                lab = s_lab[rr];
              }
              if (lab != prev && ct > 0) {  // close the run of class `prev`
                const int cr = ct - cl;
                if (crit == kEntropy) {
                  sl = sl + (cl > 0 ? T(cl) : 0.0);
                  sr = sr + (cr > 0 ? T(cr) : 0.0);
                } else {
                  ql += (int64_t)cl * cl;
                  qr += (int64_t)cr * cr;
                }
                cl = 0;
                ct = 0;
              }
              prev = lab;
              if (q < m) {
                ++ct;
                cl += s_rank[rr] <= tid ? 1 : 0;
              }
            }
            double cost = crit == kEntropy ? (T(ml) - sl) + (T(mr) - sr)
                                           : gini_term(ml, ql) + gini_term(mr, qr);
            const double tu = f_tu[j];
            double qn = __builtin_rint(cost * (1.0 / tu));
            qn = qn < 0.0 ? 0.0 : qn;
            const unsigned long long key =
                ((unsigned long long)qn << 24) | (unsigned long long)(tid - s);
            atomicMin(&f_key[j], key);
          }
        }
      }
      __syncthreads();
      for (int j = tid; j < K; j += kSfThreads) {
        const unsigned long long key = f_key[j];
        if (key != ~0ull) {
          const double tu = f_tu[j];
          const double cost = (double)(key >> 24) * tu;
          const double g = f_pterm[j] - cost;
          if (g > f_gain[j]) {  // features ascend: strict > keeps the lowest
            const int off = (int)(key & 0xffffffull);
            f_gain[j] = g;
            f_bf[j] = (int16_t)f;
            f_nl[j] = (int16_t)(off + 1);
            f_thr[j] = s_code[f_start[j] + off];
          }
          f_key[j] = ~0ull;
        }
      }
      __syncthreads();
    }
    // ---- split pass: records, next frontier (two children per split)
    int nsp = 0;
    int j0 = tid;
    if (j0 < K) nsp = (f_bf[j0] >= 0) ? 2 : 0;
    int K2;
    const int o = sf_scan_excl(nsp, s_w, &K2);  // K <= n <= 1024: one pass
    if (j0 < K && nsp) {
      const int64_t pos = f_pos[j0];
      const int nl = f_nl[j0], m = f_cnt[j0], s = f_start[j0];
      int32_t* R = node_i32 + pos * 6;
      R[0] = f_bf[j0];
      R[1] = f_thr[j0];
      R[2] = (int32_t)(pos + 1);
      R[3] = (int32_t)(pos + 2 * nl);
      n_start[o] = (int16_t)s;
      n_cnt[o] = (int16_t)nl;
      n_depth[o] = (int16_t)(f_depth[j0] + 1);
      n_pos[o] = (int32_t)(pos + 1);
      n_start[o + 1] = (int16_t)(s + nl);
      n_cnt[o + 1] = (int16_t)(m - nl);
      n_depth[o + 1] = (int16_t)(f_depth[j0] + 1);
      n_pos[o + 1] = (int32_t)(pos + 2 * nl);
    }
    // rows of split nodes: go-left flags (from the label order's positions)
    if (tid < n) {
      const int j = s_seg[tid];
      const int rr = ord_cur[(int64_t)F * n + tid];
      s_gol[rr] = (j >= 0 && f_bf[j] >= 0) ? (codeof(f_bf[j], rr) <= f_thr[j] ? 1 : 0) : 0;
    }
    __syncthreads();
    // ---- partition every order: stable left | right inside each split segment
    for (int a = 0; a < NA; ++a) {
      int rr = 0, j = -1, left = 0;
      if (tid < n) {
        rr = ord_cur[(int64_t)a * n + tid];
        j = s_seg[tid];
        left = (j >= 0 && f_bf[j] >= 0 && s_gol[rr]) ? 1 : 0;
      }
      int tot;
      const int ex = sf_scan_excl(left, s_w, &tot);
      s_key[tid] = (uint32_t)ex;  // exclusive left counts, read at segment starts
      __syncthreads();
      if (tid < n) {
        int np = tid;
        if (j >= 0 && f_bf[j] >= 0) {
          const int s = f_start[j];
          const int lbefore = ex - (int)s_key[s];  // left rows in [s, tid)
          np = left ? s + lbefore : s + f_nl[j] + (tid - s - lbefore);
        }
        ord_nxt[(int64_t)a * n + np] = (uint16_t)rr;
      }
      __syncthreads();
    }
    // ---- next frontier and its segments
    for (int q = tid; q < K2; q += kSfThreads) {
      f_start[q] = n_start[q];
      f_cnt[q] = n_cnt[q];
      f_depth[q] = n_depth[q];
      f_pos[q] = n_pos[q];
    }
    if (tid < n) s_seg[tid] = -1;
    __syncthreads();
    for (int q = 0; q < K2; ++q) {  // segments are disjoint: one pass per node
      const int s = f_start[q], m = f_cnt[q];
      if (tid >= s && tid < s + m) s_seg[tid] = (int16_t)q;
    }
    if (tid == 0) s_K = K2;
    uint16_t* t = ord_cur;
    ord_cur = ord_nxt;
    ord_nxt = t;
    __syncthreads();
  }
}

int small_fit_max_rows() { return kSfMaxRows; }

void launch_small_fit(hipStream_t stream, const void* codes_fm, int code_bytes, int64_t n_stride,
                      int n, int F, const int32_t* y, int C, int crit, int max_depth,
                      int64_t mss, int64_t msl, const double* xtab, int xtab_n, uint16_t* ord,
                      int32_t* node_i32, int32_t* node_cnt, int64_t P) {
  if (n <= 0) return;
  if (n > kSfMaxRows) throw std::runtime_error("small fit: at most 1024 rows");
  if (C > 65535) throw std::runtime_error("small fit: at most 65535 classes");
  if (code_bytes == 1)
    hipLaunchKernelGGL(small_fit_kernel<uint8_t>, dim3(1), dim3(kSfThreads), 0, stream,
                       (const uint8_t*)codes_fm, n_stride, n, F, y, C, crit, max_depth, mss, msl,
                       xtab, xtab_n, ord, node_i32, node_cnt, P);
  else
    hipLaunchKernelGGL(small_fit_kernel<uint16_t>, dim3(1), dim3(kSfThreads), 0, stream,
                       (const uint16_t*)codes_fm, n_stride, n, F, y, C, crit, max_depth, mss,
                       msl, xtab, xtab_n, ord, node_i32, node_cnt, P);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
