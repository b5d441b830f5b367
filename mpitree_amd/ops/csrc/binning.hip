// Feature binning on gfx950: bin edges and codes for the whole matrix.
//
// The reference re-derives candidate thresholds at every node with
// ``np.unique(X[:, f])`` (mpitree/tree/decision_tree.py:73). Here binning is a
// single up-front pass of two kernels:
//
// edges_kernel (one workgroup per feature): a deterministic strided row sample
//   of the column is staged in LDS. Its distinct values are first collected in
//   an LDS open-addressing hash set; when there are at most ``limit`` of them
//   (tabular data: integers, categories, quantized values) the feature is in
//   exact mode and its edges are those values, sorted. Otherwise the sample is
//   bitonic-sorted in LDS and ``limit`` quantile edges are taken (duplicates
//   dropped). Exactly the edges the host BinMapper would produce for the same
//   sample.
// bin_kernel (row tile x 16-feature tile): each thread bins 16 elements with
//   16 independent branch-free lower_bound searches over LDS edges (ILP hides
//   the LDS latency), verifies exact-mode values against their edge, flags
//   non-finite input, and writes codes row-major (histogram gathers) and
//   feature-major (partition's single-column reads) from an LDS tile.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace mt {

template <typename XT>
struct KeyOf {
  using T = typename std::conditional<sizeof(XT) == 8, unsigned long long, uint32_t>::type;
};

template <typename XT>
__device__ __forceinline__ typename KeyOf<XT>::T key_bits(XT v) {
  if constexpr (sizeof(XT) == 8) {
    return (unsigned long long)__double_as_longlong(v);
  } else {
    return __float_as_uint(v);
  }
}

template <typename XT>
__device__ __forceinline__ XT key_value(typename KeyOf<XT>::T k) {
  if constexpr (sizeof(XT) == 8) {
    return __longlong_as_double((long long)k);
  } else {
    return __uint_as_float(k);
  }
}

constexpr int kEdgeThreads = 1024;
constexpr int kEdgeHash = 2048;  // hash slots (exact mode needs <= limit <= 1024 keys)

// One workgroup per feature. smem: sample [S] XT, hash [kEdgeHash] keys.
// S = power of two >= s (padding +inf sorts last). Output: edges [F][limit]
// (+inf padded), nbins [F], exact [F].
// The edge sample, transposed: smp[f][i] = X[i n / s][f] for the s sampled rows.
// One workgroup per 64 rows x 64 features through an LDS tile: each sampled row is
// one contiguous read of its features (the per-feature workgroups of edges_kernel
// otherwise gather every value alone, from a different row -- 64 workgroups on a
// 256-CU chip, latency-bound at ~60 us for 1M x 64), and each feature's run of
// 64 values is one contiguous write.
template <typename XT>
__global__ __launch_bounds__(256) void edges_sample_kernel(const XT* __restrict__ X, int64_t n,
                                                           int F, int s,
                                                           XT* __restrict__ smp) {
  __shared__ XT tile[64][65];
  const int i0 = blockIdx.x * 64, f0 = blockIdx.y * 64;
  const int tid = threadIdx.x, c = tid & 63;
  for (int r = tid >> 6; r < 64; r += 4) {
    const int i = i0 + r, f = f0 + c;
    XT v = (XT)0;
    if (i < s && f < F) v = X[((int64_t)i * n / s) * F + f];  // (edges_kernel's sample rows)
    tile[r][c] = v;
  }
  __syncthreads();
  for (int q = tid >> 6; q < 64; q += 4) {
    const int f = f0 + q, i = i0 + c;
    if (f < F && i < s) smp[(int64_t)f * s + i] = tile[c][q];
  }
}

template <typename XT>
__global__ __launch_bounds__(kEdgeThreads) void edges_kernel(const XT* __restrict__ X, int64_t n,
                                                             int F, int s, int S, int limit,
                                                             XT* __restrict__ edges,
                                                             int32_t* __restrict__ nbins,
                                                             uint8_t* __restrict__ exact,
                                                             int probe,
                                                             const XT* __restrict__ smp) {
  using K = typename KeyOf<XT>::T;
  extern __shared__ __align__(16) uint8_t smem[];
  XT* key = reinterpret_cast<XT*>(smem);
  K* hset = reinterpret_cast<K*>(smem + (size_t)S * sizeof(XT));
  __shared__ int s_cnt, s_over;
  __shared__ int w_sum[kEdgeThreads / kWave];
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  const K kEmpty = ~(K)0;  // a NaN pattern: never a (finite) data value
  const bool use_hash = limit <= kEdgeHash / 2;
  if (tid == 0) {
    s_cnt = 0;
    s_over = use_hash ? 0 : 1;
  }
  for (int i = tid; i < kEdgeHash; i += kEdgeThreads) hset[i] = kEmpty;
  // kEdgeLoads independent gathers in flight per thread before the LDS stores:
  // each is a lone 4-8 B read from a different row, so the sample phase is
  // latency-bound (one-at-a-time issue measured 75 us of a 1M x 64 fit)
  constexpr int kEdgeLoads = 8;
  for (int i0 = tid; i0 < S; i0 += kEdgeThreads * kEdgeLoads) {
    XT v[kEdgeLoads];
#pragma unroll
    for (int u = 0; u < kEdgeLoads; ++u) {
      const int i = i0 + u * kEdgeThreads;
      v[u] = __builtin_inf();
      if (i < s) {
        if (smp != nullptr) {  // (the transposed sample: one contiguous run per feature)
          v[u] = smp[(int64_t)f * s + i];
        } else {
          const int64_t row = (int64_t)i * n / s;  // deterministic strided sample
          v[u] = X[row * F + f];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kEdgeLoads; ++u) {
      const int i = i0 + u * kEdgeThreads;
      // -0 and +0 are one value (x <= t cannot tell them apart)
      if (i < S) key[i] = v[u] == (XT)0 ? (XT)0 : v[u];
    }
  }
  __syncthreads();
  // ---- exact-mode probe: distinct values into the LDS hash set
  if (use_hash) {
    for (int i = tid; i < s && !s_over; i += kEdgeThreads) {
      const K k = key_bits<XT>(key[i]);
      uint32_t h = (uint32_t)(k ^ (k >> 29)) * 0x9E3779B1u;
      int slot = (int)(h >> 21) & (kEdgeHash - 1);
      for (int probe = 0; probe < kEdgeHash; ++probe) {
        const K cur = atomicCAS(&hset[slot], kEmpty, k);
        if (cur == kEmpty) {  // inserted a new distinct value
          if (atomicAdd(&s_cnt, 1) + 1 > limit) s_over = 1;
          break;
        }
        if (cur == k) break;
        slot = (slot + 1) & (kEdgeHash - 1);
      }
    }
  }
  __syncthreads();
  XT* out = edges + (int64_t)f * limit;
  if (probe && s_over) {
    // exact-threshold probe (core/fit.py, max_bins=None): more than `limit` values
    // send the fit to the presorted-list engine, which needs no quantile edges
    for (int i = tid; i < limit; i += kEdgeThreads) out[i] = (XT)__builtin_inf();
    if (tid == 0) {
      nbins[f] = limit;
      exact[f] = 0;
    }
    return;
  }
  if (!s_over) {
    // exact: sort the <= limit distinct values (compact them into key[] first)
    const int m = s_cnt;
    __syncthreads();
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    for (int i = tid; i < kEdgeHash; i += kEdgeThreads) {
      const K k = hset[i];
      if (k != kEmpty) key[atomicAdd(&s_cnt, 1)] = key_value<XT>(k);
    }
    __syncthreads();
    int M = 1;
    while (M < m) M <<= 1;
    for (int i = m + tid; i < M; i += kEdgeThreads) key[i] = __builtin_inf();
    __syncthreads();
    for (int k = 2; k <= M; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int q = tid; q < (M >> 1); q += kEdgeThreads) {
          const int lo = ((q & ~(j - 1)) << 1) | (q & (j - 1));
          const int hi = lo | j;
          const XT a = key[lo], b = key[hi];
          const bool up = (lo & k) == 0;
          if ((a > b) == up) {
            key[lo] = b;
            key[hi] = a;
          }
        }
        __syncthreads();
      }
    }
    for (int i = tid; i < limit; i += kEdgeThreads) out[i] = i < m ? key[i] : (XT)__builtin_inf();
    if (tid == 0) {
      nbins[f] = m;
      exact[f] = 1;
    }
    return;
  }
  // ---- quantile mode: bitonic sort of the whole sample
  for (int k = 2; k <= S; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int q = tid; q < (S >> 1); q += kEdgeThreads) {
        const int lo = ((q & ~(j - 1)) << 1) | (q & (j - 1));
        const int hi = lo | j;
        const XT a = key[lo], b = key[hi];
        const bool up = (lo & k) == 0;
        if ((a > b) == up) {
          key[lo] = b;
          key[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  // ordered compaction: out[0..) = value(i) for i in [0, R) with pick(i) true
  __shared__ int s_base;
  auto compact = [&](int R, auto pick, auto value) {
    if (tid == 0) s_base = 0;
    __syncthreads();
    for (int b0 = 0; b0 < R; b0 += kEdgeThreads) {
      const int i = b0 + tid;
      const bool keep = i < R && pick(i);
      const unsigned long long bal = __ballot(keep);
      const int lane = lane_id();
      const int wv = tid >> 6;
      if (lane == 0) w_sum[wv] = __popcll(bal);
      __syncthreads();
      int off = s_base;
      for (int w = 0; w < wv; ++w) off += w_sum[w];
      const int pos = off + __popcll(bal & ((1ull << lane) - 1ull));
      if (keep) out[pos] = value(i);
      __syncthreads();
      if (tid == kEdgeThreads - 1) s_base = pos + (keep ? 1 : 0);
      __syncthreads();
    }
    return s_base;
  };
  // distinct values of the sorted sample
  int cnt = 0;
  for (int i = tid; i < s; i += kEdgeThreads) cnt += (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
  cnt = (int)wave_sum_u32((uint32_t)cnt);
  if (lane_id() == 0) w_sum[tid >> 6] = cnt;
  __syncthreads();
  int distinct = 0;
  for (int w = 0; w < kEdgeThreads / kWave; ++w) distinct += w_sum[w];
  __syncthreads();
  const bool is_exact = distinct <= limit;
  int m;
  if (is_exact) {
    m = compact(
        s, [&](int i) { return i == 0 || key[i] != key[i - 1]; }, [&](int i) { return key[i]; });
  } else {
    // quantile k (1..limit) is sample element ceil(k s / limit) - 1; keep first of runs
    auto qi = [&](int k1) {
      const int64_t q = ((int64_t)k1 * s + limit - 1) / limit - 1;
      return (int)(q < s - 1 ? q : s - 1);
    };
    m = compact(
        limit, [&](int k) { return k == 0 || key[qi(k)] != key[qi(k + 1)]; },
        [&](int k) { return key[qi(k + 1)]; });
  }
  for (int i = m + tid; i < limit; i += kEdgeThreads) out[i] = (XT)__builtin_inf();
  if (tid == 0) {
    nbins[f] = m;
    exact[f] = is_exact ? 1 : 0;
  }
}

// skip_inexact (the exact-threshold probe): when any feature came back inexact the
// fit runs the presorted-list engine and never reads the codes; a bin workgroup then
// only checks its rows x features for non-finite values (flags bit 1).
__device__ __forceinline__ bool bin_any_inexact(const uint8_t* __restrict__ exact, int F) {
  __shared__ int s_any;
  if (threadIdx.x == 0) s_any = 0;
  __syncthreads();
  for (int f = threadIdx.x; f < F; f += blockDim.x)
    if (!exact[f]) s_any = 1;
  __syncthreads();
  return s_any != 0;
}

template <typename XT>
__device__ __forceinline__ void bin_finite_only(const XT* __restrict__ X, int F, int64_t r0,
                                                int64_t r1, int f0, int nf,
                                                int32_t* __restrict__ flags) {
  // one wave per row, lanes over the tile's features (contiguous reads), kU rows'
  // loads in flight per lane before any check
  constexpr int kU = 8;
  const int lane = lane_id(), nwv = blockDim.x / kWave;
  for (int64_t rb = r0 + (threadIdx.x >> 6); rb < r1; rb += (int64_t)nwv * kU)
    for (int f = lane; f < nf; f += kWave) {
      XT v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t r = rb + (int64_t)u * nwv;
        v[u] = r < r1 ? X[r * F + f0 + f] : (XT)0;
      }
      bool bad = false;
#pragma unroll
      for (int u = 0; u < kU; ++u) bad |= !(v[u] - v[u] == (XT)0);
      if (bad) atomicOr(&flags[f0 + f], 2);
    }
}

constexpr int kBinRows = 256;
constexpr int kBinFt = 16;                          // features per tile
constexpr int kBinPer = kBinRows * kBinFt / 256;    // elements per thread

// grid = (row tiles, feature tiles). flags[f]: bit 0 = an exact-mode value
// missed its edge (sample incomplete), bit 1 = non-finite value seen.
template <typename XT, typename CodeT, bool kLds>
__global__ __launch_bounds__(256) void bin_kernel(const XT* __restrict__ X, int64_t n, int F,
                                                  const XT* __restrict__ edges, int Bmax,
                                                  int estride, int steps0, const int32_t* __restrict__ nbins,
                                                  const uint8_t* __restrict__ exact,
                                                  CodeT* __restrict__ codes_rm, int row_elems,
                                                  CodeT* __restrict__ codes_fm,
                                                  int32_t* __restrict__ flags, int skip_inexact) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ int s_flag[kBinFt];
  if (skip_inexact && bin_any_inexact(exact, F)) {
    const int64_t a = blockIdx.x * (int64_t)kBinRows;
    bin_finite_only<XT>(X, F, a, min<int64_t>(n, a + kBinRows), blockIdx.y * kBinFt,
                        min(kBinFt, F - (int)blockIdx.y * kBinFt), flags);
    return;
  }
  __shared__ int32_t s_nb[kBinFt];
  __shared__ uint8_t s_ex[kBinFt];
  // [kBinFt][ES] when staged; the odd row stride ES spreads the 16 features'
  // concurrent searches over different LDS banks
  const int ES = Bmax | 1;
  XT* s_edges = reinterpret_cast<XT*>(smem);
  CodeT* tile = reinterpret_cast<CodeT*>(smem + (kLds ? (size_t)kBinFt * ES * sizeof(XT) : 0));
  const int64_t r0 = blockIdx.x * (int64_t)kBinRows;
  const int rows = (int)min<int64_t>(kBinRows, n - r0);
  const int f0 = blockIdx.y * kBinFt;
  const int nf = min(kBinFt, F - f0);
  if (threadIdx.x < kBinFt) {
    s_flag[threadIdx.x] = 0;
    s_nb[threadIdx.x] = threadIdx.x < nf ? nbins[f0 + threadIdx.x] : 1;
    s_ex[threadIdx.x] = threadIdx.x < nf ? exact[f0 + threadIdx.x] : 0;
  }
  if constexpr (kLds) {
    for (int e = threadIdx.x; e < nf * Bmax; e += 256) {
      const int fl = e / Bmax, b = e - fl * Bmax;
      s_edges[fl * ES + b] = edges[(int64_t)(f0 + fl) * estride + b];
    }
  }
  __syncthreads();
  // element e = threadIdx.x + 256 k -> (row e / 16, feature e % 16): a wave reads
  // 4 rows x 16 consecutive features per step
  XT v[kBinPer];
  int pos[kBinPer], nb[kBinPer];
  bool ok[kBinPer];
#pragma unroll
  for (int k = 0; k < kBinPer; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int r = e / kBinFt, fl = e % kBinFt;
    ok[k] = r < rows && fl < nf;
    v[k] = ok[k] ? X[(r0 + r) * F + f0 + fl] : (XT)0;
    // no search for padding elements: with global edges (kLds false) a lane of
    // a feature past F would read edges rows beyond the table
    nb[k] = ok[k] ? s_nb[fl] : 0;
    pos[k] = 0;  // number of edges < v (lower_bound)
  }
  for (int step = steps0; step > 0; step >>= 1) {
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
      const int fl = (threadIdx.x + 256 * k) % kBinFt;
      const int p = pos[k] + step;
      const XT* ed = kLds ? s_edges + fl * ES : edges + (int64_t)(f0 + fl) * estride;
      if (p <= nb[k] && ed[p - 1] < v[k]) pos[k] = p;
    }
  }
#pragma unroll
  for (int k = 0; k < kBinPer; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int r = e / kBinFt, fl = e % kBinFt;
    if (!ok[k]) continue;
    const XT* ed = kLds ? s_edges + fl * ES : edges + (int64_t)(f0 + fl) * estride;
    const int code = pos[k] < nb[k] ? pos[k] : nb[k] - 1;
    int fg = 0;
    if (s_ex[fl] && !(ed[code] == v[k])) fg |= 1;
    if (!isfinite(v[k])) fg |= 2;
    if (fg) atomicOr(&s_flag[fl], fg);
    tile[r * kBinFt + fl] = (CodeT)code;
  }
  __syncthreads();
  // row-major: this tile's codes of every row (+ zero padding after the last feature)
  const int pad_end = (f0 + nf == F) ? row_elems : f0 + nf;
  const int wcols = pad_end - f0;
  for (int e = threadIdx.x; e < rows * wcols; e += 256) {
    const int r = e / wcols;
    const int c = e - r * wcols;
    codes_rm[(r0 + r) * row_elems + f0 + c] = c < nf ? tile[r * kBinFt + c] : (CodeT)0;
  }
  // feature-major: kBinRows contiguous codes per feature
  for (int e = threadIdx.x; e < nf * rows; e += 256) {
    const int fl = e / rows;
    const int r = e - fl * rows;
    codes_fm[(int64_t)(f0 + fl) * n + r0 + r] = tile[r * kBinFt + fl];
  }
  if (threadIdx.x < nf && s_flag[threadIdx.x]) atomicOr(&flags[f0 + threadIdx.x], s_flag[threadIdx.x]);
}

// Row-streaming bin kernel for the common case (fp32 X, <= 256 bins, F % 4 == 0):
// each workgroup keeps the edges of up to 64 features resident in LDS and
// streams a contiguous row range in batches of kBrU x (512 / (nf / 4)) rows.
// A thread owns one float4 (4 consecutive features) of a row per pass, so X
// is read as whole 16-byte-aligned row segments, the row-major codes leave as
// one 4-byte store per thread, and the feature-major codes are transposed
// through a small LDS tile and written as 16-byte runs. The next batch's
// loads are issued before the current batch is searched (register double
// buffering) to keep enough bytes in flight per CU for HBM3E.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kBrThreads = 512;
constexpr int kBrFt = 64;  // features per tile (LDS: 64 x 257 x 4 B of edges)
constexpr int kBrU = 4;    // passes per batch

__global__ __launch_bounds__(kBrThreads) void bin_rows_kernel(
    const float* __restrict__ X, int64_t n, int F, const float* __restrict__ edges, int Bmax,
    int estride, int steps0, const int32_t* __restrict__ nbins, const uint8_t* __restrict__ exact,
    uint8_t* __restrict__ codes_rm, int row_elems, uint8_t* __restrict__ codes_fm,
    int32_t* __restrict__ flags, int64_t rows_per_block, int fm_vec, int skip_inexact) {
  extern __shared__ __align__(16) uint8_t smem[];
  if (skip_inexact && bin_any_inexact(exact, F)) {
    const int64_t a = blockIdx.x * rows_per_block;
    bin_finite_only<float>(X, F, a, min<int64_t>(n, a + rows_per_block), blockIdx.y * kBrFt,
                           min(kBrFt, F - (int)blockIdx.y * kBrFt), flags);
    return;
  }
  __shared__ int s_flag[kBrFt];
  __shared__ int s_aff[kBrFt];  // edges are e0, e0 + 1, ..., e0 + nb - 1 (integers)
  const int ES = Bmax | 1;
  const int f0 = blockIdx.y * kBrFt;
  const int nf = min(kBrFt, F - f0);  // multiple of 4
  const int tpr = nf >> 2;            // threads per row
  const int rp = kBrThreads / tpr;    // rows per pass
  const int batch = kBrU * rp;
  float* s_edges = reinterpret_cast<float*>(smem);
  uint8_t* tile = smem + (((size_t)nf * ES * 4 + 15) & ~(size_t)15);  // [batch][nf]
  const int tid = threadIdx.x;
  if (tid < kBrFt) {
    s_flag[tid] = 0;
    s_aff[tid] = 1;
  }
  for (int e = tid; e < nf * Bmax; e += kBrThreads) {
    const int fl = e / Bmax, b = e - fl * Bmax;
    s_edges[fl * ES + b] = edges[(int64_t)(f0 + fl) * estride + b];
  }
  __syncthreads();
  // Consecutive-integer edges (integer-coded / quantized / categorical columns
  // with every value present): the code is v - e0, one subtraction instead of
  // an 8-step search through LDS. Exact in fp32 while |e0| + nb < 2^24.
  for (int e = tid; e < nf * Bmax; e += kBrThreads) {
    const int fl = e / Bmax, b = e - fl * Bmax;
    if (b < nbins[f0 + fl]) {
      const float e0 = s_edges[fl * ES];
      const float eb = s_edges[fl * ES + b];
      if (!(eb == e0 + (float)b) || !(fabsf(e0) < 8388608.0f) || e0 != rintf(e0)) s_aff[fl] = 0;
    }
  }
  const int rs = tid / tpr;  // row slot within a pass
  const int q = tid - rs * tpr;
  const bool active = rs < rp;
  int nb[4], ex[4], fg[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = f0 + 4 * q + j;
    nb[j] = active ? nbins[f] : 1;
    ex[j] = active ? exact[f] : 0;
    fg[j] = 0;
  }
  __syncthreads();
  bool aff[4];
  float e0[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    aff[j] = active && s_aff[4 * q + j] != 0;
    e0[j] = s_edges[(4 * q + j) * ES];
  }
  const int64_t rbeg = blockIdx.x * rows_per_block;
  const int64_t rend = min<int64_t>(n, rbeg + rows_per_block);
  fm_vec = fm_vec && ((rbeg | batch) & 15) == 0;
  auto load = [&](int64_t b0, float4* v) {
#pragma unroll
    for (int u = 0; u < kBrU; ++u) {
      const int64_t r = b0 + u * rp + rs;
      if (active && r < rend) {
        const f32x4 t = __builtin_nontemporal_load(
            reinterpret_cast<const f32x4*>(X + r * F + f0 + 4 * q));
        v[u] = make_float4(t[0], t[1], t[2], t[3]);
      } else {
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  float4 cur[kBrU], nxt[kBrU];
  if (rbeg < rend) load(rbeg, cur);
  for (int64_t b0 = rbeg; b0 < rend; b0 += batch) {
    if (b0 + batch < rend) load(b0 + batch, nxt);
    float v[kBrU * 4];
    int pos[kBrU * 4];
#pragma unroll
    for (int u = 0; u < kBrU; ++u) {
      v[4 * u + 0] = cur[u].x;
      v[4 * u + 1] = cur[u].y;
      v[4 * u + 2] = cur[u].z;
      v[4 * u + 3] = cur[u].w;
    }
    bool hit[kBrU * 4];
    bool need = false;
#pragma unroll
    for (int k = 0; k < kBrU * 4; ++k) {
      const int j = k & 3;
      const float d = v[k] - e0[j];
      const int c = (int)d;  // v_cvt_i32_f32 saturates; NaN -> 0 (the checks reject both)
      hit[k] = aff[j] && d == (float)c && c >= 0 && c < nb[j];
      pos[k] = hit[k] ? c : 0;
      need |= active && !hit[k];
    }
    if (__ballot(need)) {  // some value is not an integer edge: lower_bound search
      for (int step = steps0; step > 0; step >>= 1) {
#pragma unroll
        for (int k = 0; k < kBrU * 4; ++k) {
          const int j = k & 3;
          const int p = pos[k] + step;
          if (!hit[k] && p <= nb[j] && s_edges[(4 * q + j) * ES + p - 1] < v[k]) pos[k] = p;
        }
      }
    }
    const int rows = (int)min<int64_t>(batch, rend - b0);
#pragma unroll
    for (int u = 0; u < kBrU; ++u) {
      const int rl = u * rp + rs;
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 4 * u + j;
        const int code = pos[k] < nb[j] ? pos[k] : nb[j] - 1;
        if (ex[j] && !hit[k] && !(s_edges[(4 * q + j) * ES + code] == v[k])) fg[j] |= 1;
        if (!isfinite(v[k])) fg[j] |= 2;
        word |= (uint32_t)code << (8 * j);
      }
      if (active && rl < rows) {
        *reinterpret_cast<uint32_t*>(codes_rm + (b0 + rl) * row_elems + f0 + 4 * q) = word;
        *reinterpret_cast<uint32_t*>(tile + rl * nf + 4 * q) = word;
      }
    }
    __syncthreads();
    // feature-major: each feature's `rows` codes are contiguous at codes_fm[f * n + b0]
    const int chunks = (rows + 15) >> 4;
    for (int e = tid; e < nf * chunks; e += kBrThreads) {
      const int fl = e % nf, c = e / nf;
      uint8_t* dst = codes_fm + (int64_t)(f0 + fl) * n + b0 + 16 * c;
      const int m = min(16, rows - 16 * c);
      if (fm_vec && m == 16) {
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          w[i] = (uint32_t)tile[(16 * c + 4 * i) * nf + fl] |
                 ((uint32_t)tile[(16 * c + 4 * i + 1) * nf + fl] << 8) |
                 ((uint32_t)tile[(16 * c + 4 * i + 2) * nf + fl] << 16) |
                 ((uint32_t)tile[(16 * c + 4 * i + 3) * nf + fl] << 24);
        *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
      } else {
        for (int i = 0; i < m; ++i) dst[i] = tile[(16 * c + i) * nf + fl];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kBrU; ++u) cur[u] = nxt[u];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (active && fg[j]) atomicOr(&s_flag[4 * q + j], fg[j]);
  __syncthreads();
  if (tid < nf && s_flag[tid]) atomicOr(&flags[f0 + tid], s_flag[tid]);
}

int edges_sample_rows(bool x64) { return x64 ? 16384 : 32768; }

// The host's view of the edges in one fp64 array: [F][limit] edges, then the
// F bin counts, then the F exact flags -- a single D2H instead of a gather.
template <typename XT>
__global__ __launch_bounds__(256) void edges_pack_kernel(const XT* __restrict__ edges,
                                                         const int32_t* __restrict__ nbins,
                                                         const uint8_t* __restrict__ exact, int F,
                                                         int limit, double* __restrict__ pack) {
  const int64_t E = (int64_t)F * limit;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < E + 2 * F; i += (int64_t)gridDim.x * 256) {
    double v;
    if (i < E)
      v = (double)edges[i];
    else if (i < E + F)
      v = (double)nbins[i - E];
    else
      v = (double)exact[i - E - F];
    pack[i] = v;
  }
}

void launch_edges(hipStream_t stream, const void* X, bool x64, int64_t n, int F, int s, int limit,
                  void* edges, int32_t* nbins, uint8_t* exact, double* pack, int probe) {
  if (probe && limit > kEdgeHash / 2) throw std::runtime_error("edges probe needs limit <= 1024");
  if (F <= 0) return;
  int S = 1;
  while (S < s) S <<= 1;
  const int xb = x64 ? 8 : 4;
  const size_t lds = (size_t)S * xb + (size_t)kEdgeHash * xb;
  if (s > edges_sample_rows(x64)) throw std::runtime_error("edges sample exceeds LDS");
  // the transposed sample (a device scratch per GPU, grown on demand; up to 256 MB --
  // wider inputs keep the per-value gathers)
  void* smp = nullptr;
  const size_t smp_bytes = (size_t)s * F * xb;
  if (smp_bytes <= ((size_t)256 << 20)) {
    static void* bufs[64] = {};
    static size_t caps[64] = {};
    int dev = 0;
    MT_HIP_CHECK(hipGetDevice(&dev));
    if (dev < 64) {
      if (caps[dev] < smp_bytes) {
        if (bufs[dev]) MT_HIP_CHECK(hipFree(bufs[dev]));
        MT_HIP_CHECK(hipMalloc(&bufs[dev], smp_bytes));
        caps[dev] = smp_bytes;
      }
      smp = bufs[dev];
    }
  }
#define MT_EDGES(XT)                                                                           \
  MT_HIP_CHECK(mt_set_max_lds((const void*)edges_kernel<XT>,                              \
                                   (int)lds));     \
  if (smp)                                                                                     \
    hipLaunchKernelGGL(edges_sample_kernel<XT>, dim3((unsigned)((s + 63) / 64),               \
                       (unsigned)((F + 63) / 64)), dim3(256), 0, stream, (const XT*)X, n, F, s, \
                       (XT*)smp);                                                              \
  hipLaunchKernelGGL(edges_kernel<XT>, dim3(F), dim3(kEdgeThreads), lds, stream, (const XT*)X, \
                     n, F, s, S, limit, (XT*)edges, nbins, exact, probe, (const XT*)smp);      \
  if (pack) {                                                                                  \
    const int64_t tot = (int64_t)F * limit + 2 * F;                                            \
    const int g = (int)std::min<int64_t>((tot + 255) / 256, 1024);                             \
    hipLaunchKernelGGL(edges_pack_kernel<XT>, dim3(g), dim3(256), 0, stream, (const XT*)edges, \
                       nbins, exact, F, limit, pack);                                          \
  }
  if (x64) {
    MT_EDGES(double)
  } else {
    MT_EDGES(float)
  }
#undef MT_EDGES
  MT_HIP_CHECK(hipGetLastError());
}

void launch_bin(hipStream_t stream, const void* X, bool x64, int64_t n, int F, const void* edges,
                int Bmax, int estride, const int32_t* nbins, const uint8_t* exact, void* codes_rm,
                int row_elems, void* codes_fm, int code_bytes, int32_t* flags, int skip_inexact) {
  if (n <= 0) return;
  const int xb = x64 ? 8 : 4;
  const size_t edge_bytes = (size_t)kBinFt * (Bmax | 1) * xb;
  const bool lds_edges = edge_bytes <= 64 * 1024;
  const size_t lds = (lds_edges ? edge_bytes : 0) + (size_t)kBinRows * kBinFt * code_bytes;
  int steps0 = 1;
  while (steps0 * 2 <= Bmax) steps0 *= 2;
  if (!x64 && code_bytes == 1 && Bmax <= 256 && (F & 3) == 0 && (row_elems & 3) == 0 &&
      ((uintptr_t)X & 15) == 0 && ((uintptr_t)codes_rm & 3) == 0) {
    const int tiles = (F + kBrFt - 1) / kBrFt;
    const int nf = std::min(kBrFt, F);
    const int batch = kBrU * (kBrThreads / (nf / 4));
    const int64_t nbatch = (n + batch - 1) / batch;
    const int64_t want = std::max<int64_t>(1, 2 * 256 / tiles);  // ~2 workgroups per CU
    const int64_t per = (nbatch + want - 1) / want;
    const int64_t rpb = per * batch;
    const unsigned gx = (unsigned)((n + rpb - 1) / rpb);
    const size_t lds2 = (((size_t)nf * (Bmax | 1) * 4 + 15) & ~(size_t)15) + (size_t)batch * nf;
    const int fm_vec = ((n & 15) == 0 && ((uintptr_t)codes_fm & 15) == 0) ? 1 : 0;
    MT_HIP_CHECK(mt_set_max_lds((const void*)bin_rows_kernel, (int)lds2));
    hipLaunchKernelGGL(bin_rows_kernel, dim3(gx, (unsigned)tiles), dim3(kBrThreads), lds2, stream,
                       (const float*)X, n, F, (const float*)edges, Bmax, estride, steps0, nbins,
                       exact, (uint8_t*)codes_rm, row_elems, (uint8_t*)codes_fm, flags, rpb,
                       fm_vec, skip_inexact);
    MT_HIP_CHECK(hipGetLastError());
    return;
  }
  dim3 grid((unsigned)((n + kBinRows - 1) / kBinRows), (unsigned)((F + kBinFt - 1) / kBinFt));
#define MT_BIN(XT, CT, L)                                                                      \
  {                                                                                            \
    MT_HIP_CHECK(mt_set_max_lds((const void*)bin_kernel<XT, CT, L>,                       \
                                     (int)lds));   \
    hipLaunchKernelGGL((bin_kernel<XT, CT, L>), grid, dim3(256), lds, stream, (const XT*)X, n, \
                       F, (const XT*)edges, Bmax, estride, steps0, nbins, exact, (CT*)codes_rm, \
                       row_elems, (CT*)codes_fm, flags, skip_inexact);                         \
  }
#define MT_BIN2(XT, CT)      \
  if (lds_edges) {           \
    MT_BIN(XT, CT, true)     \
  } else {                   \
    MT_BIN(XT, CT, false)    \
  }
  if (x64) {
    if (code_bytes == 1) {
      MT_BIN2(double, uint8_t)
    } else {
      MT_BIN2(double, uint16_t)
    }
  } else {
    if (code_bytes == 1) {
      MT_BIN2(float, uint8_t)
    } else {
      MT_BIN2(float, uint16_t)
    }
  }
#undef MT_BIN2
#undef MT_BIN
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
