// Device tree assembly: pre-order position space -> compact tree arrays.
//
// The reference builds a linked Node graph while it recurses
// (mpitree/tree/decision_tree.py:93-166) and its parallel fit pickles and
// allgathers whole subtrees (:446-477). Here a fit writes every node at its
// *pre-order position with holes*: a subtree of r rows owns 2r - 1 positions,
// the root first, then the left subtree (2 n_left - 1 positions), then the right.
// The level-wise host loop and both finisher kernels only ever need a node's
// own position and its children's row counts, so the whole tree is laid out
// without a global counter. This file removes the holes:
//
//   count_kernel   per 4096-position tile: number of written nodes (n > 0)
//   offsets_kernel one workgroup: exclusive scan of the tile counts
//   rank_kernel    per tile: each written position's final node id
//   emit_kernel    per written position: the final row of every output column,
//                  child links through the rank table, split thresholds from
//                  the padded bin-edge table, node sizes, impurities / leaf
//                  values with the same integer-form criterion as every other
//                  builder
//
// so the host receives the finished, pre-ordered tree in one pinned copy.
#include "common.h"

#include <stdexcept>
#include "criterion.h"

namespace mt {

constexpr int kAsmThreads = 256;
constexpr int kAsmPer = 16;                        // positions per thread
constexpr int kAsmTile = kAsmThreads * kAsmPer;    // positions per tile

// rec: int32 [P][6] = {feature (-1 leaf), bin, left pos, right pos, depth, n}; n == 0
// marks a position no node was written to.
// mask (optional): only positions with mask[p] != 0 count (a rank's own ranges).
__device__ __forceinline__ bool asm_live(const int32_t* __restrict__ rec,
                                         const uint8_t* __restrict__ mask, int64_t p, int64_t P) {
  return p < P && rec[p * 6 + 5] > 0 && (mask == nullptr || mask[p] != 0);
}

// {depth, n} of the thread's kAsmPer positions of a tile (and the mask bytes),
// every load issued before the first use: unconditional, clamped to P - 1 (the
// short-circuit form above compiled to one load and wait per position)
__device__ __forceinline__ void asm_load_tile(const int32_t* __restrict__ rec,
                                              const uint8_t* __restrict__ mask, int64_t base,
                                              int64_t P, bool (&live)[kAsmPer],
                                              int (&depth)[kAsmPer]) {
  int2 dn[kAsmPer];
  uint8_t mk[kAsmPer];
#pragma unroll
  for (int k = 0; k < kAsmPer; ++k) {
    const int64_t p = base + (int64_t)k * kAsmThreads + threadIdx.x;
    const int64_t pc = p < P ? p : P - 1;
    dn[k] = *reinterpret_cast<const int2*>(rec + pc * 6 + 4);
    mk[k] = 1;
  }
  if (mask != nullptr) {
#pragma unroll
    for (int k = 0; k < kAsmPer; ++k) {
      const int64_t p = base + (int64_t)k * kAsmThreads + threadIdx.x;
      mk[k] = mask[p < P ? p : P - 1];
    }
  }
#pragma unroll
  for (int k = 0; k < kAsmPer; ++k) {
    const int64_t p = base + (int64_t)k * kAsmThreads + threadIdx.x;
    live[k] = p < P && dn[k].y > 0 && mk[k] != 0;
    depth[k] = dn[k].x;
  }
}

__global__ __launch_bounds__(kAsmThreads) void asm_count_kernel(const int32_t* __restrict__ rec,
                                                                int64_t P,
                                                                int32_t* __restrict__ tile_cnt,
                                                                const uint8_t* __restrict__ mask) {
  const int64_t base = (int64_t)blockIdx.x * kAsmTile;
  int c = 0;
  bool live[kAsmPer];
  int depth[kAsmPer];
  asm_load_tile(rec, mask, base, P, live, depth);  // (coalesced positions)
#pragma unroll
  for (int k = 0; k < kAsmPer; ++k) c += live[k] ? 1 : 0;
  c = (int)wave_sum_u32((uint32_t)c);
  __shared__ int w[kAsmThreads / kWave];
  if (lane_id() == 0) w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int i = 0; i < kAsmThreads / kWave; ++i) t += w[i];
    tile_cnt[blockIdx.x] = t;
  }
}

// Exclusive scan of tile counts in place (one workgroup; tiles = P / 4096, a few
// thousand at most); total written to *total.
__global__ __launch_bounds__(kAsmThreads) void asm_offsets_kernel(int32_t* __restrict__ tile,
                                                                  int n_tiles,
                                                                  int64_t* __restrict__ total) {
  __shared__ int s_carry;
  __shared__ int w[kAsmThreads / kWave];
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int b = 0; b < n_tiles; b += kAsmThreads) {
    const int i = b + threadIdx.x;
    const int v = i < n_tiles ? tile[i] : 0;
    const int incl = (int)wave_incl_scan_u32((uint32_t)v);
    if (lane_id() == kWave - 1) w[threadIdx.x >> 6] = incl;
    __syncthreads();
    int off = s_carry;
    for (int k = 0; k < (int)(threadIdx.x >> 6); ++k) off += w[k];
    if (i < n_tiles) tile[i] = off + incl - v;
    __syncthreads();
    if (threadIdx.x == kAsmThreads - 1) s_carry = off + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    total[0] = s_carry;
    total[1] = 0;  // max depth: asm_rank_kernel reduces into it
  }
}

// Final node id of every written position (a position no node occupies gets
// ~(written positions before it), negative: the shared-host assembly ranks
// other ranks' segment roots with it), and the tree's depth (max over written positions) into total[1]. Position
// p = tile + k * kAsmThreads + thread (coalesced, the count kernel's order);
// the in-tile rank comes from per-(k, wave) ballot masks kept in LDS, and
// each workgroup adds one atomic for the depth.
__global__ __launch_bounds__(kAsmThreads) void asm_rank_kernel(const int32_t* __restrict__ rec,
                                                               int64_t P,
                                                               const int32_t* __restrict__ tile_off,
                                                               int32_t* __restrict__ rank,
                                                               int64_t* __restrict__ total,
                                                               const uint8_t* __restrict__ mask) {
  constexpr int kW = kAsmThreads / kWave;
  __shared__ unsigned long long s_mask[kAsmPer][kW];
  __shared__ int s_ktot[kAsmPer];
  __shared__ int s_dmax[kW];
  const int64_t base = (int64_t)blockIdx.x * kAsmTile;
  const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
  uint32_t flags = 0;
  int dmax = 0;
  bool live[kAsmPer];
  int depth[kAsmPer];
  asm_load_tile(rec, mask, base, P, live, depth);
#pragma unroll
  for (int k = 0; k < kAsmPer; ++k) {
    const bool v = live[k];
    flags |= (uint32_t)v << k;
    if (v) dmax = max(dmax, depth[k]);
    const unsigned long long b = __ballot(v);
    if (lane == 0) s_mask[k][wv] = b;
  }
  for (int d = kWave / 2; d > 0; d >>= 1) dmax = max(dmax, __shfl_xor(dmax, d, kWave));
  if (lane == 0) s_dmax[wv] = dmax;
  __syncthreads();
  if (threadIdx.x < kAsmPer) {
    int t = 0;
    for (int w = 0; w < kW; ++w) t += __popcll(s_mask[threadIdx.x][w]);
    s_ktot[threadIdx.x] = t;
  }
  if (threadIdx.x == 0) {
    int m = 0;
    for (int w = 0; w < kW; ++w) m = max(m, s_dmax[w]);
    if (m > 0) atomicMax(reinterpret_cast<unsigned long long*>(total) + 1, (unsigned long long)m);
  }
  __syncthreads();
  const unsigned long long below = (1ull << lane) - 1ull;
  int off = tile_off[blockIdx.x];
  for (int k = 0; k < kAsmPer; ++k) {
    const int64_t p = base + (int64_t)k * kAsmThreads + threadIdx.x;
    if (p < P) {
      int r = off + __popcll(s_mask[k][wv] & below);
      for (int w = 0; w < wv; ++w) r += __popcll(s_mask[k][w]);
      rank[p] = ((flags >> k) & 1u) ? r : ~r;  // (unwritten: ~ its exclusive rank)
    }
    off += s_ktot[k];
  }
}

// Output columns, packed back to back for one D2H; the node count N is read
// from the device (asm_offsets_kernel's total), so the emit launch needs no
// host round trip. Every column of the finished tree is emitted in its final
// dtype -- the host receives numpy views, nothing is derived after the copy:
//   n_samples i64 [N] | threshold f64 [N]
//   | impurity f64 [N] + counts i32 [N][C] (classification: rows < 2^31, half the
//     bytes of the one D2H at many classes) or leaf value f64 [N] (regression:
//     impurity is NaN for every node, the host makes it a broadcast view)
//   | feature i32 [N] | threshold_bin i32 [N] | left i32 [N] | right i32 [N]
// (thresholds: edges[feature][bin], or per position from thr_pos -- the exact
// engine's split values)
//   | depth i32 [N]
// Impurities use the integer-form criterion of every builder (criterion.h:
// (T(m) - sum_c T(c)) / m, gini (m^2 - sum c^2) / m / m), regression leaf values
// ldexp(S / m, -y_exp): the same IEEE op sequence as the host builders, so the
// columns equal theirs bit for bit. Bins are a column of their own (exact-engine
// value ranks exceed 16 bits).
struct AsmCols {
  int64_t* nsamp;
  double* threshold;
  double* impurity;
  int32_t* count;  // classification
  double* value;   // regression
  int64_t* sum;    // regression
  int32_t* feature;
  int32_t* bin;
  int32_t* left;
  int32_t* right;
  int32_t* depth;
};

__host__ __device__ inline int64_t asm_bytes(int64_t N, int C, bool reg) {
  return N * (reg ? 8 + 8 + 8 + 20 : 24 + 4 * (int64_t)C + 20);
}

__device__ inline AsmCols asm_cols(uint8_t* base, int64_t N, int C, bool reg) {
  AsmCols o;
  uint8_t* p = base;
  o.nsamp = reinterpret_cast<int64_t*>(p);
  p += N * 8;
  o.threshold = reinterpret_cast<double*>(p);
  p += N * 8;
  o.impurity = nullptr;
  o.count = nullptr;
  o.value = nullptr;
  o.sum = nullptr;
  if (reg) {  // (no impurity column: NaN for every regression node, made on the host
              //  as a broadcast view; no fixed-point sum: the value is final)
    o.value = reinterpret_cast<double*>(p);
    p += N * 8;
  } else {
    o.impurity = reinterpret_cast<double*>(p);
    p += N * 8;
    o.count = reinterpret_cast<int32_t*>(p);
    p += N * 4 * (int64_t)C;
  }
  o.feature = reinterpret_cast<int32_t*>(p);
  o.bin = o.feature + N;
  o.left = o.bin + N;
  o.right = o.left + N;
  o.depth = o.right + N;
  return o;
}

// ---------------------------------------------------------------------------
// Node-local shared-host assembly (several ranks of one node, subtree ownership;
// parallel/shared_tree.py). Rank r's position space holds the replicated prefix
// (the levels before the ownership switch) and its own segments; other ranks'
// segments are empty. With every segment's node count (one small all-gather) a
// rank knows the final id of each of its nodes: its local rank plus the nodes of
// other ranks' segments that start before it. Each rank then writes its own nodes
// (rank 0 also the prefix) straight into the node's shared host buffer (a
// registered /dev/shm mapping, zero-copy over PCIe), so no rank receives the
// other ranks' nodes over xGMI and each moves 1 / P of the tree over PCIe.
//
// tab: int64 [n][4] {lo, hi, owner, foreign nodes in segments up to and including
// this one}, ascending lo (shm_seg_prefix_kernel).
struct ShmPlace {
  bool own;
  int64_t e, lo, hi;
};

// entry index of the last segment with lo <= x (strict: lo < x), -1 if none
__device__ inline int shm_find(const int64_t* __restrict__ tab, int n, int64_t x, bool strict) {
  int lo = 0, hi = n;  // first entry with lo > x (strict: >= x)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const int64_t v = tab[(int64_t)mid * 4];
    if (strict ? v < x : v <= x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo - 1;
}

__device__ inline int64_t shm_foreign_before(const int64_t* __restrict__ tab, int n, int64_t x) {
  const int k = shm_find(tab, n, x, true);
  return k >= 0 ? tab[(int64_t)k * 4 + 3] : 0;
}

// {lo_k, hi_k, owner_k, foreign before lo_k (exclusive), foreign through k, lo_{k+1}}
// of the last segment k with lo <= p0 (k = -1: {-1, -1, -1, 0, 0, lo_0})
__device__ inline void shm_block_ctx(const int64_t* __restrict__ tab, int n, int64_t p0,
                                     int64_t* ctx) {
  const int k = shm_find(tab, n, p0, false);
  if (k >= 0) {
    ctx[0] = tab[(int64_t)k * 4 + 0];
    ctx[1] = tab[(int64_t)k * 4 + 1];
    ctx[2] = tab[(int64_t)k * 4 + 2];
    ctx[3] = k > 0 ? tab[(int64_t)(k - 1) * 4 + 3] : 0;
    ctx[4] = tab[(int64_t)k * 4 + 3];
  } else {
    ctx[0] = ctx[1] = ctx[2] = -1;
    ctx[3] = ctx[4] = 0;
  }
  ctx[5] = k + 1 < n ? tab[(int64_t)(k + 1) * 4] : INT64_MAX;
}

// where a live position p lies: inside a segment (its own, since it is written
// here) or in the replicated prefix; e = foreign nodes ranked before p
__device__ inline ShmPlace shm_place(const int64_t* __restrict__ tab, int n,
                                     const int64_t* ctx, int64_t p) {
  ShmPlace r;
  int64_t lo, hi, eb, ei;
  if (p >= ctx[0] && p < ctx[5]) {  // (the workgroup's segment context: no search)
    lo = ctx[0];
    hi = ctx[1];
    eb = ctx[3];
    ei = ctx[4];
  } else {
    const int k = shm_find(tab, n, p, false);
    lo = k >= 0 ? tab[(int64_t)k * 4 + 0] : -1;
    hi = k >= 0 ? tab[(int64_t)k * 4 + 1] : -1;
    eb = k > 0 ? tab[(int64_t)(k - 1) * 4 + 3] : 0;
    ei = k >= 0 ? tab[(int64_t)k * 4 + 3] : 0;
  }
  r.own = lo >= 0 && p < hi;
  r.lo = lo;
  r.hi = hi;
  // segments with lo < p: through k, except k itself when p is its first position
  r.e = (lo >= 0 && lo < p) ? ei : eb;
  return r;
}

// StatT: int32 class counts (classification) or int64 {count, fixed-point sum}.
template <typename StatT>
__global__ __launch_bounds__(kAsmThreads) void asm_emit_kernel(
    const int32_t* __restrict__ rec, const StatT* __restrict__ st, int64_t P, int C,
    const int32_t* __restrict__ rank, const double* __restrict__ edges, int EB,
    const int64_t* __restrict__ total, uint8_t* __restrict__ base, bool reg, int crit, int y_exp,
    const double* __restrict__ xtab, int xtab_n, const double* __restrict__ thr_pos,
    const int64_t* __restrict__ tab, int n_tab, int me, bool emit_prefix, int64_t cap_nodes) {
  const int64_t p = (int64_t)blockIdx.x * kAsmThreads + threadIdx.x;
  // shared-host assembly: the table segment around this workgroup's first position
  __shared__ int64_t s_ctx[6];
  if (tab != nullptr) {
    if (threadIdx.x == 0) shm_block_ctx(tab, n_tab, (int64_t)blockIdx.x * kAsmThreads, s_ctx);
    __syncthreads();
  }
  if (p >= P) return;
  const int j0 = rank[p];
  if (j0 < 0) return;
  const int64_t N = *total;
  if (cap_nodes > 0 && N > cap_nodes) return;  // (the host buffer is too small: re-emitted)
  int64_t j = j0;
  int64_t e_own = 0;  // foreign nodes ranked before p
  bool in_seg = false;
  int64_t seg_lo = 0, seg_hi = 0;
  if (tab != nullptr) {
    ShmPlace pl = shm_place(tab, n_tab, s_ctx, p);
    if (!pl.own && !emit_prefix) return;  // replicated prefix nodes: one rank writes them
    e_own = pl.e;
    in_seg = pl.own;
    seg_lo = pl.lo;
    seg_hi = pl.hi;
    j += e_own;
  }
  const AsmCols o = asm_cols(base, N, C, reg);
  const int32_t* R = rec + p * 6;
  const int f = R[0];
  const int b = R[1];
  // a child's final id: its local exclusive rank plus the foreign nodes before it
  auto child = [&](int64_t q) -> int32_t {
    const int rq = rank[q];
    const int64_t loc = rq >= 0 ? rq : ~rq;
    if (tab == nullptr) return (int32_t)loc;
    const int64_t e = (in_seg && q >= seg_lo && q < seg_hi) ? e_own : shm_foreign_before(tab, n_tab, q);
    return (int32_t)(loc + e);
  };
  if (f >= 0) {
    o.feature[j] = f;
    o.bin[j] = b;
    o.left[j] = child(R[2]);
    o.right[j] = child(R[3]);
    o.threshold[j] = thr_pos ? thr_pos[p] : edges[(int64_t)f * EB + b];
  } else {
    o.feature[j] = -1;
    o.bin[j] = -1;
    o.left[j] = -1;
    o.right[j] = -1;
    o.threshold[j] = __builtin_nan("");
  }
  o.depth[j] = R[4];
  const StatT* s = st + p * C;
  auto T = [&](int64_t x) -> double {
    return x < (int64_t)xtab_n ? xtab[x] : xlog2x((uint64_t)x);
  };
  if (reg) {
    const int64_t m = (int64_t)s[0], sf = (int64_t)s[1];
    o.nsamp[j] = m;
    o.value[j] = ldexp((double)sf / (double)(m > 1 ? m : 1), -y_exp);
  } else {
    int64_t m = 0, sq = 0;
    double acc = 0.0;
    for (int c = 0; c < C; ++c) {
      const int64_t v = (int64_t)s[c];
      o.count[(int64_t)j * C + c] = (int32_t)v;
      m += v;
      sq += v * v;
      acc = acc + T(v);
    }
    o.nsamp[j] = m;
    double imp = 0.0;
    if (m > 0) {
      const double term = crit == kEntropy ? T(m) - acc : gini_term(m, sq);
      imp = term / (double)m;
    }
    o.impurity[j] = imp;
  }
}

void launch_asm_rank(hipStream_t stream, const int32_t* rec, int64_t P, int32_t* tile,
                     int64_t* total, int32_t* rank, const uint8_t* mask) {
  const int n_tiles = (int)((P + kAsmTile - 1) / kAsmTile);
  if (n_tiles == 0) return;
  hipLaunchKernelGGL(asm_count_kernel, dim3(n_tiles), dim3(kAsmThreads), 0, stream, rec, P, tile,
                     mask);
  hipLaunchKernelGGL(asm_offsets_kernel, dim3(1), dim3(kAsmThreads), 0, stream, tile, n_tiles,
                     total);
  hipLaunchKernelGGL(asm_rank_kernel, dim3(n_tiles), dim3(kAsmThreads), 0, stream, rec, P, tile,
                     rank, total, mask);
  MT_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Node exchange of a multi-GPU subtree-ownership fit (ops/device_grower.py):
// rank r wrote exactly the positions inside its owned ranges; these kernels
// mark those ranges, pack the live positions in them as rows {pos, record[6],
// stats[C]} (final order from asm_rank with the mask) for one all-gather, and
// scatter every rank's rows back into the position space.
// ranges: int64 [cap][2] {lo, hi}, unused rows {0, 0}; mask: uint8 [P], zeroed.
__global__ __launch_bounds__(256) void own_mark_kernel(const int64_t* __restrict__ ranges,
                                                       uint8_t* __restrict__ mask) {
  const int64_t lo = ranges[blockIdx.x * 2 + 0], hi = ranges[blockIdx.x * 2 + 1];
  for (int64_t p = lo + threadIdx.x; p < hi; p += 256) mask[p] = 1;
}

template <typename StatT>
__global__ __launch_bounds__(kAsmThreads) void own_pack_kernel(
    const int32_t* __restrict__ rec, const StatT* __restrict__ st, int64_t P, int C,
    const int32_t* __restrict__ rank, StatT* __restrict__ rows, int64_t row_cap) {
  // row_cap: rows the buffer holds; the count past it (asm_rank's total) makes
  // the host raise on every rank, so rows beyond it are never written
  const int64_t p = (int64_t)blockIdx.x * kAsmThreads + threadIdx.x;
  if (p >= P) return;
  const int j = rank[p];
  if (j < 0 || j >= row_cap) return;
  StatT* o = rows + (int64_t)j * (7 + C);
  o[0] = (StatT)p;
  for (int k = 0; k < 6; ++k) o[1 + k] = (StatT)rec[p * 6 + k];
  for (int c = 0; c < C; ++c) o[7 + c] = st[p * C + c];
}

template <typename StatT>
__global__ __launch_bounds__(256) void own_scatter_kernel(const StatT* __restrict__ rows,
                                                          int64_t k, int C,
                                                          int32_t* __restrict__ rec,
                                                          StatT* __restrict__ st) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= k) return;
  const StatT* r = rows + i * (7 + C);
  const int64_t p = (int64_t)r[0];
  for (int q = 0; q < 6; ++q) rec[p * 6 + q] = (int32_t)r[1 + q];
  for (int c = 0; c < C; ++c) st[p * C + c] = r[7 + c];
}

void launch_own_pack(hipStream_t stream, const int64_t* ranges, int cap, uint8_t* mask,
                     const int32_t* rec, const void* st, bool st64, int64_t P, int C,
                     int32_t* tile, int64_t* total, int32_t* rank, void* rows,
                     int64_t row_cap) {
  if (cap > 0)
    hipLaunchKernelGGL(own_mark_kernel, dim3(cap), dim3(256), 0, stream, ranges, mask);
  launch_asm_rank(stream, rec, P, tile, total, rank, mask);
  const int64_t blocks = (P + kAsmThreads - 1) / kAsmThreads;
  if (blocks == 0) return;
  if (st64)
    hipLaunchKernelGGL(own_pack_kernel<int64_t>, dim3((unsigned)blocks), dim3(kAsmThreads), 0,
                       stream, rec, (const int64_t*)st, P, C, rank, (int64_t*)rows, row_cap);
  else
    hipLaunchKernelGGL(own_pack_kernel<int32_t>, dim3((unsigned)blocks), dim3(kAsmThreads), 0,
                       stream, rec, (const int32_t*)st, P, C, rank, (int32_t*)rows, row_cap);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_own_scatter(hipStream_t stream, const void* rows, int64_t k, int C, int32_t* rec,
                        void* st, bool st64) {
  if (k <= 0) return;
  const unsigned blocks = (unsigned)((k + 255) / 256);
  if (st64)
    hipLaunchKernelGGL(own_scatter_kernel<int64_t>, dim3(blocks), dim3(256), 0, stream,
                       (const int64_t*)rows, k, C, rec, (int64_t*)st);
  else
    hipLaunchKernelGGL(own_scatter_kernel<int32_t>, dim3(blocks), dim3(256), 0, stream,
                       (const int32_t*)rows, k, C, rec, (int32_t*)st);
  MT_HIP_CHECK(hipGetLastError());
}

// gvec (int64, this rank's all-gather row): [0] local tree depth, [1] and [2] left
// to the host (its free shared-buffer slots, the free bytes of its /dev/shm),
// [kShmHdr + s] nodes of segment s when this rank owns it (0 otherwise). A
// segment's count is the difference of the exclusive ranks at its ends
// (asm_rank_kernel: every position carries one).
constexpr int kShmHdr = 3;  // header words of a gathered row (shared_tree.GATHER_HDR)

__global__ __launch_bounds__(256) void shm_seg_count_kernel(const int64_t* __restrict__ segs, int S,
                                                            int me, const int32_t* __restrict__ rank,
                                                            int64_t P, const int64_t* __restrict__ total,
                                                            int64_t* __restrict__ gvec) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s == 0) gvec[0] = total[1];
  if (s >= S) return;
  const int64_t lo = segs[(int64_t)s * 3 + 0], hi = segs[(int64_t)s * 3 + 1];
  const int64_t owner = segs[(int64_t)s * 3 + 2];
  auto excl = [&](int64_t x) -> int64_t {
    if (x >= P) return total[0];
    const int r = rank[x];
    return r >= 0 ? r : ~r;
  };
  gvec[kShmHdr + s] = (owner == me && lo < hi) ? excl(hi) - excl(lo) : 0;
}

constexpr int kShmMaxSegs = 4096;  // 2 per ownership unit (grow.hip kOwnMax = 2048)
int shm_max_segs() { return kShmMaxSegs; }

// One workgroup: every segment's count (summed over the gathered rows: one owner
// each), the segments sorted by lo (bitonic, LDS), the running count of other
// ranks' nodes -> tab [S][4]; unused entries get lo = INT64_MAX (sorted last).
// total becomes the whole tree's {nodes, depth}.
__global__ __launch_bounds__(1024) void shm_seg_prefix_kernel(const int64_t* __restrict__ gall,
                                                              int nranks, int W,
                                                              const int64_t* __restrict__ segs,
                                                              int S, int me, int64_t* __restrict__ total,
                                                              int64_t* __restrict__ tab) {
  __shared__ uint64_t key[kShmMaxSegs];
  __shared__ int32_t idx[kShmMaxSegs];
  __shared__ int64_t wsum[1024 / kWave];
  __shared__ int64_t carry;
  const int tid = threadIdx.x;
  int N2 = 1;
  while (N2 < S) N2 <<= 1;
  for (int i = tid; i < N2; i += 1024) {
    uint64_t k = ~0ull;
    if (i < S) {
      const int64_t lo = segs[(int64_t)i * 3 + 0], hi = segs[(int64_t)i * 3 + 1];
      if (lo < hi) k = (uint64_t)lo;
    }
    key[i] = k;
    idx[i] = i;
  }
  __syncthreads();
  for (int size = 2; size <= N2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < N2; i += 1024) {
        const int j = i ^ stride;
        if (j > i) {
          const uint64_t ka = key[i], kb = key[j];
          const bool up = (i & size) == 0;
          if ((ka > kb) == up) {
            key[i] = kb;
            key[j] = ka;
            const int32_t t = idx[i];
            idx[i] = idx[j];
            idx[j] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int b0 = 0; b0 < S; b0 += 1024) {
    const int k = b0 + tid;
    int64_t v = 0, lo = INT64_MAX, hi = INT64_MAX, owner = -1;
    if (k < S && key[k] != ~0ull) {
      const int s = idx[k];
      lo = segs[(int64_t)s * 3 + 0];
      hi = segs[(int64_t)s * 3 + 1];
      owner = segs[(int64_t)s * 3 + 2];
      int64_t c = 0;
      for (int r = 0; r < nranks; ++r) c += gall[(int64_t)r * W + kShmHdr + s];
      v = owner != me ? c : 0;
    }
    // inclusive block scan of v
    int64_t x = v;
    for (int d = 1; d < kWave; d <<= 1) {
      const int64_t y = __shfl_up(x, d, kWave);
      if (lane_id() >= d) x += y;
    }
    if (lane_id() == kWave - 1) wsum[tid / kWave] = x;
    __syncthreads();
    int64_t off = carry;
    for (int w = 0; w < tid / kWave; ++w) off += wsum[w];
    if (k < S) {
      tab[(int64_t)k * 4 + 0] = lo;
      tab[(int64_t)k * 4 + 1] = hi;
      tab[(int64_t)k * 4 + 2] = owner;
      tab[(int64_t)k * 4 + 3] = off + x;
    }
    __syncthreads();
    if (tid == 1023) carry = off + x;
    __syncthreads();
  }
  if (tid == 0) {
    int64_t d = 0;
    for (int r = 0; r < nranks; ++r) d = max(d, gall[(int64_t)r * W]);
    total[0] += carry;
    total[1] = d;
  }
}

void launch_shm_seg_count(hipStream_t stream, const int64_t* segs, int S, int me,
                          const int32_t* rank, int64_t P, const int64_t* total, int64_t* gvec) {
  hipLaunchKernelGGL(shm_seg_count_kernel, dim3((unsigned)((S + 255) / 256 + (S == 0))), dim3(256),
                     0, stream, segs, S, me, rank, P, total, gvec);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_shm_seg_prefix(hipStream_t stream, const int64_t* gall, int nranks, int W,
                           const int64_t* segs, int S, int me, int64_t* total, int64_t* tab) {
  if (S > kShmMaxSegs) throw std::runtime_error("shared-host assembly: too many segments");
  hipLaunchKernelGGL(shm_seg_prefix_kernel, dim3(1), dim3(1024), 0, stream, gall, nranks, W, segs,
                     S, me, total, tab);
  MT_HIP_CHECK(hipGetLastError());
}

int asm_tiles(int64_t P) { return (int)((P + kAsmTile - 1) / kAsmTile); }

int64_t asm_node_bytes(int C, bool reg) { return asm_bytes(1, C, reg); }

void launch_asm_emit(hipStream_t stream, const int32_t* rec, const void* st, bool st64,
                     int64_t P, int C, const int32_t* rank, const double* edges, int EB,
                     const int64_t* total, uint8_t* base, bool reg, int crit, int y_exp,
                     const double* xtab, int xtab_n, const double* thr_pos, const int64_t* tab,
                     int n_tab, int me, bool emit_prefix, int64_t cap_nodes) {
  const int64_t blocks = (P + kAsmThreads - 1) / kAsmThreads;
  if (blocks == 0) return;
  if (st64)
    hipLaunchKernelGGL(asm_emit_kernel<int64_t>, dim3((unsigned)blocks), dim3(kAsmThreads), 0,
                       stream, rec, (const int64_t*)st, P, C, rank, edges, EB, total, base, reg,
                       crit, y_exp, xtab, xtab_n, thr_pos, tab, n_tab, me, emit_prefix, cap_nodes);
  else
    hipLaunchKernelGGL(asm_emit_kernel<int32_t>, dim3((unsigned)blocks), dim3(kAsmThreads), 0,
                       stream, rec, (const int32_t*)st, P, C, rank, edges, EB, total, base, reg,
                       crit, y_exp, xtab, xtab_n, thr_pos, tab, n_tab, me, emit_prefix, cap_nodes);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
