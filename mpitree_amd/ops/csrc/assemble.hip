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

// Final node id of every written position (positions no node occupies get -1),
// and the tree's depth (max over written positions) into total[1]. Position
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
      rank[p] = ((flags >> k) & 1u) ? r : -1;
    }
    off += s_ktot[k];
  }
}

// Output columns, packed back to back for one D2H; the node count N is read
// from the device (asm_offsets_kernel's total), so the emit launch needs no
// host round trip. Every column of the finished tree is emitted in its final
// dtype -- the host receives numpy views, nothing is derived after the copy:
//   n_samples i64 [N] | threshold f64 [N] | impurity f64 [N]
//   | counts i32 [N][C] (classification: rows < 2^31, half the bytes of the one
//     D2H at many classes) or leaf value f64 [N] + fixed-point
//     target sum i64 [N] (regression)
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
  return N * (24 + (reg ? 16 : 4 * (int64_t)C) + 20);
}

__device__ inline AsmCols asm_cols(uint8_t* base, int64_t N, int C, bool reg) {
  AsmCols o;
  uint8_t* p = base;
  o.nsamp = reinterpret_cast<int64_t*>(p);
  p += N * 8;
  o.threshold = reinterpret_cast<double*>(p);
  p += N * 8;
  o.impurity = reinterpret_cast<double*>(p);
  p += N * 8;
  o.count = nullptr;
  o.value = nullptr;
  o.sum = nullptr;
  if (reg) {
    o.value = reinterpret_cast<double*>(p);
    p += N * 8;
    o.sum = reinterpret_cast<int64_t*>(p);
    p += N * 8;
  } else {
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

// StatT: int32 class counts (classification) or int64 {count, fixed-point sum}.
template <typename StatT>
__global__ __launch_bounds__(kAsmThreads) void asm_emit_kernel(
    const int32_t* __restrict__ rec, const StatT* __restrict__ st, int64_t P, int C,
    const int32_t* __restrict__ rank, const double* __restrict__ edges, int EB,
    const int64_t* __restrict__ total, uint8_t* __restrict__ base, bool reg, int crit, int y_exp,
    const double* __restrict__ xtab, int xtab_n, const double* __restrict__ thr_pos) {
  const int64_t p = (int64_t)blockIdx.x * kAsmThreads + threadIdx.x;
  if (p >= P) return;
  const int j = rank[p];
  if (j < 0) return;
  const AsmCols o = asm_cols(base, *total, C, reg);
  const int32_t* R = rec + p * 6;
  const int f = R[0];
  const int b = R[1];
  if (f >= 0) {
    o.feature[j] = f;
    o.bin[j] = b;
    o.left[j] = rank[R[2]];
    o.right[j] = rank[R[3]];
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
    o.sum[j] = sf;
    o.value[j] = ldexp((double)sf / (double)(m > 1 ? m : 1), -y_exp);
    o.impurity[j] = __builtin_nan("");
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

int asm_tiles(int64_t P) { return (int)((P + kAsmTile - 1) / kAsmTile); }

int64_t asm_node_bytes(int C, bool reg) { return asm_bytes(1, C, reg); }

void launch_asm_emit(hipStream_t stream, const int32_t* rec, const void* st, bool st64,
                     int64_t P, int C, const int32_t* rank, const double* edges, int EB,
                     const int64_t* total, uint8_t* base, bool reg, int crit, int y_exp,
                     const double* xtab, int xtab_n, const double* thr_pos) {
  const int64_t blocks = (P + kAsmThreads - 1) / kAsmThreads;
  if (blocks == 0) return;
  if (st64)
    hipLaunchKernelGGL(asm_emit_kernel<int64_t>, dim3((unsigned)blocks), dim3(kAsmThreads), 0,
                       stream, rec, (const int64_t*)st, P, C, rank, edges, EB, total, base, reg,
                       crit, y_exp, xtab, xtab_n, thr_pos);
  else
    hipLaunchKernelGGL(asm_emit_kernel<int32_t>, dim3((unsigned)blocks), dim3(kAsmThreads), 0,
                       stream, rec, (const int32_t*)st, P, C, rank, edges, EB, total, base, reg,
                       crit, y_exp, xtab, xtab_n, thr_pos);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
