// Batched inference and feature binning on gfx950.
//
// predict: replaces the reference's per-row recursive Python ``walk`` driven
// by ``np.apply_along_axis`` (mpitree/tree/decision_tree.py:208-227) with one
// thread per row walking the flat pre-order tree arrays (root-to-leaf loads of
// 16-B node records stay in L1/L2; the raw feature value is compared in fp64,
// so ``x <= threshold`` is decided exactly as on the host).
//
// bin: replaces ``np.unique(X[:, f])`` per node (decision_tree.py:73) with a
// single up-front pass. A workgroup bins a 256-row tile: each element does a
// branch-free lower_bound over its feature's edges, codes are staged in LDS
// and written both row-major (histogram gathers) and feature-major
// (partition's single-column reads) with coalesced 1-byte-per-lane stores.
// Exact-mode features also verify that every value equals its edge, flagging
// features whose sampled edge set missed a value.
#include "common.h"

namespace mt {

struct NodeRec {
  int32_t feature;  // -1 leaf
  int32_t left;
  int32_t right;
  int32_t pad;
};

template <typename XT>
__global__ __launch_bounds__(256) void predict_kernel(const XT* __restrict__ X, int64_t n, int F,
                                                      const NodeRec* __restrict__ nodes,
                                                      const double* __restrict__ thr,
                                                      int32_t* __restrict__ leaf) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const XT* x = X + i * F;
  int32_t node = 0;
  NodeRec r = nodes[0];
  while (r.feature >= 0) {
    node = ((double)x[r.feature] <= thr[node]) ? r.left : r.right;
    r = nodes[node];
  }
  leaf[i] = node;
}

template <typename XT, typename CodeT>
__global__ __launch_bounds__(256) void bin_kernel(const XT* __restrict__ X, int64_t n, int F,
                                                  const XT* __restrict__ edges, int Bmax,
                                                  const int32_t* __restrict__ nbins,
                                                  const uint8_t* __restrict__ exact,
                                                  CodeT* __restrict__ codes_rm, int row_elems,
                                                  CodeT* __restrict__ codes_fm,
                                                  int32_t* __restrict__ bad, int tile_rows) {
  extern __shared__ uint8_t smem[];
  CodeT* tile = reinterpret_cast<CodeT*>(smem);  // [tile_rows][F] codes of this tile
  const int64_t r0 = blockIdx.x * (int64_t)tile_rows;
  const int rows = (int)min<int64_t>(tile_rows, n - r0);
  // phase 1: coalesced read of the X tile, bin, stage in LDS
  const int64_t elems = (int64_t)rows * F;
  for (int64_t e = threadIdx.x; e < elems; e += blockDim.x) {
    const int r = (int)(e / F);
    const int f = (int)(e - (int64_t)r * F);
    const XT v = X[(r0 + r) * F + f];
    const XT* ed = edges + (int64_t)f * Bmax;
    int lo = 0, cnt = nbins[f];
    while (cnt > 0) {  // lower_bound: first edge >= v
      const int half = cnt >> 1;
      if (ed[lo + half] < v) {
        lo += half + 1;
        cnt -= half + 1;
      } else {
        cnt = half;
      }
    }
    const int last = nbins[f] - 1;
    const int code = lo > last ? last : lo;
    if (exact[f] && !(ed[code] == v)) atomicOr(&bad[f], 1);
    tile[r * F + f] = (CodeT)code;
  }
  __syncthreads();
  // phase 2a: row-major codes (padded row stride)
  const int64_t rm_elems = (int64_t)rows * row_elems;
  for (int64_t e = threadIdx.x; e < rm_elems; e += blockDim.x) {
    const int r = (int)(e / row_elems);
    const int f = (int)(e - (int64_t)r * row_elems);
    codes_rm[(r0 + r) * row_elems + f] = f < F ? tile[r * F + f] : (CodeT)0;
  }
  // phase 2b: feature-major codes
  for (int64_t e = threadIdx.x; e < elems; e += blockDim.x) {
    const int f = (int)(e / rows);
    const int r = (int)(e - (int64_t)f * rows);
    codes_fm[(int64_t)f * n + r0 + r] = tile[r * F + f];
  }
}

void launch_predict(hipStream_t stream, const void* X, bool x64, int64_t n, int F,
                    const void* nodes, const double* thr, int32_t* leaf) {
  if (n <= 0) return;
  dim3 grid((unsigned)((n + 255) / 256));
  if (x64)
    hipLaunchKernelGGL(predict_kernel<double>, grid, dim3(256), 0, stream, (const double*)X, n, F,
                       (const NodeRec*)nodes, thr, leaf);
  else
    hipLaunchKernelGGL(predict_kernel<float>, grid, dim3(256), 0, stream, (const float*)X, n, F,
                       (const NodeRec*)nodes, thr, leaf);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_bin(hipStream_t stream, const void* X, bool x64, int64_t n, int F, const void* edges,
                int Bmax, const int32_t* nbins, const uint8_t* exact, void* codes_rm,
                int row_elems, void* codes_fm, int code_bytes, int32_t* bad) {
  if (n <= 0) return;
  int tile_rows = 256;
  while (tile_rows > 1 && (size_t)tile_rows * F * code_bytes > 65536) tile_rows >>= 1;
  dim3 grid((unsigned)((n + tile_rows - 1) / tile_rows));
  size_t lds = (size_t)tile_rows * F * code_bytes;
#define MT_BIN(XT, CT)                                                                         \
  {                                                                                            \
    MT_HIP_CHECK(hipFuncSetAttribute((const void*)bin_kernel<XT, CT>,                          \
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));   \
    hipLaunchKernelGGL((bin_kernel<XT, CT>), grid, dim3(256), lds, stream, (const XT*)X, n, F, \
                       (const XT*)edges, Bmax, nbins, exact, (CT*)codes_rm, row_elems,         \
                       (CT*)codes_fm, bad, tile_rows);                                         \
  }
  if (x64) {
    if (code_bytes == 1) MT_BIN(double, uint8_t) else MT_BIN(double, uint16_t)
  } else {
    if (code_bytes == 1) MT_BIN(float, uint8_t) else MT_BIN(float, uint16_t)
  }
#undef MT_BIN
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
