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

// grid = (row tiles of kBinRows, feature tiles of ft). The feature tile's
// edges are staged in LDS when they fit (else read through L1/L2), every
// element does a fixed-trip branch-free lower_bound, codes are staged in LDS
// and written row-major (the tile's bytes of each row) and feature-major
// (kBinRows contiguous bytes per feature).
constexpr int kBinRows = 256;

template <typename XT, typename CodeT>
__global__ __launch_bounds__(256) void bin_kernel(const XT* __restrict__ X, int64_t n, int F,
                                                  const XT* __restrict__ edges, int Bmax,
                                                  int steps0, const int32_t* __restrict__ nbins,
                                                  const uint8_t* __restrict__ exact,
                                                  CodeT* __restrict__ codes_rm, int row_elems,
                                                  CodeT* __restrict__ codes_fm,
                                                  int32_t* __restrict__ bad, int ft,
                                                  int edges_in_lds) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ int s_bad[64];
  XT* s_edges = reinterpret_cast<XT*>(smem);  // [ft][Bmax] when staged
  CodeT* tile = reinterpret_cast<CodeT*>(smem + (edges_in_lds ? (size_t)ft * Bmax * sizeof(XT)
                                                              : 0));  // [kBinRows][ft]
  const int64_t r0 = blockIdx.x * (int64_t)kBinRows;
  const int rows = (int)min<int64_t>(kBinRows, n - r0);
  const int f0 = blockIdx.y * ft;
  const int nf = min(ft, F - f0);
  if (threadIdx.x < 64) s_bad[threadIdx.x] = 0;
  if (edges_in_lds) {
    for (int e = threadIdx.x; e < nf * Bmax; e += blockDim.x)
      s_edges[e] = edges[(int64_t)f0 * Bmax + e];
  }
  __syncthreads();
  const int elems = rows * nf;
  for (int e = threadIdx.x; e < elems; e += blockDim.x) {
    const int r = e / nf;
    const int fl = e - r * nf;
    const int f = f0 + fl;
    const XT v = X[(r0 + r) * F + f];
    const XT* ed = edges_in_lds ? s_edges + fl * Bmax : edges + (int64_t)f * Bmax;
    const int nb = nbins[f];
    int pos = 0;  // number of edges < v  (lower_bound)
    for (int step = steps0; step > 0; step >>= 1) {
      const int p = pos + step;
      if (p <= nb && ed[p - 1] < v) pos = p;
    }
    const int code = pos < nb ? pos : nb - 1;
    if (exact[f] && !(ed[code] == v)) s_bad[fl & 63] = 1;
    tile[r * ft + fl] = (CodeT)code;
  }
  __syncthreads();
  // row-major: this tile's bytes of every row (+ zero padding after the last feature)
  const int pad_end = (f0 + nf == F) ? row_elems : f0 + nf;
  const int wcols = pad_end - f0;
  for (int e = threadIdx.x; e < rows * wcols; e += blockDim.x) {
    const int r = e / wcols;
    const int c = e - r * wcols;
    codes_rm[(r0 + r) * row_elems + f0 + c] = c < nf ? tile[r * ft + c] : (CodeT)0;
  }
  // feature-major
  for (int e = threadIdx.x; e < nf * rows; e += blockDim.x) {
    const int fl = e / rows;
    const int r = e - fl * rows;
    codes_fm[(int64_t)(f0 + fl) * n + r0 + r] = tile[r * ft + fl];
  }
  if (threadIdx.x < nf && threadIdx.x < 64 && s_bad[threadIdx.x])
    atomicOr(&bad[f0 + threadIdx.x], 1);
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
  const int xb = x64 ? 8 : 4;
  const int ft = std::min(F, 16);
  const size_t edge_bytes = (size_t)ft * Bmax * xb;
  const int edges_in_lds = edge_bytes <= 48 * 1024 ? 1 : 0;
  const size_t lds = (edges_in_lds ? edge_bytes : 0) + (size_t)kBinRows * ft * code_bytes;
  int steps0 = 1;
  while (steps0 * 2 <= Bmax) steps0 *= 2;
  dim3 grid((unsigned)((n + kBinRows - 1) / kBinRows), (unsigned)((F + ft - 1) / ft));
#define MT_BIN(XT, CT)                                                                         \
  {                                                                                            \
    MT_HIP_CHECK(hipFuncSetAttribute((const void*)bin_kernel<XT, CT>,                          \
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));   \
    hipLaunchKernelGGL((bin_kernel<XT, CT>), grid, dim3(256), lds, stream, (const XT*)X, n, F, \
                       (const XT*)edges, Bmax, steps0, nbins, exact, (CT*)codes_rm, row_elems, \
                       (CT*)codes_fm, bad, ft, edges_in_lds);                                  \
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
