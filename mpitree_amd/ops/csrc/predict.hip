// Batched inference on gfx950 (binning lives in binning.hip).
//
// predict: replaces the reference's per-row recursive Python ``walk`` driven
// by ``np.apply_along_axis`` (mpitree/tree/decision_tree.py:208-227) with one
// thread per row walking the flat pre-order tree arrays (root-to-leaf loads of
// 16-B node records stay in L1/L2; the raw feature value is compared in fp64,
// so ``x <= threshold`` is decided exactly as on the host).

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

}  // namespace mt
