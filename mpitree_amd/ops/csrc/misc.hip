// Small utility kernels.
#include "common.h"
#include "criterion.h"

namespace mt {

__global__ void xlog2x_kernel(double* __restrict__ out, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] = xlog2x((uint64_t)i);
}

// out[i] = xlog2x(i) computed on the device (bit-exactness check vs the host).
void launch_xlog2x(hipStream_t stream, double* out, int64_t n) {
  if (n <= 0) return;
  hipLaunchKernelGGL(xlog2x_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, out,
                     n);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
