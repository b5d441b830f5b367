// Small utility kernels.
#include "common.h"
#include "criterion.h"

#include <algorithm>
#include <climits>

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

// x * log2(x) in fp32 from the hardware log2 (v_log_f32), as the exact
// engine's two-class prefilter computes its terms (exact2.hip): the error bound
// its margin assumes is checked against the fp64 table for every x < n.
__global__ void hw_xlog2x_kernel(float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const float f = (float)i;
    out[i] = i > 1 ? f * __builtin_amdgcn_logf(f) : 0.0f;
  }
}

void launch_hw_xlog2x(hipStream_t stream, float* out, int n) {
  if (n <= 0) return;
  hipLaunchKernelGGL(hw_xlog2x_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, out, n);
  MT_HIP_CHECK(hipGetLastError());
}

// ---- device-resident class labels (core/fit.py prepare path) --------------
// The reference encodes labels with np.unique on every rank
// (mpitree/tree/decision_tree.py:418-421); here an int64 label column on the
// GPU is counted over its [lo, lo + R) range and re-coded through a LUT, so
// the classes, the root class counts and the int32 codes cost one small D2H.
constexpr int kLabLds = 8192;

__global__ __launch_bounds__(256) void label_count_kernel(const int64_t* __restrict__ y,
                                                          int64_t n, int64_t lo, int R,
                                                          uint32_t* __restrict__ counts,
                                                          bool checked,
                                                          int32_t* __restrict__ enc) {
  // checked: the range is a guess made before the labels' min/max reached the
  // host -- out-of-range labels are tallied in counts[R] instead of indexed
  __shared__ uint32_t h[kLabLds];
  const bool lds = R <= kLabLds;
  if (lds)
    for (int i = threadIdx.x; i < R; i += 256) h[i] = 0;
  __syncthreads();
  uint32_t oob = 0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t d = y[i] - lo;
    if (enc) enc[i] = (int32_t)d;  // (the int32 codes when the labels are 0..C-1)
    if (checked && (d < 0 || d >= R)) {
      ++oob;
      continue;
    }
    const int v = (int)d;
    if (lds)
      atomicAdd(&h[v], 1u);
    else
      atomicAdd(&counts[v], 1u);
  }
  if (checked && oob) atomicAdd(&counts[R], oob);
  if (lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < R; i += 256)
      if (h[i]) atomicAdd(&counts[i], h[i]);
  }
}

__global__ __launch_bounds__(256) void label_encode_kernel(const int64_t* __restrict__ y,
                                                           int64_t n, int64_t lo,
                                                           const int64_t* __restrict__ lut,
                                                           int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = (int32_t)lut[y[i] - lo];
}

static unsigned label_grid(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 2048));
}

void launch_label_count(hipStream_t stream, const int64_t* y, int64_t n, int64_t lo, int R,
                        uint32_t* counts, bool checked, int32_t* enc) {
  // checked: counts has R + 1 entries, the last one counts labels outside the range
  MT_HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(uint32_t) * (size_t)(R + (checked ? 1 : 0)),
                              stream));
  if (n <= 0) return;
  // LDS-privatised histograms: fewer, fuller blocks; global atomics otherwise
  const unsigned g = R <= kLabLds ? std::min(label_grid(n), 512u) : label_grid(n);
  hipLaunchKernelGGL(label_count_kernel, dim3(g), dim3(256), 0, stream, y, n, lo, R, counts,
                     checked, enc);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_label_encode(hipStream_t stream, const int64_t* y, int64_t n, int64_t lo,
                         const int64_t* lut, int32_t* out) {
  if (n <= 0) return;
  hipLaunchKernelGGL(label_encode_kernel, dim3(label_grid(n)), dim3(256), 0, stream, y, n, lo,
                     lut, out);
  MT_HIP_CHECK(hipGetLastError());
}

// ---- device-resident regression targets (ops/gpu_prepare.py) --------------
// Fixed-point int64 targets yi = rint(ldexp(y, e)) with the exponent chosen from
// max |y| (core/fit.py fixed_point_exponent), their root statistics {sum, min,
// max} and the finite check, in two launches and no host round trip: the host
// reads {finite, e, sum, min, max} together with the binning's first wait.
// st: int64 [8] = {max |y| bits, non-finite count, e, sum, min, max, -, -}.

// ceil(log2(x)) for x > 0, exact (frexp: x = m 2^k, m in [0.5, 1))
__device__ inline int ceil_log2_exact(double x) {
  int k;
  const double m = frexp(x, &k);
  return m == 0.5 ? k - 1 : k;
}

template <typename T>
__global__ __launch_bounds__(256) void target_stats_kernel(const T* __restrict__ y, int64_t n,
                                                           int64_t* __restrict__ st) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st[4] = INT64_MAX;
    st[5] = INT64_MIN;
  }
  double amax = 0.0;
  unsigned bad = 0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double v = (double)y[i];
    if (!isfinite(v)) {
      ++bad;
    } else {
      amax = fmax(amax, fabs(v));
    }
  }
  for (int d = kWave / 2; d > 0; d >>= 1) {
    amax = fmax(amax, __shfl_xor(amax, d, kWave));
    bad += __shfl_xor(bad, d, kWave);
  }
  // one atomic per workgroup (same-address atomics serialise in the L2)
  __shared__ double s_a[4];
  __shared__ unsigned s_b[4];
  if (lane_id() == 0) {
    s_a[threadIdx.x >> 6] = amax;
    s_b[threadIdx.x >> 6] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      amax = fmax(amax, s_a[w]);
      bad += s_b[w];
    }
    // non-negative doubles order as their bit patterns
    atomicMax(reinterpret_cast<unsigned long long*>(st), (unsigned long long)__double_as_longlong(amax));
    if (bad) atomicAdd(reinterpret_cast<unsigned long long*>(st) + 1, (unsigned long long)bad);
  }
}

__device__ inline int fixed_point_exponent_dev(double absmax, int64_t n) {
  if (!(absmax > 0.0) || !isfinite(absmax)) return 0;
  const int e = 62 - ceil_log2_exact((double)(n > 1 ? n : 1) + 1.0) -
                ceil_log2_exact(absmax * (1.0 + 0x1p-40));
  return e > 1000 ? 1000 : (e < -1000 ? -1000 : e);
}

template <typename T>
__global__ __launch_bounds__(256) void target_encode_kernel(const T* __restrict__ y, int64_t n,
                                                            int64_t* __restrict__ st,
                                                            int64_t* __restrict__ out) {
  const int e = fixed_point_exponent_dev(__longlong_as_double(st[0]), n);
  if (blockIdx.x == 0 && threadIdx.x == 0) st[2] = e;
  long long sum = 0, mn = LLONG_MAX, mx = LLONG_MIN;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double v = (double)y[i];
    const long long q = isfinite(v) ? (long long)rint(ldexp(v, e)) : 0;
    out[i] = q;
    sum += q;
    mn = q < mn ? q : mn;
    mx = q > mx ? q : mx;
  }
  for (int d = kWave / 2; d > 0; d >>= 1) {
    sum += __shfl_xor(sum, d, kWave);
    const long long a = __shfl_xor(mn, d, kWave), b = __shfl_xor(mx, d, kWave);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  __shared__ long long s_s[4], s_mn[4], s_mx[4];
  if (lane_id() == 0) {
    s_s[threadIdx.x >> 6] = sum;
    s_mn[threadIdx.x >> 6] = mn;
    s_mx[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      sum += s_s[w];
      mn = s_mn[w] < mn ? s_mn[w] : mn;
      mx = s_mx[w] > mx ? s_mx[w] : mx;
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(st) + 3, (unsigned long long)sum);
    atomicMin(reinterpret_cast<long long*>(st) + 4, mn);
    atomicMax(reinterpret_cast<long long*>(st) + 5, mx);
  }
}

void launch_targets(hipStream_t stream, const void* y, bool y64, int64_t n, int64_t* st,
                    int64_t* out) {
  MT_HIP_CHECK(hipMemsetAsync(st, 0, 8 * sizeof(int64_t), stream));
  if (n <= 0) return;
  const unsigned g = std::min(label_grid(n), 512u);
  if (y64) {
    hipLaunchKernelGGL(target_stats_kernel<double>, dim3(g), dim3(256), 0, stream,
                       (const double*)y, n, st);
    hipLaunchKernelGGL(target_encode_kernel<double>, dim3(g), dim3(256), 0, stream,
                       (const double*)y, n, st, out);
  } else {
    hipLaunchKernelGGL(target_stats_kernel<float>, dim3(g), dim3(256), 0, stream,
                       (const float*)y, n, st);
    hipLaunchKernelGGL(target_encode_kernel<float>, dim3(g), dim3(256), 0, stream,
                       (const float*)y, n, st, out);
  }
  MT_HIP_CHECK(hipGetLastError());
}


// ---- tiny subtrees, largest first (finish.hip / finish_reg.hip) -----------
// The tiny-subtree kernels' waves claim records in discovery order; a record's
// chain of dependent node steps grows with its rows, so a late large subtree
// leaves most waves idle at the end (a P = 8 rank has ~2 subtrees per wave).
// order[] = the record indices by rows descending (a counting sort over rows
// 0..64; unused reserved records, rows < 2, last): per-workgroup LDS counts,
// one global reservation per bucket and workgroup, LDS cursors for the places.
// scratch: int32 [2 * 65] bucket totals + cursors (zeroed by the launcher).
constexpr int kTinyOrderB = 65;
constexpr int kTinyOrderThreads = 256;

__device__ __forceinline__ int tiny_order_bucket(const int64_t* __restrict__ tiny, int64_t k) {
  const int64_t m = tiny[k * 8 + 1];
  return 64 - (int)(m < 0 ? 0 : (m > 64 ? 64 : m));
}

__global__ __launch_bounds__(kTinyOrderThreads) void tiny_order_count_kernel(
    const int64_t* __restrict__ tiny, const int32_t* __restrict__ count, int32_t* __restrict__ tot) {
  __shared__ int32_t h[kTinyOrderB];
  for (int i = threadIdx.x; i < kTinyOrderB; i += kTinyOrderThreads) h[i] = 0;
  __syncthreads();
  const int64_t K = *count;
  const int64_t per = (K + gridDim.x - 1) / gridDim.x;
  const int64_t k0 = (int64_t)blockIdx.x * per, k1 = k0 + per < K ? k0 + per : K;
  for (int64_t k = k0 + threadIdx.x; k < k1; k += kTinyOrderThreads)
    atomicAdd(&h[tiny_order_bucket(tiny, k)], 1);
  __syncthreads();
  for (int i = threadIdx.x; i < kTinyOrderB; i += kTinyOrderThreads)
    if (h[i]) atomicAdd(&tot[i], h[i]);
}

__global__ __launch_bounds__(kTinyOrderThreads) void tiny_order_place_kernel(
    const int64_t* __restrict__ tiny, const int32_t* __restrict__ count,
    const int32_t* __restrict__ tot, int32_t* __restrict__ cursor, int32_t* __restrict__ order) {
  __shared__ int32_t h[kTinyOrderB], base[kTinyOrderB];
  for (int i = threadIdx.x; i < kTinyOrderB; i += kTinyOrderThreads) h[i] = 0;
  __syncthreads();
  const int64_t K = *count;
  const int64_t per = (K + gridDim.x - 1) / gridDim.x;
  const int64_t k0 = (int64_t)blockIdx.x * per, k1 = k0 + per < K ? k0 + per : K;
  for (int64_t k = k0 + threadIdx.x; k < k1; k += kTinyOrderThreads)
    atomicAdd(&h[tiny_order_bucket(tiny, k)], 1);
  __syncthreads();
  if (threadIdx.x < kTinyOrderB) {  // (kTinyOrderB <= threads: one bucket a thread)
    const int b = threadIdx.x;
    int start = 0;
    for (int i = 0; i < b; ++i) start += tot[i];
    base[b] = start + (h[b] ? atomicAdd(&cursor[b], h[b]) : 0);
    h[b] = 0;
  }
  __syncthreads();
  for (int64_t k = k0 + threadIdx.x; k < k1; k += kTinyOrderThreads) {
    const int b = tiny_order_bucket(tiny, k);
    order[base[b] + atomicAdd(&h[b], 1)] = (int32_t)k;
  }
}

void launch_tiny_order(hipStream_t stream, const int64_t* tiny, const int32_t* count,
                       int32_t* scratch, int32_t* order, int grid) {
  MT_HIP_CHECK(hipMemsetAsync(scratch, 0, sizeof(int32_t) * 2 * kTinyOrderB, stream));
  hipLaunchKernelGGL(tiny_order_count_kernel, dim3(grid), dim3(kTinyOrderThreads), 0, stream,
                     tiny, count, scratch);
  hipLaunchKernelGGL(tiny_order_place_kernel, dim3(grid), dim3(kTinyOrderThreads), 0, stream,
                     tiny, count, scratch, scratch + kTinyOrderB, order);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
