// Setup of the exact-threshold engine (exact2.hip): per feature, the rows sorted
// by value and a per-chunk count of value changes (the dense value ranks).
//
// The reference sorts implicitly through np.unique per feature and node
// (mpitree/tree/decision_tree.py:73). Here one pass over X builds 64-bit keys
// {feature : 32 | order-preserving value bits : 32} feature-major (an LDS tile
// transpose of the row-major input), one stable rocPRIM radix sort orders all
// features at once over only the key bits that vary (32 + ceil(log2 F)) with
// 32-bit row ids as values, and two passes over the sorted keys derive the
// ranks (a per-chunk count of value changes, a per-feature scan of the chunk
// counts); xe_emit_kernel (exact2.hip) then writes the list entries.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace mt {

constexpr int kXsTile = 64;       // rows x features per transpose tile
constexpr int kXsChunk = 4096;    // sorted entries per rank chunk
constexpr int kXsThreads = 256;

// IEEE-754 order as unsigned order (-0.0 folded into +0.0 first)
__device__ __forceinline__ uint32_t xs_key_bits(float v) {
  uint32_t b = __float_as_uint(v + 0.0f);
  return (b >> 31) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float xs_key_value(uint32_t k) {
  return __uint_as_float((k >> 31) ? (k & 0x7fffffffu) : ~k);
}

// keys[f * n + i] = f << 32 | bits(X[i][f_lo + f]); rows[f * n + i] = i for the
// F features of the block starting at column f_lo of a row-major X of stride xs
__global__ __launch_bounds__(kXsThreads) void xs_keys_kernel(const float* __restrict__ X,
                                                             int64_t n, int F, int xs, int f_lo,
                                                             uint64_t* __restrict__ keys,
                                                             uint32_t* __restrict__ rows) {
  __shared__ uint32_t tile[kXsTile][kXsTile + 1];
  const int64_t i0 = (int64_t)blockIdx.x * kXsTile;
  const int f0 = blockIdx.y * kXsTile;
  const int tx = threadIdx.x & (kXsTile - 1), ty = threadIdx.x / kXsTile;  // 64 x 4
  for (int r = ty; r < kXsTile; r += kXsThreads / kXsTile) {
    const int64_t i = i0 + r;
    const int f = f0 + tx;
    tile[r][tx] = (i < n && f < F) ? xs_key_bits(X[i * xs + f_lo + f]) : 0u;
  }
  __syncthreads();
  for (int c = ty; c < kXsTile; c += kXsThreads / kXsTile) {
    const int f = f0 + c;
    const int64_t i = i0 + tx;
    if (f < F && i < n) {
      keys[(int64_t)f * n + i] = ((uint64_t)f << 32) | tile[tx][c];
      rows[(int64_t)f * n + i] = (uint32_t)i;
    }
  }
}

// Value changes per chunk: cnt[f][c] = #{j in chunk c of feature f : j is the
// first entry or keys[j] != keys[j - 1]}.
__global__ __launch_bounds__(kXsThreads) void xs_count_kernel(const uint64_t* __restrict__ keys,
                                                              int64_t n, int nc,
                                                              int32_t* __restrict__ cnt) {
  __shared__ int32_t s_w[kXsThreads / kWave];
  const int f = blockIdx.y, c = blockIdx.x;
  const int64_t base = (int64_t)f * n;
  const int64_t p0 = (int64_t)c * kXsChunk;
  const int64_t p1 = min<int64_t>(p0 + kXsChunk, n);
  int32_t k = 0;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += kXsThreads)
    k += (p == 0 || keys[base + p] != keys[base + p - 1]) ? 1 : 0;
  k = (int32_t)wave_sum_u32((uint32_t)k);
  if (lane_id() == 0) s_w[threadIdx.x >> 6] = k;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t t = 0;
    for (int w = 0; w < kXsThreads / kWave; ++w) t += s_w[w];
    cnt[(int64_t)f * nc + c] = t;
  }
}

// Per feature (one thread each): exclusive scan of the chunk counts; nuniq[f].
__global__ void xs_scan_kernel(int32_t* __restrict__ cnt, int nc, int F,
                               int32_t* __restrict__ nuniq) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  int32_t acc = 0;
  for (int c = 0; c < nc; ++c) {
    const int32_t v = cnt[(int64_t)f * nc + c];
    cnt[(int64_t)f * nc + c] = acc;
    acc += v;
  }
  nuniq[f] = acc;
}

size_t exact_setup_temp_bytes(int64_t n, int F) {
  size_t bytes = 0;
  const int64_t N = n * F;
  MT_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr,
                                                  (uint64_t*)nullptr, (const uint32_t*)nullptr,
                                                  (uint32_t*)nullptr, N, 0, 64));
  return bytes;
}

// Phase 1 (before the host learns the largest unique count): keys, sort, counts.
// keys/rows: two buffers each of n * F (ping-pong for the sort, result in [1]);
// cnt: int32 [F][nc]; nuniq: int32 [F].
void exact_setup_sort(hipStream_t stream, const float* X, int64_t n, int F, uint64_t* keys0,
                      uint64_t* keys1, uint32_t* rows0, uint32_t* rows1, void* temp,
                      size_t temp_bytes, int32_t* cnt, int32_t* nuniq, int xs, int f_lo) {
  if (xs <= 0) xs = F;
  if (n <= 0 || F <= 0) return;
  if (n >= (int64_t)1 << 24) throw std::runtime_error("exact setup: rows < 2^24");
  dim3 tg((unsigned)((n + kXsTile - 1) / kXsTile), (unsigned)((F + kXsTile - 1) / kXsTile));
  hipLaunchKernelGGL(xs_keys_kernel, tg, dim3(kXsThreads), 0, stream, X, n, F, xs, f_lo, keys0,
                     rows0);
  MT_HIP_CHECK(hipGetLastError());
  int fbits = 0;
  while ((1 << fbits) < F) ++fbits;
  const int64_t N = n * F;
  MT_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys0, keys1, rows0, rows1,
                                                  N, 0, 32 + fbits, stream));
  const int nc = (int)((n + kXsChunk - 1) / kXsChunk);
  hipLaunchKernelGGL(xs_count_kernel, dim3(nc, F), dim3(kXsThreads), 0, stream, keys1, n, nc,
                     cnt);
  MT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(xs_scan_kernel, dim3((F + 63) / 64), dim3(64), 0, stream, cnt, nc, F,
                     nuniq);
  MT_HIP_CHECK(hipGetLastError());
}

int exact_setup_chunk() { return kXsChunk; }

}  // namespace mt
