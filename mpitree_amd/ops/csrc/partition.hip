// Row partition and per-segment statistics on gfx950.
//
// Replaces the reference's ``X[region], y[region]`` / ``X[~region]`` copies
// that feed the recursion (mpitree/tree/decision_tree.py:150-164, :428-454):
// instead of copying feature rows, only the 4-B row permutation ``idx`` is
// reordered so that each child's rows are contiguous inside the parent's
// segment. The split feature is read from the feature-major code matrix, a
// single 1-byte column per node that stays L2-resident.
//
// Each workgroup handles a <= kPartChunk-row chunk of one split node's segment, counts
// its left rows with wave prefix sums, reserves space with one atomic per
// cursor (left cursor grows from the segment start, right cursor shrinks from
// the segment end) and scatters into a temporary buffer; a copy kernel writes
// the segments back. The order of rows inside a child is not stable, which is
// harmless: every statistic downstream is an integer (or fixed-point) sum.
// Permutation entries may carry the class label in their top bits
// (``row | label << shift``, see hist.hip); ``mask`` extracts the row.
#include <climits>

#include "common.h"
#include "grow.h"

namespace mt {

constexpr int kPartThreads = 256;
constexpr int kPartRows = kPartChunk / kPartThreads;  // rows per thread (grow.h)

// items: int64 [n][3] = {split j, chunk start, chunk count}
// split: int64 [k][4] = {seg start, seg count, feature, bin}
// cursors: int32 [k][2] = {left cursor, right cursor} (initialised by host)
template <typename CodeT>
__global__ __launch_bounds__(kPartThreads) void partition_kernel(
    const CodeT* __restrict__ codes_fm, int64_t n_rows, const uint32_t* __restrict__ idx,
    uint32_t* __restrict__ tmp, uint32_t mask, const int64_t* __restrict__ items,
    const int64_t* __restrict__ split, int32_t* __restrict__ cursors,
    const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.x >= *dcount) return;  // device-side item count
  __shared__ uint32_t s_left[kPartThreads / kWave];
  __shared__ uint32_t s_right[kPartThreads / kWave];
  __shared__ int32_t s_base_l, s_base_r;
  const int64_t j = items[blockIdx.x * 3 + 0];
  const int64_t c0 = items[blockIdx.x * 3 + 1];
  const int64_t cn = items[blockIdx.x * 3 + 2];
  const int64_t f = split[j * 4 + 2];
  const uint32_t bin = (uint32_t)split[j * 4 + 3];
  const CodeT* col = codes_fm + f * n_rows;
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();

  uint32_t ent[kPartRows];
  bool go[kPartRows], valid[kPartRows];
  uint32_t my_l = 0, my_r = 0;
#pragma unroll
  for (int k = 0; k < kPartRows; ++k) {
    const int64_t e = (int64_t)k * kPartThreads + threadIdx.x;
    valid[k] = e < cn;
    ent[k] = valid[k] ? idx[c0 + e] : 0u;
  }
  // the split feature's codes of all the thread's rows in flight at once
  // (unconditional gathers; a guarded one waited for each row in turn)
  uint32_t cv[kPartRows];
#pragma unroll
  for (int k = 0; k < kPartRows; ++k) cv[k] = (uint32_t)col[ent[k] & mask];
#pragma unroll
  for (int k = 0; k < kPartRows; ++k) {
    go[k] = valid[k] && cv[k] <= bin;
    my_l += (valid[k] && go[k]) ? 1u : 0u;
    my_r += (valid[k] && !go[k]) ? 1u : 0u;
  }
  uint32_t il = my_l, ir = my_r;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t ol = __shfl_up(il, d, kWave), orr = __shfl_up(ir, d, kWave);
    if (lane >= d) {
      il += ol;
      ir += orr;
    }
  }
  if (lane == kWave - 1) {
    s_left[wave] = il;
    s_right[wave] = ir;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tl = 0, tr = 0;
    for (int w = 0; w < kPartThreads / kWave; ++w) {
      const uint32_t a = s_left[w], b = s_right[w];
      s_left[w] = tl;
      s_right[w] = tr;
      tl += a;
      tr += b;
    }
    s_base_l = tl ? atomicAdd(&cursors[j * 2 + 0], (int32_t)tl) : 0;
    s_base_r = tr ? atomicSub(&cursors[j * 2 + 1], (int32_t)tr) - (int32_t)tr : 0;
  }
  __syncthreads();
  uint32_t pl = s_base_l + s_left[wave] + il - my_l;
  uint32_t pr = s_base_r + s_right[wave] + ir - my_r;
#pragma unroll
  for (int k = 0; k < kPartRows; ++k) {
    if (valid[k]) {
      if (go[k])
        tmp[pl++] = ent[k];
      else
        tmp[pr++] = ent[k];
    }
  }
}

// idx[seg] = tmp[seg] for every chunk item
__global__ __launch_bounds__(256) void copy_back_kernel(const uint32_t* __restrict__ tmp,
                                                        uint32_t* __restrict__ idx,
                                                        const int64_t* __restrict__ items,
                                                        const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.x >= *dcount) return;
  const int64_t c0 = items[blockIdx.x * 3 + 1];
  const int64_t cn = items[blockIdx.x * 3 + 2];
  for (int64_t e = threadIdx.x; e < cn; e += blockDim.x) idx[c0 + e] = tmp[c0 + e];
}

// segment statistics: items int64 [n][3] = {segment s, start, count}
// classification: out uint32 [S][C] (class counts)
// regression: out int64 [S][4] = {count, sum, min, max}
__global__ __launch_bounds__(256) void seg_stats_cls_kernel(const uint32_t* __restrict__ idx,
                                                            const int32_t* __restrict__ y,
                                                            int lab_shift,
                                                            const int64_t* __restrict__ items,
                                                            uint32_t* __restrict__ out, int C) {
  extern __shared__ uint32_t cnt[];
  const int64_t s = items[blockIdx.x * 3 + 0];
  const int64_t c0 = items[blockIdx.x * 3 + 1];
  const int64_t cn = items[blockIdx.x * 3 + 2];
  for (int c = threadIdx.x; c < C; c += blockDim.x) cnt[c] = 0;
  __syncthreads();
  for (int64_t e = threadIdx.x; e < cn; e += blockDim.x) {
    const uint32_t v = idx[c0 + e];
    const int lab = lab_shift ? (int)(v >> lab_shift) : y[v];
    atomicAdd(&cnt[lab], 1u);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    if (cnt[c]) atomicAdd(&out[s * C + c], cnt[c]);
}

__global__ __launch_bounds__(256) void seg_stats_reg_kernel(const uint32_t* __restrict__ idx,
                                                            const int64_t* __restrict__ y,
                                                            const int64_t* __restrict__ items,
                                                            int64_t* __restrict__ out) {
  __shared__ int64_t sa[4], ss[4], smin[4], smax[4];
  const int64_t s = items[blockIdx.x * 3 + 0];
  const int64_t c0 = items[blockIdx.x * 3 + 1];
  const int64_t cn = items[blockIdx.x * 3 + 2];
  int64_t a = 0, sum = 0, mn = INT64_MAX, mx = INT64_MIN;
  for (int64_t e = threadIdx.x; e < cn; e += blockDim.x) {
    const int64_t v = y[idx[c0 + e]];
    a += 1;
    sum += v;
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    a += __shfl_xor(a, d, kWave);
    sum += __shfl_xor(sum, d, kWave);
    const int64_t omn = __shfl_xor(mn, d, kWave), omx = __shfl_xor(mx, d, kWave);
    mn = omn < mn ? omn : mn;
    mx = omx > mx ? omx : mx;
  }
  const int wave = threadIdx.x >> 6;
  if (lane_id() == 0) {
    sa[wave] = a;
    ss[wave] = sum;
    smin[wave] = mn;
    smax[wave] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t A = 0, S = 0, MN = INT64_MAX, MX = INT64_MIN;
    for (int w = 0; w < 4; ++w) {
      A += sa[w];
      S += ss[w];
      MN = smin[w] < MN ? smin[w] : MN;
      MX = smax[w] > MX ? smax[w] : MX;
    }
    unsigned long long* o = reinterpret_cast<unsigned long long*>(out + s * 4);
    atomicAdd(&o[0], (unsigned long long)A);
    atomicAdd(&o[1], (unsigned long long)S);
    atomicMin(reinterpret_cast<long long*>(out + s * 4 + 2), (long long)MN);
    atomicMax(reinterpret_cast<long long*>(out + s * 4 + 3), (long long)MX);
  }
}

// idx[i] = i | y[i] << shift  (packed permutation with labels) or i
__global__ __launch_bounds__(256) void init_idx_kernel(uint32_t* __restrict__ idx,
                                                       const int32_t* __restrict__ y,
                                                       int lab_shift, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) idx[i] = lab_shift ? ((uint32_t)i | ((uint32_t)y[i] << lab_shift)) : (uint32_t)i;
}

// Regression purity: per frontier slot min / max of the fixed-point targets
// over its rows. items: int64 [n][3] {slot, start, count}; out: int64 [slot][2]
// initialised to {INT64_MAX, INT64_MIN} by the planner.
__global__ __launch_bounds__(256) void seg_minmax_kernel(const uint32_t* __restrict__ idx,
                                                         const int64_t* __restrict__ y,
                                                         const int64_t* __restrict__ items,
                                                         int64_t* __restrict__ out,
                                                         const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.x >= *dcount) return;
  const int64_t s = items[blockIdx.x * 3 + 0];
  const int64_t c0 = items[blockIdx.x * 3 + 1];
  const int64_t cn = items[blockIdx.x * 3 + 2];
  long long mn = LLONG_MAX, mx = LLONG_MIN;
  for (int64_t e = threadIdx.x; e < cn; e += blockDim.x) {
    const long long v = y[idx[c0 + e]];
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const long long a = __shfl_xor(mn, d, kWave), b = __shfl_xor(mx, d, kWave);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if (lane_id() == 0) {
    atomicMin(reinterpret_cast<long long*>(out + s * 2), mn);
    atomicMax(reinterpret_cast<long long*>(out + s * 2 + 1), mx);
  }
}

void launch_seg_minmax(hipStream_t stream, const uint32_t* idx, const int64_t* y,
                       const int64_t* items, int n_items, int64_t* out, const int32_t* dcount) {
  if (n_items <= 0) return;
  hipLaunchKernelGGL(seg_minmax_kernel, dim3(n_items), dim3(256), 0, stream, idx, y, items, out,
                     dcount);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_partition(hipStream_t stream, const void* codes_fm, int code_bytes, int64_t n_rows,
                      uint32_t* idx, uint32_t* tmp, uint32_t mask, const int64_t* items,
                      int n_items, const int64_t* split, int32_t* cursors,
                      const int32_t* dcount, bool copy_back) {
  if (n_items <= 0) return;
  if (code_bytes == 1)
    hipLaunchKernelGGL(partition_kernel<uint8_t>, dim3(n_items), dim3(kPartThreads), 0, stream,
                       (const uint8_t*)codes_fm, n_rows, idx, tmp, mask, items, split, cursors,
                       dcount);
  else
    hipLaunchKernelGGL(partition_kernel<uint16_t>, dim3(n_items), dim3(kPartThreads), 0, stream,
                       (const uint16_t*)codes_fm, n_rows, idx, tmp, mask, items, split, cursors,
                       dcount);
  MT_HIP_CHECK(hipGetLastError());
  if (!copy_back) return;  // device loop: levels alternate the two row buffers
  hipLaunchKernelGGL(copy_back_kernel, dim3(n_items), dim3(256), 0, stream, tmp, idx, items,
                     dcount);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_seg_stats(hipStream_t stream, const uint32_t* idx, const void* y, int lab_shift,
                      bool reg, const int64_t* items, int n_items, void* out, int C) {
  if (n_items <= 0) return;
  if (reg) {
    hipLaunchKernelGGL(seg_stats_reg_kernel, dim3(n_items), dim3(256), 0, stream, idx,
                       (const int64_t*)y, items, (int64_t*)out);
  } else {
    size_t lds = (size_t)C * 4;
    MT_HIP_CHECK(mt_set_max_lds((const void*)seg_stats_cls_kernel, (int)lds));
    hipLaunchKernelGGL(seg_stats_cls_kernel, dim3(n_items), dim3(256), lds, stream, idx,
                       (const int32_t*)y, lab_shift, items, (uint32_t*)out, C);
  }
  MT_HIP_CHECK(hipGetLastError());
}

void launch_init_idx(hipStream_t stream, uint32_t* idx, const int32_t* y, int lab_shift,
                     int64_t n) {
  if (n <= 0) return;
  hipLaunchKernelGGL(init_idx_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     idx, y, lab_shift, n);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
