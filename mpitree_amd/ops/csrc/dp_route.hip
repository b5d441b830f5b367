// Data-parallel subtree finishing: route each finisher job's rows to its owner.
//
// The reference gives every rank the full tree by recursing the same subtree on
// split communicators (mpitree/tree/decision_tree.py:340-362,446-477); its
// rows are never sharded. A row-sharded (strategy="data") fit here grows the
// levels with per-level histogram reductions and then finishes each subtree
// job on one owner rank, which needs that job's rows from every rank. These
// kernels do the routing on the device (ops/device_grower.py _dp_finish):
//
//   dp_plan_kernel     one workgroup: job owners (serpentine over the
//                      largest-first order), this rank's send offsets
//                      (owner-major, job order within an owner), the per-rank
//                      send / receive row counts, the owned jobs' contiguous
//                      layout and the (source, job) copy segments of the
//                      received rows;
//   dp_gather_kernel   this rank's rows of every job -> the send buffer (row-
//                      major codes + targets), grouped by destination rank;
//   dp_place_kernel    received segments -> job-contiguous rows.
//
// One host wait remains: all_to_all needs the split sizes on the host.
#include "common.h"

#include <stdexcept>

namespace mt {

constexpr int kDpThreads = 1024;

__device__ inline int dp_owner(int j, int P) {
  const int lap = j / P, off = j % P;
  return (lap & 1) == 0 ? off : P - 1 - off;
}

// exclusive block scan (kDpThreads threads) of v; returns the prefix, total in *tot
__device__ inline int64_t dp_scan(int64_t v, int64_t* s_w, int64_t* tot) {
  const int lane = lane_id(), w = threadIdx.x / kWave;
  int64_t x = v;
  for (int d = 1; d < kWave; d <<= 1) {
    const int64_t y = __shfl_up(x, d, kWave);
    if (lane >= d) x += y;
  }
  if (lane == kWave - 1) s_w[w] = x;
  __syncthreads();
  int64_t off = 0, t = 0;
  for (int k = 0; k < kDpThreads / kWave; ++k) {
    off += k < w ? s_w[k] : 0;
    t += s_w[k];
  }
  __syncthreads();
  *tot = t;
  return off + x - v;
}

// jobs: int64 [J][W], W = 5 + C + 2: {local start, rows, depth, pos, buffer,
// stats[C], local rows, src}; allc: int64 [P][J] local rows of job j on rank s.
// Outputs: soff [J] send offset of this rank's rows of job j; hdr int64 [4 + 2P]
// = {owned jobs Jm, received rows, -, -, send counts[P], recv counts[P]};
// jobs2 int64 [Jm][5 + C] = {new start, rows, depth, pos, 0, stats[C]};
// seg int64 [P * Jm][3] = {received offset, new offset, rows}, k-major.
__global__ __launch_bounds__(kDpThreads) void dp_plan_kernel(
    const int64_t* __restrict__ jobs, int J, int W, int C, const int64_t* __restrict__ allc,
    int P, int me, int64_t* __restrict__ soff, int64_t* __restrict__ hdr,
    int64_t* __restrict__ jobs2, int64_t* __restrict__ seg) {
  __shared__ int64_t s_w[kDpThreads / kWave];
  __shared__ int64_t s_carry;
  __shared__ int64_t s_rblk[64];  // received block start per source rank (P <= 64)
  const int tid = threadIdx.x;
  // send offsets, destination by destination (owner-major, job order within)
  for (int d = 0; d < P; ++d) {
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (int b0 = 0; b0 < J; b0 += kDpThreads) {
      const int j = b0 + tid;
      const bool mine = j < J && dp_owner(j, P) == d;
      const int64_t v = mine ? jobs[(int64_t)j * W + 5 + C] : 0;
      int64_t t;
      const int64_t o = dp_scan(v, s_w, &t);
      if (mine) soff[j] = o + s_carry;  // (relative to destination d's block)
      __syncthreads();
      if (tid == 0) s_carry += t;
      __syncthreads();
    }
    if (tid == 0) hdr[4 + d] = s_carry;
    __syncthreads();
  }
  // destination block starts -> absolute send offsets
  if (tid == 0) {
    int64_t a = 0;
    for (int d = 0; d < P; ++d) {
      s_rblk[d] = a;
      a += hdr[4 + d];
    }
  }
  __syncthreads();
  for (int j = tid; j < J; j += kDpThreads) soff[j] += s_rblk[dp_owner(j, P)];
  __syncthreads();
  // receive counts per source: sum of allc[s][j] over the jobs this rank owns
  for (int s = 0; s < P; ++s) {
    int64_t v = 0;
    for (int j = tid; j < J; j += kDpThreads)
      if (dp_owner(j, P) == me) v += allc[(int64_t)s * J + j];
    int64_t t;
    dp_scan(v, s_w, &t);
    if (tid == 0) hdr[4 + P + s] = t;
    __syncthreads();
  }
  if (tid == 0) {
    int64_t a = 0;
    for (int s = 0; s < P; ++s) {
      s_rblk[s] = a;
      a += hdr[4 + P + s];
    }
    hdr[1] = a;
  }
  __syncthreads();
  // owned jobs in job order: k = rank among owned jobs; their new contiguous
  // layout and the copy segments (received rows of job k from source s)
  if (tid == 0) s_carry = 0;
  __syncthreads();
  int64_t kbase = 0;  // owned jobs before this chunk
  for (int b0 = 0; b0 < J; b0 += kDpThreads) {
    const int j = b0 + tid;
    const bool mine = j < J && dp_owner(j, P) == me;
    int64_t nk;
    const int64_t k = dp_scan(mine ? 1 : 0, s_w, &nk) + kbase;
    int64_t g = 0;
    if (mine)
      for (int s = 0; s < P; ++s) g += allc[(int64_t)s * J + j];
    int64_t tg;
    const int64_t ns = dp_scan(g, s_w, &tg) + s_carry;  // new start of owned job k
    if (mine) {
      int64_t* o = jobs2 + k * (5 + C);
      const int64_t* src = jobs + (int64_t)j * W;
      o[0] = ns;
      o[1] = src[1];
      o[2] = src[2];
      o[3] = src[3];
      o[4] = 0;
      for (int c = 0; c < C; ++c) o[5 + c] = src[5 + c];
    }
    __syncthreads();
    if (tid == 0) s_carry += tg;
    __syncthreads();
    kbase += nk;
  }
  const int64_t Jm = kbase;
  if (tid == 0) hdr[0] = Jm;
  __syncthreads();
  // segments: for source s, owned job k: received offset = block(s) + rows of
  // owned jobs before k from s; new offset = new start(k) + rows of k from s' < s
  for (int s = 0; s < P; ++s) {
    if (tid == 0) s_carry = 0;
    __syncthreads();
    int64_t kb = 0;
    for (int b0 = 0; b0 < J; b0 += kDpThreads) {
      const int j = b0 + tid;
      const bool mine = j < J && dp_owner(j, P) == me;
      int64_t nk;
      const int64_t k = dp_scan(mine ? 1 : 0, s_w, &nk) + kb;
      const int64_t v = mine ? allc[(int64_t)s * J + j] : 0;
      int64_t t;
      const int64_t within = dp_scan(v, s_w, &t) + s_carry;
      if (mine) {
        int64_t before = 0;
        for (int s2 = 0; s2 < s; ++s2) before += allc[(int64_t)s2 * J + j];
        int64_t* sg = seg + ((int64_t)k * P + s) * 3;
        sg[0] = s_rblk[s] + within;
        sg[1] = jobs2[k * (5 + C)] + before;
        sg[2] = v;
      }
      __syncthreads();
      if (tid == 0) s_carry += t;
      __syncthreads();
      kb += nk;
    }
  }
}

// One workgroup per job: this rank's rows of job j (entries of idx or tmp from
// the job's local start; the low bits hold the row) -> send rows soff[j] + i.
// Rows (padded to 4-byte words) are copied a word per thread, plus the target.
template <typename YT>
__global__ __launch_bounds__(256) void dp_gather_kernel(
    const int64_t* __restrict__ jobs, int W, int C, const uint32_t* __restrict__ idx,
    const uint32_t* __restrict__ tmp, uint32_t row_mask, const uint8_t* __restrict__ codes_rm,
    int64_t row_bytes, const YT* __restrict__ y, const int64_t* __restrict__ soff,
    uint8_t* __restrict__ out_codes, YT* __restrict__ out_y) {
  const int j = blockIdx.x;
  const int64_t* J = jobs + (int64_t)j * W;
  const int64_t start = J[0], cnt = J[5 + C];
  const uint32_t* src = J[4] == 0 ? idx : tmp;
  const int64_t o = soff[j];
  const int chunks = (int)(row_bytes / 4);
  const int64_t total = cnt * chunks;
  for (int64_t t = threadIdx.x; t < total; t += 256) {
    const int64_t i = t / chunks;
    const int c = (int)(t - i * chunks);
    const uint32_t row = src[start + i] & row_mask;
    const uint32_t v = reinterpret_cast<const uint32_t*>(codes_rm + (int64_t)row * row_bytes)[c];
    reinterpret_cast<uint32_t*>(out_codes + (o + i) * row_bytes)[c] = v;
    if (c == 0) out_y[o + i] = y[row];
  }
}

// One workgroup per (owned job, source) segment: received rows -> new rows.
template <typename YT>
__global__ __launch_bounds__(256) void dp_place_kernel(const int64_t* __restrict__ seg,
                                                       const uint8_t* __restrict__ in_codes,
                                                       const YT* __restrict__ in_y,
                                                       int64_t row_bytes,
                                                       uint8_t* __restrict__ out_codes,
                                                       YT* __restrict__ out_y) {
  const int64_t* sg = seg + (int64_t)blockIdx.x * 3;
  const int64_t a = sg[0], b = sg[1], cnt = sg[2];
  const int chunks = (int)(row_bytes / 4);
  const int64_t total = cnt * chunks;
  for (int64_t t = threadIdx.x; t < total; t += 256) {
    const int64_t i = t / chunks;
    const int c = (int)(t - i * chunks);
    reinterpret_cast<uint32_t*>(out_codes + (b + i) * row_bytes)[c] =
        reinterpret_cast<const uint32_t*>(in_codes + (a + i) * row_bytes)[c];
    if (c == 0) out_y[b + i] = in_y[a + i];
  }
}

void launch_dp_plan(hipStream_t stream, const int64_t* jobs, int J, int W, int C,
                    const int64_t* allc, int P, int me, int64_t* soff, int64_t* hdr,
                    int64_t* jobs2, int64_t* seg) {
  if (P > 64) throw std::runtime_error("data-parallel routing: at most 64 ranks");
  hipLaunchKernelGGL(dp_plan_kernel, dim3(1), dim3(kDpThreads), 0, stream, jobs, J, W, C, allc,
                     P, me, soff, hdr, jobs2, seg);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_dp_gather(hipStream_t stream, const int64_t* jobs, int J, int W, int C,
                      const uint32_t* idx, const uint32_t* tmp, uint32_t row_mask,
                      const uint8_t* codes_rm, int64_t row_bytes, const void* y, bool y64,
                      const int64_t* soff, uint8_t* out_codes, void* out_y) {
  if (J <= 0) return;
  if (row_bytes % 4) throw std::runtime_error("data-parallel routing: row bytes % 4 != 0");
  if (y64)
    hipLaunchKernelGGL(dp_gather_kernel<int64_t>, dim3(J), dim3(256), 0, stream, jobs, W, C, idx,
                       tmp, row_mask, codes_rm, row_bytes, (const int64_t*)y, soff, out_codes,
                       (int64_t*)out_y);
  else
    hipLaunchKernelGGL(dp_gather_kernel<int32_t>, dim3(J), dim3(256), 0, stream, jobs, W, C, idx,
                       tmp, row_mask, codes_rm, row_bytes, (const int32_t*)y, soff, out_codes,
                       (int32_t*)out_y);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_dp_place(hipStream_t stream, const int64_t* seg, int64_t nseg, const uint8_t* in_codes,
                     const void* in_y, bool y64, int64_t row_bytes, uint8_t* out_codes,
                     void* out_y) {
  if (nseg <= 0) return;
  if (y64)
    hipLaunchKernelGGL(dp_place_kernel<int64_t>, dim3((unsigned)nseg), dim3(256), 0, stream, seg,
                       in_codes, (const int64_t*)in_y, row_bytes, out_codes, (int64_t*)out_y);
  else
    hipLaunchKernelGGL(dp_place_kernel<int32_t>, dim3((unsigned)nseg), dim3(256), 0, stream, seg,
                       in_codes, (const int32_t*)in_y, row_bytes, out_codes, (int32_t*)out_y);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
