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
//   dp_place_kernel    received rows -> job-contiguous rows (row- and feature-major).
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

// This rank's rows of job j (entries of idx or tmp from the job's local start;
// the low bits hold the row) -> send rows soff[j] + i. Workgroup (x, j) copies
// rows [64 y, 64 y + 64) of job x (the grid's y extent bounds every job's local
// rows; surplus workgroups exit), 32 threads per 128-byte row slice: coalesced
// loads and stores, and every CU busy (one workgroup per job left most idle).
template <typename YT>
__global__ __launch_bounds__(256) void dp_gather_kernel(
    const int64_t* __restrict__ jobs, int W, int C, const uint32_t* __restrict__ idx,
    const uint32_t* __restrict__ tmp, uint32_t row_mask, const uint8_t* __restrict__ codes_rm,
    int64_t row_bytes, const YT* __restrict__ y, const int64_t* __restrict__ soff,
    uint8_t* __restrict__ out_codes, YT* __restrict__ out_y) {
  __shared__ uint32_t s_row[64];
  const int j = blockIdx.x;
  const int64_t* J = jobs + (int64_t)j * W;
  const int64_t start = J[0], cnt = J[5 + C];
  const int64_t i0 = (int64_t)blockIdx.y * 64;
  if (i0 >= cnt) return;  // (block-uniform)
  const uint32_t* src = J[4] == 0 ? idx : tmp;
  const int64_t o = soff[j];
  const int tid = threadIdx.x;
  const int nr = cnt - i0 < 64 ? (int)(cnt - i0) : 64;
  if (tid < nr) {
    const uint32_t row = src[start + i0 + tid] & row_mask;
    s_row[tid] = row;
    out_y[o + i0 + tid] = y[row];
  }
  __syncthreads();
  const int words = (int)(row_bytes / 4);
  for (int e = tid; e < nr * 32; e += 256) {
    const int r = e >> 5, w0 = e & 31;
    const uint32_t* in = reinterpret_cast<const uint32_t*>(codes_rm + (int64_t)s_row[r] * row_bytes);
    uint32_t* out = reinterpret_cast<uint32_t*>(out_codes + (o + i0 + r) * row_bytes);
    for (int w = w0; w < words; w += 32) out[w] = in[w];
  }
}

// Received rows -> the owner's job-contiguous rows, in both code layouts the
// finisher reads (row-major and feature-major) plus the targets. One workgroup
// per 64 destination rows: each row's source (received) row comes from a binary
// search over the segments -- {received offset, new offset, rows}, k-major, so
// their new offsets ascend and tile [0, R) -- the tile's rows are staged through
// LDS 32 words at a time (one 128-byte row slice per 32 threads: coalesced loads
// and row-major stores), and each feature's 64 codes go out as one coalesced run
// per wave (lanes = consecutive rows), which replaces a strided device transpose.
template <typename CT, typename YT>
__global__ __launch_bounds__(256) void dp_place_kernel(const int64_t* __restrict__ seg, int64_t nseg,
                                                       int64_t R, const uint8_t* __restrict__ in_codes,
                                                       const YT* __restrict__ in_y, int row_bytes,
                                                       int F, uint8_t* __restrict__ out_rm,
                                                       CT* __restrict__ out_fm,
                                                       YT* __restrict__ out_y) {
  __shared__ int64_t s_src[64];
  __shared__ uint32_t s_tile[64 * 33];  // 64 rows x 32 words (+1: conflict-free column reads)
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  if (tid < 64) {
    const int64_t d = r0 + tid;
    int64_t src = -1;
    if (d < R) {
      int64_t lo = 0, hi = nseg - 1;  // last segment with new offset <= d
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (seg[mid * 3 + 1] <= d) lo = mid; else hi = mid - 1;
      }
      src = seg[lo * 3 + 0] + (d - seg[lo * 3 + 1]);
      out_y[d] = in_y[src];
    }
    s_src[tid] = src;
  }
  __syncthreads();
  const int words = row_bytes / 4;
  constexpr int kEpw = 4 / (int)sizeof(CT);  // codes per word
  const int i = tid & 63;                    // feature-major phase: this lane's row
  for (int w0 = 0; w0 < words; w0 += 32) {
    const int nw = words - w0 < 32 ? words - w0 : 32;
    for (int e = tid; e < 64 * 32; e += 256) {
      const int r = e >> 5, w = e & 31;
      const int64_t sr = s_src[r];
      uint32_t v = 0u;
      if (w < nw && sr >= 0) {
        v = reinterpret_cast<const uint32_t*>(in_codes + sr * row_bytes)[w0 + w];
        reinterpret_cast<uint32_t*>(out_rm + (r0 + r) * row_bytes)[w0 + w] = v;
      }
      s_tile[r * 33 + w] = v;
    }
    __syncthreads();
    const int e0 = w0 * kEpw;
    const int ne = nw * kEpw;
    if (r0 + i < R) {
      for (int fe = tid >> 6; fe < ne && e0 + fe < F; fe += 4) {
        const uint32_t word = s_tile[i * 33 + fe / kEpw];
        out_fm[(int64_t)(e0 + fe) * R + r0 + i] =
            (CT)(word >> (8 * (int)sizeof(CT) * (fe % kEpw)));
      }
    }
    __syncthreads();
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
                      const int64_t* soff, uint8_t* out_codes, void* out_y, int64_t max_rows) {
  if (J <= 0 || max_rows <= 0) return;
  if (row_bytes % 4) throw std::runtime_error("data-parallel routing: row bytes % 4 != 0");
  if (max_rows > 65535 * 64) throw std::runtime_error("data-parallel routing: job too large");
  const dim3 g((unsigned)J, (unsigned)((max_rows + 63) / 64));
  if (y64)
    hipLaunchKernelGGL(dp_gather_kernel<int64_t>, g, dim3(256), 0, stream, jobs, W, C, idx,
                       tmp, row_mask, codes_rm, row_bytes, (const int64_t*)y, soff, out_codes,
                       (int64_t*)out_y);
  else
    hipLaunchKernelGGL(dp_gather_kernel<int32_t>, g, dim3(256), 0, stream, jobs, W, C, idx,
                       tmp, row_mask, codes_rm, row_bytes, (const int32_t*)y, soff, out_codes,
                       (int32_t*)out_y);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_dp_place(hipStream_t stream, const int64_t* seg, int64_t nseg, const uint8_t* in_codes,
                     const void* in_y, bool y64, int64_t row_bytes, int64_t R, int F, int cb,
                     uint8_t* out_rm, void* out_fm, void* out_y) {
  if (nseg <= 0 || R <= 0) return;
  if (row_bytes % 4) throw std::runtime_error("data-parallel placement: row bytes % 4 != 0");
  const dim3 g((unsigned)((R + 63) / 64));
#define MT_DP_PLACE(CT, YT)                                                                  \
  hipLaunchKernelGGL((dp_place_kernel<CT, YT>), g, dim3(256), 0, stream, seg, nseg, R, in_codes, \
                     (const YT*)in_y, (int)row_bytes, F, out_rm, (CT*)out_fm, (YT*)out_y)
  if (cb == 1 && y64) MT_DP_PLACE(uint8_t, int64_t);
  else if (cb == 1) MT_DP_PLACE(uint8_t, int32_t);
  else if (y64) MT_DP_PLACE(uint16_t, int64_t);
  else MT_DP_PLACE(uint16_t, int32_t);
#undef MT_DP_PLACE
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
