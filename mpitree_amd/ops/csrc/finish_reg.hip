// Subtree finisher for regression trees (squared error) on gfx950.
//
// Same contract as the classification finisher (finish.hip): jobs are
// deferred frontier nodes with at most ``finisher_rows`` rows, every node is
// written at its pre-order position (a subtree of r rows owns 2r - 1
// positions), children at p + 1 and p + 2 n_left. Differences:
//
// * statistics are {count, fixed-point target sum} (int64); a node whose
//   targets are all equal is a leaf -- the reference-style stopping rule for
//   regression -- checked from the min / max of its rows when it is popped;
// * finish_reg_kernel (nodes above the tiny size): one 256-thread workgroup
//   per job. A node's histogram {count u32, sum i64} per (feature, bin) is
//   48 KB per 16 features, so features are processed in LDS tiles of 16: build
//   the tile from the node's rows, wave-per-feature prefix scans (DPP for the
//   counts, 64-bit shuffles for the sums), cost = -S_L^2/m_L - S_R^2/m_R with
//   the shared mse_term, then the next tile. Ties: lowest bin, lowest feature.
// * finish_tiny_reg_kernel (<= 64 rows): one wavefront per subtree with the
//   presorted per-feature lane orders of finish_tiny_sorted_kernel; per node
//   and feature one count scan and one 64-bit sum scan along the sorted order.
#include <climits>
#include <cstdlib>

#include "common.h"
#include "criterion.h"
#include "grow.h"
#include "tiny_sort.h"

namespace mt {

constexpr int kRegThreads = 256;
constexpr int kRegWaves = kRegThreads / kWave;
constexpr int kRegFT = 16;      // features per LDS tile
constexpr int kRegStack = 40;
constexpr int kRegTinyRows = 64;
constexpr int kRegTinyWaves = 4;
constexpr int kRegMaxF = 256;

// Wave-wide min / max of int64 (every lane gets the result).
__device__ __forceinline__ void wave_minmax_i64(long long& mn, long long& mx) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const long long a = __shfl_xor(mn, d, kWave), b = __shfl_xor(mx, d, kWave);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
}

// jobs: int64 [J][7] = {start, count, depth, root position, buffer, count, sum}
// node_i32: [P][6] = {feature, bin, left pos, right pos, depth, n}; node_st: int64 [P][2]
template <typename CodeT>
__global__ __launch_bounds__(kRegThreads, 2) void finish_reg_kernel(
    const uint32_t* __restrict__ codes_rm, int64_t row_words, const CodeT* __restrict__ codes_fm,
    int64_t n_rows, uint32_t* __restrict__ buf0, uint32_t* __restrict__ buf1,
    const int64_t* __restrict__ y, const int64_t* __restrict__ jobs, int J,
    int32_t* __restrict__ job_counter, const int32_t* __restrict__ nbins, int F, int B,
    int max_depth, int64_t mss, int64_t msl, int32_t* __restrict__ node_i32,
    int64_t* __restrict__ node_st, int tiny_rows, int64_t* __restrict__ tiny,
    int32_t* __restrict__ tiny_count, int64_t* __restrict__ tasks,
    int32_t* __restrict__ task_flag, int32_t epoch, int task_cap) {
  extern __shared__ __align__(16) uint8_t smem[];
  unsigned long long* t_sum = reinterpret_cast<unsigned long long*>(smem);  // [FT][B]
  uint32_t* t_cnt = reinterpret_cast<uint32_t*>(smem + (size_t)kRegFT * B * 8);  // [FT][B]
  __shared__ int32_t s_nb[kRegMaxF];
  __shared__ int s_job, s_sp;
  __shared__ int64_t s_st_start[kRegStack], s_st_sum[kRegStack];
  __shared__ int32_t s_st_count[kRegStack], s_st_depth[kRegStack], s_st_id[kRegStack],
      s_st_buf[kRegStack];
  __shared__ int64_t s_start, s_sum;
  __shared__ int32_t s_count, s_depth, s_id, s_buf;
  __shared__ long long s_min, s_max;
  __shared__ unsigned long long s_lsum;
  __shared__ double w_gain[kRegWaves];
  __shared__ int w_feat[kRegWaves], w_bin[kRegWaves];
  __shared__ int s_lc, s_rc;
  __shared__ int s_tnext, s_tend;  // this workgroup's reserved tiny records (thread 0)

  const int tid = threadIdx.x;
  if (tid == 0) s_tnext = s_tend = 0;
  // a tiny-subtree record (thread 0 only): one device atomic per kFinTinyBatch
  auto tiny_slot = [&]() -> int64_t {
    if (s_tnext == s_tend) {
      const int t = atomicAdd(tiny_count, kFinTinyBatch);
      s_tnext = t;
      s_tend = t + kFinTinyBatch;
    }
    return (int64_t)(s_tnext++);
  };
  const int wave = tid >> 6;
  const int lane = lane_id();
  const int n_tiles = (F + kRegFT - 1) / kRegFT;
  const int tile_words = kRegFT * B;  // per array
  const bool vec4 = (row_words % 4) == 0 && sizeof(CodeT) == 1;
  for (int f = tid; f < min(F, kRegMaxF); f += kRegThreads) s_nb[f] = min(B, nbins[f]);
  __syncthreads();

  // Hand-off queue (as in finish_cls_kernel): a workgroup that splits a node
  // while others idle gives them the larger child; waiters poll their own
  // publish flag and the finished word; the last completion releases them.
  unsigned long long* const q_word =
      reinterpret_cast<unsigned long long*>(job_counter + kFinCtrQueue);
  int32_t* const q_finished = job_counter + kFinCtrFinished;
  for (;;) {
    if (tid == 0) {
      const int h = atomicAdd(job_counter, 1);
      int got = h;
      if (task_cap < 0) {
        if (h >= J) got = -1;
      } else if (h >= J) {
        const uint64_t t_start = wall_clock64();
        for (uint32_t spins = 0;; ++spins) {
          if (h - J < task_cap &&
              __hip_atomic_load(task_flag + (h - J), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                  epoch) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            break;
          }
          if (__hip_atomic_load(q_finished, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) {
            got = -1;
            break;
          }
          if ((spins & 15u) == 15u && wall_clock64() - t_start > 500000000ull) {  // 5 s
            atomicExch(job_counter + kFinCtrWatch, 1);
            got = -1;
            break;
          }
          __builtin_amdgcn_s_sleep(32);
        }
      }
      s_job = got;
    }
    __syncthreads();
    const int job = s_job;
    if (job < 0) break;
    const int64_t* jb =
        job < J ? jobs + (int64_t)job * 7 : tasks + (int64_t)(job - J) * 7;
    if (tid == 0) {
      const int r = (int)jb[3];
      int32_t* R = node_i32 + (int64_t)r * 6;
      R[0] = -1;
      R[1] = -1;
      R[2] = -1;
      R[3] = -1;
      R[4] = (int32_t)jb[2];
      R[5] = (int32_t)jb[1];
      node_st[(int64_t)r * 2 + 0] = jb[5];
      node_st[(int64_t)r * 2 + 1] = jb[6];
      s_sp = 0;
      if (jb[1] <= tiny_rows) {  // the whole job goes to a wavefront
        const int t = (int)tiny_slot();
        int64_t* tr = tiny + (int64_t)t * 8;
        tr[0] = jb[0];
        tr[1] = jb[1];
        tr[2] = jb[2];
        tr[3] = jb[4];
        tr[4] = r;
      } else {
        s_sp = 1;
        s_st_start[0] = jb[0];
        s_st_count[0] = (int32_t)jb[1];
        s_st_depth[0] = (int32_t)jb[2];
        s_st_id[0] = r;
        s_st_buf[0] = (int32_t)jb[4];
        s_st_sum[0] = jb[6];
      }
    }
    __syncthreads();
    while (s_sp > 0) {
      __syncthreads();
      if (tid == 0) {
        const int sp = --s_sp;
        s_start = s_st_start[sp];
        s_count = s_st_count[sp];
        s_depth = s_st_depth[sp];
        s_id = s_st_id[sp];
        s_buf = s_st_buf[sp];
        s_sum = s_st_sum[sp];
        s_min = LLONG_MAX;
        s_max = LLONG_MIN;
        s_lc = 0;
        s_rc = 0;
        s_lsum = 0ull;
      }
      __syncthreads();
      const int64_t start = s_start;
      const int m = s_count;
      const int depth = s_depth;
      const int id = s_id;
      const int64_t S = s_sum;
      uint32_t* __restrict__ src = s_buf ? buf1 : buf0;
      uint32_t* __restrict__ dst = s_buf ? buf0 : buf1;
      const double pterm = mse_term(m, S);
      double bg = -__builtin_inf();
      int bfeat = 0x7fffffff, bbin = -1;
      bool pure = false;
      for (int t = 0; t < n_tiles; ++t) {
        const int f0 = t * kRegFT;
        const int nf = min(kRegFT, F - f0);
        {  // clear the tile (sums then counts are contiguous: 12 B per (feature, bin))
          uint4* z = reinterpret_cast<uint4*>(smem);
          const int q = tile_words * 12 / 16;
          for (int e = tid; e < q; e += kRegThreads) z[e] = make_uint4(0, 0, 0, 0);
        }
        __syncthreads();
        long long mn = LLONG_MAX, mx = LLONG_MIN;
        for (int r = tid; r < m; r += kRegThreads) {
          const uint32_t row = src[start + r];
          const long long yv = y[row];
          if (t == 0) {
            mn = yv < mn ? yv : mn;
            mx = yv > mx ? yv : mx;
          }
          uint32_t w[4];
          const uint32_t* rp = codes_rm + (int64_t)row * row_words;
          if (vec4) {
            const uint4 v = *reinterpret_cast<const uint4*>(rp + f0 / 4);
            w[0] = v.x;
            w[1] = v.y;
            w[2] = v.z;
            w[3] = v.w;
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k] = 0u;
          }
#pragma unroll
          for (int fl = 0; fl < kRegFT; ++fl) {
            if (fl < nf) {
              uint32_t code;
              if (vec4) {
                code = (w[fl >> 2] >> ((fl & 3) * 8)) & 0xffu;
              } else {
                const CodeT* cp = reinterpret_cast<const CodeT*>(rp);
                code = (uint32_t)cp[f0 + fl];
              }
              atomicAdd(&t_cnt[fl * B + (int)code], 1u);
              atomicAdd(&t_sum[fl * B + (int)code], (unsigned long long)yv);
            }
          }
        }
        if (t == 0) {
          wave_minmax_i64(mn, mx);
          if (lane == 0) {
            atomicMin(&s_min, mn);
            atomicMax(&s_max, mx);
          }
        }
        __syncthreads();
        if (t == 0 && s_min == s_max) {
          pure = true;  // all targets equal: a leaf (its record already stands)
          break;
        }
        // ---- scan the tile: wave w takes features f0 + w, f0 + w + 4, ...
        for (int fl = wave; fl < nf; fl += kRegWaves) {
          const int f = f0 + fl;
          const int nb = f < kRegMaxF ? s_nb[f] : min(B, nbins[f]);  // (wide: from memory)
          const int b0 = lane * 4;
          uint32_t cn[4];
          long long cs[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int b = b0 + k;
            cn[k] = b < nb ? t_cnt[fl * B + b] : 0u;
            cs[k] = b < nb ? (long long)t_sum[fl * B + b] : 0ll;
          }
          uint32_t pn[4];
          long long ps[4];
          pn[0] = cn[0];
          ps[0] = cs[0];
#pragma unroll
          for (int k = 1; k < 4; ++k) {
            pn[k] = pn[k - 1] + cn[k];
            ps[k] = ps[k - 1] + cs[k];
          }
          const uint32_t en = wave_incl_scan_dpp(pn[3]) - pn[3];
          const long long es = (long long)wave_incl_scan_i64((int64_t)ps[3]) - ps[3];
          double best_cost = __builtin_inf();
          int best_bin = 0x7fffffff;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int64_t ml = (int64_t)(en + pn[k]);
            const int64_t sl = (int64_t)(es + ps[k]);
            const int64_t mr = (int64_t)m - ml;
            if (b0 + k < nb && cn[k] > 0 && ml >= msl && mr >= msl) {
              const double cost = mse_term(ml, sl) + mse_term(mr, S - sl);
              if (cost < best_cost) {
                best_cost = cost;
                best_bin = b0 + k;
              }
            }
          }
          wave_argmin_dpp(best_cost, best_bin);  // lanes own ascending bins (B <= 256)
          if (best_cost < __builtin_inf()) {
            const double g = pterm - best_cost;
            if (g > bg) {  // features ascend within a wave: strict > keeps the lowest
              bg = g;
              bfeat = f;
              bbin = best_bin;
            }
          }
        }
        __syncthreads();  // every wave is done with the tile before it is cleared
      }
      if (lane == 0) {
        w_gain[wave] = bg;
        w_feat[wave] = bfeat;
        w_bin[wave] = bbin;
      }
      __syncthreads();
      int bf, bb;
      {
        double g = w_gain[0];
        bf = w_feat[0];
        bb = w_bin[0];
        for (int w = 1; w < kRegWaves; ++w) {
          if (w_gain[w] > g || (w_gain[w] == g && w_feat[w] < bf)) {
            g = w_gain[w];
            bf = w_feat[w];
            bb = w_bin[w];
          }
        }
        if (!(g > -__builtin_inf()) || pure) bf = -1;
      }
      if (bf >= 0) {
        // ---- partition rows src -> dst; left targets summed on the way
        const CodeT* col = codes_fm + (int64_t)bf * n_rows;
        const unsigned long long lt = (1ull << lane) - 1ull;
        unsigned long long lsum = 0ull;
        for (int r0 = 0; r0 < m; r0 += kRegThreads) {
          const int r = r0 + tid;
          const bool valid = r < m;
          const uint32_t ent = valid ? src[start + r] : 0u;
          const bool go = valid && (uint32_t)col[ent] <= (uint32_t)bb;
          if (go) lsum += (unsigned long long)y[ent];
          const unsigned long long bl = __ballot(go);
          const unsigned long long br = __ballot(valid && !go);
          int basel = 0, baser = 0;
          if (lane == 0) {
            const int nl = __popcll(bl), nr = __popcll(br);
            basel = nl ? atomicAdd(&s_lc, nl) : 0;
            baser = nr ? atomicAdd(&s_rc, nr) : 0;
          }
          basel = __builtin_amdgcn_readfirstlane(basel);
          baser = __builtin_amdgcn_readfirstlane(baser);
          if (valid) {
            if (go)
              dst[start + basel + __popcll(bl & lt)] = ent;
            else
              dst[start + m - 1 - (baser + __popcll(br & lt))] = ent;
          }
        }
        lsum = (unsigned long long)wave_sum_i64((int64_t)lsum);
        if (lane == 0) atomicAdd(&s_lsum, lsum);
      }
      __syncthreads();
      if (tid == 0 && bf >= 0) {
        const int nl = s_lc;
        const int nr = m - nl;
        const int64_t sl = (int64_t)s_lsum, sr = S - sl;
        const int lid = id + 1, rid = id + 2 * nl;
        int32_t* P = node_i32 + (int64_t)id * 6;
        P[0] = bf;
        P[1] = bb;
        P[2] = lid;
        P[3] = rid;
        const int cd = depth + 1;
        int32_t* L = node_i32 + (int64_t)lid * 6;
        int32_t* Rr = node_i32 + (int64_t)rid * 6;
        L[0] = -1; L[1] = -1; L[2] = -1; L[3] = -1; L[4] = cd; L[5] = nl;
        Rr[0] = -1; Rr[1] = -1; Rr[2] = -1; Rr[3] = -1; Rr[4] = cd; Rr[5] = nr;
        node_st[(int64_t)lid * 2 + 0] = nl;
        node_st[(int64_t)lid * 2 + 1] = sl;
        node_st[(int64_t)rid * 2 + 0] = nr;
        node_st[(int64_t)rid * 2 + 1] = sr;
        const bool depth_stop = max_depth >= 0 && cd >= max_depth;
        const bool tlf = depth_stop || nl < mss || nl < 2 * msl;
        const bool trf = depth_stop || nr < mss || nr < 2 * msl;
        const bool left_small = nl <= nr;
        for (int pass = 0; pass < 2; ++pass) {
          const bool is_left = (pass == 0) ? !left_small : left_small;
          if (is_left ? tlf : trf) continue;
          const int cm = is_left ? nl : nr;
          const int64_t cstart = is_left ? start : start + nl;
          if (pass == 0 && cm > 2 * tiny_rows && task_cap > 0) {
            const int head =
                __hip_atomic_load(job_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int pushed = (int)(__hip_atomic_load(q_word, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT) >> 32);
            if (head > J + pushed && pushed < task_cap) {
              const int k = (int)(__hip_atomic_fetch_add(q_word, 1ull << 32, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) >> 32);
              if (k < task_cap) {
                int64_t* T = tasks + (int64_t)k * 7;
                T[0] = cstart;
                T[1] = cm;
                T[2] = cd;
                T[3] = is_left ? lid : rid;
                T[4] = s_buf ^ 1;
                T[5] = cm;
                T[6] = is_left ? sl : sr;
                __threadfence();  // the child's rows and record, chip-wide, before the flag
                __hip_atomic_store(task_flag + k, epoch, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
                continue;
              }
              __hip_atomic_fetch_add(q_word, ~0ull << 32, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          if (cm <= tiny_rows) {
            const int t = (int)tiny_slot();
            int64_t* tr = tiny + (int64_t)t * 8;
            tr[0] = cstart;
            tr[1] = cm;
            tr[2] = cd;
            tr[3] = s_buf ^ 1;
            tr[4] = is_left ? lid : rid;
            continue;
          }
          const int sp = s_sp++;
          s_st_start[sp] = cstart;
          s_st_count[sp] = cm;
          s_st_depth[sp] = cd;
          s_st_id[sp] = is_left ? lid : rid;
          s_st_buf[sp] = s_buf ^ 1;
          s_st_sum[sp] = is_left ? sl : sr;
        }
      }
      __syncthreads();
    }
    if (tid == 0 && task_cap >= 0) {
      const unsigned long long q =
          __hip_atomic_fetch_add(q_word, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(uint32_t)q + 1 == J + (int)(q >> 32))
        __hip_atomic_store(q_finished, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tid == 0)  // reserved records left unused: empty (m = 0), skipped by the tiny kernel
    for (int k = s_tnext; k < s_tend; ++k) tiny[(int64_t)k * 8 + 1] = 0;
}

// ---------------------------------------------------------------------------
// Tiny regression subtrees (<= 64 rows): one wavefront per subtree, one row
// per lane, presorted per-feature lane orders (the bitonic network of
// finish_tiny_sorted_kernel): srt[f][k] = {code : 8, run end : 1, -, lane : 6}
// for sorted position k, computed once per subtree (a child's rows are a
// subset of its parent's, so the order never changes).
//
// Per node, the split cost -(S_L^2 / m_L + S_R^2 / m_R) needs two fp64
// divisions and an int64 prefix per candidate; the exact form is the shared
// mse_term and must stay bit-identical to the host builders. So every feature
// is first scored in fp32 (one packed count scan, one fp32 target-sum scan, two
// v_rcp_f32 per position), and only features whose fp32 minimum lies within
// the fp32 error bound of the node's fp32 minimum are re-scored exactly (int64
// DPP prefix, mse_term). Bound, with A = sum |y| over the node: each converted
// target carries 2^-24 relative error, a 64-term fp32 prefix <= 65 * 2^-24 A,
// so S_L, S_R are off by <= 2^-17.9 A and each term S^2/m by <= 2^-16.9 A^2
// (+ 2^-22 A^2 of rounding in the square, reciprocal and product): the cost by
// <= 2^-15.8 A^2. A feature can hold the exact optimum (or a candidate whose
// gain rounds equal to it) only if its fp32 minimum is within twice that of
// the node's; the threshold uses 2^-13 A^2. Every candidate of a re-scored
// feature is compared exactly, with the (gain, feature, cost, code) order of
// the block finisher, so the tree is the host builder's bit for bit.
constexpr int kRegTinyStack = 16;
constexpr int kRegSmallNode = 16;  // nodes of 3..16 rows: one lane per feature

__host__ __device__ inline int reg_tiny_wave_bytes(int F) {
  // srt [F][64] u16 | targets [64] int64 | per-feature fp32 minima [F] | flags [64]
  return F * kWave * 2 + kWave * 8 + ((F * 4 + 15) & ~15) + kWave;
}

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int64_t dpp_i64_zero(int64_t v) {
  const uint64_t x = (uint64_t)v;
  const uint32_t lo = dpp_u32<CTRL, ROW_MASK>(0u, (uint32_t)x);
  const uint32_t hi = dpp_u32<CTRL, ROW_MASK>(0u, (uint32_t)(x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Inclusive wave64 prefix sums in DPP steps (int64 exact, fp32 approximate).
__device__ __forceinline__ int64_t wave_incl_scan_i64_dpp(int64_t v) {
  v += dpp_i64_zero<kDppRowShr + 1>(v);
  v += dpp_i64_zero<kDppRowShr + 2>(v);
  v += dpp_i64_zero<kDppRowShr + 4>(v);
  v += dpp_i64_zero<kDppRowShr + 8>(v);
  v += dpp_i64_zero<kDppRowBcast15, 0xa>(v);
  v += dpp_i64_zero<kDppRowBcast31, 0xc>(v);
  return v;
}

__device__ __forceinline__ float wave_incl_scan_f32_dpp(float v) {
  auto add = [](float x, uint32_t o) { return x + __uint_as_float(o); };
  v = add(v, dpp_u32<kDppRowShr + 1>(0u, __float_as_uint(v)));
  v = add(v, dpp_u32<kDppRowShr + 2>(0u, __float_as_uint(v)));
  v = add(v, dpp_u32<kDppRowShr + 4>(0u, __float_as_uint(v)));
  v = add(v, dpp_u32<kDppRowShr + 8>(0u, __float_as_uint(v)));
  v = add(v, dpp_u32<kDppRowBcast15, 0xa>(0u, __float_as_uint(v)));
  v = add(v, dpp_u32<kDppRowBcast31, 0xc>(0u, __float_as_uint(v)));
  return v;
}

__global__ __launch_bounds__(256) void finish_tiny_reg_kernel(
    const uint32_t* __restrict__ codes_rm, int64_t row_words, const uint32_t* __restrict__ buf0,
    const uint32_t* __restrict__ buf1, const int64_t* __restrict__ y,
    const int64_t* __restrict__ tiny, const int32_t* __restrict__ tiny_count,
    int32_t* __restrict__ tiny_counter, int F, int max_depth, int64_t mss, int64_t msl,
    int32_t* __restrict__ node_i32, int64_t* __restrict__ node_st,
    const int32_t* __restrict__ order) {
  extern __shared__ __align__(16) uint8_t dyn_reg[];
  __shared__ unsigned long long s_mask[kRegTinyWaves][kRegTinyStack];
  __shared__ int32_t s_dep[kRegTinyWaves][kRegTinyStack], s_slot[kRegTinyWaves][kRegTinyStack];
  const int lane = lane_id();
  const int wave = threadIdx.x >> 6;
  uint8_t* wb = dyn_reg + (size_t)wave * reg_tiny_wave_bytes(F);
  uint16_t* srt = reinterpret_cast<uint16_t*>(wb);
  long long* s_y = reinterpret_cast<long long*>(wb + F * kWave * 2);
  float* s_fmin = reinterpret_cast<float*>(wb + F * kWave * 2 + kWave * 8);
  uint8_t* flag = wb + F * kWave * 2 + kWave * 8 + ((F * 4 + 15) & ~15);
  const int K = *tiny_count;
  const int nwords = (F + 3) >> 2;
  const int mslw = (int)(msl < 65 ? msl : 65);
  WaveClaim claim;
  const int claim_batch = wave_claim_batch(K);
  for (;;) {
    const int k = wave_claim_next(claim, tiny_counter, K, claim_batch);
    if (k >= K) break;
    // order (optional): the records by rows descending (launch_tiny_order)
    const int64_t* rec = tiny + (int64_t)(order ? order[k] : k) * 8;
    const int64_t start = rec[0];
    const int m = (int)rec[1];
    if (m < 2) continue;  // (an unused reserved record)
    const int depth0 = (int)rec[2];
    const uint32_t* src = rec[3] ? buf1 : buf0;
    const int64_t root_slot = rec[4];
    const bool act = lane < m;
    uint32_t row = 0;
    long long yv = 0;
    if (act) {
      row = src[start + lane];
      yv = y[row];
    }
    const float yf = (float)yv;
    s_y[lane] = yv;
    // ---- presort: keys {code : 8, lane : 8} are unique, so the network is stable
    const uint32_t* rowp = codes_rm + (int64_t)row * row_words;
    int lg = 1;
    while ((1 << lg) < m) ++lg;
    for (int w = 0; w < nwords; ++w) {
      const uint32_t word = act ? rowp[w] : 0u;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int f = w * 4 + 2 * h;
        if (f >= F) break;
        const uint32_t ka = ((word >> (16 * h)) & 0xffu) << 8 | (uint32_t)lane;
        const uint32_t kb = ((word >> (16 * h + 8)) & 0xffu) << 8 | (uint32_t)lane;
        uint32_t v = act ? (ka | (kb << 16)) : 0xffffffffu;
        v = bitonic64_pk_u16(v, lane, lg);
        const uint32_t nv = (uint32_t)__shfl_down((int)v, 1, kWave);
        const bool endl = lane == m - 1;
        const uint32_t ea = (endl || ((nv >> 8) & 0xffu) != ((v >> 8) & 0xffu)) ? 0x80u : 0u;
        const uint32_t eb = (endl || (nv >> 24) != (v >> 24)) ? 0x80u : 0u;
        // positions past the subtree: lane 63 (never a node row there), no run end
        srt[f * kWave + lane] = act ? (uint16_t)((v & 0xffffu) | ea) : (uint16_t)0xff3fu;
        if (f + 1 < F)
          srt[(f + 1) * kWave + lane] = act ? (uint16_t)((v >> 16) | eb) : (uint16_t)0xff3fu;
      }
    }
    if (lane == 0) {
      s_mask[wave][0] = m == 64 ? ~0ull : ((1ull << m) - 1ull);
      s_dep[wave][0] = depth0;
      s_slot[wave][0] = (int32_t)root_slot;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int sp = 1;
    while (sp > 0) {
      --sp;
      const unsigned long long M = s_mask[wave][sp];
      const int d = s_dep[wave][sp];
      const int64_t slot = s_slot[wave][sp];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const bool mine = act && ((M >> lane) & 1ull);
      const int mm = __popcll(M);
      const int64_t S = wave_sum_i64(mine ? (int64_t)yv : 0);
      long long mn = mine ? yv : LLONG_MAX, mx = mine ? yv : LLONG_MIN;
      wave_minmax_i64(mn, mx);
      if (mn == mx) continue;  // all targets equal: leaf (record written at creation)
      int bf = -1;
      uint32_t bb = 0xffffffffu;
      unsigned long long LM = 0ull;
      if (mm == 2) {
        // Two rows (about half the internal nodes of a subtree grown to single
        // rows): the only partition is {a} | {b}, so every feature whose codes
        // differ scores the same cost bit for bit (fp64 addition commutes) and
        // the lowest such feature wins, at the smaller code -- no scans.
        const int a = __ffsll((long long)M) - 1, b = 63 - __clzll((long long)M);
        if (msl <= 1) {
          const uint32_t ra = (uint32_t)__builtin_amdgcn_readlane((int)row, a);
          const uint32_t rb = (uint32_t)__builtin_amdgcn_readlane((int)row, b);
          for (int w0 = 0; w0 < nwords; w0 += kWave) {
            const int w = w0 + lane;
            uint32_t x = 0u, wa = 0u;
            if (w < nwords) {
              wa = codes_rm[(int64_t)ra * row_words + w];
              x = wa ^ codes_rm[(int64_t)rb * row_words + w];
            }
            const unsigned long long nz = __ballot(x != 0u);
            if (nz) {
              const int wl = __ffsll((long long)nz) - 1;
              const uint32_t xw = (uint32_t)__builtin_amdgcn_readlane((int)x, wl);
              const uint32_t aw = (uint32_t)__builtin_amdgcn_readlane((int)wa, wl);
              const int byte = (__ffs((int)xw) - 1) >> 3;
              const int f = (w0 + wl) * 4 + byte;
              if (f < F) {  // (bytes past F are row padding)
                const uint32_t ca = (aw >> (8 * byte)) & 0xffu;
                const uint32_t cb = ca ^ ((xw >> (8 * byte)) & 0xffu);
                bf = f;
                bb = ca < cb ? ca : cb;
                LM = ca < cb ? (1ull << a) : (1ull << b);
              }
              break;
            }
          }
        }
        if (bf < 0) continue;  // identical rows (or min_samples_leaf > 1): leaf
      } else if (mm <= kRegSmallNode) {
        // Small node: one lane per feature. Lane f reads the node rows' codes of
        // feature f (coalesced bytes of each row) and scores every distinct
        // code as a threshold from the exact int64 left sums -- mm^2 integer
        // steps and mm exact costs per lane instead of a wave scan per feature.
        // Same exact costs and the same (gain, feature, cost, code) order.
        uint32_t rj[kRegSmallNode];
        int64_t yj[kRegSmallNode];
        unsigned long long rest = M;
#pragma unroll
        for (int t = 0; t < kRegSmallNode; ++t) {
          const int j = rest ? __ffsll((long long)rest) - 1 : 0;
          rest &= rest - 1ull;
          rj[t] = (uint32_t)__builtin_amdgcn_readlane((int)row, j);
          yj[t] = (int64_t)s_y[j];
        }
        const double pterm = mse_term(mm, S);
        double bg = -__builtin_inf(), bc = __builtin_inf();
        bf = 0x7fffffff;
        const uint8_t* cb8 = reinterpret_cast<const uint8_t*>(codes_rm);
        const int64_t rb = row_words * 4;
        for (int f0 = 0; f0 < F; f0 += kWave) {
          const int f = f0 + lane;
          uint32_t code[kRegSmallNode];
#pragma unroll
          for (int t = 0; t < kRegSmallNode; ++t)
            code[t] = (t < mm && f < F) ? (uint32_t)cb8[(int64_t)rj[t] * rb + f] : 0xffffu;
          if (f < F) {
#pragma unroll
            for (int i = 0; i < kRegSmallNode; ++i) {
              if (i >= mm) break;
              const uint32_t c = code[i];
              int ml = 0;
              int64_t sl = 0;
#pragma unroll
              for (int t = 0; t < kRegSmallNode; ++t) {
                const bool le = code[t] <= c;  // (padding entries are 0xffff: never)
                ml += le ? 1 : 0;
                sl += le ? yj[t] : 0;
              }
              const int mr = mm - ml;
              if (ml >= mslw && mr >= mslw) {
                const double cost = mse_term(ml, sl) + mse_term(mr, S - sl);
                const double g = pterm - cost;
                if (g > bg || (g == bg && (f < bf || (f == bf && (cost < bc ||
                                                               (cost == bc && c < bb)))))) {
                  bg = g;
                  bf = f;
                  bc = cost;
                  bb = c;
                }
              }
            }
          }
        }
#pragma unroll
        for (int dd = kWave / 2; dd > 0; dd >>= 1) {
          const double og = __shfl_xor(bg, dd, kWave);
          const int of = __shfl_xor(bf, dd, kWave);
          const double oc = __shfl_xor(bc, dd, kWave);
          const uint32_t ob = (uint32_t)__shfl_xor((int)bb, dd, kWave);
          const bool take =
              og > bg ||
              (og == bg && (of < bf || (of == bf && (oc < bc || (oc == bc && ob < bb)))));
          if (take) {
            bg = og;
            bf = of;
            bc = oc;
            bb = ob;
          }
        }
        bf = __builtin_amdgcn_readfirstlane(bf);
        bb = (uint32_t)__builtin_amdgcn_readfirstlane((int)bb);
        if (!(bg > -__builtin_inf()) || bf < 0 || bf >= F) continue;
        {
          const uint32_t v = srt[bf * kWave + lane];
          if (act) flag[v & 0x3fu] = (uint8_t)((v >> 8) <= bb);
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
        LM = M & __ballot(act && flag[lane]);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      } else {
        // ---- pass 1: fp32 minimum cost of every feature
        const float ym = mine ? yf : 0.0f;
        const float Sf = (float)S;
        const float Af = __uint_as_float((uint32_t)__builtin_amdgcn_readlane(
            (int)__float_as_uint(wave_incl_scan_f32_dpp(fabsf(ym))), 63));
        const float fmm = (float)mm;
        float nmin = __builtin_inff();
        auto approx = [&](uint32_t v, uint32_t ml, float sl) -> float {
          const float fl = (float)ml, fr = fmm - fl, sr = Sf - sl;
          const bool ok = (v & 0x80u) && (int)ml >= mslw && mm - (int)ml >= mslw;
          const float c = -((sl * sl) * __builtin_amdgcn_rcpf(fl) +
                            (sr * sr) * __builtin_amdgcn_rcpf(fr));
          return ok ? c : __builtin_inff();
        };
        for (int f = 0; f < F; f += 2) {
          const bool two = f + 1 < F;
          const uint32_t va = srt[f * kWave + lane];
          const uint32_t vb = two ? (uint32_t)srt[(f + 1) * kWave + lane] : 0xff3fu;
          const uint32_t sa = va & 0x3fu, sb = vb & 0x3fu;
          const uint32_t ia = (uint32_t)(M >> sa) & 1u, ib = (uint32_t)(M >> sb) & 1u;
          const float ya = __shfl(ym, (int)sa, kWave), yb = __shfl(ym, (int)sb, kWave);
          const uint32_t cnt = wave_incl_scan_dpp(ia | (ib << 16));
          const float sla = wave_incl_scan_f32_dpp(ya), slb = wave_incl_scan_f32_dpp(yb);
          const float fa = wave_min_f32_dpp(approx(va, cnt & 0xffffu, sla));
          const float fb = wave_min_f32_dpp(approx(vb, cnt >> 16, slb));
          if (lane == 0) {
            s_fmin[f] = fa;
            if (two) s_fmin[f + 1] = fb;
          }
          nmin = fminf(nmin, two ? fminf(fa, fb) : fa);
        }
        if (!(nmin < __builtin_inff())) continue;  // no admissible split: leaf
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const float thr = nmin + 0x1p-13f * (Af * Af);
        // ---- pass 2: exact costs of the features that can hold the optimum
        const double pterm = mse_term(mm, S);
        double bg = -__builtin_inf(), bc = __builtin_inf();
        bf = 0x7fffffff;
        for (int f = 0; f < F; ++f) {
          if (!(s_fmin[f] <= thr)) continue;  // wave-uniform
          const uint32_t v = srt[f * kWave + lane];
          const uint32_t s = v & 0x3fu;
          const uint32_t in = (uint32_t)(M >> s) & 1u;
          const int64_t ys = in ? (int64_t)s_y[s] : 0;
          const int ml = (int)wave_incl_scan_dpp(in);
          const int64_t sl = wave_incl_scan_i64_dpp(ys);
          const int mr = mm - ml;
          double cost = __builtin_inf();
          if ((v & 0x80u) && ml >= mslw && mr >= mslw)
            cost = mse_term(ml, sl) + mse_term(mr, S - sl);
          const double g = pterm - cost;
          if (g > bg) {  // features ascend: strict > keeps the lowest
            bg = g;
            bf = f;
            bc = cost;
            bb = v >> 8;
          }
        }
#pragma unroll
        for (int dd = kWave / 2; dd > 0; dd >>= 1) {
          const double og = __shfl_xor(bg, dd, kWave);
          const int of = __shfl_xor(bf, dd, kWave);
          const double oc = __shfl_xor(bc, dd, kWave);
          const uint32_t ob = (uint32_t)__shfl_xor((int)bb, dd, kWave);
          const bool take =
              og > bg ||
              (og == bg && (of < bf || (of == bf && (oc < bc || (oc == bc && ob < bb)))));
          if (take) {
            bg = og;
            bf = of;
            bc = oc;
            bb = ob;
          }
        }
        bf = __builtin_amdgcn_readfirstlane(bf);
        bb = (uint32_t)__builtin_amdgcn_readfirstlane((int)bb);
        if (!(bg > -__builtin_inf()) || bf < 0) continue;
        // left rows: sorted positions of feature bf with code <= bb, scattered back to lanes
        {
          const uint32_t v = srt[bf * kWave + lane];
          if (act) flag[v & 0x3fu] = (uint8_t)((v >> 8) <= bb);
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
        LM = M & __ballot(act && flag[lane]);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      const unsigned long long RM = M & ~LM;
      const int nl = __popcll(LM), nr = __popcll(RM);
      // a split always leaves rows on both sides; anything else is a kernel bug --
      // stop here instead of re-splitting into positions outside the subtree
      if (nl == 0 || nr == 0) continue;
      const int64_t ls = slot + 1, rs = slot + 2 * nl;
      const int64_t SL = wave_sum_i64(((LM >> lane) & 1ull) ? (int64_t)yv : 0);
      const int cd = d + 1;
      if (lane == 0) {
        int32_t* P = node_i32 + slot * 6;
        P[0] = bf;
        P[1] = (int32_t)bb;
        P[2] = (int32_t)ls;
        P[3] = (int32_t)rs;
        int32_t* L = node_i32 + ls * 6;
        int32_t* Rr = node_i32 + rs * 6;
        L[0] = -1; L[1] = -1; L[2] = -1; L[3] = -1; L[4] = cd; L[5] = nl;
        Rr[0] = -1; Rr[1] = -1; Rr[2] = -1; Rr[3] = -1; Rr[4] = cd; Rr[5] = nr;
        node_st[ls * 2 + 0] = nl;
        node_st[ls * 2 + 1] = SL;
        node_st[rs * 2 + 0] = nr;
        node_st[rs * 2 + 1] = S - SL;
      }
      const bool depth_stop = max_depth >= 0 && cd >= max_depth;
      const bool tlf = depth_stop || nl < mss || nl < 2 * msl;
      const bool trf = depth_stop || nr < mss || nr < 2 * msl;
      const bool left_small = nl <= nr;
      for (int pass = 0; pass < 2; ++pass) {
        const bool is_left = (pass == 0) ? !left_small : left_small;
        if (is_left ? tlf : trf) continue;
        if (lane == 0) {
          s_mask[wave][sp] = is_left ? LM : RM;
          s_dep[wave][sp] = cd;
          s_slot[wave][sp] = (int32_t)(is_left ? ls : rs);
        }
        ++sp;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

int finish_reg_lds_bytes(int B) { return kRegFT * B * 12; }

// Resident block-finisher workgroups per CU for B bins (LDS tile and VGPRs): the
// persistent grid is this many per CU (1M x 64, B = 256: 3 per CU, 9.35 -> 8.83
// ms per fit against the former fixed 2).
int finish_reg_blocks_per_cu(int B, int code_bytes) {
  const void* k = code_bytes == 1 ? (const void*)finish_reg_kernel<uint8_t>
                                  : (const void*)finish_reg_kernel<uint16_t>;
  const int lds = finish_reg_lds_bytes(B);
  MT_HIP_CHECK(mt_set_max_lds(k, lds));
  int per_cu = 0;
  MT_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kRegThreads, lds));
  return per_cu < 1 ? 1 : per_cu;
}

static int reg_env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// counter: int32 [4] = {job cursor, tiny count, tiny cursor, -}, zeroed by the host.
void launch_finish_reg(hipStream_t stream, const void* codes_rm, int64_t row_words,
                       const void* codes_fm, int code_bytes, int64_t n_rows, uint32_t* buf0,
                       uint32_t* buf1, const int64_t* y, const int64_t* jobs, int J,
                       int32_t* counter, const int32_t* nbins, int F, int B, int max_depth,
                       int64_t mss, int64_t msl, int32_t* node_i32, int64_t* node_st, int grid,
                       int tiny_rows, int64_t* tiny, int tiny_grid, int64_t* tasks,
                       int32_t* task_flag, int32_t epoch, int task_cap, int32_t* tiny_order) {
  if (J <= 0) return;
  if (code_bytes != 1) tiny_rows = 0;
  // the tiny kernel keeps every feature's lane order in LDS: workgroups of fewer
  // waves past 4 x that (2 waves up to ~590 features, 1 up to ~1180; the grid keeps
  // the total wave count), and past one wave's worth the block kernel grows the
  // subtrees to the leaves (MPITREE_REG_TINY_WAVES caps the width: A/B)
  int tw = std::max(1, std::min(kRegTinyWaves, reg_env_int("MPITREE_REG_TINY_WAVES",
                                                          kRegTinyWaves)));
  while (tw > 1 && (size_t)tw * reg_tiny_wave_bytes(F) > 160 * 1024) tw >>= 1;
  if ((size_t)tw * reg_tiny_wave_bytes(F) > 160 * 1024 ||
      (tw < kRegTinyWaves && reg_env_int("MPITREE_REG_TINY_NARROW", 1) == 0))
    tiny_rows = 0;
  tiny_rows = std::min(tiny_rows, kRegTinyRows);
  const size_t lds = (size_t)finish_reg_lds_bytes(B);
#define MT_FR(CT)                                                                           \
  MT_HIP_CHECK(mt_set_max_lds((const void*)finish_reg_kernel<CT>,                      \
                                   (int)lds));  \
  hipLaunchKernelGGL(finish_reg_kernel<CT>, dim3(grid), dim3(kRegThreads), lds, stream,     \
                     (const uint32_t*)codes_rm, row_words, (const CT*)codes_fm, n_rows, buf0, \
                     buf1, y, jobs, J, counter, nbins, F, B, max_depth, mss, msl, node_i32,  \
                     node_st, tiny_rows, tiny, counter + 1, tasks, task_flag, epoch, task_cap);
  if (code_bytes == 1) {
    MT_FR(uint8_t)
  } else {
    MT_FR(uint16_t)
  }
#undef MT_FR
  MT_HIP_CHECK(hipGetLastError());
  if (tiny_rows > 0) {
    const size_t tl = (size_t)tw * reg_tiny_wave_bytes(F);
    const int tg = std::max(1, tiny_grid * kRegTinyWaves / tw);
    MT_HIP_CHECK(mt_set_max_lds((const void*)finish_tiny_reg_kernel, (int)tl));
    int32_t* order = nullptr;  // (tiny_order: [2 * 65] scratch, then the order)
    if (tiny_order) {
      order = tiny_order + 2 * 65;
      launch_tiny_order(stream, tiny, counter + 1, tiny_order, order, 128);
    }
    hipLaunchKernelGGL(finish_tiny_reg_kernel, dim3(tg), dim3(tw * kWave), tl,
                       stream, (const uint32_t*)codes_rm, row_words, buf0, buf1, y, tiny,
                       counter + 1, counter + 2, F, max_depth, mss, msl, node_i32, node_st,
                       order);
    MT_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace mt
