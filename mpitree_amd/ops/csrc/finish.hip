// Subtree finisher: one workgroup grows an entire small subtree on gfx950.
//
// The reference recurses node by node to the leaves
// (mpitree/tree/decision_tree.py:150-164), and its parallel version hands
// whole subtrees to MPI sub-communicators (:446-477). Here, once a frontier
// node has at most ``finisher_rows`` rows, the level-wise engine stops
// launching per-level kernels for it and enqueues it as a *job*; a persistent
// grid of 256-thread workgroups (two per CU, so each CU overlaps two
// independent node pipelines) pulls jobs, largest first, from an atomic
// counter and grows each subtree depth-first with no further launches or
// host round trips:
//
//   per node: LDS histogram of all features (two 16-bit classes per word) ->
//   wave-per-feature prefix scan with the shared integer-form criterion and
//   an LDS-resident x*log2(x) table -> workgroup argmax (ties: lowest
//   feature) -> unstable partition of the node's rows from one row buffer
//   into the other (ping-pong, no copy-back) -> child records, terminal
//   checks, push the larger child first so the DFS stack stays O(log rows).
//
// Class counts travel on the DFS stack (known from the parent's split), so a
// node needs five workgroup barriers. Node ids are local to the job and
// allocated in processing order, which depends only on the data, so results
// are deterministic; the host re-numbers the tree into pre-order. Every job
// owns a disjoint output region of 2*rows-1 node slots.
#include "common.h"
#include "criterion.h"

namespace mt {

constexpr int kFinThreads = 256;
constexpr int kFinWaves = kFinThreads / kWave;
constexpr int kFinStack = 40;    // >= log2(max job rows) + 2
constexpr int kFinMaxC = 16;     // classes supported by the finisher
constexpr int kFinTab = 1024;    // LDS x*log2(x) entries

struct FinRowLab {
  uint32_t mask;
  int shift;
};

// jobs: int64 [J][5 + C] = {start, count, depth, base, buffer, counts[C]}
// node_i32: [slots][6] = {feature, bin, left, right, depth, n}; node_cnt: [slots][C]
template <typename CodeT>
__global__ __launch_bounds__(kFinThreads, 2) void finish_cls_kernel(
    const uint32_t* __restrict__ codes_rm, int64_t row_words, const CodeT* __restrict__ codes_fm,
    int64_t n_rows, uint32_t* __restrict__ buf0, uint32_t* __restrict__ buf1,
    const int32_t* __restrict__ y, FinRowLab rl, const int64_t* __restrict__ jobs, int J,
    int32_t* __restrict__ job_counter, const int32_t* __restrict__ nbins, int F, int B, int C,
    int crit, int max_depth, int64_t mss, int64_t msl, const double* __restrict__ xtab,
    int xtab_n, int32_t* __restrict__ node_i32, int32_t* __restrict__ node_cnt,
    int32_t* __restrict__ job_nodes) {
  extern __shared__ __align__(16) uint32_t hist[];  // [F][B*W + 1] packed class pairs
  __shared__ double s_tab[kFinTab];
  __shared__ int s_job;
  __shared__ int64_t s_st_start[kFinStack];
  __shared__ int32_t s_st_count[kFinStack], s_st_depth[kFinStack], s_st_id[kFinStack];
  __shared__ int32_t s_st_buf[kFinStack];
  __shared__ int32_t s_st_cnt[kFinStack][kFinMaxC];
  __shared__ int s_sp, s_next;
  __shared__ int64_t s_start;
  __shared__ int32_t s_count, s_depth, s_id, s_buf;
  __shared__ int32_t s_cnt[kFinMaxC], s_left[kFinMaxC];
  __shared__ double s_pterm;
  __shared__ double w_gain[kFinWaves];
  __shared__ int w_feat[kFinWaves], w_bin[kFinWaves];
  __shared__ int s_bf, s_bb;
  __shared__ int s_lc, s_rc;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = lane_id();
  const int W = (C + 1) >> 1;
  const int fstride = B * W + 1;
  constexpr int cpw = 4 / sizeof(CodeT);
  const int words = (F + cpw - 1) / cpw;
  const int tn = min(kFinTab, xtab_n);
  const int JW = 5 + C;

  for (int i = tid; i < tn; i += kFinThreads) s_tab[i] = xtab[i];
  for (int e = tid; e < F * fstride; e += kFinThreads) hist[e] = 0u;

  auto tl = [&](uint64_t x) -> double {
    return x < (uint64_t)tn ? s_tab[x] : (x < (uint64_t)xtab_n ? __ldg(xtab + x) : xlog2x(x));
  };

  for (;;) {
    if (tid == 0) s_job = atomicAdd(job_counter, 1);
    __syncthreads();
    const int job = s_job;
    if (job >= J) break;
    const int64_t* jb = jobs + (int64_t)job * JW;
    const int64_t base = jb[3];
    int32_t* ni = node_i32 + base * 6;
    int32_t* nc = node_cnt + base * C;
    if (tid == 0) {
      s_sp = 1;
      s_st_start[0] = jb[0];
      s_st_count[0] = (int32_t)jb[1];
      s_st_depth[0] = (int32_t)jb[2];
      s_st_id[0] = 0;
      s_st_buf[0] = (int32_t)jb[4];
      s_next = 1;
      ni[0] = -1;
      ni[1] = -1;
      ni[2] = -1;
      ni[3] = -1;
      ni[4] = (int32_t)jb[2];
      ni[5] = (int32_t)jb[1];
    }
    if (tid < C) {
      s_st_cnt[0][tid] = (int32_t)jb[5 + tid];
      nc[tid] = (int32_t)jb[5 + tid];
    }
    __syncthreads();
    while (s_sp > 0) {
      __syncthreads();  // everyone has read s_sp before thread 0 pops
      // ---- pop + node term (thread 0); the histogram is already zero
      if (tid == 0) {
        const int sp = --s_sp;
        s_start = s_st_start[sp];
        s_count = s_st_count[sp];
        s_depth = s_st_depth[sp];
        s_id = s_st_id[sp];
        s_buf = s_st_buf[sp];
        double acc = 0.0;
        int64_t mm = 0, sq = 0;
        for (int c = 0; c < C; ++c) {
          const int64_t t = s_st_cnt[sp][c];
          s_cnt[c] = (int32_t)t;
          mm += t;
          acc = acc + tl((uint64_t)t);
          sq += t * t;
        }
        s_pterm = crit == kEntropy ? tl((uint64_t)mm) - acc : gini_term(mm, sq);
        s_lc = 0;
        s_rc = 0;
      }
      __syncthreads();
      const int64_t start = s_start;
      const int m = s_count;
      const int depth = s_depth;
      const int id = s_id;
      uint32_t* __restrict__ src = s_buf ? buf1 : buf0;
      uint32_t* __restrict__ dst = s_buf ? buf0 : buf1;
      // ---- histogram of this node's rows (all features)
      for (int e = tid; e < m * words; e += kFinThreads) {
        const int r = e / words;
        const int wi = e - r * words;
        const uint32_t ent = src[start + r];
        const uint32_t row = rl.shift ? (ent & rl.mask) : ent;
        const int lab = rl.shift ? (int)(ent >> rl.shift) : y[row];
        const uint32_t wv = codes_rm[(int64_t)row * row_words + wi];
        const uint32_t inc = 1u << ((lab & 1) * 16);
#pragma unroll
        for (int j = 0; j < cpw; ++j) {
          const int f = wi * cpw + j;
          if (f < F) {
            const uint32_t code =
                (wv >> (j * 8 * sizeof(CodeT))) & ((sizeof(CodeT) == 1) ? 0xffu : 0xffffu);
            atomicAdd(&hist[f * fstride + (int)code * W + (lab >> 1)], inc);
          }
        }
      }
      __syncthreads();
      const double pterm = s_pterm;
      // ---- wave-per-feature scan (B <= 256: one 256-bin pass)
      double bg = -__builtin_inf();
      int bfeat = 0x7fffffff, bbin = -1;
      for (int f = wave; f < F; f += kFinWaves) {
        const int nb = min(B, nbins[f]);
        const uint32_t* h = hist + f * fstride;
        double best_cost = __builtin_inf();
        int best_bin = 0x7fffffff;
        const int b0 = lane * 4;
        uint32_t mL[4] = {0, 0, 0, 0}, ne[4] = {0, 0, 0, 0};
        double sL[4] = {0.0, 0.0, 0.0, 0.0}, sR[4] = {0.0, 0.0, 0.0, 0.0};
        int64_t qL[4] = {0, 0, 0, 0}, qR[4] = {0, 0, 0, 0};
        for (int w = 0; w < W; ++w) {
          uint32_t vlo[4], vhi[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int b = b0 + k;
            const uint32_t v = b < nb ? h[b * W + w] : 0u;
            vlo[k] = v & 0xffffu;
            vhi[k] = v >> 16;
          }
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int c = 2 * w + half;
            if (c >= C) break;
            const uint32_t* vv = half ? vhi : vlo;
            uint32_t p[4];
            p[0] = vv[0];
            p[1] = p[0] + vv[1];
            p[2] = p[1] + vv[2];
            p[3] = p[2] + vv[3];
            const uint32_t incl = wave_incl_scan_dpp(p[3]);
            const uint32_t excl = incl - p[3];
            const uint32_t tc = (uint32_t)s_cnt[c];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t L = excl + p[k];
              const uint32_t R = tc - L;
              mL[k] += L;
              ne[k] |= vv[k];
              if (crit == kEntropy) {
                sL[k] = sL[k] + tl(L);
                sR[k] = sR[k] + tl(R);
              } else {
                qL[k] += (int64_t)L * L;
                qR[k] += (int64_t)R * R;
              }
            }
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int b = b0 + k;
          const int64_t ml = mL[k];
          const int64_t mr = (int64_t)m - ml;
          if (b < nb && ne[k] && ml >= msl && mr >= msl) {
            double cost;
            if (crit == kEntropy)
              cost = (tl((uint64_t)ml) - sL[k]) + (tl((uint64_t)mr) - sR[k]);
            else
              cost = gini_term(ml, qL[k]) + gini_term(mr, qR[k]);
            if (cost < best_cost) {
              best_cost = cost;
              best_bin = b;
            }
          }
        }
        wave_argmin_dpp(best_cost, best_bin);  // single 256-bin pass: lanes own ascending bins
        if (best_cost < __builtin_inf()) {
          const double g = pterm - best_cost;
          if (g > bg) {  // features visited in increasing order: strict > keeps the lowest
            bg = g;
            bfeat = f;
            bbin = best_bin;
          }
        }
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
        for (int w = 1; w < kFinWaves; ++w) {
          if (w_gain[w] > g || (w_gain[w] == g && w_feat[w] < bf)) {
            g = w_gain[w];
            bf = w_feat[w];
            bb = w_bin[w];
          }
        }
        if (!(g > -__builtin_inf())) bf = -1;
      }
      if (bf >= 0) {
        // ---- left class counts of the winning split
        for (int c = wave; c < C; c += kFinWaves) {
          uint32_t s = 0;
          const uint32_t* h = hist + bf * fstride;
          for (int b = lane; b <= bb; b += kWave) {
            const uint32_t v = h[b * W + (c >> 1)];
            s += (c & 1) ? (v >> 16) : (v & 0xffffu);
          }
          s = wave_sum_u32(s);
          if (lane == 0) s_left[c] = (int32_t)s;
        }
        // ---- partition rows src -> dst (unstable; left from the front, right from the back)
        const CodeT* col = codes_fm + (int64_t)bf * n_rows;
        for (int r0 = 0; r0 < m; r0 += kFinThreads) {
          const int r = r0 + tid;
          const bool valid = r < m;
          const uint32_t ent = valid ? src[start + r] : 0u;
          const bool go = valid && (uint32_t)col[ent & rl.mask] <= (uint32_t)bb;
          const unsigned long long bl = __ballot(go);
          const unsigned long long br = __ballot(valid && !go);
          const unsigned long long lt = (1ull << lane) - 1ull;
          int basel = 0, baser = 0;
          if (lane == 0) {
            const int nl = __popcll(bl), nr = __popcll(br);
            basel = nl ? atomicAdd(&s_lc, nl) : 0;
            baser = nr ? atomicAdd(&s_rc, nr) : 0;
          }
          basel = __shfl(basel, 0, kWave);
          baser = __shfl(baser, 0, kWave);
          if (valid) {
            if (go)
              dst[start + basel + __popcll(bl & lt)] = ent;
            else
              dst[start + m - 1 - (baser + __popcll(br & lt))] = ent;
          }
        }
      }
      __syncthreads();
      // ---- clear the histogram for the next node (all scan reads are done)
      for (int e = tid; e < F * fstride; e += kFinThreads) hist[e] = 0u;
      // ---- children
      if (tid == 0 && bf >= 0) {
        const int nl = s_lc;
        const int nr = m - nl;
        const int lid = s_next, rid = s_next + 1;
        s_next += 2;
        ni[id * 6 + 0] = bf;
        ni[id * 6 + 1] = bb;
        ni[id * 6 + 2] = lid;
        ni[id * 6 + 3] = rid;
        int nzl = 0, nzr = 0;
        for (int c = 0; c < C; ++c) {
          const int32_t lc = s_left[c], rc = s_cnt[c] - s_left[c];
          nc[lid * C + c] = lc;
          nc[rid * C + c] = rc;
          nzl += lc > 0;
          nzr += rc > 0;
        }
        const int cd = depth + 1;
        const bool depth_stop = max_depth >= 0 && cd >= max_depth;
        const bool tlf = depth_stop || nl < mss || nl < 2 * msl || nzl <= 1;
        const bool trf = depth_stop || nr < mss || nr < 2 * msl || nzr <= 1;
        int32_t* L = ni + lid * 6;
        int32_t* Rr = ni + rid * 6;
        L[0] = -1; L[1] = -1; L[2] = -1; L[3] = -1; L[4] = cd; L[5] = nl;
        Rr[0] = -1; Rr[1] = -1; Rr[2] = -1; Rr[3] = -1; Rr[4] = cd; Rr[5] = nr;
        // push the larger child first so the smaller one is processed next
        const bool left_small = nl <= nr;
        for (int pass = 0; pass < 2; ++pass) {
          const bool is_left = (pass == 0) ? !left_small : left_small;
          if (is_left ? tlf : trf) continue;
          const int sp = s_sp++;
          s_st_start[sp] = is_left ? start : start + nl;
          s_st_count[sp] = is_left ? nl : nr;
          s_st_depth[sp] = cd;
          s_st_id[sp] = is_left ? lid : rid;
          s_st_buf[sp] = s_buf ^ 1;
          for (int c = 0; c < C; ++c)
            s_st_cnt[sp][c] = is_left ? s_left[c] : s_cnt[c] - s_left[c];
        }
      }
      __syncthreads();
    }
    if (tid == 0) job_nodes[job] = s_next;
    __syncthreads();
  }
}

int finish_lds_bytes(int F, int B, int C) { return F * (B * ((C + 1) / 2) + 1) * 4; }
int finish_max_classes() { return kFinMaxC; }

void launch_finish(hipStream_t stream, const void* codes_rm, int64_t row_words,
                   const void* codes_fm, int code_bytes, int64_t n_rows, uint32_t* buf0,
                   uint32_t* buf1, const int32_t* y, int lab_shift, const int64_t* jobs, int J,
                   int32_t* counter, const int32_t* nbins, int F, int B, int C, int crit,
                   int max_depth, int64_t mss, int64_t msl, const double* xtab, int xtab_n,
                   int32_t* node_i32, int32_t* node_cnt, int32_t* job_nodes, int grid) {
  if (J <= 0) return;
  if (C > kFinMaxC) throw std::runtime_error("finisher supports at most 16 classes");
  FinRowLab rl{lab_shift ? ((1u << lab_shift) - 1u) : 0xffffffffu, lab_shift};
  const size_t lds = (size_t)finish_lds_bytes(F, B, C);
#define MT_FIN(CT)                                                                            \
  MT_HIP_CHECK(hipFuncSetAttribute((const void*)finish_cls_kernel<CT>,                        \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));    \
  hipLaunchKernelGGL(finish_cls_kernel<CT>, dim3(grid), dim3(kFinThreads), lds, stream,       \
                     (const uint32_t*)codes_rm, row_words, (const CT*)codes_fm, n_rows, buf0, \
                     buf1, y, rl, jobs, J, counter, nbins, F, B, C, crit, max_depth, mss,     \
                     msl, xtab, xtab_n, node_i32, node_cnt, job_nodes);
  if (code_bytes == 1) {
    MT_FIN(uint8_t)
  } else {
    MT_FIN(uint16_t)
  }
#undef MT_FIN
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
