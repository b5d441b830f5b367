// Per-node feature histograms on gfx950.
//
// Replaces the reference's per-threshold masking + row copies + np.unique
// entropy loop (mpitree/tree/decision_tree.py:73-86): one pass over a node's
// rows accumulates [F, B, C] class counts, after which every threshold's left
// and right class distributions are prefix sums (split_scan.hip).
//
// Design (CDNA4):
//  * rows of a node are addressed through the row permutation ``idx``. For
//    classification with n < 2^24 rows and <= 256 classes the label rides in
//    the top byte of the permutation entry (row | label << 24), so one
//    coalesced 4-B load yields both and no label gather is needed;
//  * the row-major code matrix is read with 16-B loads (4 lanes per 64-B row
//    for 64 u8 features), each lane keeping 4 rows in flight, so a 512-thread
//    workgroup has 512 row gathers outstanding to hide HBM/L2 latency;
//  * each workgroup privatises the histogram of its feature tile in LDS.
//    Classification packs two classes per 32-bit LDS word (16-bit halves; a
//    work item is at most 65535 rows so a half never overflows), halving LDS
//    footprint and atomics; the feature stride is padded by one word so lanes
//    of one row with equal codes land in different banks;
//  * no global atomics on the hot path: a work item that covers a whole node
//    writes the final histogram with plain stores; items of a multi-item node
//    write their packed LDS image to a private slab, and ``hist_reduce``
//    sums groups of slabs in parallel (integer sums: order-free, bitwise
//    deterministic);
//  * histograms that cannot fit one feature in LDS (very large B*C) fall back
//    to direct global atomics.
#include "common.h"

#ifndef MT_HIST_ROWS_CAP  // class-tiled histograms: capped item row (A/B: 0)
#define MT_HIST_ROWS_CAP 1
#endif
#ifndef MT_RED_ROWS_CAP  // device-planned slab reduction: capped row count (A/B: 0)
#define MT_RED_ROWS_CAP 1
#endif

namespace mt {

constexpr int kHistThreads = 512;
constexpr int kUnroll = 4;  // rows in flight per lane

struct RowLab {
  uint32_t mask;
  int shift;  // > 0: label packed in the permutation entry
};

// items: int64 [n_items][4] = {slot, start, count, dest}; dest < 0 -> unpack
// into hist[slot], dest >= 0 -> raw packed LDS image into slab[dest].
template <typename CodeT, int VEC>
__global__ __launch_bounds__(kHistThreads) void hist_cls_lds_kernel(
    const uint32_t* __restrict__ codes, int64_t row_words, const uint32_t* __restrict__ idx,
    const int32_t* __restrict__ y, RowLab rl, const int64_t* __restrict__ items,
    uint32_t* __restrict__ hist, uint32_t* __restrict__ slab, int F_h, int f_lo, int B, int C,
    int ft, int lane_shift, const int32_t* __restrict__ dcount, const int64_t* __restrict__ zred,
    const int32_t* __restrict__ zcount, int64_t zE, int ct) {
  // ct: classes per LDS tile (C: no class tiling). With many classes a single
  // feature's [B][C] counts exceed the LDS budget: grid.y then covers feature
  // tiles x class tiles of ct classes (ct even), each workgroup counting the rows
  // whose label falls in its class range (the codes are read once per tile)
  // zred (optional, device-planned levels): zero the multi-item slots {slot, -, -}
  // [*zcount] that the following slab reduction adds into -- one launch less per
  // level. This kernel writes single-item slots and slabs only, never a zred slot.
  // The zeroing is spread over the active workgroups (at least one).
  if (zred) {
    const int act = max(1, dcount ? min(*dcount, (int)gridDim.x) : (int)gridDim.x);
    if ((int)blockIdx.x < act) {
      const int64_t per = zE >> 2;  // uint4 per slot (zE % 4 == 0, host-checked)
      const int64_t total = (int64_t)(*zcount) * per;
      const int64_t stride = (int64_t)act * gridDim.y * blockDim.x;
      for (int64_t i = ((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * blockDim.x + threadIdx.x;
           i < total; i += stride) {
        const int64_t z = i / per;
        reinterpret_cast<uint4*>(hist + zred[z * 3] * zE)[i - z * per] = make_uint4(0, 0, 0, 0);
      }
    }
  }
  // dcount (optional): device-side item count; the grid is an upper bound, or (the
  // class-tiled launch) a capped row of workgroups that strides over the items
  const int n_it = dcount ? *dcount : (int)gridDim.x;
  if ((int)blockIdx.x >= n_it) return;
  extern __shared__ uint32_t lds[];
  constexpr int cpw = 4 / sizeof(CodeT);  // codes per 32-bit word
  const int n_ct = (C + ct - 1) / ct;
  const int c_tile = (int)blockIdx.y % n_ct;
  const int c_lo = c_tile * ct, c_hi = min(C, c_lo + ct);
  const int W = (c_hi - c_lo + 1) >> 1;  // words of this tile's classes
  const int Wall = (C + 1) >> 1;         // words of every class (slab layout)
  const int fstride = B * W + 1;
  const int t0 = (int)(blockIdx.y / n_ct) * ft;
  const int t1 = min(F_h, t0 + ft);
  const int nf = t1 - t0;
  const int g0 = f_lo + t0, g1 = f_lo + t1;
  const int gw0 = (g0 / cpw) & ~(VEC - 1);  // first (VEC-aligned) code word
  const int nwords = (g1 + cpw - 1) / cpw - gw0;
  for (int it = blockIdx.x; it < n_it; it += gridDim.x) {
  const int64_t slot = items[it * 4 + 0];
  const int64_t start = items[it * 4 + 1];
  const int64_t count = items[it * 4 + 2];
  const int64_t dest = items[it * 4 + 3];

  const int lds_words = nf * fstride;
  for (int e = threadIdx.x; e < lds_words; e += blockDim.x) lds[e] = 0u;
  __syncthreads();

  const int L = 1 << lane_shift;  // lanes per row
  const int sub = threadIdx.x & (L - 1);
  const int rpp = blockDim.x >> lane_shift;  // rows per block pass
  const int my_w = gw0 + sub * VEC;
  const bool active = sub * VEC < nwords;
  for (int64_t base = threadIdx.x >> lane_shift; base < count; base += (int64_t)rpp * kUnroll) {
    uint32_t ent[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t r = base + (int64_t)u * rpp;
      ent[u] = (active && r < count) ? idx[start + r] : 0xffffffffu;
    }
    uint32_t w[kUnroll][VEC];
    int lab[kUnroll];
    // every row gather of the unrolled rows in flight before the first use: the
    // loads are unconditional (an absent row reads row 0) -- a guarded load made
    // the compiler wait for each row's gather in turn
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const bool ok = ent[u] != 0xffffffffu;
      const uint32_t row = ok ? (rl.shift ? (ent[u] & rl.mask) : ent[u]) : 0u;
      lab[u] = rl.shift ? (int)(ent[u] >> rl.shift) : y[row];
      if constexpr (VEC == 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(codes + (int64_t)row * row_words + my_w);
        w[u][0] = v.x;
        w[u][1] = v.y;
        w[u][2] = v.z;
        w[u][3] = v.w;
      } else {
        w[u][0] = codes[(int64_t)row * row_words + my_w];
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (ent[u] == 0xffffffffu || lab[u] < c_lo || lab[u] >= c_hi) continue;
      const int lt = lab[u] - c_lo;  // (c_lo even: the class keeps its half-word)
      const uint32_t inc = 1u << ((lt & 1) * 16);
      const int off = lt >> 1;
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
#pragma unroll
        for (int j = 0; j < cpw; ++j) {
          const int gf = (my_w + v) * cpw + j;
          if (gf >= g0 && gf < g1) {
            const uint32_t code = (w[u][v] >> (j * 8 * sizeof(CodeT))) &
                                  ((sizeof(CodeT) == 1) ? 0xffu : 0xffffu);
            atomicAdd(&lds[(gf - g0) * fstride + (int)code * W + off], inc);
          }
        }
      }
    }
  }
  __syncthreads();

  const int per_f = B * W;
  if (dest >= 0) {  // packed image -> slab [F_h][B][Wall] (this tile's words of it)
    uint32_t* out = slab + dest * (int64_t)F_h * B * Wall + (int64_t)t0 * B * Wall;
    for (int e = threadIdx.x; e < nf * per_f; e += blockDim.x) {
      const int f = e / per_f;
      const int rem = e - f * per_f;
      const int b = rem / W;
      const int w = rem - b * W;
      out[((int64_t)f * B + b) * Wall + (c_lo >> 1) + w] = lds[f * fstride + rem];
    }
  } else {
    uint32_t* out = hist + slot * (int64_t)F_h * B * C;
    for (int e = threadIdx.x; e < nf * per_f; e += blockDim.x) {
      const int f = e / per_f;
      const int rem = e - f * per_f;
      const int b = rem / W;
      const int wc = rem - b * W;
      const uint32_t v = lds[f * fstride + rem];
      const int c = c_lo + 2 * wc;
      const int64_t o = ((int64_t)(t0 + f) * B + b) * C + c;
      out[o] = v & 0xffffu;
      if (c + 1 < c_hi) out[o + 1] = v >> 16;
    }
  }
  __syncthreads();  // (the next item zeroes the LDS image these loops read)
  }
}

// Regression payload: per bin {count, fixed-point target sum} as two int64.
template <typename CodeT>
__global__ __launch_bounds__(kHistThreads) void hist_reg_lds_kernel(
    const CodeT* __restrict__ codes, int64_t row_words, const uint32_t* __restrict__ idx,
    const int64_t* __restrict__ y, const int64_t* __restrict__ items,
    int64_t* __restrict__ hist, int64_t* __restrict__ slab, int F_h, int f_lo, int B, int ft,
    int lane_shift, const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.x >= *dcount) return;
  extern __shared__ uint32_t lds[];
  constexpr int cpw = 4 / sizeof(CodeT);
  const int t0 = blockIdx.y * ft;
  const int t1 = min(F_h, t0 + ft);
  const int nf = t1 - t0;
  const int g0 = f_lo + t0, g1 = f_lo + t1;
  const int gw0 = g0 / cpw;
  const int nwords = (g1 + cpw - 1) / cpw - gw0;
  const int64_t slot = items[blockIdx.x * 4 + 0];
  const int64_t start = items[blockIdx.x * 4 + 1];
  const int64_t count = items[blockIdx.x * 4 + 2];
  const int64_t dest = items[blockIdx.x * 4 + 3];
  // layout: sums (u64) [nf][B] first (8-B aligned), then counts (u32) [nf][B+1]
  unsigned long long* sums = reinterpret_cast<unsigned long long*>(lds);
  uint32_t* cnts = lds + 2 * nf * B;
  const int cstride = B + 1;
  for (int e = threadIdx.x; e < nf * B; e += blockDim.x) sums[e] = 0ull;
  for (int e = threadIdx.x; e < nf * cstride; e += blockDim.x) cnts[e] = 0u;
  __syncthreads();
  const uint32_t* __restrict__ cw = reinterpret_cast<const uint32_t*>(codes);
  const int L = 1 << lane_shift;
  const int sub = threadIdx.x & (L - 1);
  const int rpp = blockDim.x >> lane_shift;
  if (sub < nwords) {
    for (int64_t r = threadIdx.x >> lane_shift; r < count; r += rpp) {
      const uint32_t row = idx[start + r];
      const unsigned long long yv = (unsigned long long)y[row];
      const uint32_t word = cw[(int64_t)row * row_words + gw0 + sub];
#pragma unroll
      for (int j = 0; j < cpw; ++j) {
        const int gf = (gw0 + sub) * cpw + j;
        if (gf >= g0 && gf < g1) {
          const uint32_t code = (word >> (j * 8 * sizeof(CodeT))) &
                                ((sizeof(CodeT) == 1) ? 0xffu : 0xffffu);
          atomicAdd(&cnts[(gf - g0) * cstride + (int)code], 1u);
          atomicAdd(&sums[(gf - g0) * B + (int)code], yv);
        }
      }
    }
  }
  __syncthreads();
  int64_t* out = dest < 0 ? hist + slot * (int64_t)F_h * B * 2 : slab + dest * (int64_t)F_h * B * 2;
  for (int e = threadIdx.x; e < nf * B; e += blockDim.x) {
    const int f = e / B;
    const int b = e - f * B;
    const int64_t o = ((int64_t)(t0 + f) * B + b) * 2;
    out[o] = (int64_t)cnts[f * cstride + b];
    out[o + 1] = (int64_t)sums[e];
  }
}

// Fallback: direct global atomics (B*C too large for an LDS feature tile).
template <typename CodeT>
__global__ __launch_bounds__(256) void hist_cls_global_kernel(
    const CodeT* __restrict__ codes, int64_t row_elems, const uint32_t* __restrict__ idx,
    const int32_t* __restrict__ y, RowLab rl, const int64_t* __restrict__ items,
    uint32_t* __restrict__ hist, int F_h, int f_lo, int B, int C) {
  const int64_t slot = items[blockIdx.x * 4 + 0];
  const int64_t start = items[blockIdx.x * 4 + 1];
  const int64_t count = items[blockIdx.x * 4 + 2];
  uint32_t* out = hist + slot * (int64_t)F_h * B * C;
  const int64_t total = count * F_h;
  for (int64_t e = threadIdx.x; e < total; e += blockDim.x) {
    const int64_t r = e / F_h;
    const int f = (int)(e - r * F_h);
    const uint32_t ent = idx[start + r];
    const uint32_t row = rl.shift ? (ent & rl.mask) : ent;
    const int lab = rl.shift ? (int)(ent >> rl.shift) : y[row];
    const int code = (int)codes[(int64_t)row * row_elems + f_lo + f];
    atomicAdd(&out[((int64_t)f * B + code) * C + lab], 1u);
  }
}

template <typename CodeT>
__global__ __launch_bounds__(256) void hist_reg_global_kernel(
    const CodeT* __restrict__ codes, int64_t row_elems, const uint32_t* __restrict__ idx,
    const int64_t* __restrict__ y, const int64_t* __restrict__ items,
    int64_t* __restrict__ hist, int F_h, int f_lo, int B) {
  const int64_t slot = items[blockIdx.x * 4 + 0];
  const int64_t start = items[blockIdx.x * 4 + 1];
  const int64_t count = items[blockIdx.x * 4 + 2];
  unsigned long long* out =
      reinterpret_cast<unsigned long long*>(hist + slot * (int64_t)F_h * B * 2);
  const int64_t total = count * F_h;
  for (int64_t e = threadIdx.x; e < total; e += blockDim.x) {
    const int64_t r = e / F_h;
    const int f = (int)(e - r * F_h);
    const uint32_t row = idx[start + r];
    const int code = (int)codes[(int64_t)row * row_elems + f_lo + f];
    atomicAdd(&out[((int64_t)f * B + code) * 2], 1ull);
    atomicAdd(&out[((int64_t)f * B + code) * 2 + 1], (unsigned long long)y[row]);
  }
}

// ---------------------------------------------------------------- reduction
// red: int64 [n][3] = {slot, first slab, k slabs}.
// Classification slabs hold the packed [F_h][B][W] LDS image (two 16-bit
// classes per word); grid = (word chunks, red entries, slab groups). Each
// thread unpacks and sums up to G slabs of one word and adds the result to
// the (zeroed) histogram.
__global__ __launch_bounds__(256) void zero_slots_kernel(const int64_t* __restrict__ red,
                                                         uint32_t* __restrict__ hist,
                                                         int64_t E,
                                                         const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.y >= *dcount) return;
  const int64_t slot = red[blockIdx.y * 3 + 0];
  if ((E & 3) == 0) {  // every slot base is 16-B aligned
    uint4* h = reinterpret_cast<uint4*>(hist + slot * E);
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E / 4;
         e += (int64_t)gridDim.x * blockDim.x)
      h[e] = make_uint4(0, 0, 0, 0);
    return;
  }
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x)
    hist[slot * E + e] = 0;
}

// With ``tasks`` (device-planned levels) each grid row is one task {slot,
// first slab, slabs <= G} and z is 1; otherwise row y is reduction entry y and
// z selects its group of G slabs.
__global__ __launch_bounds__(256) void hist_reduce_cls_kernel(
    const int64_t* __restrict__ red, const uint32_t* __restrict__ slab,
    uint32_t* __restrict__ hist, int64_t Ep, int C, int W, int G,
    const int32_t* __restrict__ dcount) {
  // rows past the grid's y extent: the device count can exceed the launch's rows
  // (device-planned levels launch a capped row count and stride over the tasks)
  const int ny = dcount ? *dcount : (int)gridDim.y;
  const int64_t Eu = (Ep / W) * C;
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= Ep) return;
  for (int ty = blockIdx.y; ty < ny; ty += gridDim.y) {
  const int64_t slot = red[ty * 3 + 0];
  const int64_t first = red[ty * 3 + 1];
  const int64_t k = red[ty * 3 + 2];
  const int64_t k0 = (int64_t)blockIdx.z * G;
  if (k0 >= k) continue;
  const int64_t k1 = min(k, k0 + G);
  uint32_t a0 = 0, a1 = 0;
  // every slab load of the group in flight before the first add (a rolled loop
  // waited for each load in turn: one L2 / MALL round trip per slab)
  constexpr int kGMax = 16;
  for (int64_t jb = k0; jb < k1; jb += kGMax) {
    uint32_t v[kGMax];
#pragma unroll
    for (int u = 0; u < kGMax; ++u) {
      const int64_t j = jb + u;
      v[u] = j < k1 ? slab[(first + j) * Ep + e] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kGMax; ++u) {
      a0 += v[u] & 0xffffu;
      a1 += v[u] >> 16;
    }
  }
  const int64_t fb = e / W;
  const int wc = (int)(e - fb * W);
  uint32_t* out = hist + slot * Eu + fb * C + 2 * wc;
  if (a0) atomicAdd(out, a0);
  if (a1 && 2 * wc + 1 < C) atomicAdd(out + 1, a1);
  }
}

// regression slabs are already [F][B][2] int64
__global__ __launch_bounds__(256) void hist_reduce_reg_kernel(const int64_t* __restrict__ red,
                                                              const int64_t* __restrict__ slab,
                                                              int64_t* __restrict__ hist,
                                                              int64_t E,
                                                              const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.y >= *dcount) return;
  const int64_t slot = red[blockIdx.y * 3 + 0];
  const int64_t first = red[blockIdx.y * 3 + 1];
  const int64_t k = red[blockIdx.y * 3 + 2];
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t acc = 0;
    for (int64_t j = 0; j < k; ++j) acc += slab[(first + j) * E + e];
    hist[slot * E + e] = acc;
  }
}

// hist[slot] = prev[parent] - hist[sibling] ; der: int64 [n][3]
template <typename T>
__global__ __launch_bounds__(256) void hist_derive_kernel(const int64_t* __restrict__ der,
                                                          const T* __restrict__ prev,
                                                          T* __restrict__ hist, int64_t E,
                                                          const int32_t* __restrict__ dcount) {
  if (dcount && (int)blockIdx.y >= *dcount) return;
  const int64_t slot = der[blockIdx.y * 3 + 0];
  const int64_t ps = der[blockIdx.y * 3 + 1];
  const int64_t ss = der[blockIdx.y * 3 + 2];
  // 16-B vectors (E is a multiple of 4 elements for every histogram shape we allocate
  // whenever B*C % 4 == 0; the scalar tail handles the rest)
  constexpr int V = 16 / sizeof(T);
  const int64_t nv = E / V;
  using VT = uint4;
  const VT* pp = reinterpret_cast<const VT*>(prev + ps * E);
  const VT* sp = reinterpret_cast<const VT*>(hist + ss * E);
  VT* op = reinterpret_cast<VT*>(hist + slot * E);
  const bool aligned = (E % V) == 0;
  if (aligned) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nv;
         e += (int64_t)gridDim.x * blockDim.x) {
      const VT a = pp[e], b = sp[e];
      VT r;
      if (sizeof(T) == 4) {
        r.x = a.x - b.x;
        r.y = a.y - b.y;
        r.z = a.z - b.z;
        r.w = a.w - b.w;
      } else {
        const uint64_t a0 = ((uint64_t)a.y << 32) | a.x, a1 = ((uint64_t)a.w << 32) | a.z;
        const uint64_t b0 = ((uint64_t)b.y << 32) | b.x, b1 = ((uint64_t)b.w << 32) | b.z;
        const uint64_t r0 = a0 - b0, r1 = a1 - b1;
        r.x = (uint32_t)r0;
        r.y = (uint32_t)(r0 >> 32);
        r.z = (uint32_t)r1;
        r.w = (uint32_t)(r1 >> 32);
      }
      op[e] = r;
    }
    return;
  }
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    hist[slot * E + e] = prev[ps * E + e] - hist[ss * E + e];
  }
}

}  // namespace mt

// ----------------------------------------------------------------- launchers
namespace mt {

static int ceil_pow2_shift(int v) {
  int s = 0;
  while ((1 << s) < v) ++s;
  return s;
}

// Features per LDS tile for the histogram kernel (0 -> global-atomic fallback).
// At most 128: a row's tile is read by at most 64 lanes of one word each
// (16-bit codes, unaligned rows), so wider tiles would drop features.
int hist_feature_tile(int F_h, int B, int C, bool reg, int lds_budget) {
  int per_f = reg ? (B * 8 + (B + 1) * 4) : (B * ((C + 1) / 2) + 1) * 4;
  int ft = std::min(lds_budget / per_f, 128);
  if (ft <= 0) return 0;
  if (ft >= F_h) return F_h;
  if (ft >= 16) ft &= ~15;
  else if (ft >= 4) ft &= ~3;
  return ft;
}

// Classes per LDS tile of the classification histogram kernel: C when a
// feature's whole [B][C] histogram fits the budget (hist_feature_tile > 0), else
// the largest even count that fits one feature (0: not even two classes fit).
int hist_class_tile(int F_h, int B, int C, bool reg, int lds_budget) {
  if (reg) return hist_feature_tile(F_h, B, C, reg, lds_budget) > 0 ? 2 : 0;
  if (hist_feature_tile(F_h, B, C, reg, lds_budget) > 0) return C;
  const int words = lds_budget / 4 - 1;  // per feature: B * ct / 2 + 1 words
  int ct = 2 * (words / std::max(B, 1));
  return ct >= 2 ? std::min(ct, C) : 0;
}

// Words of the packed classification slab per work item ([F_h][B][W]).
int64_t hist_slab_words(int F_h, int B, int C, bool reg) {
  return reg ? (int64_t)F_h * B * 2 : (int64_t)F_h * B * ((C + 1) / 2);
}

void launch_hist(hipStream_t stream, const void* codes, int code_bytes, int64_t row_stride_bytes,
                 const uint32_t* idx, const void* y, int lab_shift, const int64_t* items,
                 int n_items, void* hist, void* slab, int F_h, int f_lo, int B, int C, bool reg,
                 int lds_budget, const int32_t* dcount, const int64_t* zred, int zred_bound,
                 const int32_t* zcount) {
  // zred / zcount (classification, optional): the multi-item slots to zero before
  // the slab reduction (launch_hist_reduce_tasks with zero = false) -- fused into
  // the LDS histogram kernel, else a zero_slots_kernel launch here
  if (n_items <= 0) return;
  const int ft = hist_feature_tile(F_h, B, C, reg, lds_budget);
  const int64_t Eu = (int64_t)F_h * B * C;
  const bool fuse_zero = zred && zred_bound > 0 && !reg &&
                         (ft != 0 || hist_class_tile(F_h, B, C, reg, lds_budget) > 0) &&
                         (Eu & 3) == 0;
  if (zred && zred_bound > 0 && !fuse_zero) {
    hipLaunchKernelGGL(zero_slots_kernel,
                       dim3((unsigned)std::min<int64_t>((Eu / 4 + 255) / 256, 64), zred_bound),
                       dim3(256), 0, stream, zred, (uint32_t*)hist, Eu, zcount);
    MT_HIP_CHECK(hipGetLastError());
  }
  RowLab rl{lab_shift ? ((1u << lab_shift) - 1u) : 0xffffffffu, lab_shift};
  // many classes: class-tiled LDS histograms (one feature per tile)
  const int ct = reg ? 0 : hist_class_tile(F_h, B, C, reg, lds_budget);
  if (ft == 0 && ct > 0 && ct < C) {
    const int n_ct = (C + ct - 1) / ct;
    const int64_t row_words = row_stride_bytes / 4;
    const int cpw = 4 / code_bytes;
    int words = 1;
    for (int f = 0; f < F_h; ++f) {
      const int a = f_lo + f, b = a + 1;
      words = std::max(words, (b + cpw - 1) / cpw - a / cpw);
    }
    const int shift = std::min(ceil_pow2_shift(words), 6);
    const size_t lds = (size_t)(B * ((ct + 1) / 2) + 1) * 4;
    // (a capped row of workgroups striding over the items: the item bound times
    // F_h x class tiles launched ~1M workgroups a level at C = 300, most of them
    // only reading the device count)
    const int gx = MT_HIST_ROWS_CAP ? std::max(1, std::min(n_items, 32768 / (F_h * n_ct) + 1))
                                    : n_items;
    dim3 grid(gx, F_h * n_ct);
#define MT_CLS_CT(CT)                                                                         \
  MT_HIP_CHECK(mt_set_max_lds((const void*)hist_cls_lds_kernel<CT, 1>, (int)lds));           \
  hipLaunchKernelGGL((hist_cls_lds_kernel<CT, 1>), grid, dim3(kHistThreads), lds, stream,     \
                     (const uint32_t*)codes, row_words, idx, (const int32_t*)y, rl, items,    \
                     (uint32_t*)hist, (uint32_t*)slab, F_h, f_lo, B, C, 1, shift, dcount,    \
                     fuse_zero ? zred : nullptr, zcount, Eu, ct);
    if (code_bytes == 1) {
      MT_CLS_CT(uint8_t)
    } else {
      MT_CLS_CT(uint16_t)
    }
#undef MT_CLS_CT
    MT_HIP_CHECK(hipGetLastError());
    return;
  }
  if (ft == 0) {
    dim3 grid(n_items);
    const int64_t row_elems = row_stride_bytes / code_bytes;
#define MT_GLOBAL(CT)                                                                          \
  if (reg)                                                                                     \
    hipLaunchKernelGGL(hist_reg_global_kernel<CT>, grid, dim3(256), 0, stream,                 \
                       (const CT*)codes, row_elems, idx, (const int64_t*)y, items,             \
                       (int64_t*)hist, F_h, f_lo, B);                                          \
  else                                                                                         \
    hipLaunchKernelGGL(hist_cls_global_kernel<CT>, grid, dim3(256), 0, stream,                 \
                       (const CT*)codes, row_elems, idx, (const int32_t*)y, rl, items,         \
                       (uint32_t*)hist, F_h, f_lo, B, C);
    if (code_bytes == 1) {
      MT_GLOBAL(uint8_t)
    } else {
      MT_GLOBAL(uint16_t)
    }
#undef MT_GLOBAL
    MT_HIP_CHECK(hipGetLastError());
    return;
  }
  const int n_tiles = (F_h + ft - 1) / ft;
  const int cpw = 4 / code_bytes;
  const int64_t row_words = row_stride_bytes / 4;
  dim3 grid(n_items, n_tiles);
  if (reg) {
    int words = 1;
    for (int t = 0; t < n_tiles; ++t) {
      const int a = f_lo + t * ft, b = f_lo + std::min(F_h, (t + 1) * ft);
      words = std::max(words, (b + cpw - 1) / cpw - a / cpw);
    }
    int shift = std::min(ceil_pow2_shift(words), 9);
    size_t lds = (size_t)ft * (B * 8 + (B + 1) * 4);
#define MT_REG(CT)                                                                            \
  MT_HIP_CHECK(mt_set_max_lds((const void*)hist_reg_lds_kernel<CT>,                      \
                                   (int)lds));    \
  hipLaunchKernelGGL(hist_reg_lds_kernel<CT>, grid, dim3(kHistThreads), lds, stream,          \
                     (const CT*)codes, row_words, idx, (const int64_t*)y, items,              \
                     (int64_t*)hist, (int64_t*)slab, F_h, f_lo, B, ft, shift, dcount);
    if (code_bytes == 1) {
      MT_REG(uint8_t)
    } else {
      MT_REG(uint16_t)
    }
#undef MT_REG
    MT_HIP_CHECK(hipGetLastError());
    return;
  }
  // 16-B row loads when every tile's word range is 4-word aligned
  bool vec4 = (row_words % 4) == 0;
  int words = 1;
  for (int t = 0; t < n_tiles; ++t) {
    const int a = f_lo + t * ft, b = f_lo + std::min(F_h, (t + 1) * ft);
    const int w0 = (a / cpw) & ~3;
    words = std::max(words, (b + cpw - 1) / cpw - (vec4 ? w0 : a / cpw));
  }
  const int vec = vec4 ? 4 : 1;
  const int lanes = (words + vec - 1) / vec;
  const int shift = std::min(ceil_pow2_shift(lanes), 6);
  size_t lds = (size_t)ft * (B * ((C + 1) / 2) + 1) * 4;
#define MT_CLS(CT, V)                                                                         \
  MT_HIP_CHECK(mt_set_max_lds((const void*)hist_cls_lds_kernel<CT, V>,                   \
                                   (int)lds));    \
  hipLaunchKernelGGL((hist_cls_lds_kernel<CT, V>), grid, dim3(kHistThreads), lds, stream,     \
                     (const uint32_t*)codes, row_words, idx, (const int32_t*)y, rl, items,    \
                     (uint32_t*)hist, (uint32_t*)slab, F_h, f_lo, B, C, ft, shift, dcount,   \
                     fuse_zero ? zred : nullptr, zcount, Eu, C);
  if (code_bytes == 1) {
    if (vec4) {
      MT_CLS(uint8_t, 4)
    } else {
      MT_CLS(uint8_t, 1)
    }
  } else {
    if (vec4) {
      MT_CLS(uint16_t, 4)
    } else {
      MT_CLS(uint16_t, 1)
    }
  }
#undef MT_CLS
  MT_HIP_CHECK(hipGetLastError());
}

void launch_hist_reduce(hipStream_t stream, const int64_t* red, int n_red, int max_k,
                        const void* slab, void* hist, int F_h, int B, int C, bool reg,
                        const int32_t* dcount) {
  if (n_red <= 0) return;
  if (reg) {
    const int64_t E = (int64_t)F_h * B * 2;
    int gx = (int)std::min<int64_t>((E + 255) / 256, 1024);
    hipLaunchKernelGGL(hist_reduce_reg_kernel, dim3(gx, n_red), dim3(256), 0, stream, red,
                       (const int64_t*)slab, (int64_t*)hist, E, dcount);
    MT_HIP_CHECK(hipGetLastError());
    return;
  }
  const int W = (C + 1) / 2;
  const int64_t Ep = (int64_t)F_h * B * W;
  const int64_t Eu = (int64_t)F_h * B * C;
  hipLaunchKernelGGL(zero_slots_kernel, dim3((unsigned)std::min<int64_t>((Eu / 4 + 255) / 256, 256),
                                             n_red),
                     dim3(256), 0, stream, red, (uint32_t*)hist, Eu, dcount);
  MT_HIP_CHECK(hipGetLastError());
  const int G = 16;
  const int groups = (max_k + G - 1) / G;
  dim3 grid((unsigned)((Ep + 255) / 256), n_red, groups);
  hipLaunchKernelGGL(hist_reduce_cls_kernel, grid, dim3(256), 0, stream, red,
                     (const uint32_t*)slab, (uint32_t*)hist, Ep, C, W, G, dcount);
  MT_HIP_CHECK(hipGetLastError());
}

// Device-planned reduction: zero the multi-item slots (red entries), then one
// workgroup row per task {slot, first slab, <= 16 slabs} adds into them.
void launch_hist_reduce_tasks(hipStream_t stream, const int64_t* red, int red_bound,
                              const int64_t* tasks, int task_bound, const void* slab, void* hist,
                              int F_h, int B, int C, const int32_t* dred, const int32_t* dtasks,
                              bool zero) {
  if (red_bound <= 0 || task_bound <= 0) return;
  const int W = (C + 1) / 2;
  const int64_t Ep = (int64_t)F_h * B * W;
  const int64_t Eu = (int64_t)F_h * B * C;
  if (zero) {  // else launch_hist already zeroed the slots (zred)
    hipLaunchKernelGGL(zero_slots_kernel,
                       dim3((unsigned)std::min<int64_t>((Eu / 4 + 255) / 256, 64), red_bound),
                       dim3(256), 0, stream, red, (uint32_t*)hist, Eu, dred);
    MT_HIP_CHECK(hipGetLastError());
  }
  // rows: the task bound, capped so the grid holds ~32k workgroups (many classes:
  // ~10k column blocks a row, and a bound of hundreds of rows launched millions of
  // workgroups that only checked the device count -- 2.6 ms a level at C = 300)
  const int64_t xb = (Ep + 255) / 256;
  const int rows = (int)std::max<int64_t>(
      1, std::min<int64_t>(task_bound, MT_RED_ROWS_CAP ? (32768 + xb - 1) / xb : task_bound));
  dim3 grid((unsigned)xb, rows, 1);
  hipLaunchKernelGGL(hist_reduce_cls_kernel, grid, dim3(256), 0, stream, tasks,
                     (const uint32_t*)slab, (uint32_t*)hist, Ep, C, W, 16, dtasks);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_hist_derive(hipStream_t stream, const int64_t* der, int n_der, const void* prev,
                        void* hist, int64_t E, bool is64, const int32_t* dcount) {
  if (n_der <= 0) return;
  int gx = (int)std::min<int64_t>((E / 4 + 255) / 256, 256);
  if (gx < 1) gx = 1;
  dim3 grid(gx, n_der);
  if (is64)
    hipLaunchKernelGGL(hist_derive_kernel<int64_t>, grid, dim3(256), 0, stream, der,
                       (const int64_t*)prev, (int64_t*)hist, E, dcount);
  else
    hipLaunchKernelGGL(hist_derive_kernel<uint32_t>, grid, dim3(256), 0, stream, der,
                       (const uint32_t*)prev, (uint32_t*)hist, E, dcount);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
