// Per-node feature histograms on gfx950.
//
// Replaces the reference's per-threshold masking + row copies + np.unique
// entropy loop (mpitree/tree/decision_tree.py:73-86): one pass over a node's
// rows accumulates [F, B, C] class counts, after which every threshold's left
// and right class distributions are prefix sums (split_scan.hip).
//
// Design (CDNA4):
//  * rows of a node are addressed through the row permutation ``idx`` and
//    read as 32-bit words of the row-major code matrix, several lanes per row
//    (one lane per 4 u8 codes), so a wave touches whole 64-B rows;
//  * each workgroup privatises the histogram of its feature tile in LDS.
//    Classification packs two classes per 32-bit LDS word (16-bit halves;
//    a work item is at most 65535 rows so a half never overflows), halving
//    LDS footprint and atomics; the feature stride is padded by one word so
//    lanes of one row with equal codes hit different banks;
//  * no global atomics: a work item that covers a whole node writes the
//    final histogram with plain stores, items of a multi-item node write a
//    private slab that ``hist_reduce`` sums (integer, so order-free and
//    bitwise deterministic);
//  * histograms that cannot fit one feature in LDS (very large B*C) fall back
//    to direct global atomics.
#include "common.h"

namespace mt {

// items: int64 [n_items][4] = {slot, start, count, dest}; dest < 0 -> write
// hist[slot], dest >= 0 -> write slab[dest].
template <typename CodeT>
__global__ __launch_bounds__(256) void hist_cls_lds_kernel(
    const CodeT* __restrict__ codes, int64_t row_words, const int32_t* __restrict__ idx,
    const int32_t* __restrict__ y, const int64_t* __restrict__ items,
    uint32_t* __restrict__ hist, uint32_t* __restrict__ slab, int F_h, int f_lo, int B,
    int C, int ft, int wpr_shift) {
  extern __shared__ uint32_t lds[];
  constexpr int cpw = 4 / sizeof(CodeT);  // codes per 32-bit word
  const int W = (C + 1) >> 1;
  const int fstride = B * W + 1;
  const int tile = blockIdx.y;
  const int t0 = tile * ft;                       // first hist feature of tile
  const int t1 = min(F_h, t0 + ft);               // end (exclusive)
  const int g0 = f_lo + t0;                       // global feature index
  const int gw0 = g0 / cpw;                       // first code word
  const int nwords = (f_lo + t1 + cpw - 1) / cpw - gw0;
  const int64_t slot = items[blockIdx.x * 4 + 0];
  const int64_t start = items[blockIdx.x * 4 + 1];
  const int64_t count = items[blockIdx.x * 4 + 2];
  const int64_t dest = items[blockIdx.x * 4 + 3];

  const int lds_words = (t1 - t0) * fstride;
  for (int e = threadIdx.x; e < lds_words; e += blockDim.x) lds[e] = 0u;
  __syncthreads();

  const uint32_t* __restrict__ cw = reinterpret_cast<const uint32_t*>(codes);
  const int wpr = 1 << wpr_shift;
  const int sub = threadIdx.x & (wpr - 1);
  const int rows_per_pass = blockDim.x >> wpr_shift;
  if (sub < nwords) {
    for (int64_t r = threadIdx.x >> wpr_shift; r < count; r += rows_per_pass) {
      const int32_t row = idx[start + r];
      const int32_t lab = y[row];
      const uint32_t word = cw[(int64_t)row * row_words + gw0 + sub];
      const uint32_t inc = 1u << ((lab & 1) * 16);
      const int cw_off = lab >> 1;
#pragma unroll
      for (int j = 0; j < cpw; ++j) {
        const int gf = (gw0 + sub) * cpw + j;
        if (gf >= g0 && gf < f_lo + t1) {
          const uint32_t code = (word >> (j * 8 * sizeof(CodeT))) &
                                ((sizeof(CodeT) == 1) ? 0xffu : 0xffffu);
          atomicAdd(&lds[(gf - g0) * fstride + (int)code * W + cw_off], inc);
        }
      }
    }
  }
  __syncthreads();

  uint32_t* out = dest < 0 ? hist + slot * (int64_t)F_h * B * C : slab + dest * (int64_t)F_h * B * C;
  const int per_f = B * W;
  for (int e = threadIdx.x; e < lds_words - (t1 - t0); e += blockDim.x) {
    const int f = e / per_f;
    const int rem = e - f * per_f;
    const int b = rem / W;
    const int wc = rem - b * W;
    const uint32_t v = lds[f * fstride + rem];
    const int64_t o = ((int64_t)(t0 + f) * B + b) * C + 2 * wc;
    out[o] = v & 0xffffu;
    if (2 * wc + 1 < C) out[o + 1] = v >> 16;
  }
}

// Regression payload: per bin {count, fixed-point target sum} as two int64.
template <typename CodeT>
__global__ __launch_bounds__(256) void hist_reg_lds_kernel(
    const CodeT* __restrict__ codes, int64_t row_words, const int32_t* __restrict__ idx,
    const int64_t* __restrict__ y, const int64_t* __restrict__ items,
    int64_t* __restrict__ hist, int64_t* __restrict__ slab, int F_h, int f_lo, int B, int ft,
    int wpr_shift) {
  extern __shared__ uint32_t lds[];
  constexpr int cpw = 4 / sizeof(CodeT);
  const int tile = blockIdx.y;
  const int t0 = tile * ft;
  const int t1 = min(F_h, t0 + ft);
  const int nf = t1 - t0;
  const int g0 = f_lo + t0;
  const int gw0 = g0 / cpw;
  const int nwords = (f_lo + t1 + cpw - 1) / cpw - gw0;
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
  const int wpr = 1 << wpr_shift;
  const int sub = threadIdx.x & (wpr - 1);
  const int rows_per_pass = blockDim.x >> wpr_shift;
  if (sub < nwords) {
    for (int64_t r = threadIdx.x >> wpr_shift; r < count; r += rows_per_pass) {
      const int32_t row = idx[start + r];
      const unsigned long long yv = (unsigned long long)y[row];
      const uint32_t word = cw[(int64_t)row * row_words + gw0 + sub];
#pragma unroll
      for (int j = 0; j < cpw; ++j) {
        const int gf = (gw0 + sub) * cpw + j;
        if (gf >= g0 && gf < f_lo + t1) {
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
    const CodeT* __restrict__ codes, int64_t row_elems, const int32_t* __restrict__ idx,
    const int32_t* __restrict__ y, const int64_t* __restrict__ items,
    uint32_t* __restrict__ hist, int F_h, int f_lo, int B, int C) {
  const int64_t slot = items[blockIdx.x * 4 + 0];
  const int64_t start = items[blockIdx.x * 4 + 1];
  const int64_t count = items[blockIdx.x * 4 + 2];
  uint32_t* out = hist + slot * (int64_t)F_h * B * C;
  const int64_t total = count * F_h;
  for (int64_t e = threadIdx.x; e < total; e += blockDim.x) {
    const int64_t r = e / F_h;
    const int f = (int)(e - r * F_h);
    const int32_t row = idx[start + r];
    const int code = (int)codes[(int64_t)row * row_elems + f_lo + f];
    atomicAdd(&out[((int64_t)f * B + code) * C + y[row]], 1u);
  }
}

template <typename CodeT>
__global__ __launch_bounds__(256) void hist_reg_global_kernel(
    const CodeT* __restrict__ codes, int64_t row_elems, const int32_t* __restrict__ idx,
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
    const int32_t row = idx[start + r];
    const int code = (int)codes[(int64_t)row * row_elems + f_lo + f];
    atomicAdd(&out[((int64_t)f * B + code) * 2], 1ull);
    atomicAdd(&out[((int64_t)f * B + code) * 2 + 1], (unsigned long long)y[row]);
  }
}

// hist[slot] = sum of slab[first .. first+k) ; red: int64 [n][3] = {slot, first, k}
template <typename T>
__global__ __launch_bounds__(256) void hist_reduce_kernel(const int64_t* __restrict__ red,
                                                          const T* __restrict__ slab,
                                                          T* __restrict__ hist, int64_t E) {
  const int64_t slot = red[blockIdx.y * 3 + 0];
  const int64_t first = red[blockIdx.y * 3 + 1];
  const int64_t k = red[blockIdx.y * 3 + 2];
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    T acc = 0;
    for (int64_t j = 0; j < k; ++j) acc += slab[(first + j) * E + e];
    hist[slot * E + e] = acc;
  }
}

// hist[slot] = prev[parent] - hist[sibling] ; der: int64 [n][3]
template <typename T>
__global__ __launch_bounds__(256) void hist_derive_kernel(const int64_t* __restrict__ der,
                                                          const T* __restrict__ prev,
                                                          T* __restrict__ hist, int64_t E) {
  const int64_t slot = der[blockIdx.y * 3 + 0];
  const int64_t ps = der[blockIdx.y * 3 + 1];
  const int64_t ss = der[blockIdx.y * 3 + 2];
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    hist[slot * E + e] = prev[ps * E + e] - hist[ss * E + e];
  }
}

}  // namespace mt

// ----------------------------------------------------------------- launchers
namespace mt {

static int floor_pow2_shift(int v) {
  int s = 0;
  while ((1 << (s + 1)) <= v) ++s;
  return s;
}
static int ceil_pow2_shift(int v) {
  int s = 0;
  while ((1 << s) < v) ++s;
  return s;
}

// Returns the features-per-tile used by the LDS kernel (0 -> global fallback).
int hist_feature_tile(int F_h, int B, int C, bool reg, int lds_budget) {
  int per_f = reg ? (B * 8 + (B + 1) * 4) : (B * ((C + 1) / 2) + 1) * 4;
  int ft = lds_budget / per_f;
  if (ft <= 0) return 0;
  if (ft >= F_h) return F_h;
  if (ft >= 4) ft &= ~3;
  return ft;
}

void launch_hist(hipStream_t stream, const void* codes, int code_bytes, int64_t row_stride_bytes,
                 const int32_t* idx, const void* y, const int64_t* items, int n_items, void* hist,
                 void* slab, int F_h, int f_lo, int B, int C, bool reg, int lds_budget) {
  if (n_items <= 0) return;
  const int ft = hist_feature_tile(F_h, B, C, reg, lds_budget);
  dim3 block(256);
  if (ft == 0) {
    dim3 grid(n_items);
    const int64_t row_elems = row_stride_bytes / code_bytes;
#define MT_GLOBAL(CT)                                                                        \
  if (reg)                                                                                   \
    hipLaunchKernelGGL(hist_reg_global_kernel<CT>, grid, block, 0, stream, (const CT*)codes, \
                       row_elems, idx, (const int64_t*)y, items, (int64_t*)hist, F_h, f_lo, B); \
  else                                                                                       \
    hipLaunchKernelGGL(hist_cls_global_kernel<CT>, grid, block, 0, stream, (const CT*)codes, \
                       row_elems, idx, (const int32_t*)y, items, (uint32_t*)hist, F_h, f_lo, B, \
                       C);
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
  // 32-bit code words spanned by the widest tile; lanes per row = pow2 >= that
  int words = 1;
  for (int t = 0; t < n_tiles; ++t) {
    const int a = f_lo + t * ft, b = f_lo + std::min(F_h, (t + 1) * ft);
    words = std::max(words, (b + cpw - 1) / cpw - a / cpw);
  }
  int wpr_shift = ceil_pow2_shift(words);
  if (wpr_shift > 8) wpr_shift = 8;
  (void)floor_pow2_shift;
  size_t lds = reg ? (size_t)ft * (B * 8 + (B + 1) * 4)
                   : (size_t)ft * (B * ((C + 1) / 2) + 1) * 4;
  dim3 grid(n_items, n_tiles);
  const int64_t row_words = row_stride_bytes / 4;
#define MT_LDS(CT)                                                                            \
  if (reg) {                                                                                  \
    MT_HIP_CHECK(hipFuncSetAttribute((const void*)hist_reg_lds_kernel<CT>,                    \
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));  \
    hipLaunchKernelGGL(hist_reg_lds_kernel<CT>, grid, block, lds, stream, (const CT*)codes,   \
                       row_words, idx, (const int64_t*)y, items, (int64_t*)hist,              \
                       (int64_t*)slab, F_h, f_lo, B, ft, wpr_shift);                          \
  } else {                                                                                    \
    MT_HIP_CHECK(hipFuncSetAttribute((const void*)hist_cls_lds_kernel<CT>,                    \
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));  \
    hipLaunchKernelGGL(hist_cls_lds_kernel<CT>, grid, block, lds, stream, (const CT*)codes,   \
                       row_words, idx, (const int32_t*)y, items, (uint32_t*)hist,             \
                       (uint32_t*)slab, F_h, f_lo, B, C, ft, wpr_shift);                      \
  }
  if (code_bytes == 1) {
    MT_LDS(uint8_t)
  } else {
    MT_LDS(uint16_t)
  }
#undef MT_LDS
  MT_HIP_CHECK(hipGetLastError());
}

void launch_hist_reduce(hipStream_t stream, const int64_t* red, int n_red, const void* slab,
                        void* hist, int64_t E, bool is64) {
  if (n_red <= 0) return;
  int gx = (int)std::min<int64_t>((E + 255) / 256, 512);
  dim3 grid(gx, n_red);
  if (is64)
    hipLaunchKernelGGL(hist_reduce_kernel<int64_t>, grid, dim3(256), 0, stream, red,
                       (const int64_t*)slab, (int64_t*)hist, E);
  else
    hipLaunchKernelGGL(hist_reduce_kernel<uint32_t>, grid, dim3(256), 0, stream, red,
                       (const uint32_t*)slab, (uint32_t*)hist, E);
  MT_HIP_CHECK(hipGetLastError());
}

void launch_hist_derive(hipStream_t stream, const int64_t* der, int n_der, const void* prev,
                        void* hist, int64_t E, bool is64) {
  if (n_der <= 0) return;
  int gx = (int)std::min<int64_t>((E + 255) / 256, 512);
  dim3 grid(gx, n_der);
  if (is64)
    hipLaunchKernelGGL(hist_derive_kernel<int64_t>, grid, dim3(256), 0, stream, der,
                       (const int64_t*)prev, (int64_t*)hist, E);
  else
    hipLaunchKernelGGL(hist_derive_kernel<uint32_t>, grid, dim3(256), 0, stream, der,
                       (const uint32_t*)prev, (uint32_t*)hist, E);
  MT_HIP_CHECK(hipGetLastError());
}

}  // namespace mt
