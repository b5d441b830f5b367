// Setup of the exact-threshold engine (exact2.hip): per feature, the rows sorted
// by value and a per-chunk count of value changes (the dense value ranks).
//
// The reference sorts implicitly through np.unique per feature and node
// (mpitree/tree/decision_tree.py:73). Here one pass over X writes 32-bit
// order-preserving value keys feature-major (an LDS tile transpose of the
// row-major input), and a batched LSD radix sort orders every feature's column at
// once: four stable 8-bit passes over 8192-key tiles (F x ceil(n / 8192) of them),
// each a reduce-then-scan -- per-tile digit counts, a per-(feature, digit) scan
// over the tiles, then a pass that ranks each tile's keys in registers (wave
// ballots) and writes every digit's run contiguously from LDS. Row ids travel as
// values (pass 0 generates them). The feature never enters the key, so a pass
// moves 16 bytes per entry instead of the 24 of a {feature, value} 64-bit key
// sort with 32-bit payloads, in 4 passes instead of 5. (A one-sweep variant that
// took each tile's prefix by decoupled look-back instead of the count + scan
// kernels measured 0.4 ms per pass against 0.21 ms without the look-back: its
// tiles wait on cross-XCD status visibility, profiles/kernel_experiments.md.)
// Two passes over the sorted keys then derive the ranks (a per-chunk count of
// value changes, a per-feature scan of the chunk counts); xe_emit_kernel
// (exact2.hip) writes the list entries.
#include "common.h"

namespace mt {

constexpr int kXsTile = 64;       // rows x features per transpose tile
constexpr int kXsChunk = 4096;    // sorted entries per rank chunk
constexpr int kXsThreads = 256;
constexpr int kRsItems = 16;                       // keys per lane of a sort tile
constexpr int kRsPasses = 4;                       // 8-bit digits of a 32-bit key
constexpr int kRsScanGroups = 16;                  // tile groups per scan workgroup

// IEEE-754 order as unsigned order (-0.0 folded into +0.0 first)
__device__ __forceinline__ uint32_t xs_key_bits(float v) {
  uint32_t b = __float_as_uint(v + 0.0f);
  return (b >> 31) ? ~b : (b | 0x80000000u);
}

// keys[f * n + i] = bits(X[i][f_lo + f]) for the F features of the block starting
// at column f_lo of a row-major X of stride xs
__global__ __launch_bounds__(kXsThreads) void xs_keys_kernel(const float* __restrict__ X,
                                                             int64_t n, int F, int xs, int f_lo,
                                                             uint32_t* __restrict__ keys) {
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
    if (f < F && i < n) keys[(int64_t)f * n + i] = tile[tx][c];
  }
}

// counts[(f * T + t) * 256 + d]: keys of tile t (kNT * 16 keys) of feature f whose
// digit (key >> shift) & 255 is d (per-wave LDS counts).
template <int kNT>
__global__ __launch_bounds__(kNT) void xs_tile_count_kernel(const uint32_t* __restrict__ keys,
                                                            int64_t n, int T, int shift,
                                                            uint32_t* __restrict__ counts) {
  constexpr int kW = kNT / kWave, kTile = kNT * kRsItems;
  __shared__ uint32_t h[kW][256];
  const int tid = threadIdx.x, w = tid >> 6;
  for (int i = tid; i < kW * 256; i += kNT) (&h[0][0])[i] = 0u;
  __syncthreads();
  const int f = blockIdx.x / T, t = blockIdx.x % T;
  const int64_t p0 = (int64_t)t * kTile;
  const int cnt = (int)min<int64_t>(kTile, n - p0);
  const uint32_t* k = keys + (int64_t)f * n + p0;
  uint32_t v[kRsItems];
#pragma unroll
  for (int u = 0; u < kRsItems; ++u) {
    const int i = u * kNT + tid;
    v[u] = i < cnt ? k[i] : 0u;
  }
#pragma unroll
  for (int u = 0; u < kRsItems; ++u)
    if (u * kNT + tid < cnt) atomicAdd(&h[w][(v[u] >> shift) & 255u], 1u);
  __syncthreads();
  if (tid < 256) {
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < kW; ++q) s += h[q][tid];
    counts[(int64_t)blockIdx.x * 256 + tid] = s;
  }
}

// In place: counts[f][t][d] -> the exclusive prefix over the feature's earlier tiles;
// totals[f][d] = the feature's count of digit d. Grid (F, 4): 64 digits x 16 tile
// groups per workgroup.
__global__ __launch_bounds__(kWave * kRsScanGroups) void xs_tile_scan_kernel(
    uint32_t* __restrict__ counts, int T, uint32_t* __restrict__ totals) {
  __shared__ uint32_t s_g[kRsScanGroups][kWave];
  const int dl = threadIdx.x & (kWave - 1), g = threadIdx.x >> 6;
  const int f = blockIdx.x, d = blockIdx.y * kWave + dl;
  const int per = (T + kRsScanGroups - 1) / kRsScanGroups;
  const int t0 = g * per, t1 = min(T, t0 + per);
  uint32_t* c = counts + (int64_t)f * T * 256 + d;
  uint32_t sum = 0;
  for (int t = t0; t < t1; ++t) sum += c[(int64_t)t * 256];
  s_g[g][dl] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (int q = 0; q < g; ++q) run += s_g[q][dl];
  for (int t = t0; t < t1; ++t) {
    const uint32_t v = c[(int64_t)t * 256];
    c[(int64_t)t * 256] = run;
    run += v;
  }
  if (g == kRsScanGroups - 1) totals[(int64_t)f * 256 + d] = run;
}

// One stable counting pass on digit (key >> shift) & 255: tile t (kNT * 16 keys) of
// feature f puts its keys with digit d at the feature's digit base + pref[f][t][d]
// onwards. Dynamic LDS: the tile's keys and rows in digit order (kNT * 128 bytes).
template <int kNT, bool kFirst, bool kLab>
__global__ __launch_bounds__(kNT) void xs_scatter_kernel(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ rin,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ rout, int64_t n, int T, int shift,
    const uint32_t* __restrict__ pref, const uint32_t* __restrict__ totals,
    const int32_t* __restrict__ ylab) {
  constexpr int kW = kNT / kWave, kTile = kNT * kRsItems;
  extern __shared__ uint32_t s_dyn[];
  uint32_t* const s_key = s_dyn;
  uint32_t* const s_row = s_dyn + kTile;
  __shared__ uint32_t s_wh[kW][256];  // per-wave digit counts -> wave offsets
  __shared__ uint32_t s_tex[256];     // tile-local start of each digit's run
  __shared__ int32_t s_goff[256];     // feature position of a run's entry 0 minus its start
  __shared__ uint64_t s_tot[4];
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  for (int i = tid; i < kW * 256; i += kNT) (&s_wh[0][0])[i] = 0u;
  const int f = blockIdx.x / T, t = blockIdx.x % T;
  const int64_t base = (int64_t)f * n;
  const int64_t p0 = (int64_t)t * kTile;
  const int cnt = (int)min<int64_t>(kTile, n - p0);
  __syncthreads();

  // ---- load (wave-striped: item k of lane l is tile entry w * 1024 + k * 64 + l)
  uint32_t key[kRsItems], row[kRsItems], rk[kRsItems];
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const int i = w * (kWave * kRsItems) + k * kWave + lane;
    const bool in = i < cnt;
    key[k] = in ? kin[base + p0 + i] : 0u;
    if constexpr (kFirst) {  // row ids (packed labels join them at the store)
      row[k] = (uint32_t)(p0 + i);
    } else {
      row[k] = in ? rin[base + p0 + i] : 0u;
    }
  }
  // ---- rank: lanes with equal digits found by 8 ballots; the lowest one bumps the count
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const int i = w * (kWave * kRsItems) + k * kWave + lane;
    const bool in = i < cnt;
    const uint32_t d = (key[k] >> shift) & 255u;
    unsigned long long m = __ballot(in);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const unsigned long long bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    const uint32_t c = s_wh[w][d];
    rk[k] = c + (uint32_t)__popcll(m & lt);
    if (in && (m & lt) == 0ull) s_wh[w][d] = c + (uint32_t)__popcll(m);
  }
  __syncthreads();

  // ---- per digit (threads 0..255 = digits): wave offsets, tile and feature prefixes
  const int d = tid;
  uint32_t tc = 0;
  int64_t pv = 0, incl = 0;
  if (tid < 256) {
#pragma unroll
    for (int q = 0; q < kW; ++q) {
      const uint32_t v = s_wh[q][d];
      s_wh[q][d] = tc;
      tc += v;
    }
    pv = ((int64_t)totals[(int64_t)f * 256 + d] << 32) | tc;
    incl = wave_incl_scan_i64(pv);
    if (lane == kWave - 1) s_tot[w] = (uint64_t)incl;
  }
  __syncthreads();
  if (tid < 256) {
    int64_t excl = incl - pv;
    for (int q = 0; q < w; ++q) excl += (int64_t)s_tot[q];
    const uint32_t tex = (uint32_t)(excl & 0xffffffffll);
    const uint32_t dbase = (uint32_t)(excl >> 32);
    s_tex[d] = tex;
    s_goff[d] = (int32_t)(dbase + pref[(int64_t)blockIdx.x * 256 + d]) - (int32_t)tex;
  }
  __syncthreads();

  // ---- stage in digit order, then store each digit's run contiguously
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const int i = w * (kWave * kRsItems) + k * kWave + lane;
    if (i < cnt) {
      const uint32_t dk = (key[k] >> shift) & 255u;
      const uint32_t lp = s_tex[dk] + s_wh[w][dk] + rk[k];
      s_key[lp] = key[k];
      s_row[lp] = row[k];
    }
  }
  __syncthreads();
  // 4 entries per lane per step: their label reads (pass 0 with packed labels: rows
  // of this tile, a local window) are in flight together
  constexpr int kS = 4;
  for (int i0 = tid; i0 < cnt; i0 += kNT * kS) {
    uint32_t kk[kS], rv[kS];
#pragma unroll
    for (int u = 0; u < kS; ++u) {
      const int i = i0 + u * kNT;
      kk[u] = i < cnt ? s_key[i] : 0u;
      rv[u] = i < cnt ? s_row[i] : 0u;
    }
    if constexpr (kLab) {
#pragma unroll
      for (int u = 0; u < kS; ++u)
        if (i0 + u * kNT < cnt) rv[u] |= (uint32_t)ylab[rv[u]] << 25;
    }
#pragma unroll
    for (int u = 0; u < kS; ++u) {
      const int i = i0 + u * kNT;
      if (i < cnt) {
        const int64_t dst = base + (int64_t)(s_goff[(kk[u] >> shift) & 255u] + i);
        kout[dst] = kk[u];
        rout[dst] = rv[u];
      }
    }
  }
}

// Value changes per chunk: cnt[f][c] = #{j in chunk c of feature f : j is the
// first entry or keys[j] != keys[j - 1]}.
__global__ __launch_bounds__(kXsThreads) void xs_count_kernel(const uint32_t* __restrict__ keys,
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

// Per feature (one wave each): exclusive scan of the chunk counts; nuniq[f].
__global__ __launch_bounds__(kWave) void xs_scan_kernel(int32_t* __restrict__ cnt, int nc,
                                                        int32_t* __restrict__ nuniq) {
  const int f = blockIdx.x, lane = lane_id();
  int32_t* c = cnt + (int64_t)f * nc;
  uint32_t carry = 0;
  for (int b = 0; b < nc; b += kWave) {
    const int i = b + lane;
    const uint32_t v = i < nc ? (uint32_t)c[i] : 0u;
    const uint32_t incl = wave_incl_scan_dpp(v);
    if (i < nc) c[i] = (int32_t)(carry + incl - v);
    carry += __shfl(incl, kWave - 1, kWave);
  }
  if (lane == 0) nuniq[f] = (int32_t)carry;
}

// Sort tile: kNT threads x 16 keys (MPITREE_SORT_TILE=4096 / 8192 / 16384, default 8192).
static int xs_nt() {
  static const int nt = [] {
    const char* v = std::getenv("MPITREE_SORT_TILE");
    const int t = v ? std::atoi(v) : 8192;
    return t == 4096 ? 256 : t == 16384 ? 1024 : 512;
  }();
  return nt;
}
static int64_t xs_tiles(int64_t n) {
  const int64_t tile = (int64_t)xs_nt() * kRsItems;
  return (n + tile - 1) / tile;
}

// temp: [counts F * T * 256 | totals F * 256] u32 (every word written before it is read)
size_t exact_setup_temp_bytes(int64_t n, int F) {
  const int64_t T = xs_tiles(n);
  return (size_t)((int64_t)F * T * 256 + (int64_t)F * 256) * 4;
}

template <int kNT>
static void xs_sort_passes(hipStream_t stream, int64_t n, int F, int64_t T, uint32_t* keys0,
                           uint32_t* keys1, uint32_t* rows0, uint32_t* rows1, uint32_t* counts,
                           uint32_t* totals, const int32_t* ylab) {
  // keys 1 -> 0 -> 1 -> 0 -> 1; rows (generated) -> 0 -> 1 -> 0 -> 1
  uint32_t* kb[2] = {keys0, keys1};
  uint32_t* rb[2] = {rows0, rows1};
  const unsigned grid = (unsigned)(F * T);
  const int lds = kNT * kRsItems * 2 * 4;
  MT_HIP_CHECK(mt_set_max_lds((const void*)xs_scatter_kernel<kNT, true, false>, lds));
  MT_HIP_CHECK(mt_set_max_lds((const void*)xs_scatter_kernel<kNT, true, true>, lds));
  MT_HIP_CHECK(mt_set_max_lds((const void*)xs_scatter_kernel<kNT, false, false>, lds));
  for (int q = 0; q < kRsPasses; ++q) {
    const int src = (q & 1) ? 0 : 1, dst = src ^ 1;
    hipLaunchKernelGGL(xs_tile_count_kernel<kNT>, dim3(grid), dim3(kNT), 0, stream, kb[src], n,
                       (int)T, 8 * q, counts);
    MT_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(xs_tile_scan_kernel, dim3(F, 256 / kWave), dim3(kWave * kRsScanGroups), 0,
                       stream, counts, (int)T, totals);
    MT_HIP_CHECK(hipGetLastError());
    if (q == 0 && ylab) {
      hipLaunchKernelGGL((xs_scatter_kernel<kNT, true, true>), dim3(grid), dim3(kNT), lds, stream,
                         kb[src], nullptr, kb[dst], rb[dst], n, (int)T, 8 * q, counts, totals,
                         ylab);
    } else if (q == 0) {
      hipLaunchKernelGGL((xs_scatter_kernel<kNT, true, false>), dim3(grid), dim3(kNT), lds,
                         stream, kb[src], nullptr, kb[dst], rb[dst], n, (int)T, 8 * q, counts,
                         totals, nullptr);
    } else {
      hipLaunchKernelGGL((xs_scatter_kernel<kNT, false, false>), dim3(grid), dim3(kNT), lds, stream,
                         kb[src], rb[src], kb[dst], rb[dst], n, (int)T, 8 * q, counts, totals,
                         nullptr);
    }
    MT_HIP_CHECK(hipGetLastError());
  }
}

// Phase 1 (before the host learns the largest unique count): keys, sort, counts.
// keys/rows: two u32 buffers each of n * F (ping-pong; the result is in [1]);
// cnt: int32 [F][nc]; nuniq: int32 [F]; ylab (or null): labels < 128 carried in bits
// 25..31 of the sorted row values.
void exact_setup_sort(hipStream_t stream, const float* X, int64_t n, int F, uint32_t* keys0,
                      uint32_t* keys1, uint32_t* rows0, uint32_t* rows1, void* temp,
                      size_t temp_bytes, int32_t* cnt, int32_t* nuniq, int xs, int f_lo,
                      const int32_t* ylab) {
  if (xs <= 0) xs = F;
  if (n <= 0 || F <= 0) return;
  if (n >= (int64_t)1 << 24) throw std::runtime_error("exact setup: rows < 2^24");
  if (temp_bytes < exact_setup_temp_bytes(n, F))
    throw std::runtime_error("exact setup: temp buffer too small");
  const int64_t T = xs_tiles(n);
  if ((int64_t)F * T >= ((int64_t)1 << 31)) throw std::runtime_error("exact setup: too many tiles");
  uint32_t* counts = static_cast<uint32_t*>(temp);
  uint32_t* totals = counts + (int64_t)F * T * 256;
  dim3 tg((unsigned)((n + kXsTile - 1) / kXsTile), (unsigned)((F + kXsTile - 1) / kXsTile));
  hipLaunchKernelGGL(xs_keys_kernel, tg, dim3(kXsThreads), 0, stream, X, n, F, xs, f_lo, keys1);
  MT_HIP_CHECK(hipGetLastError());
  if (xs_nt() == 256) {
    xs_sort_passes<256>(stream, n, F, T, keys0, keys1, rows0, rows1, counts, totals, ylab);
  } else if (xs_nt() == 1024) {
    xs_sort_passes<1024>(stream, n, F, T, keys0, keys1, rows0, rows1, counts, totals, ylab);
  } else {
    xs_sort_passes<512>(stream, n, F, T, keys0, keys1, rows0, rows1, counts, totals, ylab);
  }
  const int nc = (int)((n + kXsChunk - 1) / kXsChunk);
  hipLaunchKernelGGL(xs_count_kernel, dim3(nc, F), dim3(kXsThreads), 0, stream, keys1, n, nc,
                     cnt);
  MT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(xs_scan_kernel, dim3(F), dim3(kWave), 0, stream, cnt, nc, nuniq);
  MT_HIP_CHECK(hipGetLastError());
}

int exact_setup_chunk() { return kXsChunk; }

}  // namespace mt
