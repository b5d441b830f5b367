// Probe: can gfx950 integer MFMA build a many-class node histogram faster than
// the finisher's LDS atomics? (C = 64 spends its block
// finisher in 16 LDS feature-tile histogram passes per node.)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/mfma_hist_probe.hip -o /tmp/mfma_hist
//   ./mfma_hist [nodes] [rows] [classes] [reps]
//
// Workload: `nodes` independent nodes of `rows` rows, 64 features, 256 bins, C
// classes (a C = 64 finisher job is <= 4096 rows). Output per node and feature:
// the [256 bins][C] class histogram, checked by a per-(node, feature) digest and
// in full for node 0 against the host.
//
//   atomic  the finisher's method: one 512-thread workgroup per node, features in
//           LDS tiles of [tile][256][C / 2] words (two 16-bit class counts a
//           word), one ds_add per (row, feature); the tile's rows re-read per tile
//   mfma    H_f = onehot(codes_f)^T onehot(y) on v_mfma_i32_32x32x32_i8: M = bins
//           (8 blocks of 32), N = classes (blocks of 32), K = rows (32 per step);
//           one-hot fragments built in registers from 16-byte code / label loads
//           (codes feature-major for the probe: each lane loads 16 rows at once)
//
// The one-hot product does bins x classes multiply-adds per (row, feature) where
// the atomic pass does one add: 256 x 64 = 16384 MACs against one LDS atomic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

constexpr int kF = 64, kB = 256;
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// digest of one [256][C] histogram: sum of count * (cell + 1), wrapping
__device__ __host__ inline uint32_t cell_w(int b, int c, int C) { return (uint32_t)(b * C + c) * 2654435761u + 1u; }

// ---- atomic: the finisher's LDS histogram, FT features a tile
template <int FT, bool kDigest>
__global__ __launch_bounds__(512) void hist_atomic(const uint8_t* __restrict__ codes_rm,  // [node][rows][64]
                                                   const uint8_t* __restrict__ y, int rows, int C,
                                                   uint32_t* __restrict__ digest) {
  extern __shared__ uint32_t h[];  // [FT][256][W]
  const int node = blockIdx.x, tid = threadIdx.x;
  const int W = (C + 1) / 2;
  const uint8_t* cr = codes_rm + (size_t)node * rows * kF;
  const uint8_t* yl = y + (size_t)node * rows;
  for (int f0 = 0; f0 < kF; f0 += FT) {
    for (int e = tid; e < FT * kB * W; e += 512) h[e] = 0;
    __syncthreads();
    // one thread per (row, feature of the tile)
    for (int t = tid; t < rows * FT; t += 512) {
      const int r = t / FT, fl = t % FT;
      const int code = cr[(size_t)r * kF + f0 + fl];
      const int c = yl[r];
      atomicAdd(&h[(fl * kB + code) * W + (c >> 1)], 1u << (16 * (c & 1)));
    }
    __syncthreads();
    if (!kDigest) {  // (timing: keep one word per tile live)
      if (tid == 0) digest[node * kF + f0] = h[(node + f0) % (FT * kB * W)];
      __syncthreads();
      continue;
    }
    for (int fl = tid >> 6; fl < FT; fl += 8) {  // one wave per feature: its digest
      uint32_t d = 0;
      for (int e = (tid & 63); e < kB * C; e += 64) {
        const int b = e / C, c = e % C;
        d += ((h[(fl * kB + b) * W + (c >> 1)] >> (16 * (c & 1))) & 0xffffu) * cell_w(b, c, C);
      }
      for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      if ((tid & 63) == 0) digest[node * kF + f0 + fl] = d;
    }
    __syncthreads();
  }
}

// ---- mfma: one wave per feature (8 waves, 8 features each), bins in two halves
// of 4 blocks (128 accumulator registers), classes in CB blocks of 32.
template <int CB>
__global__ __launch_bounds__(512) void hist_mfma(const uint8_t* __restrict__ codes_fm,  // [node][64][rows]
                                                 const uint8_t* __restrict__ y, int rows, int C,
                                                 uint32_t* __restrict__ digest,
                                                 int32_t* __restrict__ full0) {
  const int node = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const uint8_t* yl = y + (size_t)node * rows;
  for (int f = wave; f < kF; f += 8) {
    const uint8_t* cf = codes_fm + ((size_t)node * kF + f) * rows;
    uint32_t d = 0;
    for (int half = 0; half < 2; ++half) {
      v16i acc[4][CB];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j) acc[i][j] = v16i{};
      for (int k0 = 0; k0 < rows; k0 += 32) {
        // lane half hh holds rows k0 + 16 hh + [0, 16): 16 codes, 16 labels
        const uint4 cv = *reinterpret_cast<const uint4*>(cf + k0 + 16 * hh);
        const uint4 lv = *reinterpret_cast<const uint4*>(yl + k0 + 16 * hh);
        const uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w}, lw[4] = {lv.x, lv.y, lv.z, lv.w};
        v4i bf[CB];
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          const uint32_t want = (uint32_t)(cb * 32 + r);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) x |= (((lw[q] >> (8 * j)) & 0xffu) == want ? 1u : 0u) << (8 * j);
            bf[cb][q] = (int)x;
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t want = (uint32_t)((half * 4 + i) * 32 + r);
          v4i af;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) x |= (((cw[q] >> (8 * j)) & 0xffu) == want ? 1u : 0u) << (8 * j);
            af[q] = (int)x;
          }
#pragma unroll
          for (int cb = 0; cb < CB; ++cb)
            acc[i][cb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, bf[cb], acc[i][cb], 0, 0, 0);
        }
      }
      // C/D map: col = lane & 31 (class), row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5) (bin)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int b = (half * 4 + i) * 32 + (g & 3) + 8 * (g >> 2) + 4 * hh;
            const int c = cb * 32 + r;
            const int v = acc[i][cb][g];
            if (c < C) {
              d += (uint32_t)v * cell_w(b, c, C);
              if (node == 0 && full0) full0[((size_t)f * kB + b) * C + c] = v;
            }
          }
    }
    for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
    if (lane == 0) digest[node * kF + f] = d;
  }
}

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? std::atoi(argv[1]) : 512;
  const int rows = argc > 2 ? std::atoi(argv[2]) : 2048;  // multiple of 32
  const int C = argc > 3 ? std::atoi(argv[3]) : 64;       // <= 64 (two 32-class blocks)
  const int reps = argc > 4 ? std::atoi(argv[4]) : 10;
  if (rows % 32 || C > 64 || C < 2) {
    std::fprintf(stderr, "rows must be a multiple of 32, 2 <= C <= 64\n");
    return 2;
  }
  const size_t ncode = (size_t)nodes * rows * kF;
  std::vector<uint8_t> crm(ncode), cfm(ncode), yl((size_t)nodes * rows);
  uint64_t s = 88172645463325252ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  for (int nd = 0; nd < nodes; ++nd)
    for (int r = 0; r < rows; ++r) {
      yl[(size_t)nd * rows + r] = (uint8_t)(rnd() % C);
      for (int f = 0; f < kF; ++f) {
        const uint8_t v = (uint8_t)(rnd() & 255);
        crm[((size_t)nd * rows + r) * kF + f] = v;
        cfm[((size_t)nd * kF + f) * rows + r] = v;
      }
    }
  uint8_t *d_rm, *d_fm, *d_y;
  uint32_t *d_da, *d_dm;
  int32_t* d_full;
  CK(hipMalloc(&d_rm, ncode));
  CK(hipMalloc(&d_fm, ncode));
  CK(hipMalloc(&d_y, yl.size()));
  CK(hipMalloc(&d_da, (size_t)nodes * kF * 4));
  CK(hipMalloc(&d_dm, (size_t)nodes * kF * 4));
  CK(hipMalloc(&d_full, (size_t)kF * kB * C * 4));
  CK(hipMemcpy(d_rm, crm.data(), ncode, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_fm, cfm.data(), ncode, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_y, yl.data(), yl.size(), hipMemcpyHostToDevice));
  constexpr int FT = 4;
  const int W = (C + 1) / 2;
  const size_t lds = (size_t)FT * kB * W * 4;
  CK(hipFuncSetAttribute((const void*)hist_atomic<FT, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)hist_atomic<FT, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_it = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  // build only (the finisher then scans the tile), and build + a full read of every tile
  const float ta = time_it([&] {
    hipLaunchKernelGGL((hist_atomic<FT, false>), dim3(nodes), dim3(512), lds, 0, d_rm, d_y, rows, C, d_da);
  });
  const float tad = time_it([&] {
    hipLaunchKernelGGL((hist_atomic<FT, true>), dim3(nodes), dim3(512), lds, 0, d_rm, d_y, rows, C, d_da);
  });
  const float tm = time_it([&] {
    if (C > 32)
      hipLaunchKernelGGL(hist_mfma<2>, dim3(nodes), dim3(512), 0, 0, d_fm, d_y, rows, C, d_dm, d_full);
    else
      hipLaunchKernelGGL(hist_mfma<1>, dim3(nodes), dim3(512), 0, 0, d_fm, d_y, rows, C, d_dm, d_full);
  });
  std::vector<uint32_t> da((size_t)nodes * kF), dm((size_t)nodes * kF);
  std::vector<int32_t> full((size_t)kF * kB * C);
  CK(hipMemcpy(da.data(), d_da, da.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(dm.data(), d_dm, dm.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(full.data(), d_full, full.size() * 4, hipMemcpyDeviceToHost));
  // host check of node 0 and of every digest
  std::vector<int32_t> ref((size_t)kF * kB * C, 0);
  for (int r = 0; r < rows; ++r)
    for (int f = 0; f < kF; ++f) ++ref[((size_t)f * kB + crm[(size_t)r * kF + f]) * C + yl[r]];
  long bad_full = 0;
  for (size_t i = 0; i < ref.size(); ++i) bad_full += ref[i] != full[i];
  uint32_t d0 = 0;
  for (int f = 0; f < 1; ++f)
    for (int b = 0; b < kB; ++b)
      for (int c = 0; c < C; ++c) d0 += (uint32_t)ref[((size_t)f * kB + b) * C + c] * cell_w(b, c, C);
  long bad_dig = 0;
  for (size_t i = 0; i < da.size(); ++i) bad_dig += da[i] != dm[i];
  const double row_feat = (double)nodes * rows * kF;
  const double macs = row_feat * kB * (C > 32 ? 64 : 32);
  std::printf("nodes=%d rows=%d C=%d features=%d bins=%d\n", nodes, rows, C, kF, kB);
  std::printf("atomic: %.3f ms  (%.2f G row-features/s); with every cell read back: %.3f ms\n", ta,
              row_feat / ta / 1e6, tad);
  std::printf("mfma:   %.3f ms  (%.2f G row-features/s, %.1f TMAC/s i8 incl. one-hot build)\n", tm,
              row_feat / tm / 1e6, macs / tm / 1e9);
  std::printf("mfma / atomic time: %.1fx (build only), %.1fx (with read-back)\n", tm / ta, tm / tad);
  std::printf("check: node 0 full histogram mismatches %ld of %zu; digest mismatches %ld of %zu; "
              "node 0 feature 0 digest host %u atomic %u mfma %u\n",
              bad_full, ref.size(), bad_dig, da.size(), d0, da[0], dm[0]);
  return (bad_full || bad_dig) ? 1 : 0;
}
