// Shared helpers for the gfx950 kernels (wave64 CDNA4; never warp32 idioms).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <map>
#include <mutex>
#include <string>
#include <utility>

#define MT_HIP_CHECK(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess)                                                         \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

namespace mt {

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device,
// size): the driver call costs microseconds of host time and the level loop
// launches half a dozen LDS kernels per level. Sizes only grow (a larger
// maximum serves every smaller launch).
inline hipError_t mt_set_max_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  std::lock_guard<std::mutex> g(mu);
  auto it = done.find({fn, dev});
  if (it != done.end() && it->second >= bytes) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done[{fn, dev}] = bytes;
  return e;
}

constexpr int kWave = 64;  // CDNA wavefront width

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Work claims of a wave: `batch` consecutive items per atomic on one counter (each
// atomic on a shared counter serialises, ~10 ns), and no claim after a batch that
// reached the end. Returns the next item; >= K: done.
struct WaveClaim {
  int k = 0, end = 0;
};
__device__ __forceinline__ int wave_claim_next(WaveClaim& c, int32_t* counter, int K, int batch) {
  if (c.k >= c.end) {
    if (c.end >= K && c.end > 0) return K;
    int v = 0;
    if ((threadIdx.x & (kWave - 1)) == 0) v = atomicAdd(counter, batch);
    v = __builtin_amdgcn_readfirstlane(v);
    c.k = v;
    c.end = v + batch;
  }
  return c.k++;
}
// Items per claim: up to 4 while every wave still gets >= 4 claims.
__device__ __forceinline__ int wave_claim_batch(int K) {
  const int waves = (int)(gridDim.x * (blockDim.x / kWave));
  return max(1, min(4, K / max(1, 4 * waves)));
}

// Inclusive wave64 prefix sum (Hillis-Steele over __shfl_up).
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t o = __shfl_up(v, d, kWave);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ int64_t wave_incl_scan_i64(int64_t v) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    int64_t o = __shfl_up(v, d, kWave);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}

// ---------------------------------------------------------------------------
// DPP wave primitives (GFX9-family DPP: row_shr within 16-lane rows, then
// row_bcast:15 / row_bcast:31 across rows). Each step is a VALU op with a
// few cycles of latency instead of an LDS round trip through ds_bpermute.
constexpr int kDppRowShr = 0x110;   // + n, n in 1..15
constexpr int kDppRowBcast15 = 0x142;
constexpr int kDppRowBcast31 = 0x143;

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, 0xf, false);
}

// Inclusive wave64 prefix sum in 6 DPP steps.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
  v += dpp_u32<kDppRowShr + 1>(0u, v);
  v += dpp_u32<kDppRowShr + 2>(0u, v);
  v += dpp_u32<kDppRowShr + 4>(0u, v);
  v += dpp_u32<kDppRowShr + 8>(0u, v);
  v += dpp_u32<kDppRowBcast15, 0xa>(0u, v);
  v += dpp_u32<kDppRowBcast31, 0xc>(0u, v);
  return v;
}

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_f64(double old, double v) {
  const uint64_t o = (uint64_t)__double_as_longlong(old);
  const uint64_t x = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = dpp_u32<CTRL, ROW_MASK>((uint32_t)o, (uint32_t)x);
  const uint32_t hi = dpp_u32<CTRL, ROW_MASK>((uint32_t)(o >> 32), (uint32_t)(x >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Wave-wide minimum of a double (every lane gets the result).
__device__ __forceinline__ double wave_min_f64_dpp(double v) {
  v = fmin(v, dpp_f64<kDppRowShr + 1>(v, v));
  v = fmin(v, dpp_f64<kDppRowShr + 2>(v, v));
  v = fmin(v, dpp_f64<kDppRowShr + 4>(v, v));
  v = fmin(v, dpp_f64<kDppRowShr + 8>(v, v));
  v = fmin(v, dpp_f64<kDppRowBcast15, 0xa>(v, v));
  v = fmin(v, dpp_f64<kDppRowBcast31, 0xc>(v, v));
  const uint64_t x = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Wave-wide minimum of a float (every lane gets the result).
__device__ __forceinline__ float wave_min_f32_dpp(float v) {
  auto step = [](float x, uint32_t o) { return fminf(x, __uint_as_float(o)); };
  v = step(v, dpp_u32<kDppRowShr + 1>(__float_as_uint(v), __float_as_uint(v)));
  v = step(v, dpp_u32<kDppRowShr + 2>(__float_as_uint(v), __float_as_uint(v)));
  v = step(v, dpp_u32<kDppRowShr + 4>(__float_as_uint(v), __float_as_uint(v)));
  v = step(v, dpp_u32<kDppRowShr + 8>(__float_as_uint(v), __float_as_uint(v)));
  v = step(v, dpp_u32<kDppRowBcast15, 0xa>(__float_as_uint(v), __float_as_uint(v)));
  v = step(v, dpp_u32<kDppRowBcast31, 0xc>(__float_as_uint(v), __float_as_uint(v)));
  return __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(v), 63));
}

// (cost, bin) argmin with ties to the lowest bin, for bins owned by lanes in
// increasing order (lane l holds only bins below lane l+1's): the minimum
// cost, then the lowest lane holding it. Result broadcast to every lane.
__device__ __forceinline__ void wave_argmin_dpp(double& cost, int& bin) {
  const double mn = wave_min_f64_dpp(cost);
  const unsigned long long hit = __ballot(cost == mn);
  const int src = hit ? __ffsll((long long)hit) - 1 : 0;
  bin = __builtin_amdgcn_readlane(bin, src);
  cost = mn;
}

// (cost, bin) lexicographic min across the wave; ties go to the lower bin.
__device__ __forceinline__ void wave_argmin(double& cost, int& bin) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    double oc = __shfl_xor(cost, d, kWave);
    int ob = __shfl_xor(bin, d, kWave);
    if (oc < cost || (oc == cost && ob < bin)) {
      cost = oc;
      bin = ob;
    }
  }
}

// (gain, feature) lexicographic max; ties go to the lower feature.
__device__ __forceinline__ void wave_argmax(double& gain, int& feat, int& bin) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    double og = __shfl_xor(gain, d, kWave);
    int of = __shfl_xor(feat, d, kWave);
    int ob = __shfl_xor(bin, d, kWave);
    if (og > gain || (og == gain && of < feat)) {
      gain = og;
      feat = of;
      bin = ob;
    }
  }
}

}  // namespace mt
