// Shared helpers for the gfx950 kernels (wave64 CDNA4; never warp32 idioms).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

#define MT_HIP_CHECK(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess)                                                         \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

namespace mt {

constexpr int kWave = 64;  // CDNA wavefront width

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

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
