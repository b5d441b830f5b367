// Wave-level sort helpers shared by the tiny-subtree kernels (finish.hip,
// finish_reg.hip): a 64-lane bitonic network over two packed 16-bit keys.
#pragma once
#include "common.h"

namespace mt {

// Lane l's value from lane l ^ J (DPP within rows, swizzle, bpermute across halves).
template <int J>
__device__ __forceinline__ uint32_t lane_xor_u32(uint32_t v) {
  if constexpr (J == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // quad [1,0,3,2]
  } else if constexpr (J == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // quad [2,3,0,1]
  } else if constexpr (J == 4) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F);  // xor 4 (bit mode)
  } else if constexpr (J == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
  } else if constexpr (J == 16) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);  // xor 16
  } else {
    return (uint32_t)__shfl_xor((int)v, 32, kWave);
  }
}

typedef unsigned short mt_u16x2 __attribute__((ext_vector_type(2)));

template <int K, int J>
__device__ __forceinline__ uint32_t bitonic_step_pk(uint32_t v, int lane) {
  const uint32_t p = lane_xor_u32<J>(v);
  const mt_u16x2 a = __builtin_bit_cast(mt_u16x2, v), b = __builtin_bit_cast(mt_u16x2, p);
  const uint32_t lo = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(a, b));
  const uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(a, b));
  const bool keep_min = ((lane & K) == 0) == ((lane & J) == 0);
  return keep_min ? lo : hi;
}

// Ascending bitonic sort of 64 lanes, two independent 16-bit keys per lane.
// lg (wave-uniform) = ceil(log2(active lanes)): every lane >= 2^lg holds the
// all-ones key, so the stages that merge blocks larger than 2^lg are skipped --
// after stage 2^lg lanes [0, 2^lg) are ascending and the rest are equal maxima
// (a 32-row subtree runs 15 of the 21 steps, a 16-row one 10).
__device__ __forceinline__ uint32_t bitonic64_pk_u16(uint32_t v, int lane, int lg) {
  v = bitonic_step_pk<2, 1>(v, lane);
  if (lg < 2) return v;
  v = bitonic_step_pk<4, 2>(v, lane);
  v = bitonic_step_pk<4, 1>(v, lane);
  if (lg < 3) return v;
  v = bitonic_step_pk<8, 4>(v, lane);
  v = bitonic_step_pk<8, 2>(v, lane);
  v = bitonic_step_pk<8, 1>(v, lane);
  if (lg < 4) return v;
  v = bitonic_step_pk<16, 8>(v, lane);
  v = bitonic_step_pk<16, 4>(v, lane);
  v = bitonic_step_pk<16, 2>(v, lane);
  v = bitonic_step_pk<16, 1>(v, lane);
  if (lg < 5) return v;
  v = bitonic_step_pk<32, 16>(v, lane);
  v = bitonic_step_pk<32, 8>(v, lane);
  v = bitonic_step_pk<32, 4>(v, lane);
  v = bitonic_step_pk<32, 2>(v, lane);
  v = bitonic_step_pk<32, 1>(v, lane);
  if (lg < 6) return v;
  v = bitonic_step_pk<64, 32>(v, lane);
  v = bitonic_step_pk<64, 16>(v, lane);
  v = bitonic_step_pk<64, 8>(v, lane);
  v = bitonic_step_pk<64, 4>(v, lane);
  v = bitonic_step_pk<64, 2>(v, lane);
  v = bitonic_step_pk<64, 1>(v, lane);
  return v;
}

template <int K, int J>
__device__ __forceinline__ uint32_t bitonic_step_u32(uint32_t v, int lane) {
  const uint32_t p = lane_xor_u32<J>(v);
  const bool keep_min = ((lane & K) == 0) == ((lane & J) == 0);
  return keep_min ? (v < p ? v : p) : (v < p ? p : v);
}

// Ascending bitonic sort of 64 lanes, one 32-bit key per lane (16-bit codes);
// lg as for bitonic64_pk_u16.
__device__ __forceinline__ uint32_t bitonic64_u32(uint32_t v, int lane, int lg) {
  v = bitonic_step_u32<2, 1>(v, lane);
  if (lg < 2) return v;
  v = bitonic_step_u32<4, 2>(v, lane);
  v = bitonic_step_u32<4, 1>(v, lane);
  if (lg < 3) return v;
  v = bitonic_step_u32<8, 4>(v, lane);
  v = bitonic_step_u32<8, 2>(v, lane);
  v = bitonic_step_u32<8, 1>(v, lane);
  if (lg < 4) return v;
  v = bitonic_step_u32<16, 8>(v, lane);
  v = bitonic_step_u32<16, 4>(v, lane);
  v = bitonic_step_u32<16, 2>(v, lane);
  v = bitonic_step_u32<16, 1>(v, lane);
  if (lg < 5) return v;
  v = bitonic_step_u32<32, 16>(v, lane);
  v = bitonic_step_u32<32, 8>(v, lane);
  v = bitonic_step_u32<32, 4>(v, lane);
  v = bitonic_step_u32<32, 2>(v, lane);
  v = bitonic_step_u32<32, 1>(v, lane);
  if (lg < 6) return v;
  v = bitonic_step_u32<64, 32>(v, lane);
  v = bitonic_step_u32<64, 16>(v, lane);
  v = bitonic_step_u32<64, 8>(v, lane);
  v = bitonic_step_u32<64, 4>(v, lane);
  v = bitonic_step_u32<64, 2>(v, lane);
  v = bitonic_step_u32<64, 1>(v, lane);
  return v;
}

}  // namespace mt
