// Split criteria shared bit-for-bit by the host C++ builder and the gfx950 kernels.
//
// The reference scores a threshold with numpy entropy over probabilities
// (reference: mpitree/tree/decision_tree.py:37-51, 76-91). Probabilities make
// the result depend on summation order and on the BLAS used by np.dot, so we
// score with the integer form instead:
//
//   entropy term  E(counts) = T(m) - sum_c T(c_c),   T(x) = x*log2(x)
//   gini term     G(counts) = (m*m - sum_c c_c^2) / m
//   mse term      V(S, m)   = -(S*S)/m   (plus the constant sum y^2)
//
// Each term equals m * impurity(node). A split's cost is term(L) + term(R) and
// its gain is term(parent) - cost, which is (m/1) times the reference's
// information gain, so argmin/argmax decisions are the same while every
// quantity is computed from integers with one fixed sequence of IEEE
// operations. This file is compiled with -ffp-contract=off for both g++ and
// hipcc, so the host oracle, the host builder and the device kernels produce
// identical bits (tests/test_criterion.py checks the numpy mirror as well).
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define MT_HD __host__ __device__ __forceinline__
#else
#define MT_HD static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace mt {

enum Criterion : int32_t { kEntropy = 0, kGini = 1, kSquaredError = 2 };

MT_HD double bits_to_double(uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __longlong_as_double((long long)b);
#else
  double d;
  memcpy(&d, &b, sizeof(d));
  return d;
#endif
}

MT_HD uint64_t double_to_bits(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint64_t)__double_as_longlong(d);
#else
  uint64_t b;
  memcpy(&b, &d, sizeof(b));
  return b;
#endif
}

// x * log2(x) for an integer count x >= 0 (T(0) = T(1) = 0).
// atanh series on m in [1/sqrt2, sqrt2): log(m) = 2 s (1 + z/3 + z^2/5 + ...),
// s = (m-1)/(m+1), z = s^2 <= 0.0295; 11 terms put the truncation below 1 ulp.
MT_HD double xlog2x(uint64_t x) {
  if (x <= 1) return 0.0;
  const double d = (double)x;
  const uint64_t bits = double_to_bits(d);
  int e = (int)((bits >> 52) & 0x7ff) - 1023;
  double m = bits_to_double((bits & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
  if (m > 1.4142135623730951) {
    m = m * 0.5;
    e = e + 1;
  }
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  double p = 0.047619047619047616;  // 1/21
  p = p * z + 0.05263157894736842;  // 1/19
  p = p * z + 0.058823529411764705; // 1/17
  p = p * z + 0.06666666666666667;  // 1/15
  p = p * z + 0.07692307692307693;  // 1/13
  p = p * z + 0.09090909090909091;  // 1/11
  p = p * z + 0.1111111111111111;   // 1/9
  p = p * z + 0.14285714285714285;  // 1/7
  p = p * z + 0.2;                  // 1/5
  p = p * z + 0.3333333333333333;   // 1/3
  p = p * z + 1.0;
  const double lnm = (2.0 * s) * p;
  const double l2 = (double)e + lnm * 1.4426950408889634;  // 1/ln(2)
  return d * l2;
}

// Gini term from the total m and sum of squared class counts (exact ints).
MT_HD double gini_term(int64_t m, int64_t sumsq) {
  if (m <= 0) return 0.0;
  return (double)(m * m - sumsq) / (double)m;
}

// Canonical ties (every classification engine). Splits whose costs are
// mathematically equal can still round differently -- e.g. left/right counts
// [1,2]/[6,1] vs [4,3]/[3,0]: T(3)+T(7)-T(6)-2 == T(7)-8-T(3) since
// T(6) = 2T(3)+6 -- so each node's candidate costs are compared on a grid of
// 2^-32 * (T(m) + m): such ties become exact and the first candidate in
// (feature, threshold) order wins everywhere, which is the reference's stated
// rule (np.argmin over thresholds, np.argmax over features;
// mpitree/tree/decision_tree.py:88-90, 140). rint is round-half-even on host
// and device; the multiply / rint / multiply sequence is the same IEEE ops.
MT_HD double tie_unit(double tm, int64_t m) {
  return (tm + (double)m) * 2.3283064365386963e-10;  // 2^-32
}

MT_HD double tie_round(double cost, double inv_unit, double unit) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_rint(cost * inv_unit) * unit;
#else
  return rint(cost * inv_unit) * unit;
#endif
}

// Squared-error term: -(S^2)/m with S the fixed-point target sum.
MT_HD double mse_term(int64_t m, int64_t s_fixed) {
  if (m <= 0) return 0.0;
  const double s = (double)s_fixed;
  return -((s * s) / (double)m);
}

}  // namespace mt
