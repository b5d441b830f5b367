// Exhaustive accuracy of the VALU x*log2(x) term (v_log_f32) over every count the
// finisher's fp32 first pass can see (0 <= x < 2^24). The pass's candidate
// threshold is proven from a per-term relative error bound; this measures it.
//
//   hipcc --offload-arch=gfx950 -O3 tools/probes/vlog_probe.hip -o tools/probes/vlog_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ float tv(uint32_t x) {
  const float f = (float)x;
  return f * __builtin_amdgcn_logf(fmaxf(f, 1.0f));
}

__global__ void probe(uint32_t n, unsigned long long* out) {
  // out[0]: max relative error (double bits, x >= 2); out[1]: max error in ulps of
  // the correctly rounded value; out[2]: count of x with a non-exact result
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n) return;
  const double ex = x < 2 ? 0.0 : (double)x * log2((double)x);
  const float v = tv(x);
  const float r = (float)ex;  // correctly rounded
  if (x >= 2) {
    const double rel = fabs((double)v - ex) / ex;
    atomicMax(out, (unsigned long long)__double_as_longlong(rel));
  } else if (v != 0.0f) {
    atomicMax(out + 3, 1ull);
  }
  const int du = abs(__float_as_int(v) - __float_as_int(r));
  atomicMax(out + 1, (unsigned long long)du);
  if (v != r) atomicAdd(out + 2, 1ull);
}

int main() {
  const uint32_t n = 1u << 24;
  unsigned long long* d;
  hipMalloc(&d, 4 * sizeof(unsigned long long));
  hipMemset(d, 0, 4 * sizeof(unsigned long long));
  probe<<<n / 256, 256>>>(n, d);
  unsigned long long h[4];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  double rel;
  memcpy(&rel, &h[0], 8);
  printf("x in [0, 2^24): max rel err %.3e (= %.2f * 2^-24), max ulps vs rounded %llu, "
         "inexact %llu of %u, T(0..1) != 0: %llu\n",
         rel, rel / std::ldexp(1.0, -24), h[1], h[2], n, h[3]);
  hipFree(d);
  return 0;
}
