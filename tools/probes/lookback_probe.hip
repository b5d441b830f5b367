// Standalone probe of the exact engine's decoupled look-back primitive on one
// GPU: ticketed workgroups publish chunk aggregates / inclusive prefixes into
// tagged status words and walk back for their exclusive prefix; the host checks
// every prefix. Also reports the wall_clock64 rate (watchdog units).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr uint64_t kAgg = 1, kIncl = 2;

__device__ void publish(uint64_t* w, uint32_t tag, uint64_t state, uint32_t v) {
  __hip_atomic_store(w, ((uint64_t)tag << 34) | (state << 32) | (uint64_t)v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void lb_kernel(uint64_t* st, int32_t* tick, int n_chunks, uint32_t tag,
                          int64_t* prefix, int32_t* watch) {
  __shared__ int s_t;
  for (;;) {
    if (threadIdx.x == 0) s_t = atomicAdd(tick, 1);
    __syncthreads();
    const int t = s_t;
    __syncthreads();
    if (t >= n_chunks) break;
    if (threadIdx.x < 64) {
      const uint32_t agg = (uint32_t)(t % 7 + 1);
      if (threadIdx.x == 0) publish(st + t, tag, t == 0 ? kIncl : kAgg, agg);
      int64_t acc = 0;
      if (threadIdx.x == 0 && t > 0) {
        const uint64_t t0 = wall_clock64();
        for (int d = 1; d <= t; ++d) {
          uint64_t s = 0;
          bool dead = false;
          for (uint32_t spins = 0;; ++spins) {
            s = __hip_atomic_load(st + t - d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(s >> 34) == tag) break;
            if ((spins & 63u) == 63u && wall_clock64() - t0 > 200000000ull) {
              atomicExch(watch, 1);
              dead = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (dead) break;
          acc += (uint32_t)s;
          if (((s >> 32) & 3ull) == kIncl) break;
        }
        publish(st + t, tag, kIncl, (uint32_t)(acc + agg));
      }
      if (threadIdx.x == 0) prefix[t] = acc;
    }
  }
}

__global__ void clock_kernel(uint64_t* out) {
  const uint64_t a = wall_clock64();
  const long long c0 = clock64();
  while (clock64() - c0 < 100000000LL) {
  }
  out[0] = wall_clock64() - a;
  out[1] = (uint64_t)(clock64() - c0);
}

int main() {
  const int n = 20000;
  uint64_t* st;
  int32_t* tick;
  int64_t* pre;
  int32_t* watch;
  uint64_t* clk;
  hipMalloc(&st, n * 8);
  hipMalloc(&tick, 4);
  hipMalloc(&pre, n * 8);
  hipMalloc(&watch, 4);
  hipMalloc(&clk, 16);
  hipMemset(st, 0, n * 8);
  hipMemset(watch, 0, 4);
  int bad = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(tick, 0, 4);
    hipLaunchKernelGGL(lb_kernel, dim3(2048), dim3(256), 0, 0, st, tick, n, 7u + rep, pre, watch);
    hipError_t e = hipDeviceSynchronize();
    std::vector<int64_t> h(n);
    hipMemcpy(h.data(), pre, n * 8, hipMemcpyDeviceToHost);
    int64_t want = 0;
    for (int t = 0; t < n; ++t) {
      if (h[t] != want) ++bad;
      want += t % 7 + 1;
    }
    int w = 0;
    hipMemcpy(&w, watch, 4, hipMemcpyDeviceToHost);
    printf("rep %d: err=%s bad=%d watchdog=%d\n", rep, hipGetErrorString(e), bad, w);
  }
  hipLaunchKernelGGL(clock_kernel, dim3(1), dim3(64), 0, 0, clk);
  hipDeviceSynchronize();
  uint64_t c[2];
  hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
  printf("wall_clock64 ticks %llu over %llu shader clocks\n", (unsigned long long)c[0],
         (unsigned long long)c[1]);
  return bad != 0;
}
