// Probe: cost of a device-wide barrier in a cooperative persistent kernel vs a
// chain of dependent kernel launches on one stream (the level loop's choice).
//
//   hipcc --offload-arch=gfx950 -O3 tools/probes/gridbar_probe.hip -o /tmp/gridbar
//   ./gridbar [blocks_per_cu] [phases] [words_per_block]
//
// Every phase each workgroup writes `words` 32-bit words of its own slab and then
// reads the slab of workgroup (b + 37) % nb written in the previous phase, so the
// barrier must publish dirty data across XCDs (agent-scope release / acquire),
// which is what a fused hist -> scan -> plan -> partition level needs. Every wait
// is bounded by a wall-clock timeout (the kernel reports it instead of hanging).
#include <hip/hip_runtime.h>

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

struct Bar {
  unsigned* count;
  unsigned* gen;
  int* timeout;
};

__device__ __forceinline__ bool grid_sync(const Bar& b, unsigned nb) {
  __syncthreads();
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // release this workgroup's writes, then arrive
    const unsigned a =
        __hip_atomic_fetch_add(b.count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    if (a == nb - 1) {
      __hip_atomic_store(b.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(b.gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > 200000000ull) {  // 2 s at 100 MHz
          atomicExch(b.timeout, 1);
          ok = 0;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

__global__ void persistent_kernel(Bar b, unsigned* slab, int words, int phases) {
  const unsigned nb = gridDim.x;
  for (int p = 0; p < phases; ++p) {
    unsigned* mine = slab + (size_t)blockIdx.x * words;
    for (int i = threadIdx.x; i < words; i += blockDim.x) mine[i] = p * 7 + i;
    if (!grid_sync(b, nb)) return;
    const unsigned* other = slab + (size_t)((blockIdx.x + 37) % nb) * words;
    unsigned acc = 0;
    for (int i = threadIdx.x; i < words; i += blockDim.x) acc += other[i];
    if (acc == 0xdeadbeefu) slab[0] = acc;  // keep the reads
    if (!grid_sync(b, nb)) return;
  }
}

__global__ void phase_write(unsigned* slab, int words, int p) {
  unsigned* mine = slab + (size_t)blockIdx.x * words;
  for (int i = threadIdx.x; i < words; i += blockDim.x) mine[i] = p * 7 + i;
}

__global__ void phase_read(unsigned* slab, int words) {
  const unsigned* other = slab + (size_t)((blockIdx.x + 37) % gridDim.x) * words;
  unsigned acc = 0;
  for (int i = threadIdx.x; i < words; i += blockDim.x) acc += other[i];
  if (acc == 0xdeadbeefu) slab[0] = acc;
}

int main(int argc, char** argv) {
  const int per_cu = argc > 1 ? std::atoi(argv[1]) : 1;
  const int phases = argc > 2 ? std::atoi(argv[2]) : 200;
  const int words = argc > 3 ? std::atoi(argv[3]) : 4096;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persistent_kernel, 256, 0));
  const int nb = cus * std::min(per_cu, occ);
  unsigned *slab, *cnt;
  int* to;
  CK(hipMalloc(&slab, (size_t)nb * words * 4 + 4));
  CK(hipMalloc(&cnt, 256));
  CK(hipMalloc(&to, 4));
  CK(hipMemset(cnt, 0, 256));
  CK(hipMemset(to, 0, 4));
  Bar b{cnt, cnt + 32, to};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    void* args[] = {&b, &slab, (void*)&words, (void*)&phases};
    CK(hipEventRecord(e0));
    CK(hipLaunchCooperativeKernel((const void*)persistent_kernel, dim3(nb), dim3(256), args, 0,
                                  0));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    int t = 0;
    CK(hipMemcpy(&t, to, 4, hipMemcpyDeviceToHost));
    std::printf("persistent: %d blocks (%d CUs), %d phases x 2 barriers, %d words/block: "
                "%.2f us per barrier%s\n",
                nb, cus, phases, words, ms * 1e3 / (2 * phases), t ? " TIMEOUT" : "");
    CK(hipEventRecord(e0));
    for (int p = 0; p < phases; ++p) {
      hipLaunchKernelGGL(phase_write, dim3(nb), dim3(256), 0, 0, slab, words, p);
      hipLaunchKernelGGL(phase_read, dim3(nb), dim3(256), 0, 0, slab, words);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("launch chain: %d x 2 kernels of %d blocks: %.2f us per kernel\n", phases, nb,
                ms * 1e3 / (2 * phases));
  }
  return 0;
}
