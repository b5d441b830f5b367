// Probe: how fast can a kernel write a finished tree's columns straight into
// host memory (zero-copy over PCIe) compared with a device write + one D2H DMA?
// And does that hold for a POSIX shared-memory mapping registered with
// hipHostRegister (what several ranks of one node would share)?
//
//   hipcc --offload-arch=gfx950 -O3 tools/probes/zc_probe.hip -o /tmp/zc_probe
//   ./zc_probe [MB] [reps]
//
// Cases (each the median of `reps`):
//   dev+D2H      kernel writes a device buffer, hipMemcpyAsync to pinned host
//   zc pinned    kernel writes hipHostMalloc'd memory through its device pointer
//   zc shm       kernel writes a /dev/shm mapping registered with hipHostRegister
//   zc shm/8     the same, 1/8 of the bytes (one rank's share at P = 8)
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

// one 16-byte vector store per thread and iteration, grid-stride, coalesced
__global__ __launch_bounds__(256) void fill(int4* __restrict__ out, long long n16, int seed) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16;
       i += (long long)gridDim.x * 256) {
    const int v = (int)i ^ seed;
    out[i] = make_int4(v, v + 1, v + 2, v + 3);
  }
}

static float time_fill(int4* dst, long long n16, int grid, hipStream_t s, int seed,
                       void* d2h_src = nullptr, void* d2h_dst = nullptr) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  hipLaunchKernelGGL(fill, dim3(grid), dim3(256), 0, s, dst, n16, seed);
  if (d2h_src) CK(hipMemcpyAsync(d2h_dst, d2h_src, n16 * 16, hipMemcpyDeviceToHost, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms;
}

static float median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const long long mb = argc > 1 ? atoll(argv[1]) : 120;
  const int reps = argc > 2 ? atoi(argv[2]) : 7;
  const long long bytes = mb << 20;
  const long long n16 = bytes / 16;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  int4* dev;
  CK(hipMalloc(&dev, bytes));
  void* pinned;
  CK(hipHostMalloc(&pinned, bytes, hipHostMallocMapped));
  int4* pinned_d;
  CK(hipHostGetDevicePointer((void**)&pinned_d, pinned, 0));
  // shared memory, as the ranks of one node would map it
  char name[64];
  std::snprintf(name, sizeof name, "/zc_probe_%d", (int)getpid());
  const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, bytes) != 0) {
    std::perror("shm");
    return 1;
  }
  void* shm = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  shm_unlink(name);
  if (shm == MAP_FAILED) {
    std::perror("mmap");
    return 1;
  }
  std::memset(shm, 0, bytes);  // fault the pages in (as a reused buffer would be)
  // registration cost (once per pooled buffer)
  const auto c0 = std::chrono::steady_clock::now();
  CK(hipHostRegister(shm, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  const double reg_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
  int4* shm_d;
  CK(hipHostGetDevicePointer((void**)&shm_d, shm, 0));
  int dev_id = 0, n_cu = 0;
  CK(hipGetDevice(&dev_id));
  CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev_id));
  std::printf("bytes %lld MB, CUs %d, hipHostRegister %.2f ms\n", mb, n_cu, reg_ms);
  for (int grid_mul : {1, 4, 16}) {
    const int grid = n_cu * grid_mul;
    std::vector<float> a, b, c, d;
    for (int r = 0; r < reps; ++r) {
      a.push_back(time_fill(dev, n16, grid, s, r, dev, pinned));
      b.push_back(time_fill(pinned_d, n16, grid, s, r));
      c.push_back(time_fill(shm_d, n16, grid, s, r));
      d.push_back(time_fill(shm_d, n16 / 8, grid, s, r));
    }
    // correctness of the shm writes (last rep wrote seed reps - 1 over the 1/8 prefix)
    const int4* h = (const int4*)shm;
    long long bad = 0;
    for (long long i = 0; i < n16 / 8; i += 4097) {
      const int v = (int)i ^ (reps - 1);
      if (h[i].x != v || h[i].w != v + 3) ++bad;
    }
    const double gb = bytes / 1e9;
    std::printf("grid %5d: dev+D2H %.3f ms (%.1f GB/s) | zc pinned %.3f ms (%.1f GB/s) | "
                "zc shm %.3f ms (%.1f GB/s) | zc shm/8 %.3f ms (%.1f GB/s) | bad %lld\n",
                grid, median(a), gb / median(a) * 1e3, median(b), gb / median(b) * 1e3,
                median(c), gb / median(c) * 1e3, median(d), gb / 8 / median(d) * 1e3, bad);
  }
  CK(hipHostUnregister(shm));
  munmap(shm, bytes);
  CK(hipHostFree(pinned));
  CK(hipFree(dev));
  return 0;
}
