// Host-sanitizer harness for the native tree builder (cpu_builder_core.h).
//
// Built by tests/test_sanitizers.py with g++ -fsanitize=address,undefined
// (GPU sanitizers are unavailable on the MI355X pool, so the host code is
// what gets sanitized). Reads one problem from a binary file, grows the tree
// with the same Builder the _cpu extension uses, and writes the node table
// back so the test can compare it with the extension's result bit for bit.
//
// input : int64 header {n, F, C, crit, max_depth, mss, msl, threads, code_bytes}
//         codes [n][F] (u8 or u16) | labels int32 [n] (or fixed-point int64 [n]
//         for squared error) | nbins int32 [F]
// output: int64 N, then per node {feature, bin, depth, left, right, nsamp,
//         stats[S]} as int64 (S = C, or 2 for regression)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cpu_builder_core.h"

template <typename T>
static std::vector<T> read_vec(FILE* f, size_t n) {
  std::vector<T> v(n);
  if (n && std::fread(v.data(), sizeof(T), n, f) != n) {
    std::fprintf(stderr, "short read\n");
    std::exit(2);
  }
  return v;
}

template <typename CodeT>
static int run(FILE* in, FILE* out, const int64_t* h) {
  const int64_t n = h[0], F = h[1];
  const int C = (int)h[2], crit = (int)h[3];
  const bool reg = crit == mt::kSquaredError;
  auto codes = read_vec<CodeT>(in, (size_t)(n * F));
  std::vector<int32_t> ylab;
  std::vector<int64_t> yfix;
  if (reg)
    yfix = read_vec<int64_t>(in, (size_t)n);
  else
    ylab = read_vec<int32_t>(in, (size_t)n);
  auto nbins = read_vec<int32_t>(in, (size_t)F);
  mt::host::Builder<CodeT> b;
  b.codes = codes.data();
  b.n = n;
  b.F = F;
  b.ylab = reg ? nullptr : ylab.data();
  b.yfix = reg ? yfix.data() : nullptr;
  b.nbins = nbins.data();
  b.p = mt::host::Params{crit, (int)h[4], h[5], h[6] < 1 ? 1 : h[6], C, reg};
  b.run(h[7] < 1 ? 1 : (int)h[7]);
  const int64_t N = (int64_t)b.feat.size();
  const int S = reg ? 2 : C;
  std::fwrite(&N, sizeof(N), 1, out);
  for (int64_t i = 0; i < N; ++i) {
    int64_t row[6] = {b.feat[i], b.bin[i], b.depth[i], b.left[i], b.right[i], b.nsamp[i]};
    std::fwrite(row, sizeof(int64_t), 6, out);
    std::fwrite(&b.stats[(size_t)i * S], sizeof(int64_t), (size_t)S, out);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s input.bin output.bin\n", argv[0]);
    return 2;
  }
  FILE* in = std::fopen(argv[1], "rb");
  FILE* out = std::fopen(argv[2], "wb");
  if (!in || !out) return 2;
  auto h = read_vec<int64_t>(in, 9);
  const int rc = h[8] == 1 ? run<uint8_t>(in, out, h.data()) : run<uint16_t>(in, out, h.data());
  std::fclose(in);
  std::fclose(out);
  return rc;
}
