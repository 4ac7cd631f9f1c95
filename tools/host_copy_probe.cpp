// Host memcpy rate into pinned staging (measurement only): 16 threads copying a
// 512 MiB pageable source into buffers from hipHostMalloc (default / non-coherent
// / coherent flags) and into plain malloc'd memory, as the scanner's parallel
// range reads do (scanner.cpp read_full: 16 MiB pieces).
// Build: hipcc -O3 tools/host_copy_probe.cpp -o tools/_build_hcp/hcp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

static double copy_rate(uint8_t *dst, const uint8_t *src, size_t n, int nt) {
  const size_t piece = 16ull << 20, np = (n + piece - 1) / piece;
  double best = 0;
  for (int rep = 0; rep < 4; rep++) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
      th.emplace_back([=] {
        for (size_t i = t; i < np; i += nt) {
          const size_t o = i * piece, len = n - o < piece ? n - o : piece;
          memcpy(dst + o, src + o, len);
        }
      });
    for (auto &x : th) x.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (n / s / 1e9 > best) best = n / s / 1e9;
  }
  return best;
}

int main() {
  const size_t n = 512ull << 20;
  uint8_t *src = (uint8_t *)malloc(n);
  memset(src, 1, n);
  struct { const char *name; unsigned flags; } kinds[] = {
      {"hipHostMallocDefault", hipHostMallocDefault},
      {"hipHostMallocNonCoherent", hipHostMallocNonCoherent},
      {"hipHostMallocCoherent", hipHostMallocCoherent}};
  for (int nt : {8, 16}) {
    for (auto &k : kinds) {
      uint8_t *dst = nullptr;
      if (hipHostMalloc((void **)&dst, n, k.flags) != hipSuccess) {
        printf("{\"kind\":\"%s\",\"error\":1}\n", k.name);
        continue;
      }
      memset(dst, 0, n);
      printf("{\"kind\":\"%s\",\"threads\":%d,\"GBs\":%.1f}\n", k.name, nt, copy_rate(dst, src, n, nt));
      hipHostFree(dst);
    }
    uint8_t *dst = (uint8_t *)malloc(n);
    memset(dst, 0, n);
    printf("{\"kind\":\"malloc\",\"threads\":%d,\"GBs\":%.1f}\n", nt, copy_rate(dst, src, n, nt));
    free(dst);
  }
  return 0;
}
