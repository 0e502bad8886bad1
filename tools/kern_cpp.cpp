// tools/kern_cpp.cpp -- device-resident C1 kernel time from a C++ host on the
// system HIP runtime (compare bench.py's kernel_ms under torch's runtime).
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include "kvh.h"
int main() {
  const size_t n = 100000000, L = 16;
  void *dk, *dout;
  if (hipMalloc(&dk, n * L) != hipSuccess || hipMalloc(&dout, n * 16) != hipSuccess) return 1;
  {
    std::vector<uint64_t> h(n * L / 8);
    uint64_t x = 88172645463325252ull;
    for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    if (hipMemcpy(dk, h.data(), n * L, hipMemcpyHostToDevice) != hipSuccess) return 1;
  }
  hipStream_t st; if (hipStreamCreate(&st) != hipSuccess) return 1;
  hipEvent_t a, b; if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
  for (int i = 0; i < 20; i++) kvh_meow128_fixed(dk, L, n, 1, 2, (uint64_t*)dout, 0, st);
  hipEvent_t ea[50], eb[50];
  for (int i = 0; i < 50; i++) if (hipEventCreate(&ea[i]) != hipSuccess || hipEventCreate(&eb[i]) != hipSuccess) return 1;
  for (int mode = 0; mode < 4; mode++) {
    // 0: own stream, one event pair around 50 launches; 1: own stream, a pair
    // per launch; 2/3: the null stream, the same two ways
    hipStream_t s = mode < 2 ? st : nullptr;
    float tot = 0;
    if (mode % 2 == 0) {
      if (hipEventRecord(a, s) != hipSuccess) return 1;
      for (int i = 0; i < 50; i++) kvh_meow128_fixed(dk, L, n, 1, 2, (uint64_t*)dout, 0, s);
      if (hipEventRecord(b, s) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return 1;
      if (hipEventElapsedTime(&tot, a, b) != hipSuccess) return 1;
    } else {
      for (int i = 0; i < 50; i++) {
        if (hipEventRecord(ea[i], s) != hipSuccess) return 1;
        kvh_meow128_fixed(dk, L, n, 1, 2, (uint64_t*)dout, 0, s);
        if (hipEventRecord(eb[i], s) != hipSuccess) return 1;
      }
      if (hipEventSynchronize(eb[49]) != hipSuccess) return 1;
      for (int i = 0; i < 50; i++) { float ms = 0; if (hipEventElapsedTime(&ms, ea[i], eb[i]) != hipSuccess) return 1; tot += ms; }
    }
    printf("mode %d: %.4f ms/launch  %.1f G hash/s\n", mode, tot / 50, n / (tot / 50) / 1e6);
  }
  return 0;
}
