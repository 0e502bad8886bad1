// tools/pcie_probe.hip -- pinned hipMemcpyAsync bandwidth on the GPU box:
// H2D alone, D2H alone, and both directions at once on two streams (the
// ceiling for the host pipeline kvh_meow128_fixed_host).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <chrono>
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %d\n", #x, (int)e_); return 1; } } while (0)
int main() {
  const size_t B = 1ull << 30;
  void *h1, *h2, *d1, *d2;
  HC(hipHostMalloc(&h1, B, 0)); HC(hipHostMalloc(&h2, B, 0));
  HC(hipMalloc(&d1, B)); HC(hipMalloc(&d2, B));
  memset(h1, 1, B); memset(h2, 2, B);
  hipStream_t s1, s2; HC(hipStreamCreate(&s1)); HC(hipStreamCreate(&s2));
  for (int rep = 0; rep < 2; rep++) {
    auto t0 = std::chrono::steady_clock::now();
    HC(hipMemcpyAsync(d1, h1, B, hipMemcpyHostToDevice, s1)); HC(hipStreamSynchronize(s1));
    auto t1 = std::chrono::steady_clock::now();
    HC(hipMemcpyAsync(h2, d2, B, hipMemcpyDeviceToHost, s2)); HC(hipStreamSynchronize(s2));
    auto t2 = std::chrono::steady_clock::now();
    HC(hipMemcpyAsync(d1, h1, B, hipMemcpyHostToDevice, s1));
    HC(hipMemcpyAsync(h2, d2, B, hipMemcpyDeviceToHost, s2));
    HC(hipStreamSynchronize(s1)); HC(hipStreamSynchronize(s2));
    auto t3 = std::chrono::steady_clock::now();
    const double a = std::chrono::duration<double>(t1 - t0).count(), b = std::chrono::duration<double>(t2 - t1).count(),
                 c = std::chrono::duration<double>(t3 - t2).count();
    printf("H2D %.1f GB/s  D2H %.1f GB/s  both at once %.1f GB/s total\n", B / a / 1e9, B / b / 1e9, 2 * B / c / 1e9);
  }
  // chunked: 16 MiB pieces alternating streams
  const size_t C = 16u << 20;
  auto t0 = std::chrono::steady_clock::now();
  for (size_t o = 0; o < B; o += C) {
    HC(hipMemcpyAsync((char*)d1 + o, (char*)h1 + o, C, hipMemcpyHostToDevice, s1));
    HC(hipMemcpyAsync((char*)h2 + o, (char*)d2 + o, C, hipMemcpyDeviceToHost, s2));
  }
  HC(hipStreamSynchronize(s1)); HC(hipStreamSynchronize(s2));
  auto t1 = std::chrono::steady_clock::now();
  printf("chunked 16 MiB both directions: %.1f GB/s total\n", 2 * B / std::chrono::duration<double>(t1 - t0).count() / 1e9);
  return 0;
}
