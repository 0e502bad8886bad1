// tools/copy_peak.hip -- the achievable HBM streaming rate for the key-hash
// traffic shape on this box (measurement infrastructure for bench.py's
// roofline.achievable_peak; not part of the product).
//
// Copies n 16-byte items in -> out (16 B read + 16 B written per item, the
// C1 bytes per key) with the access pattern of k_fixed (wave-chunked: wave w
// owns runs of 64*U consecutive items, every load/store instruction moves a
// contiguous 1 KiB, non-temporal), after a settle period so the engine clock
// has left its post-idle transient.  Prints one JSON line.
//
// usage: copy_peak [n_items=100000000] [settle_ms=500] [reps=50]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <chrono>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int U>
__global__ void __launch_bounds__(1024) copy_chunked(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6, last = n - 1;
  for (uint64_t b = wave * 64 * U; b < n; b += nw * 64 * U) {
    v4u X[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      X[u] = __builtin_nontemporal_load(in + (j < last ? j : last));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = b + 64 * u + lane;
      v4u v = X[u];
      v.x ^= 0x9e3779b9u;
      __builtin_nontemporal_store(v, out + (j < last ? j : last));
    }
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;
  const double settle_ms = argc > 2 ? atof(argv[2]) : 500.0;
  const int reps = argc > 3 ? atoi(argv[3]) : 50;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  v4u *in = nullptr, *out = nullptr;
  CK(hipMalloc(&in, n * 16));
  CK(hipMalloc(&out, n * 16));
  CK(hipMemset(in, 1, n * 16));
  const dim3 grid(cus), block(1024);
  auto t0 = std::chrono::steady_clock::now();
  int settle = 0;
  for (;;) {
    hipLaunchKernelGGL(copy_chunked<4>, grid, block, 0, 0, in, out, n);
    CK(hipDeviceSynchronize());
    settle++;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms >= settle_ms) break;
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(copy_chunked<4>, grid, block, 0, 0, in, out, n);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double per = ms / reps;
  printf("{\"copy_GBps\": %.1f, \"ms_per_copy\": %.4f, \"bytes_per_copy\": %llu, \"items\": %llu, "
         "\"settle_launches\": %d, \"reps\": %d, \"pattern\": \"wave-chunked 64x4 x 16 B, nt loads/stores, grid = CUs x 1024\"}\n",
         32.0 * (double)n / (per * 1e-3) / 1e9, per, (unsigned long long)(32 * n), (unsigned long long)n, settle, reps);
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
