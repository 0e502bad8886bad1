// tools/copy_peak.hip -- the achievable HBM streaming rate for the key-hash
// traffic shape on this box (measurement infrastructure for bench.py's
// roofline.achievable_peak; not part of the product).
//
// Copies n 16-byte items in -> out (16 B read + 16 B written per item, the
// C1 bytes per key) with the access pattern of k_fixed_q (round 4):
// persistent 1024-thread workgroups, each workgroup-iteration (16 waves x
// 64*U items, every load/store instruction a contiguous 1 KiB, non-temporal)
// taken in address order from one ticket counter, the next ticket fetched one
// iteration ahead -- the fastest streaming form measured on this part
// (6.7 TB/s vs 5.2-5.4 for the static per-wave order and 6.2-6.5 for a
// one-shot grid, tools/stream_forms.hip) -- after a settle period so the
// engine clock has left its post-idle transient.  Prints
// one JSON line.
//
// usage: copy_peak [n_items=100000000] [settle_ms=500] [reps=50]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <chrono>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int U>
__global__ void __launch_bounds__(1024) copy_q(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n,
                                               unsigned long long* tk) {
  __shared__ unsigned long long tkl[2];
  const uint32_t tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, wpb = blockDim.x >> 6;
  const uint64_t last = n - 1, per_it = (uint64_t)wpb * 64 * U;
  if (tid == 0) tkl[0] = atomicAdd(tk, 1ull);
  __syncthreads();
  for (uint32_t it = 0;; it++) {
    const uint64_t t = tkl[it & 1];
    if (tid == 0) tkl[(it + 1) & 1] = atomicAdd(tk, 1ull);
    if (t * per_it >= n) break;
    const uint64_t b = t * per_it + (uint64_t)wv * 64 * U;
    if (b < n) {
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
    __syncthreads();
  }
  if (tid == 0) {
    __threadfence();
    if (atomicAdd(tk + 1, 1ull) == (unsigned long long)gridDim.x - 1) {
      atomicExch(tk, 0ull);
      atomicExch(tk + 1, 0ull);
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
  unsigned long long* tk = nullptr;
  CK(hipMalloc(&tk, 16));
  CK(hipMemset(tk, 0, 16));
  CK(hipMalloc(&in, n * 16));
  CK(hipMalloc(&out, n * 16));
  CK(hipMemset(in, 1, n * 16));
  const dim3 grid(cus), block(1024);
  auto t0 = std::chrono::steady_clock::now();
  int settle = 0;
  for (;;) {
    hipLaunchKernelGGL(copy_q<4>, grid, block, 0, 0, in, out, n, tk);
    CK(hipDeviceSynchronize());
    settle++;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms >= settle_ms) break;
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(copy_q<4>, grid, block, 0, 0, in, out, n, tk);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double per = ms / reps;
  printf("{\"copy_GBps\": %.1f, \"ms_per_copy\": %.4f, \"bytes_per_copy\": %llu, \"items\": %llu, "
         "\"settle_launches\": %d, \"reps\": %d, \"pattern\": \"k_fixed_q: in-order workgroup tickets, 16 waves x 64x4 x 16 B, nt loads/stores, grid = CUs x 1024\"}\n",
         32.0 * (double)n / (per * 1e-3) / 1e9, per, (unsigned long long)(32 * n), (unsigned long long)n, settle, reps);
  CK(hipFree(tk));
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
