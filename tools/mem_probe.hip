// tools/mem_probe.hip -- streaming 16-B-in/16-B-out copy patterns on MI355X:
// which access shape reaches the HBM roof (the key-hash kernel moves the same
// bytes).  Prints TB/s (read + write) per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(1024) copy_pp(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x, US = U * S, last = n - 1;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  v4u A[U], B[U];
  auto ld = [&](uint64_t b, v4u (&X)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) { uint64_t j = b + u * S; j = j < last ? j : last;
      X[u] = NTL ? __builtin_nontemporal_load(in + j) : in[j]; }
  };
  auto st = [&](uint64_t b, const v4u (&X)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) { uint64_t j = b + u * S; j = j < last ? j : last;
      v4u v = X[u]; v.x ^= 0x9e3779b9u;
      if (NTS) __builtin_nontemporal_store(v, out + j); else out[j] = v; }
  };
  ld(i, A);
  do {
    ld(i + US, B); st(i, A);
    ld(i + 2 * US, A); st(i + US, B);
    i += 2 * US;
  } while (i < n);
}

// contiguous per-lane chunk: lane handles U consecutive 16-B items per step (wave covers U KB)
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(1024) copy_blk(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t b = wave * 64 * U; b < n; b += nw * 64 * U) {
    v4u X[U];
#pragma unroll
    for (int u = 0; u < U; u++) { uint64_t j = b + u * 64 + lane; if (j < n) X[u] = NTL ? __builtin_nontemporal_load(in + j) : in[j]; }
#pragma unroll
    for (int u = 0; u < U; u++) { uint64_t j = b + u * 64 + lane; v4u v = X[u]; v.x ^= 1u;
      if (j < n) { if (NTS) __builtin_nontemporal_store(v, out + j); else out[j] = v; } }
  }
}

template <class F>
void timeit(const char* name, F f, uint64_t n, int grid) {
  f(grid); hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 10; r++) f(grid);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 10;
  printf("%-28s grid=%5d  %.3f ms  %.2f TB/s\n", name, grid, ms, 32.0 * n / ms / 1e9);
}

int main() {
  const uint64_t n = 100000000;  // 1.6 GB in, 1.6 GB out
  v4u *in, *out;
  hipMalloc(&in, n * 16); hipMalloc(&out, n * 16);
  hipMemset(in, 1, n * 16);
  for (int grid : {512, 1024, 2048}) {
#define PP(U, L, S) timeit("pp U=" #U " ntl=" #L " nts=" #S, [&](int g) { hipLaunchKernelGGL((copy_pp<U, L, S>), dim3(g), dim3(1024), 0, 0, in, out, n); }, n, grid);
    PP(1, false, false) PP(2, false, false) PP(4, false, false) PP(1, true, true) PP(2, true, true) PP(4, true, true)
    PP(2, false, true) PP(2, true, false)
#define BL(U, L, S) timeit("blk U=" #U " ntl=" #L " nts=" #S, [&](int g) { hipLaunchKernelGGL((copy_blk<U, L, S>), dim3(g), dim3(1024), 0, 0, in, out, n); }, n, grid);
    BL(1, false, false) BL(4, false, false) BL(8, false, false) BL(4, true, true) BL(8, true, true)
  }
  // hipMemcpy D2D reference
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipMemcpy(out, in, n * 16, hipMemcpyDeviceToDevice);
  hipEventRecord(a);
  for (int r = 0; r < 10; r++) hipMemcpy(out, in, n * 16, hipMemcpyDeviceToDevice);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 10;
  printf("hipMemcpy D2D              %.3f ms  %.2f TB/s\n", ms, 32.0 * n / ms / 1e9);
  return 0;
}
