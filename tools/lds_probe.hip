// tools/lds_probe.hip -- microbenchmark: AES-round throughput from LDS tables
// (no global memory in the loop).  Reports rounds/s and lookups/clk/CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <chrono>
#include "../raikv_amd/csrc/meow_dev.hpp"
using namespace kvh;

template <int NT, int U>
__global__ void __launch_bounds__(1024) probe(uint32_t* out, int rounds) {
  __shared__ uint32_t lds[LdsTab<NT>::kWords];
  fill_tables<NT>(lds);
  __syncthreads();
  const LdsTab<NT> T(lds);
  Blk s[U], k;
  for (int u = 0; u < U; u++) for (int c = 0; c < 4; c++) s[u].w[c] = threadIdx.x * 2654435761u + u * 977 + c;
  for (int c = 0; c < 4; c++) k.w[c] = blockIdx.x + c;
  for (int r = 0; r < rounds; r++) {
#pragma unroll
    for (int u = 0; u < U; u++) s[u] = aesdec(s[u], k, T);
  }
  uint32_t x = 0;
  for (int u = 0; u < U; u++) x ^= s[u].w[0] ^ s[u].w[1] ^ s[u].w[2] ^ s[u].w[3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int NT, int U>
void run(int wgs, int rounds, int block) {
  uint32_t* d; hipMalloc(&d, (size_t)wgs * 1024 * 4);
  hipLaunchKernelGGL((probe<NT, U>), dim3(wgs), dim3(block), 0, 0, d, rounds);
  hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  for (int i = 0; i < 5; i++) hipLaunchKernelGGL((probe<NT, U>), dim3(wgs), dim3(block), 0, 0, d, rounds);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
  double lanerounds = (double)wgs * block * U * rounds;
  printf("NT=%d U=%d wgs=%d block=%d: %.3f ms  %.1f G lane-rounds/s  %.2f lookups/ns/CU\n", NT, U, wgs, block, ms,
         lanerounds / ms / 1e6, lanerounds * 16 / (ms * 1e6) / 256);
  hipFree(d);
}

int main() {
  const int R = 4000;
  run<4, 1>(256, R, 1024); run<4, 2>(256, R, 1024); run<4, 4>(256, R, 1024);
  run<2, 1>(512, R, 1024); run<2, 2>(512, R, 1024); run<2, 4>(512, R, 1024);
  run<4, 1>(512, R, 512); run<4, 2>(512, R, 512);
  run<2, 1>(256, R, 1024); run<2, 2>(256, R, 1024);
  return 0;
}
