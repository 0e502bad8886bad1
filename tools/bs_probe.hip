// tools/bs_probe.hip -- microbenchmark: bitsliced AESDEC round throughput
// (raikv_amd/csrc/bs_aes.hpp, 8 keys per lane) against the LDS T-table round
// (tools/lds_probe.hip).  No memory traffic in the loop; prints key-rounds/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../raikv_amd/csrc/bs_prelude.hpp"
using namespace kvh;

__device__ __forceinline__ uint32_t rotb(uint32_t x, int r) {  // rotate left by 8r bits
  return r == 0 ? x : __builtin_amdgcn_alignbit(x, x, 32 - 8 * r);
}

template <int S, int UNR = 1>
__global__ void __launch_bounds__(256) probe(uint32_t* out, const uint32_t* keys, int rounds) {
  uint32_t kk[32];
#pragma unroll
  for (int i = 0; i < 32; i++) kk[i] = __builtin_amdgcn_readfirstlane(keys[i]);
  uint32_t u[S][32], v[32];
#pragma unroll
  for (int s = 0; s < S; s++)
#pragma unroll
    for (int i = 0; i < 32; i++) u[s][i] = (threadIdx.x + 1) * 2654435761u + i * 977u + s;
  for (int r = 0; r < rounds; r += UNR) {
#pragma unroll
    for (int s = 0; s < S * UNR; s++) {
#pragma unroll
      for (int row = 0; row < 4; row++) {
        uint32_t t[8];
        bs::inv8(&u[s % S][8 * row], t);
#pragma unroll
        for (int i = 0; i < 8; i++) v[8 * row + i] = rotb(t[i], row);
      }
      bs::lin(v, kk, u[s % S]);
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int s = 0; s < S; s++)
#pragma unroll
    for (int i = 0; i < 32; i++) x ^= u[s][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int S, int UNR = 1>
void run(int wgs, int block, int rounds, uint32_t* keys) {
  uint32_t* d; (void)hipMalloc(&d, (size_t)wgs * block * 4);
  hipLaunchKernelGGL((probe<S, UNR>), dim3(wgs), dim3(block), 0, 0, d, keys, rounds);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  for (int i = 0; i < 5; i++) hipLaunchKernelGGL((probe<S, UNR>), dim3(wgs), dim3(block), 0, 0, d, keys, rounds);
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 5;
  const double kr = (double)wgs * block * 8 * S * rounds;  // 8 keys per lane per state
  printf("bitsliced UNR=%d S=%d wgs=%d block=%d: %.3f ms  %.1f G key-rounds/s (%.2f key-rounds/ns/CU)\n", UNR, S, wgs, block,
         ms, kr / ms / 1e6, kr / (ms * 1e6) / 256);
  (void)hipFree(d);
}

int main() {
  uint32_t h[32];
  for (int i = 0; i < 32; i++) h[i] = (i * 0x9e3779b9u) & 0xff00ff00u;
  uint32_t* keys; (void)hipMalloc(&keys, sizeof h);
  (void)hipMemcpy(keys, h, sizeof h, hipMemcpyHostToDevice);
  const int R = 400;
  // waves per SIMD = wgs / 256 (256-thread workgroups: one wave per SIMD each)
  run<1, 1>(256, 256, R, keys); run<1, 1>(512, 256, R, keys); run<1, 1>(1024, 256, R, keys);
  run<1, 1>(1536, 256, R, keys);
  run<1, 10>(256, 256, R, keys); run<1, 10>(512, 256, R, keys); run<1, 10>(1024, 256, R, keys);
  run<1, 10>(1536, 256, R, keys);
  run<2, 1>(256, 256, R, keys); run<2, 1>(512, 256, R, keys);
  return 0;
}
