// scatter_probe: what 32-byte record scatters cost on this GPU (design data
// for the f2 bucketed sort).  n records of 32 bytes move from
// a coalesced source to: (seq) the same index, (bkB) bucket positions for
// 2^B buckets of uniform random keys with 64K-element tiles (LDS-ranked, as
// k_bk_scatter), (perm) a uniform random permutation.  Prints ms per pass.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

struct __attribute__((aligned(16))) Rec { uint64_t a, b, c, d; };

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

__global__ void k_seq(const Rec* __restrict__ in, Rec* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = in[i];
}
__global__ void k_perm(const Rec* __restrict__ in, Rec* __restrict__ out, uint64_t n, uint64_t mask) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[mix(i) & mask] = in[i];  // n = mask + 1: a random map (collisions ok for timing)
}
// tile-ranked bucket scatter: pos[b] preloaded with the tile's bucket bases
__global__ void __launch_bounds__(1024) k_bk(const Rec* __restrict__ in, Rec* __restrict__ out, uint64_t n,
                                             uint32_t B, uint32_t tile) {
  __shared__ uint32_t pos[1 << 14];
  const uint32_t nb = 1u << B;
  const uint64_t per = n / nb;  // bucket b owns [b * per, (b + 1) * per); tiles write their share
  const uint32_t ntiles = (uint32_t)(n / tile);
  for (uint32_t b = threadIdx.x; b < nb; b += 1024) pos[b] = (uint32_t)(b * per + (uint64_t)blockIdx.x * (per / ntiles));
  __syncthreads();
  const uint64_t i0 = (uint64_t)blockIdx.x * tile;
  for (uint32_t t = threadIdx.x; t < tile; t += 1024) {
    const uint64_t i = i0 + t;
    const Rec r = in[i];
    const uint32_t b = (uint32_t)(mix(r.a ^ i) >> (64 - B));  // the input is constant: key off the index
    const uint32_t p = atomicAdd(&pos[b], 1u);
    out[p % n] = r;
  }
}

int main(int argc, char** argv) {
  const uint64_t n = 1ull << 27;  // 134M records, 4 GiB each way
  Rec *in, *out;
  if (hipMalloc(&in, n * sizeof(Rec)) != hipSuccess || hipMalloc(&out, n * sizeof(Rec)) != hipSuccess) return 2;
  hipMemset(in, 0x5a, n * sizeof(Rec));
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto&& launch) {
    launch(); hipDeviceSynchronize();
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    printf("{\"probe\": \"%s\", \"ms\": %.3f, \"GBps_rw\": %.0f}\n", name, best, 2.0 * n * sizeof(Rec) / best / 1e6);
  };
  const uint32_t g = (uint32_t)((n + 255) / 256);
  timeit("seq", [&] { hipLaunchKernelGGL(k_seq, dim3(g), dim3(256), 0, 0, in, out, n); });
  timeit("perm", [&] { hipLaunchKernelGGL(k_perm, dim3(g), dim3(256), 0, 0, in, out, n, n - 1); });
  for (uint32_t B : {6u, 8u, 10u, 12u, 14u})
    for (uint32_t tile : {65536u, 262144u}) {
      char nm[64];
      snprintf(nm, sizeof nm, "bk%u_tile%uk", B, tile / 1024);
      timeit(nm, [&] { hipLaunchKernelGGL(k_bk, dim3((uint32_t)(n / tile)), dim3(1024), 0, 0, in, out, n, B, tile); });
    }
  return 0;
}
