// tools/gather_probe.hip -- microbenchmark: can the vector-memory path (L1/TCP)
// serve part of the AES T-table lookups beside the LDS?  Variant G of the
// round takes G of its 4 lookups per column from a global 1 KiB Td0 table
// (rotated in VALU), the rest from the replicated LDS tables.  Reports
// lane-rounds/s; no HBM traffic in the loop.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../raikv_amd/csrc/meow_dev.hpp"
using namespace kvh;

__device__ uint32_t g_td0[256];

template <int G>
struct MixTab {
  LdsTab<2> L;
  const uint32_t* g;
  __device__ MixTab(const uint32_t* lds, const uint32_t* gt) : L(lds), g(gt) {}
  __device__ __forceinline__ uint32_t gl(uint32_t x, int r) const {
    const uint32_t v = g[x];
    return rotl32(v, 8 * r);
  }
  __device__ __forceinline__ uint32_t col(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
    uint32_t t0, t1, t2, t3;
    t0 = L.ld(__builtin_amdgcn_perm(a, L.lw[0], LdsTab<2>::sel<0>()));
    t1 = L.ld(__builtin_amdgcn_perm(b, L.lw[1], LdsTab<2>::sel<1>()));
    if (G >= 2) t2 = gl((c >> 16) & 255, 2); else t2 = rotl32(L.ld(__builtin_amdgcn_perm(c, L.lw[0], LdsTab<2>::sel<2>())), 16);
    if (G >= 1) t3 = gl(d >> 24, 3); else t3 = rotl32(L.ld(__builtin_amdgcn_perm(d, L.lw[1], LdsTab<2>::sel<3>())), 16);
    return xor3(t0, t1, k) ^ t2 ^ t3;
  }
};

// G = 0..2 global lookups per column; Q: only every Q-th column uses global
template <int G, int U, int Q>
__global__ void __launch_bounds__(1024) probe(uint32_t* out, int rounds) {
  __shared__ uint32_t lds[LdsTab<2>::kWords];
  fill_tables<2>(lds);
  __syncthreads();
  const MixTab<G> TG(lds, g_td0);
  const MixTab<0> TL(lds, g_td0);
  Blk s[U], k;
  for (int u = 0; u < U; u++) for (int c = 0; c < 4; c++) s[u].w[c] = threadIdx.x * 2654435761u + u * 977 + c;
  for (int c = 0; c < 4; c++) k.w[c] = blockIdx.x + c;
  for (int r = 0; r < rounds; r++) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      Blk o;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        if (c % Q == 0)
          o.w[c] = TG.col(s[u].w[c], s[u].w[(c + 3) & 3], s[u].w[(c + 2) & 3], s[u].w[(c + 1) & 3], k.w[c]);
        else
          o.w[c] = TL.col(s[u].w[c], s[u].w[(c + 3) & 3], s[u].w[(c + 2) & 3], s[u].w[(c + 1) & 3], k.w[c]);
      }
      s[u] = o;
    }
  }
  uint32_t x = 0;
  for (int u = 0; u < U; u++) x ^= s[u].w[0] ^ s[u].w[1] ^ s[u].w[2] ^ s[u].w[3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int G, int U, int Q>
void run(int wgs, int rounds) {
  uint32_t* d; hipMalloc(&d, (size_t)wgs * 1024 * 4);
  hipLaunchKernelGGL((probe<G, U, Q>), dim3(wgs), dim3(1024), 0, 0, d, rounds);
  hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  for (int i = 0; i < 5; i++) hipLaunchKernelGGL((probe<G, U, Q>), dim3(wgs), dim3(1024), 0, 0, d, rounds);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
  double lanerounds = (double)wgs * 1024 * U * rounds;
  printf("G=%d Q=%d U=%d: %.3f ms  %.1f G lane-rounds/s (%.2f lane-rounds/ns/CU)\n", G, Q, U, ms,
         lanerounds / ms / 1e6, lanerounds / (ms * 1e6) / 256);
  hipFree(d);
}

int main() {
  uint32_t h[256];
  for (int i = 0; i < 256; i++) h[i] = kTd0.v[i];
  hipMemcpyToSymbol(HIP_SYMBOL(g_td0), h, sizeof h);
  const int R = 2000;
  run<0, 2, 1>(512, R);
  run<1, 2, 4>(512, R);
  run<1, 2, 2>(512, R);
  run<1, 2, 1>(512, R);
  run<2, 2, 2>(512, R);
  run<2, 2, 1>(512, R);
  run<0, 4, 1>(512, R);
  run<1, 4, 2>(512, R);
  run<1, 4, 1>(512, R);
  return 0;
}
