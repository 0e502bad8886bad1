// tools/fetch_calib.hip -- calibration of rocprofv3 FETCH_SIZE for the
// access patterns of the variable-length kernels (MI355X_MICROARCH.md §HBM:
// "other access widths are uncalibrated: calibrate on a known byte count in
// your own access pattern").  Each kernel reads every byte of a 4 GiB buffer
// (far past the 256 MiB Infinity Cache) exactly once, so the true HBM read
// bytes per dispatch are known; FETCH_SIZE per dispatch / 4 GiB is the factor
// for that pattern.  Not part of the product.
//   k_stream   16 B per lane, wave-chunked coalesced runs (k_fixed's loads)
//   k_gather16 each wave owns 12 KiB windows (k_var6: 256 keys x ~47 B) and
//              reads the window's 768 16-byte pieces in a scrambled order,
//              12 pieces per lane (sorted-window key gathers)
//   k_gather4  the same windows read as 4-byte dwords in a scrambled order
//              (partial-chunk loads, load_bytes)
// usage: fetch_calib [which=all|stream|gather16|gather4] [reps=3]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr uint64_t kBytes = 4ull << 30;
constexpr uint32_t kWin = 12288;  // bytes per window

__global__ void __launch_bounds__(1024) k_stream(const v4u* __restrict__ in, uint32_t* __restrict__ sink) {
  const uint64_t n = kBytes / 16, lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (uint64_t b = wave * 256; b < n; b += nw * 256) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const v4u v = __builtin_nontemporal_load(in + b + 64 * u + lane);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads, never true for the fill pattern
}

template <int W>
__global__ void __launch_bounds__(1024) k_gather(const uint8_t* __restrict__ in, uint32_t* __restrict__ sink) {
  constexpr uint32_t pieces = kWin / W, per_lane = pieces / 64;
  const uint64_t nwin = kBytes / kWin, lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (uint64_t w = wave; w < nwin; w += nw) {
    const uint8_t* base = in + w * kWin;
#pragma unroll 4
    for (uint32_t j = 0; j < per_lane; j++) {
      const uint32_t p = ((j * 64 + (uint32_t)lane) * 97u) % pieces;  // 97 is coprime with pieces: a permutation
      if constexpr (W == 16) {
        const v4u v = *(const v4u*)(base + 16 * (uint64_t)p);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      } else {
        acc ^= *(const uint32_t*)(base + 4 * (uint64_t)p);
      }
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const char* which = argc > 1 ? argv[1] : "all";
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
  uint8_t* buf = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  if (hipMemset(buf, 0x5a, kBytes) != hipSuccess) return 1;
  const dim3 grid(cus * 2), block(1024);
  for (int r = 0; r < reps; r++) {
    if (!strcmp(which, "all") || !strcmp(which, "stream"))
      hipLaunchKernelGGL(k_stream, grid, block, 0, 0, (const v4u*)buf, sink);
    if (!strcmp(which, "all") || !strcmp(which, "gather16"))
      hipLaunchKernelGGL(k_gather<16>, grid, block, 0, 0, buf, sink);
    if (!strcmp(which, "all") || !strcmp(which, "gather4"))
      hipLaunchKernelGGL(k_gather<4>, grid, block, 0, 0, buf, sink);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("{\"bytes_read_per_dispatch\": %llu, \"reps\": %d}\n", (unsigned long long)kBytes, reps);
  (void)hipFree(buf);
  (void)hipFree(sink);
  return 0;
}
