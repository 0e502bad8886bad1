// tools/pcie_probe2.hip -- which part of a 3-stage H2D -> kernel -> D2H
// pipeline stops the two PCIe directions from overlapping?  16 MiB chunks,
// 1 GiB in total each way, pinned host memory.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <chrono>
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %d\n", #x, (int)e_); return 1; } } while (0)
__global__ void touch(uint32_t* p, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] ^= 1u;
}
int main() {
  const size_t B = 1ull << 30, C = 16u << 20, NC = B / C;
  void *h1, *h2, *d1, *d2;
  HC(hipHostMalloc(&h1, B, 0)); HC(hipHostMalloc(&h2, B, 0));
  HC(hipMalloc(&d1, B)); HC(hipMalloc(&d2, B));
  memset(h1, 1, B); memset(h2, 2, B);
  hipStream_t si, sk, so; HC(hipStreamCreateWithFlags(&si, hipStreamNonBlocking));
  HC(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking)); HC(hipStreamCreateWithFlags(&so, hipStreamNonBlocking));
  hipEvent_t ei[64], ek[64];
  for (int i = 0; i < 64; i++) { HC(hipEventCreateWithFlags(&ei[i], hipEventDisableTiming)); HC(hipEventCreateWithFlags(&ek[i], hipEventDisableTiming)); }
  for (int mode = 0; mode < 4; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      auto t0 = std::chrono::steady_clock::now();
      for (size_t c = 0; c < NC; c++) {
        char* hi = (char*)h1 + c * C; char* ho = (char*)h2 + c * C;
        char* di = (char*)d1 + c * C; char* dout = (char*)d2 + c * C;
        HC(hipMemcpyAsync(di, hi, C, hipMemcpyHostToDevice, si));
        if (mode == 0) {  // independent directions
          HC(hipMemcpyAsync(ho, dout, C, hipMemcpyDeviceToHost, so));
        } else if (mode == 1) {  // D2H waits for the chunk's H2D
          HC(hipEventRecord(ei[c], si)); HC(hipStreamWaitEvent(so, ei[c], 0));
          HC(hipMemcpyAsync(ho, dout, C, hipMemcpyDeviceToHost, so));
        } else {  // H2D -> kernel (small or full-chip grid) -> D2H
          HC(hipEventRecord(ei[c], si)); HC(hipStreamWaitEvent(sk, ei[c], 0));
          const size_t n = C / 4;
          const int grid = mode == 2 ? 64 : (int)((n + 255) / 256);
          hipLaunchKernelGGL(touch, dim3(grid), dim3(256), 0, sk, (uint32_t*)dout, mode == 2 ? (size_t)64 * 256 : n);
          HC(hipEventRecord(ek[c], sk)); HC(hipStreamWaitEvent(so, ek[c], 0));
          HC(hipMemcpyAsync(ho, dout, C, hipMemcpyDeviceToHost, so));
        }
      }
      HC(hipDeviceSynchronize());
      auto t1 = std::chrono::steady_clock::now();
      printf("mode %d: %.1f GB/s total\n", mode, 2.0 * B / std::chrono::duration<double>(t1 - t0).count() / 1e9);
    }
  }
  return 0;
}
