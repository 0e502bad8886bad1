// e2e_host.cpp -- the PCIe-inclusive rate of the host pipeline
// (kvh_meow128_fixed_host) from a plain C++ host, i.e. the way raikv's C/C++
// would call the C-ABI, on the system HIP runtime.  (A Python process that
// imports torch runs torch's bundled HIP runtime instead, whose copies
// overlap less: bench.py reports both.)  Keys and hashes live in pinned host
// memory from kvh_host_alloc; the output is checked word for word against
// the device-resident kernel on the same keys before timing.
//   usage: e2e_host [n=50000000] [key_len=16] [reps=5]
// prints one JSON line.
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>
#include "kvh.h"

static int fail(const char* what) {
  printf("{\"error\": \"%s\", \"kvh\": %d}\n", what, kvh_last_error());
  return 1;
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 50000000ull;
  const uint32_t L = argc > 2 ? (uint32_t)atoi(argv[2]) : 16u;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const uint64_t s1 = 0xa8e0bcc94d1855f5ull, s2 = 0xad3bec1e8de4a1a3ull;
  void *hk = nullptr, *ho = nullptr;
  if (kvh_host_alloc(&hk, n * L) || kvh_host_alloc(&ho, n * 16)) return fail("kvh_host_alloc");
  uint64_t x = 0x9E3779B97F4A7C15ull;
  uint64_t* k64 = (uint64_t*)hk;
  for (size_t i = 0; i < n * L / 8; i++) {  // xorshift64 key bytes
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    k64[i] = x;
  }
  // reference: the device-resident kernel on the same keys
  void *dk = nullptr, *dout = nullptr;
  if (hipMalloc(&dk, n * L) != hipSuccess || hipMalloc(&dout, n * 16) != hipSuccess) return fail("hipMalloc");
  if (hipMemcpy(dk, hk, n * L, hipMemcpyHostToDevice) != hipSuccess) return fail("hipMemcpy");
  if (kvh_meow128_fixed(dk, L, n, s1, s2, (uint64_t*)dout, 0, nullptr)) return fail("kvh_meow128_fixed");
  std::vector<uint64_t> ref(2 * n);
  if (hipMemcpy(ref.data(), dout, n * 16, hipMemcpyDeviceToHost) != hipSuccess) return fail("hipMemcpy");
  (void)hipFree(dk); (void)hipFree(dout);
  if (kvh_meow128_fixed_host(hk, L, n, s1, s2, (uint64_t*)ho, 0)) return fail("kvh_meow128_fixed_host");
  if (memcmp(ho, ref.data(), n * 16)) return fail("host pipeline output differs from the device kernel");
  std::vector<double> ts;
  for (int r = 0; r < reps; r++) {
    auto t0 = std::chrono::steady_clock::now();
    if (kvh_meow128_fixed_host(hk, L, n, s1, s2, (uint64_t*)ho, 0)) return fail("kvh_meow128_fixed_host");
    ts.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  std::sort(ts.begin(), ts.end());
  const double dt = ts[ts.size() / 2];
  printf("{\"hash_per_s\": %.6g, \"GB_per_s_h2d_plus_d2h\": %.4g, \"keys\": %zu, \"key_len\": %u, \"reps\": %d, "
         "\"runtime\": \"system HIP (C++ host)\"}\n",
         n / dt, n * (L + 16.0) / dt / 1e9, n, L, reps);
  (void)kvh_host_free(hk); (void)kvh_host_free(ho);
  return 0;
}
