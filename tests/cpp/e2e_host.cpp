// e2e_host.cpp -- the PCIe-inclusive rate of the host pipelines
// (kvh_meow128_fixed_host, kvh_meow128_var_host and their _multi forms)
// from a plain C++ host, i.e. the way raikv's C/C++ would call the C-ABI, on
// the system HIP runtime.  (A Python process that imports torch runs torch's
// bundled HIP runtime instead, whose copies overlap less: bench.py reports
// both.)  Keys, offsets and hashes live in pinned host memory from
// kvh_host_alloc; the output is checked word for word against the
// device-resident kernel on the same keys before timing.
//   usage: e2e_host [n=50000000] [key_len=16, 0 = zipf 8-256 B] [reps=5] [devices=0]
//   (devices: comma list for the _multi entries, e.g. 0,1,2,3; default: the
//   single-device entry on the current device)
// prints one JSON line.
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <string>
#include <vector>
#include "kvh.h"

static int fail(const char* what) {
  printf("{\"error\": \"%s\", \"kvh\": %d}\n", what, kvh_last_error());
  return 1;
}

// YCSB zipfian(theta 0.99) over `items` ranks, the generator the reference
// ports in include/raikv/zipf.h:8-81 (raikv_amd/workload.py zipf_lengths):
// key length = 8 + rank, 8-256 B (config C2's distribution).
struct Zipf {
  double theta = 0.99, alpha, zetan = 0, eta, base1;
  uint64_t items;
  explicit Zipf(uint64_t n) : items(n) {
    for (uint64_t i = 1; i <= n; i++) zetan += 1.0 / pow((double)i, theta);
    const double zeta2 = 1.0 + 1.0 / pow(2.0, theta);
    alpha = 1.0 / (1.0 - theta);
    eta = (1 - pow(2.0 / n, 1 - theta)) / (1 - zeta2 / zetan);
    base1 = 1.0 + pow(0.5, theta);
  }
  uint64_t rank(double u) const {
    const double uz = u * zetan;
    if (uz < 1.0) return 0;
    if (uz < base1) return 1;
    return std::min<uint64_t>(items - 1, (uint64_t)(items * pow(eta * u - eta + 1.0, alpha)));
  }
};

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 50000000ull;
  const uint32_t L = argc > 2 ? (uint32_t)atoi(argv[2]) : 16u;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  std::vector<int> devs;
  if (argc > 4) {
    std::string s = argv[4];
    for (size_t p = 0; p < s.size();) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      devs.push_back(atoi(s.substr(p, q - p).c_str()));
      p = q + 1;
    }
  }
  const bool var = L == 0;
  const uint64_t s1 = 0xa8e0bcc94d1855f5ull, s2 = 0xad3bec1e8de4a1a3ull;
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  void *hf = nullptr;
  uint64_t* offs = nullptr;
  size_t nbytes = n * L;
  if (var) {
    if (kvh_host_alloc(&hf, 8 * (n + 1))) return fail("kvh_host_alloc");
    offs = (uint64_t*)hf;
    Zipf z(249);
    offs[0] = 0;
    for (size_t i = 0; i < n; i++) offs[i + 1] = offs[i] + 8 + z.rank((rnd() >> 11) * 0x1.0p-53);
    nbytes = offs[n];
  }
  void *hk = nullptr, *ho = nullptr;
  if (kvh_host_alloc(&hk, nbytes + 8) || kvh_host_alloc(&ho, n * 16)) return fail("kvh_host_alloc");
  uint64_t* k64 = (uint64_t*)hk;
  for (size_t i = 0; i < (nbytes + 7) / 8; i++) k64[i] = rnd();  // xorshift64 key bytes
  // reference: the device-resident kernel on the same keys
  void *dk = nullptr, *dout = nullptr, *doff = nullptr;
  if (hipMalloc(&dk, nbytes + 8) != hipSuccess || hipMalloc(&dout, n * 16) != hipSuccess) return fail("hipMalloc");
  if (hipMemcpy(dk, hk, nbytes, hipMemcpyHostToDevice) != hipSuccess) return fail("hipMemcpy");
  if (var) {
    if (hipMalloc(&doff, 8 * (n + 1)) != hipSuccess) return fail("hipMalloc");
    if (hipMemcpy(doff, offs, 8 * (n + 1), hipMemcpyHostToDevice) != hipSuccess) return fail("hipMemcpy");
    if (kvh_meow128_var(dk, (const uint64_t*)doff, n, s1, s2, (uint64_t*)dout, 0, nullptr)) return fail("kvh_meow128_var");
  } else if (kvh_meow128_fixed(dk, L, n, s1, s2, (uint64_t*)dout, 0, nullptr)) {
    return fail("kvh_meow128_fixed");
  }
  std::vector<uint64_t> ref(2 * n);
  if (hipMemcpy(ref.data(), dout, n * 16, hipMemcpyDeviceToHost) != hipSuccess) return fail("hipMemcpy");
  (void)hipFree(dk); (void)hipFree(dout); (void)hipFree(doff);
  auto call = [&]() -> int {
    if (!devs.empty())
      return var ? kvh_meow128_var_host_multi(hk, offs, n, s1, s2, (uint64_t*)ho, 0, devs.data(), (int)devs.size())
                 : kvh_meow128_fixed_host_multi(hk, L, n, s1, s2, (uint64_t*)ho, 0, devs.data(), (int)devs.size());
    return var ? kvh_meow128_var_host(hk, offs, n, s1, s2, (uint64_t*)ho, 0)
               : kvh_meow128_fixed_host(hk, L, n, s1, s2, (uint64_t*)ho, 0);
  };
  memset(ho, 0, n * 16);
  if (call()) return fail("host pipeline");
  if (memcmp(ho, ref.data(), n * 16)) return fail("host pipeline output differs from the device kernel");
  std::vector<double> ts;
  for (int r = 0; r < reps; r++) {
    auto t0 = std::chrono::steady_clock::now();
    if (call()) return fail("host pipeline");
    ts.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  std::sort(ts.begin(), ts.end());
  const double dt = ts[ts.size() / 2];
  const double moved = (double)nbytes + (var ? 8.0 * (n + 1) : 0.0) + 16.0 * n;
  std::string dl;
  for (size_t i = 0; i < devs.size(); i++) dl += (i ? "," : "") + std::to_string(devs[i]);
  printf("{\"hash_per_s\": %.6g, \"GB_per_s_h2d_plus_d2h\": %.4g, \"keys\": %zu, \"key_len\": %s, "
         "\"key_bytes\": %zu, \"reps\": %d, \"devices\": \"%s\", \"runtime\": \"system HIP (C++ host)\"}\n",
         n / dt, moved / dt / 1e9, n, var ? "\"zipf 8-256\"" : std::to_string(L).c_str(), nbytes, reps,
         devs.empty() ? "current" : dl.c_str());
  (void)kvh_host_free(hk); (void)kvh_host_free(ho);
  if (hf) (void)kvh_host_free(hf);
  return 0;
}
