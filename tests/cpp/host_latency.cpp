// host_latency.cpp -- per-call latency and rate of the host-memory pipelines
// (kvh_meow128_fixed_host / kvh_meow128_var_host) at raikv's own batch sizes,
// beside the reference CPU path on the same keys, from a plain C++ host on
// the system HIP runtime (how raikv's C/C++ calls the C-ABI).
//
// raikv hashes 8 keys per prefetch pipe (include/raikv/ev_net.h:442,
// drained in src/ev_net.cpp:677-735) and up to 16K frags per ctest batch
// (test/ctest.c:34, :76-104); this times n = 8 .. 50M keys per call:
//   host_pipe    keys and hashes in pinned host memory (kvh_host_alloc), or
//                pageable (malloc) with "pageable"
//   device_call  the same batch device-resident: kvh_meow128_{fixed,var} on a
//                stream + hipStreamSynchronize (launch + kernel floor)
//   copy_rt      one H2D of the batch's bytes + one D2H of its hashes on one
//                stream + sync, no kernel (the PCIe round-trip floor)
//   ref_cpu_1t   the reference's kv_hash_meow128 over the batch on this
//                thread (oracle/_ref/libkvref.so: the unmodified
//                src/key_hash.c, dlopen'ed as the timed CPU baseline only)
// Outputs of every host-pipeline call size are compared word for word with
// the device-resident kernel before timing.  One JSON line per size.
//   usage: host_latency [key_len=16, 0 = zipf 8-256 B] [pinned|pageable] [sizes] [tiny-path limit, knob 21]
#include <dlfcn.h>
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

// YCSB zipfian(theta 0.99) over 249 ranks (include/raikv/zipf.h:8-81): key
// length 8 + rank, config C2's distribution
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

using clk = std::chrono::steady_clock;
static double secs(clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); }

struct Stat {
  double med, p10, p90;
};
template <class F>
static Stat timed(int reps, F f) {
  std::vector<double> ts;
  for (int r = 0; r < reps; r++) {
    const auto t0 = clk::now();
    if (f()) return {-1, -1, -1};
    ts.push_back(secs(t0));
  }
  std::sort(ts.begin(), ts.end());
  return {ts[ts.size() / 2], ts[ts.size() / 10], ts[ts.size() * 9 / 10]};
}

typedef void (*ref_meow_t)(const void*, size_t, uint64_t*, uint64_t*);

int main(int argc, char** argv) {
  const uint32_t L = argc > 1 ? (uint32_t)atoi(argv[1]) : 16u;
  const bool pageable = argc > 2 && !strcmp(argv[2], "pageable");
  std::vector<size_t> sizes = {8, 64, 1024, 16384, 262144, 4194304, 50000000};
  if (argc > 3) {
    sizes.clear();
    std::string s = argv[3];
    for (size_t p = 0; p < s.size();) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      sizes.push_back(strtoull(s.substr(p, q - p).c_str(), nullptr, 10));
      p = q + 1;
    }
  }
  const bool var = L == 0;
  const int tiny = argc > 4 ? atoi(argv[4]) : -1;
  if (tiny >= 0 && kvh_set_tuning(21, tiny) < 0) return fail("knob 21");
  const size_t nmax = *std::max_element(sizes.begin(), sizes.end());
  const uint64_t s1 = 0xa8e0bcc94d1855f5ull, s2 = 0xad3bec1e8de4a1a3ull;
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  auto halloc = [&](void** p, size_t b) -> int {
    if (pageable) { *p = malloc(b); return *p ? 0 : -1; }
    return kvh_host_alloc(p, b);
  };
  uint64_t* offs = nullptr;
  size_t nbytes = nmax * L;
  if (var) {
    if (halloc((void**)&offs, 8 * (nmax + 1))) return fail("alloc offsets");
    Zipf z(249);
    offs[0] = 0;
    for (size_t i = 0; i < nmax; i++) offs[i + 1] = offs[i] + 8 + z.rank((rnd() >> 11) * 0x1.0p-53);
    nbytes = offs[nmax];
  }
  uint8_t* hk = nullptr;
  uint64_t* ho = nullptr;
  if (halloc((void**)&hk, nbytes + 8) || halloc((void**)&ho, nmax * 16)) return fail("alloc");
  for (size_t i = 0; i < (nbytes + 7) / 8; i++) ((uint64_t*)hk)[i] = rnd();
  void *dk = nullptr, *dout = nullptr, *doff = nullptr;
  if (hipMalloc(&dk, nbytes + 8) != hipSuccess || hipMalloc(&dout, nmax * 16) != hipSuccess) return fail("hipMalloc");
  if (hipMemcpy(dk, hk, nbytes, hipMemcpyHostToDevice) != hipSuccess) return fail("hipMemcpy");
  if (var) {
    if (hipMalloc(&doff, 8 * (nmax + 1)) != hipSuccess) return fail("hipMalloc");
    if (hipMemcpy(doff, offs, 8 * (nmax + 1), hipMemcpyHostToDevice) != hipSuccess) return fail("hipMemcpy");
  }
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return fail("stream");
  // the reference CPU path (test-only baseline): src/key_hash.c's kv_hash_meow128
  ref_meow_t ref_meow = nullptr;
  {
    std::string self = argv[0];
    const size_t sl = self.rfind('/');
    const std::string dir = sl == std::string::npos ? "." : self.substr(0, sl);
    void* h = dlopen((dir + "/../../oracle/_ref/libkvref.so").c_str(), RTLD_NOW | RTLD_LOCAL);
    if (h) ref_meow = (ref_meow_t)dlsym(h, "kv_hash_meow128");
  }
  std::vector<uint64_t> ref(2 * nmax);
  for (size_t n : sizes) {
    auto dev_call = [&]() -> int {
      int rc = var ? kvh_meow128_var(dk, (const uint64_t*)doff, n, s1, s2, (uint64_t*)dout, 0, st)
                   : kvh_meow128_fixed(dk, L, n, s1, s2, (uint64_t*)dout, 0, st);
      return rc ? rc : (hipStreamSynchronize(st) != hipSuccess);
    };
    auto host_call = [&]() -> int {
      return var ? kvh_meow128_var_host(hk, offs, n, s1, s2, ho, 0) : kvh_meow128_fixed_host(hk, L, n, s1, s2, ho, 0);
    };
    const size_t kb = var ? offs[n] : n * L;
    auto copy_rt = [&]() -> int {
      if (hipMemcpyAsync(dk, hk, kb, hipMemcpyHostToDevice, st) != hipSuccess) return 1;
      if (hipMemcpyAsync(ho, dout, 16 * n, hipMemcpyDeviceToHost, st) != hipSuccess) return 1;
      return hipStreamSynchronize(st) != hipSuccess;
    };
    if (dev_call()) return fail("device call");
    if (hipMemcpy(ref.data(), dout, 16 * n, hipMemcpyDeviceToHost) != hipSuccess) return fail("hipMemcpy");
    memset(ho, 0, 16 * n);
    if (host_call()) return fail("host pipeline");
    if (memcmp(ho, ref.data(), 16 * n)) return fail("host pipeline output differs from the device kernel");
    const int reps = (int)std::max<size_t>(5, std::min<size_t>(2000, 20000000 / std::max<size_t>(n, 1)));
    for (int w = 0; w < 3; w++) { host_call(); dev_call(); }
    const Stat h = timed(reps, host_call);
    const Stat d = timed(reps, dev_call);
    const Stat c = timed(reps, copy_rt);
    if (dev_call()) return fail("device call");  // copy_rt overwrote the device keys' bytes with the same data
    double cpu1 = -1;
    if (ref_meow) {
      const int creps = (int)std::max<size_t>(3, std::min<size_t>(2000, 20000000 / std::max<size_t>(n, 1)));
      const Stat r = timed(creps, [&]() -> int {
        for (size_t i = 0; i < n; i++) {
          uint64_t a = s1, b = s2;
          const size_t o = var ? offs[i] : i * L, len = var ? offs[i + 1] - offs[i] : L;
          ref_meow(hk + o, len, &a, &b);
          ho[2 * i] = a; ho[2 * i + 1] = b;
        }
        return 0;
      });
      cpu1 = r.med;
      if (memcmp(ho, ref.data(), 16 * n)) return fail("reference CPU output differs from the device kernel");
    }
    printf("{\"n\": %zu, \"key_len\": %s, \"host_mem\": \"%s\", \"host_pipe_us\": %.2f, \"host_pipe_p10_us\": %.2f, "
           "\"host_pipe_p90_us\": %.2f, \"host_pipe_hash_per_s\": %.4g, \"device_call_us\": %.2f, "
           "\"copy_roundtrip_us\": %.2f, \"ref_cpu_1t_us\": %.2f, \"ref_cpu_1t_hash_per_s\": %.4g, "
           "\"gpu_faster_than_1_cpu_thread\": %s, \"tiny_limit\": %d, \"reps\": %d}\n",
           n, var ? "\"zipf 8-256\"" : std::to_string(L).c_str(), pageable ? "pageable" : "pinned", h.med * 1e6,
           h.p10 * 1e6, h.p90 * 1e6, n / h.med, d.med * 1e6, c.med * 1e6, cpu1 * 1e6, cpu1 > 0 ? n / cpu1 : -1.0,
           cpu1 > 0 && h.med < cpu1 ? "true" : "false", tiny, reps);
    fflush(stdout);
  }
  return 0;
}
