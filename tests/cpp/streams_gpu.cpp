// streams_gpu.cpp -- TEST: the ticket state of the in-order streaming kernels
// for every kind of stream a caller can pass:
//   1. four host threads hashing at once on hipStreamPerThread (one handle
//      value, four different streams), fixed and variable length, ragged
//      sizes, into outputs poisoned with 0xA5 bytes; every launch equals the
//      oracle and leaves the words past its n untouched;
//   2. launches captured into graphs on one stream (whose ticket words already
//      exist) and replayed on two other streams at once while direct launches
//      run on the capture stream;
//   3. kvh_stream_release before a stream is destroyed, and a new stream after.
// The oracle (oracle/liboracle.so, test infrastructure) is the checker.
// Runs under pytest -m gpu (tests/test_gpu_parity.py::test_streams_program).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <atomic>
#include <thread>
#include <vector>
#include "kvh.h"

extern "C" {
void orc_batch_fixed(const uint8_t* keys, size_t len, size_t n, uint64_t s1, uint64_t s2, uint64_t* out, int fixup);
void orc_batch_var(const uint8_t* keys, const uint64_t* offs, size_t n, uint64_t s1, uint64_t s2, uint64_t* out,
                   int fixup);
}

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)
#define KV(x)                                                                                 \
  do {                                                                                        \
    int r_ = (x);                                                                             \
    if (r_ != 0) {                                                                            \
      fprintf(stderr, "%s:%d %s: %d (%s)\n", __FILE__, __LINE__, #x, r_, kvh_strerror(r_));   \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)

static const uint64_t S1 = 0xA8E0BCC94D1855F5ull, S2 = 0xAD3BEC1E8DE4A1A3ull;
static const uint64_t POISON = 0xA5A5A5A5A5A5A5A5ull;

struct Batch {
  size_t nf = 0, nv = 0;
  std::vector<uint8_t> kf, kv;
  std::vector<uint64_t> offs, wf, wv;  // oracle hashes
  uint8_t *dkf = nullptr, *dkv = nullptr;
  uint64_t* doffs = nullptr;
};

static uint64_t rnd(uint64_t& s) {
  s ^= s << 13; s ^= s >> 7; s ^= s << 17;
  return s;
}

static void make(Batch& B, size_t nf, size_t nv) {
  uint64_t r = 88172645463325252ull;
  B.nf = nf;
  B.nv = nv;
  B.kf.resize(nf * 16);
  for (auto& b : B.kf) b = (uint8_t)rnd(r);
  B.offs.resize(nv + 1);
  B.offs[0] = 0;
  for (size_t i = 0; i < nv; i++) B.offs[i + 1] = B.offs[i] + (rnd(r) % 121);  // 0..120-byte keys
  B.kv.resize(B.offs[nv] + 1);
  for (auto& b : B.kv) b = (uint8_t)rnd(r);
  B.wf.resize(2 * nf);
  B.wv.resize(2 * nv);
  orc_batch_fixed(B.kf.data(), 16, nf, S1, S2, B.wf.data(), 0);
  orc_batch_var(B.kv.data(), B.offs.data(), nv, S1, S2, B.wv.data(), 0);
  CK(hipMalloc(&B.dkf, B.kf.size()));
  CK(hipMalloc(&B.dkv, B.kv.size()));
  CK(hipMalloc(&B.doffs, 8 * B.offs.size()));
  CK(hipMemcpy(B.dkf, B.kf.data(), B.kf.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(B.dkv, B.kv.data(), B.kv.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(B.doffs, B.offs.data(), 8 * B.offs.size(), hipMemcpyHostToDevice));
}

// words [0, 2n) equal want, words [2n, cap) still the poison; returns the bad count
static long check(const std::vector<uint64_t>& got, const std::vector<uint64_t>& want, size_t n, size_t cap) {
  long bad = 0;
  for (size_t i = 0; i < 2 * n; i++) bad += got[i] != want[i];
  for (size_t i = 2 * n; i < 2 * cap; i++) bad += got[i] != POISON;
  return bad;
}

// 1. hipStreamPerThread from four threads at once
static long per_thread_streams(const Batch& B, int iters) {
  std::atomic<long> bad{0};
  std::atomic<int> ready{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 4; t++) {
    th.emplace_back([&, t] {
      const size_t cap = B.nf > B.nv ? B.nf : B.nv;
      uint64_t* d = nullptr;
      CK(hipMalloc(&d, 16 * cap));
      std::vector<uint64_t> h(2 * cap);
      ready++;
      while (ready.load() < 4) std::this_thread::yield();  // start together
      for (int it = 0; it < iters; it++) {
        const bool var = ((it + t) & 1) != 0;
        const size_t N = var ? B.nv : B.nf;
        const size_t n = N - ((size_t)t * 7919 + (size_t)it * 104729) % (N / 3);  // ragged, per thread
        CK(hipMemsetAsync(d, 0xA5, 16 * cap, hipStreamPerThread));
        if (var)
          KV(kvh_meow128_var(B.dkv, B.doffs, n, S1, S2, d, 0, (void*)hipStreamPerThread));
        else
          KV(kvh_meow128_fixed(B.dkf, 16, n, S1, S2, d, 0, (void*)hipStreamPerThread));
        CK(hipMemcpyAsync(h.data(), d, 16 * cap, hipMemcpyDeviceToHost, hipStreamPerThread));
        CK(hipStreamSynchronize(hipStreamPerThread));
        const long b = check(h, var ? B.wv : B.wf, n, cap);
        if (b) fprintf(stderr, "thread %d iter %d (%s n=%zu): %ld bad words\n", t, it, var ? "var" : "fixed", n, b);
        bad += b;
      }
      CK(hipFree(d));
    });
  }
  for (auto& x : th) x.join();
  return bad.load();
}

// 2. graphs captured on one stream, replayed on two others while the capture
// stream runs direct launches
static long graphs(const Batch& B, int rounds) {
  hipStream_t cap, sa, sb;
  CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  const size_t nf = B.nf, nv = B.nv;
  uint64_t *of[3], *ov[2];
  for (auto& p : of) CK(hipMalloc(&p, 16 * nf));
  for (auto& p : ov) CK(hipMalloc(&p, 16 * nv));
  // a direct launch first: the capture stream's ticket words exist (round 4
  // baked them into the graphs)
  KV(kvh_meow128_fixed(B.dkf, 16, nf, S1, S2, of[2], 0, cap));
  CK(hipStreamSynchronize(cap));
  hipGraphExec_t ex[2];
  for (int g = 0; g < 2; g++) {
    hipGraph_t gr;
    CK(hipStreamBeginCapture(cap, hipStreamCaptureModeGlobal));
    CK(hipMemsetAsync(of[g], 0xA5, 16 * nf, cap));
    CK(hipMemsetAsync(ov[g], 0xA5, 16 * nv, cap));
    KV(kvh_meow128_fixed(B.dkf, 16, nf, S1, S2, of[g], 0, cap));
    KV(kvh_meow128_var(B.dkv, B.doffs, nv, S1, S2, ov[g], 0, cap));
    CK(hipStreamEndCapture(cap, &gr));
    CK(hipGraphInstantiate(&ex[g], gr, nullptr, nullptr, 0));
    CK(hipGraphDestroy(gr));
  }
  long bad = 0;
  std::vector<uint64_t> h(2 * (nf > nv ? nf : nv));
  for (int r = 0; r < rounds; r++) {
    CK(hipGraphLaunch(ex[r & 1], sa));
    CK(hipGraphLaunch(ex[(r & 1) ^ 1], sb));
    for (int k = 0; k < 3; k++) {
      CK(hipMemsetAsync(of[2], 0xA5, 16 * nf, cap));
      KV(kvh_meow128_fixed(B.dkf, 16, nf, S1, S2, of[2], 0, cap));
    }
    CK(hipDeviceSynchronize());
    for (int g = 0; g < 3; g++) {
      CK(hipMemcpy(h.data(), of[g], 16 * nf, hipMemcpyDeviceToHost));
      const long b = check(h, B.wf, nf, nf);
      if (b) fprintf(stderr, "round %d fixed output %d: %ld bad words\n", r, g, b);
      bad += b;
    }
    for (int g = 0; g < 2; g++) {
      CK(hipMemcpy(h.data(), ov[g], 16 * nv, hipMemcpyDeviceToHost));
      const long b = check(h, B.wv, nv, nv);
      if (b) fprintf(stderr, "round %d var output %d: %ld bad words\n", r, g, b);
      bad += b;
    }
  }
  for (auto& e : ex) CK(hipGraphExecDestroy(e));
  for (auto& p : of) CK(hipFree(p));
  for (auto& p : ov) CK(hipFree(p));
  KV(kvh_stream_release(cap));
  CK(hipStreamDestroy(cap));
  CK(hipStreamDestroy(sa));
  CK(hipStreamDestroy(sb));
  return bad;
}

// 3. release, destroy, and a new stream (which may get the same handle value)
static long release_cycle(const Batch& B) {
  long bad = 0;
  uint64_t* d = nullptr;
  CK(hipMalloc(&d, 16 * B.nf));
  std::vector<uint64_t> h(2 * B.nf);
  for (int k = 0; k < 6; k++) {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(hipMemsetAsync(d, 0xA5, 16 * B.nf, s));
    KV(kvh_meow128_fixed(B.dkf, 16, B.nf, S1, S2, d, 0, s));
    KV(kvh_stream_release(s));  // synchronises s first
    CK(hipMemcpy(h.data(), d, 16 * B.nf, hipMemcpyDeviceToHost));
    bad += check(h, B.wf, B.nf, B.nf);
    CK(hipStreamDestroy(s));
  }
  KV(kvh_stream_release(nullptr));
  KV(kvh_stream_release((void*)hipStreamPerThread));
  CK(hipFree(d));
  return bad;
}

int main() {
  Batch B;
  make(B, 2000003, 300001);
  long total = 0, b;
  b = per_thread_streams(B, 24);
  printf("hipStreamPerThread x 4 threads: %ld bad words\n", b);
  total += b;
  const int prev = kvh_set_tuning(26, 6);  // ticket fetches of every other ticket delayed (tickets.hpp)
  b = per_thread_streams(B, 8);
  kvh_set_tuning(26, prev);
  printf("hipStreamPerThread x 4 threads, fetch delay: %ld bad words\n", b);
  total += b;
  b = graphs(B, 8);
  printf("graphs replayed on two streams + direct launches on the capture stream: %ld bad words\n", b);
  total += b;
  b = release_cycle(B);
  printf("kvh_stream_release / destroy / new stream: %ld bad words\n", b);
  total += b;
  printf("%s\n", total ? "FAIL" : "OK");
  return total ? 1 : 0;
}
