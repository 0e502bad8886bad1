// streams_gpu.cpp -- TEST: the ticket state of the in-order streaming kernels
// for every kind of stream a caller can pass,
// over every entry point whose kernel takes its chunks through wave tickets:
// fixed length (k_fixed_qw), runtime length (k_fixed_rt), variable length
// (k_var9), multi-seed (k_fixed_lanes), fused hash + positions (k_fixed_pos),
// CRC32C fixed / variable (k_crc_fixed_ct, k_crc_var_sorted) and spans
// (k_spans):
//   1. four host threads calling at once on hipStreamPerThread (one handle
//      value, four different streams), ragged sizes, into outputs poisoned
//      with 0xA5 bytes: every launch equals the oracle and leaves the bytes
//      past its n untouched; then again with the knob-26 fetch delay;
//   2. launches captured into graphs on one stream (whose ticket words
//      already exist) and replayed on two other streams at once while direct
//      launches run on the capture stream;
//   3. kvh_stream_release before a stream is destroyed, and a new stream after;
//   4. more new streams than the word pool holds, during another thread's
//      global-mode graph capture (which must stay valid).
// The oracle (oracle/liboracle.so, test infrastructure) is the checker.
// Runs under pytest -m gpu (tests/test_gpu_parity.py::test_streams_program).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <functional>
#include <string>
#include <thread>
#include <vector>
#include "kvh.h"

extern "C" {
void orc_batch_fixed(const uint8_t* keys, size_t len, size_t n, uint64_t s1, uint64_t s2, uint64_t* out, int fixup);
void orc_batch_var(const uint8_t* keys, const uint64_t* offs, size_t n, uint64_t s1, uint64_t s2, uint64_t* out,
                   int fixup);
void orc_batch_multiseed(const uint8_t* keys, size_t len, size_t n, const uint64_t* seeds, size_t arity,
                         uint64_t* out, int fixup);
void orc_crc_batch_fixed(const uint8_t* keys, size_t len, size_t n, const uint32_t* seeds, uint32_t seed,
                         uint32_t* out);
void orc_crc_batch_var(const uint8_t* keys, const uint64_t* offs, size_t n, const uint32_t* seeds, uint32_t seed,
                       uint32_t* out);
typedef struct {
  uint64_t ht_size, ht_mod_mask, ht_mod_fraction;
  uint32_t ht_mod_shift;
  uint16_t cuckoo_buckets;
  uint8_t cuckoo_arity, pad;
} orc_geom_t;
int orc_ht_geom(uint64_t map_size, uint32_t entry_size, float ratio, uint16_t buckets, uint8_t arity, orc_geom_t* g);
uint32_t orc_positions_per_key(const orc_geom_t* g);
void orc_cuckoo_positions(const orc_geom_t* g, const uint64_t* hashes, size_t n, uint64_t* pos);
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
static const uint64_t MS[8] = {1, 2, 3, 4, 0x1234, 0x5678, 0x9abcdef0ull, 0x0fedcba9ull};

static uint64_t rnd(uint64_t& s) {
  s ^= s << 13; s ^= s >> 7; s ^= s << 17;
  return s;
}

// one ticketed entry point: launch(n, out, stream) writes `per` bytes per
// key into out; want holds the oracle's bytes for all `cap` keys
struct Job {
  std::string name;
  size_t cap, per;
  std::vector<uint8_t> want;
  std::function<void(size_t, void*, hipStream_t)> launch;
};

struct Data {
  size_t nf = 2000003, nv = 300001;
  std::vector<uint8_t> kf, kv;
  std::vector<uint64_t> offs;
  std::vector<uint32_t> lens;
  uint8_t *dkf = nullptr, *dkv = nullptr;
  uint64_t* doffs = nullptr;
  uint32_t* dlens = nullptr;
  kvh_ht_geom_t geom;
  std::vector<Job> jobs;
};

template <class T>
static std::vector<uint8_t> bytes_of(const std::vector<T>& v) {
  std::vector<uint8_t> b(v.size() * sizeof(T));
  memcpy(b.data(), v.data(), b.size());
  return b;
}

static void make(Data& D) {
  uint64_t r = 88172645463325252ull;
  D.kf.resize(D.nf * 16);
  for (auto& b : D.kf) b = (uint8_t)rnd(r);
  D.offs.resize(D.nv + 1);
  D.lens.resize(D.nv);
  D.offs[0] = 0;
  for (size_t i = 0; i < D.nv; i++) {
    D.lens[i] = (uint32_t)(rnd(r) % 121);  // 0..120-byte keys
    D.offs[i + 1] = D.offs[i] + D.lens[i];
  }
  D.kv.resize(D.offs[D.nv] + 1);
  for (auto& b : D.kv) b = (uint8_t)rnd(r);
  CK(hipMalloc(&D.dkf, D.kf.size()));
  CK(hipMalloc(&D.dkv, D.kv.size()));
  CK(hipMalloc(&D.doffs, 8 * D.offs.size()));
  CK(hipMalloc(&D.dlens, 4 * D.lens.size()));
  CK(hipMemcpy(D.dkf, D.kf.data(), D.kf.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(D.dkv, D.kv.data(), D.kv.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(D.doffs, D.offs.data(), 8 * D.offs.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(D.dlens, D.lens.data(), 4 * D.lens.size(), hipMemcpyHostToDevice));
  const uint8_t* kf = D.dkf;
  const uint8_t* kv = D.dkv;
  const uint64_t* of = D.doffs;
  const uint32_t* ln = D.dlens;
  {  // fixed 16 B (k_fixed_qw)
    std::vector<uint64_t> w(2 * D.nf);
    orc_batch_fixed(D.kf.data(), 16, D.nf, S1, S2, w.data(), 0);
    D.jobs.push_back({"fixed16", D.nf, 16, bytes_of(w), [kf](size_t n, void* o, hipStream_t s) {
                        KV(kvh_meow128_fixed(kf, 16, n, S1, S2, (uint64_t*)o, 0, s));
                      }});
  }
  {  // runtime length 20 B (k_fixed_rt)
    const size_t n20 = D.nf * 16 / 20;
    std::vector<uint64_t> w(2 * n20);
    orc_batch_fixed(D.kf.data(), 20, n20, S1, S2, w.data(), 0);
    D.jobs.push_back({"fixed20", n20, 16, bytes_of(w), [kf](size_t n, void* o, hipStream_t s) {
                        KV(kvh_meow128_fixed(kf, 20, n, S1, S2, (uint64_t*)o, 0, s));
                      }});
  }
  {  // variable length (k_var9)
    std::vector<uint64_t> w(2 * D.nv);
    orc_batch_var(D.kv.data(), D.offs.data(), D.nv, S1, S2, w.data(), 0);
    D.jobs.push_back({"var", D.nv, 16, bytes_of(w), [kv, of](size_t n, void* o, hipStream_t s) {
                        KV(kvh_meow128_var(kv, of, n, S1, S2, (uint64_t*)o, 0, s));
                      }});
    // the same keys as (offset, length) spans (k_spans): the same hashes
    D.jobs.push_back({"spans", D.nv, 16, bytes_of(w), [kv, of, ln](size_t n, void* o, hipStream_t s) {
                        KV(kvh_meow128_spans(kv, of, ln, n, S1, S2, (uint64_t*)o, 0, s));
                      }});
  }
  {  // multi-seed, 32 B x 4 seeds (k_fixed_lanes)
    const size_t n32 = D.nf / 2;
    std::vector<uint64_t> w(8 * n32);
    orc_batch_multiseed(D.kf.data(), 32, n32, MS, 4, w.data(), 0);
    D.jobs.push_back({"multiseed", n32, 64, bytes_of(w), [kf](size_t n, void* o, hipStream_t s) {
                        KV(kvh_meow128_multiseed(kf, 32, n, MS, 4, (uint64_t*)o, 0, s));
                      }});
  }
  {  // CRC32C fixed 16 B and variable length (k_crc_fixed_ct, k_crc_var_sorted)
    std::vector<uint32_t> w(D.nf), wv(D.nv);
    orc_crc_batch_fixed(D.kf.data(), 16, D.nf, nullptr, 7, w.data());
    orc_crc_batch_var(D.kv.data(), D.offs.data(), D.nv, nullptr, 7, wv.data());
    D.jobs.push_back({"crc16", D.nf, 4, bytes_of(w), [kf](size_t n, void* o, hipStream_t s) {
                        KV(kvh_crc_c_fixed(kf, 16, n, nullptr, 7, (uint32_t*)o, s));
                      }});
    D.jobs.push_back({"crc_var", D.nv, 4, bytes_of(wv), [kv, of](size_t n, void* o, hipStream_t s) {
                        KV(kvh_crc_c_var(kv, of, n, nullptr, 7, (uint32_t*)o, s));
                      }});
  }
  {  // fused hash + cuckoo positions (k_fixed_pos): hashes (fixed up) then positions, one buffer
    KV(kvh_ht_geom_init(1ull << 30, 64, 1.0f, 4, 4, &D.geom));
    orc_geom_t og;
    if (orc_ht_geom(1ull << 30, 64, 1.0f, 4, 4, &og) != 0) { fprintf(stderr, "orc_ht_geom\n"); exit(2); }
    const uint32_t pk = orc_positions_per_key(&og);
    const size_t n = D.nf / 2;
    std::vector<uint64_t> h(2 * n), p((size_t)pk * n);
    orc_batch_fixed(D.kf.data(), 16, n, S1, S2, h.data(), 1);
    orc_cuckoo_positions(&og, h.data(), n, p.data());
    // per key: 16 hash bytes, then 8 * pk position bytes (the job's buffer is
    // split in two regions by the launcher; the check interleaves nothing)
    std::vector<uint8_t> w(n * (16 + 8 * (size_t)pk));
    for (size_t i = 0; i < n; i++) {
      memcpy(&w[i * 16], &h[2 * i], 16);
      memcpy(&w[n * 16 + i * 8 * pk], &p[(size_t)pk * i], 8 * pk);
    }
    const kvh_ht_geom_t* g = &D.geom;
    // this job's output regions depend on cap, not on the ragged n: launch
    // writes hashes at [0, 16 n) and positions at [16 cap, ...)
    D.jobs.push_back({"fused_pos", n, 16 + 8 * (size_t)pk, w, [kf, g, n](size_t m, void* o, hipStream_t s) {
                        KV(kvh_meow128_fixed_positions(kf, 16, m, S1, S2, g, (uint64_t*)o,
                                                       (uint8_t*)o + 16 * n, 0, s));
                      }});
  }
}

// bytes of `job` for keys [0, n) equal the oracle; every other byte of the
// poisoned buffer still 0xA5; returns the bad byte count (memcmp first: the
// buffers are tens of MB)
static long range_bad(const uint8_t* got, const uint8_t* want, size_t len) {
  if (memcmp(got, want, len) == 0) return 0;
  long bad = 0;
  for (size_t i = 0; i < len; i++) bad += got[i] != want[i];
  return bad;
}
static long poison_bad(const uint8_t* got, size_t len) {
  static std::vector<uint8_t> p(1 << 20, 0xA5);
  long bad = 0;
  for (size_t o = 0; o < len; o += p.size()) {
    const size_t m = std::min(p.size(), len - o);
    if (memcmp(got + o, p.data(), m) != 0)
      for (size_t i = 0; i < m; i++) bad += got[o + i] != 0xA5;
  }
  return bad;
}
static long check(const Job& J, const std::vector<uint8_t>& got, size_t n) {
  if (J.name == "fused_pos") {  // two regions (hashes, positions), each a prefix of its cap-sized area
    const size_t ph = J.per - 16, hb = 16 * J.cap;
    return range_bad(got.data(), J.want.data(), 16 * n) + poison_bad(got.data() + 16 * n, 16 * (J.cap - n)) +
           range_bad(got.data() + hb, J.want.data() + hb, ph * n) +
           poison_bad(got.data() + hb + ph * n, ph * (J.cap - n));
  }
  return range_bad(got.data(), J.want.data(), J.per * n) + poison_bad(got.data() + J.per * n, J.per * (J.cap - n));
}

// 1. hipStreamPerThread from four threads at once, every job in turn
static long per_thread_streams(const Data& D, int iters) {
  std::atomic<long> bad{0};
  std::atomic<int> ready{0};
  size_t maxb = 0;
  for (const Job& J : D.jobs) maxb = std::max(maxb, J.per * J.cap);
  std::vector<std::thread> th;
  for (int t = 0; t < 4; t++) {
    th.emplace_back([&, t] {
      uint8_t* d = nullptr;
      CK(hipMalloc(&d, maxb));
      std::vector<uint8_t> h(maxb);
      ready++;
      while (ready.load() < 4) std::this_thread::yield();  // start together
      for (int it = 0; it < iters; it++) {
        const Job& J = D.jobs[(it + 3 * t) % D.jobs.size()];
        const size_t n = J.cap - ((size_t)t * 7919 + (size_t)it * 104729) % (J.cap / 3);  // ragged, per thread
        const size_t nb = J.per * J.cap;
        CK(hipMemsetAsync(d, 0xA5, nb, hipStreamPerThread));
        J.launch(n, d, hipStreamPerThread);
        CK(hipMemcpyAsync(h.data(), d, nb, hipMemcpyDeviceToHost, hipStreamPerThread));
        CK(hipStreamSynchronize(hipStreamPerThread));
        const long b = check(J, h, n);
        if (b) fprintf(stderr, "thread %d iter %d (%s n=%zu): %ld bad bytes\n", t, it, J.name.c_str(), n, b);
        bad += b;
      }
      CK(hipFree(d));
    });
  }
  for (auto& x : th) x.join();
  return bad.load();
}

// 2. graphs captured on one stream (every job, whole batches), replayed on
// two others at once while the capture stream runs direct launches
static long graphs(const Data& D, int rounds) {
  hipStream_t cap, sa, sb;
  CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  const size_t nj = D.jobs.size();
  std::vector<uint8_t*> g0(nj), g1(nj), dir(nj);
  for (size_t j = 0; j < nj; j++) {
    const size_t nb = D.jobs[j].per * D.jobs[j].cap;
    CK(hipMalloc(&g0[j], nb));
    CK(hipMalloc(&g1[j], nb));
    CK(hipMalloc(&dir[j], nb));
    D.jobs[j].launch(D.jobs[j].cap, dir[j], cap);  // the capture stream's ticket words exist before capture
  }
  CK(hipStreamSynchronize(cap));
  hipGraphExec_t ex[2];
  for (int g = 0; g < 2; g++) {
    hipGraph_t gr;
    CK(hipStreamBeginCapture(cap, hipStreamCaptureModeGlobal));
    for (size_t j = 0; j < nj; j++) {
      uint8_t* o = g ? g1[j] : g0[j];
      CK(hipMemsetAsync(o, 0xA5, D.jobs[j].per * D.jobs[j].cap, cap));
      D.jobs[j].launch(D.jobs[j].cap, o, cap);  // no call is refused during a capture
    }
    CK(hipStreamEndCapture(cap, &gr));
    CK(hipGraphInstantiate(&ex[g], gr, nullptr, nullptr, 0));
    CK(hipGraphDestroy(gr));
  }
  long bad = 0;
  std::vector<uint8_t> h;
  for (int r = 0; r < rounds; r++) {
    CK(hipGraphLaunch(ex[r & 1], sa));
    CK(hipGraphLaunch(ex[(r & 1) ^ 1], sb));
    for (size_t j = 0; j < nj; j++) {
      CK(hipMemsetAsync(dir[j], 0xA5, D.jobs[j].per * D.jobs[j].cap, cap));
      D.jobs[j].launch(D.jobs[j].cap, dir[j], cap);
    }
    CK(hipDeviceSynchronize());
    for (size_t j = 0; j < nj; j++) {
      const Job& J = D.jobs[j];
      h.resize(J.per * J.cap);
      for (uint8_t* o : {g0[j], g1[j], dir[j]}) {
        CK(hipMemcpy(h.data(), o, h.size(), hipMemcpyDeviceToHost));
        const long b = check(J, h, J.cap);
        if (b) fprintf(stderr, "round %d %s: %ld bad bytes\n", r, J.name.c_str(), b);
        bad += b;
      }
    }
  }
  for (auto& e : ex) CK(hipGraphExecDestroy(e));
  for (size_t j = 0; j < nj; j++) {
    CK(hipFree(g0[j]));
    CK(hipFree(g1[j]));
    CK(hipFree(dir[j]));
  }
  KV(kvh_stream_release(cap));
  CK(hipStreamDestroy(cap));
  CK(hipStreamDestroy(sa));
  CK(hipStreamDestroy(sb));
  return bad;
}

// 3. release, destroy, and a new stream (which may get the same handle value)
static long release_cycle(const Data& D) {
  long bad = 0;
  const Job& J = D.jobs[0];
  uint8_t* d = nullptr;
  CK(hipMalloc(&d, J.per * J.cap));
  std::vector<uint8_t> h(J.per * J.cap);
  for (int k = 0; k < 6; k++) {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(hipMemsetAsync(d, 0xA5, h.size(), s));
    J.launch(J.cap, d, s);
    KV(kvh_stream_release(s));  // synchronises s first
    CK(hipMemcpy(h.data(), d, h.size(), hipMemcpyDeviceToHost));
    bad += check(J, h, J.cap);
    CK(hipStreamDestroy(s));
  }
  KV(kvh_stream_release(nullptr));
  KV(kvh_stream_release((void*)hipStreamPerThread));
  CK(hipFree(d));
  return bad;
}

// 4. more streams than a device's ticket-word pool holds (1024 sets), each
// taking words on its first call, while another thread holds a
// hipStreamCaptureModeGlobal capture open.  No library
// call may allocate or synchronise then (either would invalidate that
// capture); the streams past the pool take the static chunk order.  Buffers
// and streams are made before the capture and every result is read after it.
static long pool_dry_under_capture(const Data& D) {
  const Job& J = D.jobs[0];  // fixed 16-byte keys
  const size_t n = 20011, ns = 1100, per = J.per * n;
  std::vector<hipStream_t> ss(ns);
  for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipStream_t cs;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  uint8_t *d = nullptr, *gout = nullptr;
  CK(hipMalloc(&d, per * ns));
  CK(hipMalloc(&gout, per));
  CK(hipMemset(d, 0xA5, per * ns));
  CK(hipMemset(gout, 0xA5, per));
  CK(hipDeviceSynchronize());
  std::atomic<int> phase{0};
  hipError_t end_err = hipSuccess;
  hipGraph_t graph = nullptr;
  std::thread capt([&] {
    CK(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
    J.launch(n, gout, cs);  // captured: the static order, no words
    phase = 1;
    while (phase.load() < 2) std::this_thread::yield();
    end_err = hipStreamEndCapture(cs, &graph);
  });
  while (phase.load() < 1) std::this_thread::yield();
  for (size_t i = 0; i < ns; i++) J.launch(n, d + per * i, ss[i]);  // first call on each stream
  phase = 2;
  capt.join();
  long bad = 0;
  if (end_err != hipSuccess || !graph) {
    fprintf(stderr, "capture invalidated: %s\n", hipGetErrorString(end_err));
    bad++;
  } else {
    hipGraphExec_t ex;
    CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ex, cs));
    CK(hipStreamSynchronize(cs));
    CK(hipGraphExecDestroy(ex));
    CK(hipGraphDestroy(graph));
  }
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> h(per);
  for (size_t i = 0; i <= ns; i++) {
    CK(hipMemcpy(h.data(), i < ns ? d + per * i : gout, per, hipMemcpyDeviceToHost));
    const long b = range_bad(h.data(), J.want.data(), per);
    if (b) fprintf(stderr, "%s %zu: %ld bad bytes\n", i < ns ? "stream" : "graph", i, b);
    bad += b;
  }
  for (auto& s : ss) {
    KV(kvh_stream_release(s));
    CK(hipStreamDestroy(s));
  }
  CK(hipStreamDestroy(cs));
  CK(hipFree(d));
  CK(hipFree(gout));
  return bad;
}

int main() {
  Data D;
  make(D);
  long total = 0, b;
  b = per_thread_streams(D, 32);
  printf("hipStreamPerThread x 4 threads, %zu entry points: %ld bad bytes\n", D.jobs.size(), b);
  total += b;
  const int prev = kvh_set_tuning(26, 6);  // ticket fetches of every other ticket delayed (tickets.hpp)
  b = per_thread_streams(D, 16);
  kvh_set_tuning(26, prev);
  printf("hipStreamPerThread x 4 threads, fetch delay: %ld bad bytes\n", b);
  total += b;
  b = graphs(D, 4);
  printf("graphs replayed on two streams + direct launches on the capture stream: %ld bad bytes\n", b);
  total += b;
  b = release_cycle(D);
  printf("kvh_stream_release / destroy / new stream: %ld bad bytes\n", b);
  total += b;
  b = pool_dry_under_capture(D);
  printf("1100 new streams (past the 1024-set pool) during another thread's global-mode capture: %ld bad\n", b);
  total += b;
  printf("%s\n", total ? "FAIL" : "OK");
  return total ? 1 : 0;
}
