// kvh.hip -- gfx950 kernels and the C-ABI (include/kvh.h) of the batched
// Meow128 key-hash engine.  See DESIGN.md for the data layout in HBM, the
// kernels' rooflines and the folding argument; meow_dev.hpp for the round.
//
// Kernels
//   k_fixed<L,NT,A16,U>   fixed length L in {8,16,..,64}, one seed, constants
//                         folded into SGPRs (configs C1, C4)
//   k_fixed_lanes         LA lanes per key, one seed each (config C3)
//   k_fixed_ms            one lane per key, `arity` seeds (C3 fallback)
//   k_fixed_rt            any fixed length below one block (runtime L)
//   k_generic<VAR,NT>     any length: fixed stride or u64 offsets
//   k_var9, k_var6        variable length, per-wave length-sorted windows (C2)
//   k_seeded              straight-line restatement, per-key seeds, constant
//                         memory tables (drop-ins, x2/x4/x8 variants)
//   k_stream_*            streaming init/update/final state transitions
//
// libkvh.so holds only kernels some call of include/kvh.h launches.  The
// research kernels that lost their A/B and the ablation builds whose outputs
// are not hashes live in tools/exp/ (`make experiments` -> tools/libkvh_exp.so,
// which links these objects plus tools/exp/*.o; see rt::g_exp).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <atomic>
#include <map>
#include <mutex>
#include <thread>
#include <condition_variable>
#include <deque>
#include <functional>
#include <vector>
#include <algorithm>
#include "meow_dev.hpp"
#include "kvh_internal.hpp"
#include "kvh_var.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

#ifndef KVH_VERSION
#define KVH_VERSION "raikv_amd-kvh 0.1 (gfx950)"
#endif

namespace {

// straight-line restatement, one thread per key, per-key seeds
__global__ void __launch_bounds__(256)
k_seeded(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint64_t n,
         const uint64_t* __restrict__ seeds, uint64_t* __restrict__ out, uint32_t flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ConstTab T;
  const uint64_t o0 = offs[i], o1 = offs[i + 1];
  const Blk h = meow_literal(keys + o0, o1 - o0, seeds[2 * i], seeds[2 * i + 1], T);
  store_h(out, i, h, (flags & KVH_FIXUP) != 0);
}

// Tiny host batches (raikv's 8-key prefetch pipes, ev_net.h:442; a ctest
// batch of a few thousand frags, ctest.c:34): keys, offsets and hashes stay
// in coherent pinned host memory and the kernel reads and writes them
// across PCIe itself -- one launch and one synchronize, no DMA copies, no
// LDS table fill (constant-memory tables, the literal restatement).  Key i
// is keys[offs[i] - offs[0] ..) (variable length) or keys[i * key_len ..).
// Each workgroup first copies its 256 keys' offsets and then their bytes
// into LDS with coalesced 16-byte reads (two PCIe round trips for the whole
// workgroup; one lane per key reading its own pieces across PCIe costs a
// round trip per 16 bytes), then hashes from LDS; a workgroup whose keys
// hold more than kTinyLds bytes reads them from host memory per lane.
constexpr uint32_t kTinyLds = 32768;
__global__ void __launch_bounds__(256)
k_tiny(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint32_t key_len, uint64_t n, uint64_t s1,
       uint64_t s2, uint64_t* __restrict__ out, uint32_t flags) {
  __shared__ uint64_t so[257];
  __shared__ __attribute__((aligned(16))) uint32_t buf[(kTinyLds + 32) / 4];
  const uint32_t tid = threadIdx.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * 256;
  const uint32_t cnt = (uint32_t)(n - i0 < 256 ? n - i0 : 256);
  const uint64_t o0 = offs ? offs[0] : 0;
  for (uint32_t t = tid; t <= cnt; t += 256) so[t] = offs ? offs[i0 + t] - o0 : (i0 + t) * key_len;
  __syncthreads();
  const uint64_t lo = so[0] & ~(uint64_t)15, hi = so[cnt], bytes = hi - lo;
  const ConstTab T;
  const bool fix = (flags & KVH_FIXUP) != 0;
  if (bytes <= kTinyLds) {
    // 16-byte reads of [lo, hi rounded up): inside the caller's batch buffer,
    // which the host side pads to a 16-byte multiple
    for (uint64_t x = tid * 16; x < bytes; x += 256 * 16) {
      const uint4 v = *(const uint4*)(keys + lo + x);
      *(uint4*)((uint8_t*)buf + x) = v;
    }
    __syncthreads();
    if (tid < cnt) {
      const uint64_t a = so[tid] - lo, L = so[tid + 1] - so[tid];
      store_h(out, i0 + tid, meow_literal((const uint8_t*)buf + a, L, s1, s2, T, LdsBytes{}), fix);
    }
  } else if (tid < cnt) {
    store_h(out, i0 + tid, meow_literal(keys + so[tid], so[tid + 1] - so[tid], s1, s2, T), fix);
  }
}

// streaming: state[16 words] in/out; absorb nblk full 64-byte blocks
__global__ void k_stream_absorb(uint32_t* st, const uint8_t* data, uint64_t nblk) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const ConstTab T;
  MeowState s;
  for (int i = 0; i < 4; i++) for (int c = 0; c < 4; c++) s.S[i].w[c] = st[4 * i + c];
  absorb_blocks(s, data, nblk, T);
  for (int i = 0; i < 4; i++) for (int c = 0; c < 4; c++) st[4 * i + c] = s.S[i].w[c];
}

// streaming final: Meow_Loop over the buffered `off` bytes, then finish
// with the Mixer of (k1, k2, total) (key_hash.c:1541-1568)
__global__ void k_stream_final(const uint32_t* st, const uint8_t* block, uint64_t off,
                               uint64_t k1, uint64_t k2, uint64_t total, uint64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const ConstTab T;
  MeowState s;
  for (int i = 0; i < 4; i++) for (int c = 0; c < 4; c++) s.S[i].w[c] = st[4 * i + c];
  if (off > 0) absorb_loop(s, block, off, T);
  const Blk h = finish(s, mixer(k1, k2, total), T);
  out[0] = (uint64_t)h.w[0] | ((uint64_t)h.w[1] << 32);
  out[1] = (uint64_t)h.w[2] | ((uint64_t)h.w[3] << 32);
}

}  // namespace

// ------------------------------------------------------------ host runtime (kvh_internal.hpp)
namespace kvh {
namespace rt {

thread_local int t_last_err = 0;
ExpHooks g_exp{};

struct DevInfo {
  int cus = 0;
};
std::mutex g_mu;
std::vector<DevInfo> g_dev;

int set_err(int e) { t_last_err = e; return e; }
int hip_err(hipError_t e) { return set_err(KVH_EHIP_BASE - (int)e); }

int device_cus(int* cus) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  std::lock_guard<std::mutex> g(g_mu);
  if ((int)g_dev.size() <= dev) g_dev.resize(dev + 1);
  if (g_dev[dev].cus == 0) {
    int c = 0;
    e = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return hip_err(e);
    g_dev[dev].cus = c > 0 ? c : 1;
  }
  *cus = g_dev[dev].cus;
  return 0;
}

// Ticket words for the in-order streaming kernels (tickets.hpp): four u64
// per (device, stream), zero between launches -- the kernel's last
// workgroup puts the counters back to zero as it exits, so no memset precedes
// a launch.  Launches on one stream are serialised, so a stream's words are
// never used by two kernels at once.  Two kinds of handle do not name one
// serialised queue, and are resolved here:
//  - hipStreamPerThread is one handle value for a different stream on every
//    host thread: its words are kept per (calling thread, device) and go back
//    to the pool when the thread exits;
//  - a launch captured into a graph may be replayed on any stream, and
//    several replays may run at once: a captured launch takes the static
//    chunk order (*tk = nullptr; the launchers then run the static form).
// No allocation and no synchronisation on the launch path (VERDICT r5 item 6,
// ADVICE r5): each device's pool of kTkQuads word sets is allocated ONCE, on
// the device's first ticketed call, and zeroed by a hipMemsetAsync on that
// call's stream; an event recorded after it is waited on (hipStreamWaitEvent,
// no host wait) by every stream that takes words before it has completed.  A
// pool that runs dry makes the call take the static chunk order (the same
// hashes); it never grows.  Lookups are one map search under the device's
// own lock.  kvh_stream_release hands a stream's words back (before the stream
// is destroyed).  Word 2 holds the test-only fetch delay of knob 26, written
// asynchronously on the stream that takes the words.
constexpr int kTkDev = 64;
constexpr size_t kTkQuads = 1024;  // word sets per device (32 KiB): streams that can hold words at once
struct Spare {
  unsigned long long* p;
  uint32_t dbg;     // the delay word it holds
  hipEvent_t done;  // a thread's last launch with it (nullptr: released after a synchronize)
};
struct TicketPool {
  std::mutex mu;
  unsigned long long* words = nullptr;  // kTkQuads x 4, allocated on the device's first ticketed call
  hipEvent_t zeroed = nullptr;           // after the pool's memset, until known complete
  std::vector<Spare> spare;              // released (zero counters)
  std::map<std::pair<uintptr_t, uint32_t>, unsigned long long*> by_stream;  // (stream, delay) -> words
  size_t used = 0;
};
TicketPool g_tickets[kTkDev];
std::atomic<int> g_tune_tkdbg{0};  // knob 26: test-only ticket fetch delay (tickets.hpp word 2)
std::atomic<int> g_tune_refwg{0};  // knob 27 (experiments build): earlier many-batch exact-order forms (128, 256)

// words of device P for stream st, word 2 = dbg; caller holds P.mu.  *out = nullptr (0 returned) when the
// pool is dry: the caller's launch takes the static order.
int new_words(TicketPool& P, hipStream_t st, uint32_t dbg, unsigned long long** out) {
  hipError_t e;
  *out = nullptr;
  if (!P.words) {  // once per device, on its first ticketed call
    unsigned long long* w = nullptr;
    if ((e = hipMalloc((void**)&w, kTkQuads * 4 * sizeof(unsigned long long))) != hipSuccess) return hip_err(e);
    if ((e = hipMemsetAsync(w, 0, kTkQuads * 4 * sizeof(unsigned long long), st)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&P.zeroed, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventRecord(P.zeroed, st)) != hipSuccess) {
      (void)hipFree(w);
      P.zeroed = nullptr;
      return hip_err(e);
    }
    P.words = w;
  }
  unsigned long long* p = nullptr;
  uint32_t had = 0;
  if (!P.spare.empty()) {
    const Spare sp = P.spare.back();
    P.spare.pop_back();
    p = sp.p;
    had = sp.dbg;
    if (sp.done) {  // a finished thread's words: its last launch may still run
      e = hipStreamWaitEvent(st, sp.done, 0);
      (void)hipEventDestroy(sp.done);
      if (e != hipSuccess) return hip_err(e);
    }
  } else {
    if (P.used == kTkQuads) return 0;  // dry: the static order for this call
    p = P.words + 4 * P.used++;
    if (P.zeroed) {  // the pool's memset, until it is known to be done
      if (hipEventQuery(P.zeroed) == hipSuccess) {
        (void)hipEventDestroy(P.zeroed);
        P.zeroed = nullptr;
      } else if ((e = hipStreamWaitEvent(st, P.zeroed, 0)) != hipSuccess) {
        return hip_err(e);
      }
    }
  }
  if (had != dbg && (e = hipMemsetD32Async((hipDeviceptr_t)(p + 2), dbg, 1, st)) != hipSuccess)
    return hip_err(e);  // word 2's high half stays 0 (the delay is < 2^32)
  *out = p;
  return 0;
}

// hipStreamPerThread's words of this thread, per device.  When the thread
// exits they go back to the pool behind an event recorded on the thread's
// stream, so the next taker waits for the thread's last launch on the device.
struct PerThreadWords {
  unsigned long long* p[kTkDev] = {};
  uint32_t dbg[kTkDev] = {};
  ~PerThreadWords() {
    for (int d = 0; d < kTkDev; d++) {
      if (!p[d]) continue;
      int cur = 0;
      hipEvent_t ev = nullptr;
      if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(d) != hipSuccess) continue;  // leave them: never reused
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess &&
          hipEventRecord(ev, hipStreamPerThread) == hipSuccess) {
        std::lock_guard<std::mutex> g(g_tickets[d].mu);
        g_tickets[d].spare.push_back({p[d], dbg[d], ev});
      } else if (ev) {
        (void)hipEventDestroy(ev);
      }
      (void)hipSetDevice(cur);
    }
  }
};
thread_local PerThreadWords t_pts;

int stream_tickets(hipStream_t st, unsigned long long** tk) {
  *tk = nullptr;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  if (dev < 0 || dev >= kTkDev) return set_err(KVH_EINVAL);
  if (st != nullptr && st != hipStreamLegacy) {  // the legacy null stream is never captured
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if ((e = hipStreamIsCapturing(st, &cs)) != hipSuccess) return hip_err(e);
    if (cs != hipStreamCaptureStatusNone) return 0;  // captured: the static order
  }
  const uint32_t dbg = (uint32_t)g_tune_tkdbg.load(std::memory_order_relaxed);
  TicketPool& P = g_tickets[dev];
  if (st == hipStreamPerThread) {
    if (t_pts.p[dev] && t_pts.dbg[dev] == dbg) { *tk = t_pts.p[dev]; return 0; }
    std::lock_guard<std::mutex> g(P.mu);
    if (t_pts.p[dev]) {  // another delay (tests only): the old set goes back (this thread's stream is ordered)
      hipEvent_t ev = nullptr;
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hip_err(e);
      if ((e = hipEventRecord(ev, hipStreamPerThread)) != hipSuccess) {
        (void)hipEventDestroy(ev);
        return hip_err(e);
      }
      P.spare.push_back({t_pts.p[dev], t_pts.dbg[dev], ev});
      t_pts.p[dev] = nullptr;
    }
    unsigned long long* p = nullptr;
    if (int rc = new_words(P, st, dbg, &p)) return rc;
    if (p) {
      t_pts.p[dev] = p;
      t_pts.dbg[dev] = dbg;
    }
    *tk = p;
    return 0;
  }
  std::lock_guard<std::mutex> g(P.mu);
  const auto key = std::make_pair((uintptr_t)st, dbg);
  auto it = P.by_stream.find(key);
  if (it != P.by_stream.end()) { *tk = it->second; return 0; }
  unsigned long long* p = nullptr;
  if (int rc = new_words(P, st, dbg, &p)) return rc;
  if (p) P.by_stream.emplace(key, p);
  *tk = p;
  return 0;
}

int stream_release(hipStream_t st) {
  if (st == nullptr || st == hipStreamLegacy || st == hipStreamPerThread) return set_err(0);
  hipError_t e = hipStreamSynchronize(st);  // every launch that holds the words has finished
  if (e != hipSuccess) return hip_err(e);
  for (int d = 0; d < kTkDev; d++) {
    TicketPool& P = g_tickets[d];
    std::lock_guard<std::mutex> g(P.mu);
    for (auto it = P.by_stream.begin(); it != P.by_stream.end();) {
      if (it->first.first == (uintptr_t)st) {
        P.spare.push_back({it->second, it->first.second, nullptr});
        it = P.by_stream.erase(it);
      } else {
        ++it;
      }
    }
  }
  return set_err(0);
}

int launch_done() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(e);
  return set_err(0);
}

}  // namespace rt
}  // namespace kvh

namespace {

// ------------------------------------------------------------ host side
// Tuning knobs (kvh_set_tuning): process-wide, read once per call with
// relaxed atomic loads, so a knob set on one thread never races a launch on
// another (a call in flight keeps the value it read).
}  // namespace

// Tuning knobs (kvh_set_tuning): process-wide, read once per call with
// relaxed atomic loads, so a knob set on one thread never races a launch on
// another (a call in flight keeps the value it read).  The kernel-selection
// knobs are shared with kvh_fixed.hip / kvh_varlen.hip (kvh_internal.hpp).
using Knob = std::atomic<int>;

namespace kvh {
namespace rt {
Knob g_tune_nt{0};        // tables per LDS: 2 or 4 (0 = per-length default)
Knob g_tune_order{0};     // knob 24: fixed-length chunk order: 0 = per-length default; 1 = static per wave (k_fixed); 2 = in address order through wave tickets (k_fixed_qw); 3/4/5 = in address order, one workgroup barrier per ticket of 1/4/16 rounds (k_fixed_q)
Knob g_tune_wgmul{1};     // workgroups per CU multiplier
Knob g_tune_generic{0};   // force the generic kernel
Knob g_tune_kpl{0};       // keys per lane per chunk in k_fixed (0 = per-length default)
Knob g_tune_ms_lanes{1};  // multi-seed: 1 = lanes-per-key kernel, 0 = one lane per key
Knob g_tune_var{46};      // var-length kernel: 46 = k_var9 with windows in address order (wave tickets); 23 = k_var9 static order (16 waves; 24 = 12 waves, 25 = 12 waves + block prefetch); 44 four tables x 16 copies, 45 clamped loads; 13 = k_var6 windows sorted by 16-byte length class; 7 = by exact length; 0 = unsorted k_generic
}  // namespace rt
}  // namespace kvh

namespace {

// Pinned/device staging for the synchronous host drop-ins.
struct Staging {
  std::mutex mu;
  uint8_t* dev = nullptr;
  size_t cap = 0;
  int device = -1;
};
Staging g_stage;

int stage_reserve(size_t bytes) {  // caller holds g_stage.mu
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  if (g_stage.dev && g_stage.device == dev && g_stage.cap >= bytes) return 0;
  if (g_stage.dev) {
    int cur = dev;
    (void)hipSetDevice(g_stage.device);  // best-effort release of the old staging buffer
    (void)hipFree(g_stage.dev);
    (void)hipSetDevice(cur);
    g_stage.dev = nullptr;
  }
  size_t cap = std::max<size_t>(bytes, 1 << 20);
  e = hipMalloc(&g_stage.dev, cap);
  if (e != hipSuccess) { g_stage.dev = nullptr; g_stage.cap = 0; return hip_err(e); }
  g_stage.cap = cap;
  g_stage.device = dev;
  return 0;
}

size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// Hash `n` host keys (pointers + lengths) with per-key seeds on the GPU via
// k_seeded; out gets 2n words.  Synchronous.
int seeded_host(const void* const* ptrs, const size_t* lens, size_t n, const uint64_t* seeds,
                uint64_t* out, uint32_t flags) {
  if (n == 0) return set_err(0);
  size_t kbytes = 0;
  for (size_t i = 0; i < n; i++) {
    if (lens[i] && !ptrs[i]) return set_err(KVH_EINVAL);
    kbytes += lens[i];
  }
  std::vector<uint8_t> host(al16(kbytes) + al16(8 * (n + 1)) + al16(16 * n));
  std::vector<uint64_t> offs(n + 1);
  size_t o = 0;
  for (size_t i = 0; i < n; i++) {
    offs[i] = o;
    if (lens[i]) memcpy(host.data() + o, ptrs[i], lens[i]);
    o += lens[i];
  }
  offs[n] = o;
  const size_t off_offs = al16(kbytes), off_seeds = off_offs + al16(8 * (n + 1)),
               off_out = off_seeds + al16(16 * n);
  memcpy(host.data() + off_offs, offs.data(), 8 * (n + 1));
  memcpy(host.data() + off_seeds, seeds, 16 * n);
  std::lock_guard<std::mutex> g(g_stage.mu);
  int rc = stage_reserve(off_out + 16 * n);
  if (rc) return rc;
  uint8_t* d = g_stage.dev;
  hipError_t e = hipMemcpy(d, host.data(), off_out, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_err(e);
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL(k_seeded, dim3(grid), dim3(256), 0, 0, d, (const uint64_t*)(d + off_offs), (uint64_t)n,
                     (const uint64_t*)(d + off_seeds), (uint64_t*)(d + off_out), flags);
  rc = launch_done();
  if (rc) return rc;
  e = hipMemcpy(out, d + off_out, 16 * n, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_err(e);
  return set_err(0);
}

int same_len_host(const void* const* ptrs, size_t cnt, size_t sz, const uint64_t* seed_pairs,
                  bool per_key_seed, uint64_t* x) {
  std::vector<size_t> lens(cnt, sz);
  std::vector<uint64_t> seeds(2 * cnt);
  for (size_t i = 0; i < cnt; i++) {
    seeds[2 * i] = per_key_seed ? seed_pairs[2 * i] : seed_pairs[0];
    seeds[2 * i + 1] = per_key_seed ? seed_pairs[2 * i + 1] : seed_pairs[1];
  }
  return seeded_host(ptrs, lens.data(), cnt, seeds.data(), x, 0);
}

// Host pipeline state (kvh_meow128_{fixed,var}_host): streams, events and
// buffer slots, grown on demand and kept for the process lifetime.  Each
// device has kPipesPerDev of them, so that several host threads may drive one
// device at once (kvh_*_host_multi with a device listed twice); a call holds
// one pipeline for its duration.
constexpr int kPipeSlots = 16;  // buffer slots allocated; g_tune_pipe_slots of them used
constexpr int kMaxDev = 64;
constexpr int kPipesPerDev = 4;
Knob g_tune_pipe_mib{16};   // key bytes per pipeline chunk, MiB (knob 15)
Knob g_tune_pipe_slots{4};  // chunks in flight (knob 16)
Knob g_tune_tiny{16384};    // host batches of at most this many keys take the zero-copy tiny path (knob 21; 0 = off)
constexpr size_t kTinyBytes = 512 << 10;  // ... and at most this many key bytes
struct HostPipe {
  std::mutex mu;
  hipStream_t s_in = nullptr, s_k = nullptr, s_out = nullptr;
  hipEvent_t ev_in[kPipeSlots] = {}, ev_k[kPipeSlots] = {}, ev_out[kPipeSlots] = {};
  uint8_t* dk[kPipeSlots] = {};      // key bytes (device)
  uint64_t* doff[kPipeSlots] = {};   // key offsets (device, variable length)
  uint64_t* dout[kPipeSlots] = {};   // hashes (device)
  uint8_t* tiny = nullptr;           // coherent pinned keys | offsets | hashes of the tiny path
  size_t tinycap = 0;
  uint8_t* hk[kPipeSlots] = {};      // pinned bounce buffers for pageable callers
  uint64_t* hoff[kPipeSlots] = {};
  uint64_t* ho[kPipeSlots] = {};
  size_t kcap = 0, fcap = 0, ocap = 0, hkcap = 0, hfcap = 0, hocap = 0;
  // slots [0, ns) of buffer array b hold `want` bytes each (grow-only)
  template <class T, class A, class F>
  static hipError_t regrow(T* (&b)[kPipeSlots], size_t& cap, size_t want, int ns, A alloc, F release) {
    if (cap < want) {
      for (int s = 0; s < kPipeSlots; s++) if (b[s]) { (void)release(b[s]); b[s] = nullptr; }
      cap = want;
    }
    for (int s = 0; s < ns; s++) {
      if (b[s]) continue;
      const hipError_t e = alloc((void**)&b[s], cap);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // streams, events and ns slots for chunks of kb key bytes, fb offset bytes
  // (0: fixed length) and ob hash bytes on the current device
  int reserve(int ns, size_t kb, size_t fb, size_t ob, bool need_hk, bool need_hf, bool need_ho) {
    hipError_t e = hipSuccess;
    for (hipStream_t* st : {&s_in, &s_k, &s_out})
      if (e == hipSuccess && !*st) e = hipStreamCreateWithFlags(st, hipStreamNonBlocking);
    for (int s = 0; s < kPipeSlots && e == hipSuccess; s++)
      for (hipEvent_t* ev : {&ev_in[s], &ev_k[s], &ev_out[s]})
        if (e == hipSuccess && !*ev) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    auto dmal = [](void** p, size_t b) { return hipMalloc(p, b); };
    auto dfree = [](void* p) { return hipFree(p); };
    auto hmal = [](void** p, size_t b) { return hipHostMalloc(p, b, 0); };
    auto hfree = [](void* p) { return hipHostFree(p); };
    if (e == hipSuccess) e = regrow(dk, kcap, std::max<size_t>(kb, 16), ns, dmal, dfree);
    if (e == hipSuccess && fb) e = regrow(doff, fcap, fb, ns, dmal, dfree);
    if (e == hipSuccess) e = regrow(dout, ocap, ob, ns, dmal, dfree);
    if (e == hipSuccess && need_hk) e = regrow(hk, hkcap, std::max<size_t>(kb, 16), ns, hmal, hfree);
    if (e == hipSuccess && need_hf) e = regrow(hoff, hfcap, fb, ns, hmal, hfree);
    if (e == hipSuccess && need_ho) e = regrow(ho, hocap, ob, ns, hmal, hfree);
    return e == hipSuccess ? 0 : hip_err(e);
  }
};
HostPipe g_pipe[kMaxDev][kPipesPerDev];

// a free pipeline of the current device (blocks on pipeline 0 when all are busy)
std::unique_lock<std::mutex> pick_pipe(int dev, HostPipe** P) {
  for (int i = 0; i < kPipesPerDev; i++) {
    std::unique_lock<std::mutex> lk(g_pipe[dev][i].mu, std::try_to_lock);
    if (lk.owns_lock()) { *P = &g_pipe[dev][i]; return lk; }
  }
  *P = &g_pipe[dev][0];
  return std::unique_lock<std::mutex>(g_pipe[dev][0].mu);
}

// Page-locked ranges made through this API (kvh_host_alloc,
// kvh_host_register), by base: a batch lying inside ONE of them is DMA'd
// directly.
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pin_ranges;
void pin_track(const void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pin_ranges[(uintptr_t)p] = bytes;
}
void pin_untrack(const void* p) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pin_ranges.erase((uintptr_t)p);
}

bool pinned_byte(const void* p) {
  hipPointerAttribute_t a;
  const bool pin = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  return pin;
}

// [p, p + bytes) may be DMA'd without a bounce copy: it lies inside one range
// registered or allocated through this API, or (page-locked memory from
// elsewhere, e.g. hipHostMalloc) both its ends are page-locked AND the
// runtime's allocation holding p covers the whole range.  Two registrations
// with a pageable gap between them therefore take the bounce buffers, never a
// DMA across the gap; so does a range registered only in part.
bool is_pinned(const void* p, size_t bytes) {
  if (!bytes) return true;
  const uintptr_t a = (uintptr_t)p;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pin_ranges.upper_bound(a);
    if (it != g_pin_ranges.begin()) {
      --it;
      if (a >= it->first && a - it->first <= it->second && bytes <= it->second - (a - it->first)) return true;
    }
  }
  if (!pinned_byte(p) || (bytes > 1 && !pinned_byte((const uint8_t*)p + bytes - 1))) return false;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  const bool ok = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess;
  (void)hipGetLastError();
  const uintptr_t b = (uintptr_t)base;
  return ok && size && a >= b && a - b <= size && bytes <= size - (a - b);
}

// One host batch through H2D -> kernel -> D2H on the current device.
// Chunk c is keys [lo_c, hi_c): fixed length (key_len > 0) in chunks of
// `chunk_keys` keys, variable length (offs != nullptr, n+1 host offsets) in
// chunks of at most `budget` key bytes and `chunk_keys` keys (a longer key
// is a chunk of its own, the buffers grow to hold it).  Three streams (H2D,
// kernel, D2H) linked by per-slot events, `slots` chunks in flight: chunk c
// is copied in on s_in, hashed on s_k once its copy-in event fired, copied
// out on s_out once its kernel event fired; a slot is refilled once its
// previous chunk's copy-out event fired.  One stream per DMA direction lets
// both PCIe directions run at once (full duplex).
int host_pipeline(const uint8_t* keys, uint32_t key_len, const uint64_t* offs, size_t n, uint64_t s1, uint64_t s2,
                  uint64_t* out, uint32_t flags) {
  if (n == 0) return set_err(0);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  if (dev < 0 || dev >= kMaxDev) return set_err(KVH_EINVAL);
  HostPipe* P = nullptr;
  std::unique_lock<std::mutex> lk = pick_pipe(dev, &P);
  const bool var = offs != nullptr;
  if (n <= (size_t)knob(g_tune_tiny) && (var ? offs[n] - offs[0] : (uint64_t)n * key_len) <= kTinyBytes) {
    // tiny batch: copy into the pipeline's coherent pinned buffer, one
    // kernel reading and writing host memory, one synchronize
    const size_t kb = var ? (size_t)(offs[n] - offs[0]) : n * (size_t)key_len;
    const size_t o_off = al16(kb), o_out = o_off + al16(var ? 8 * (n + 1) : 0), need = o_out + 16 * n;
    if (P->tinycap < need) {
      if (P->tiny) (void)hipHostFree(P->tiny);
      P->tiny = nullptr;
      P->tinycap = 0;
      const size_t cap = std::max<size_t>(need, (1 << 20) + 64);
      if ((e = hipHostMalloc((void**)&P->tiny, cap, hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess)
        return hip_err(e);
      P->tinycap = cap;
    }
    if (!P->s_k && (e = hipStreamCreateWithFlags(&P->s_k, hipStreamNonBlocking)) != hipSuccess) return hip_err(e);
    if (kb) memcpy(P->tiny, keys + (var ? offs[0] : 0), kb);
    memset(P->tiny + kb, 0, al16(kb) - kb);  // k_tiny reads whole 16-byte groups
    if (var) memcpy(P->tiny + o_off, offs, 8 * (n + 1));
    hipLaunchKernelGGL(k_tiny, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, P->s_k, (const uint8_t*)P->tiny,
                       var ? (const uint64_t*)(P->tiny + o_off) : (const uint64_t*)nullptr, key_len, (uint64_t)n, s1,
                       s2, (uint64_t*)(P->tiny + o_out), flags);
    int rc = launch_done();
    if ((e = hipStreamSynchronize(P->s_k)) != hipSuccess && !rc) rc = hip_err(e);
    if (rc) return rc;
    memcpy(out, P->tiny + o_out, 16 * n);
    return set_err(0);
  }
  const size_t budget = (size_t)knob(g_tune_pipe_mib) << 20;
  const size_t chunk_keys = var ? std::max<size_t>(1, budget / 8) : std::max<size_t>(1, budget / key_len);
  // chunk boundaries; the largest chunk sizes the buffers
  std::vector<size_t> bounds{0};
  size_t max_bytes = 0, max_keys = 0;
  while (bounds.back() < n) {
    const size_t lo = bounds.back();
    size_t hi = std::min(n, lo + chunk_keys);
    if (var) {  // at most `budget` key bytes, at least one key
      const uint64_t lim = offs[lo] + budget;
      hi = std::max(lo + 1, (size_t)(std::upper_bound(offs + lo, offs + hi + 1, lim) - offs) - 1);
      max_bytes = std::max<size_t>(max_bytes, offs[hi] - offs[lo]);
    } else {
      max_bytes = std::max<size_t>(max_bytes, (hi - lo) * key_len);
    }
    max_keys = std::max(max_keys, hi - lo);
    bounds.push_back(hi);
  }
  const uint64_t kb0 = var ? offs[0] : 0, kb1 = var ? offs[n] : (uint64_t)n * key_len;
  const bool pin_k = is_pinned(keys + kb0, kb1 - kb0), pin_o = is_pinned(out, 16 * n),
             pin_f = var && is_pinned(offs, 8 * (n + 1));
  const int slots = std::min(std::max(knob(g_tune_pipe_slots), 2), kPipeSlots);
  int rc = P->reserve(slots, max_bytes, var ? 8 * (max_keys + 1) : 0, 16 * max_keys, !pin_k, var && !pin_f, !pin_o);
  if (rc) return rc;
  if (bounds.size() == 2) {
    // one chunk (raikv's batches: 8 keys per prefetch pipe, ev_net.h:442; up
    // to 16K frags per ctest batch, ctest.c:34): H2D, kernel and D2H in order
    // on one stream and one synchronize, no cross-stream events
    const uint8_t* src = keys + kb0;
    const size_t nbytes = (size_t)(kb1 - kb0);
    if (!pin_k && nbytes) { memcpy(P->hk[0], src, nbytes); src = P->hk[0]; }
    const uint64_t* fsrc = offs;
    if (var && !pin_f) { memcpy(P->hoff[0], offs, 8 * (n + 1)); fsrc = P->hoff[0]; }
    uint64_t* dst = pin_o ? out : P->ho[0];
    if ((nbytes && (e = hipMemcpyAsync(P->dk[0], src, nbytes, hipMemcpyHostToDevice, P->s_k)) != hipSuccess) ||
        (var && (e = hipMemcpyAsync(P->doff[0], fsrc, 8 * (n + 1), hipMemcpyHostToDevice, P->s_k)) != hipSuccess)) {
      rc = hip_err(e);
      (void)hipStreamSynchronize(P->s_k);  // a copy already queued may still read hk[0]
      return rc;
    }
    rc = var ? kvh_meow128_var((const uint8_t*)((uintptr_t)P->dk[0] - (uintptr_t)kb0), P->doff[0], n, s1, s2,
                               P->dout[0], flags, P->s_k)
             : kvh_meow128_fixed(P->dk[0], key_len, n, s1, s2, P->dout[0], flags, P->s_k);
    if (!rc && (e = hipMemcpyAsync(dst, P->dout[0], 16 * n, hipMemcpyDeviceToHost, P->s_k)) != hipSuccess)
      rc = hip_err(e);
    if ((e = hipStreamSynchronize(P->s_k)) != hipSuccess && !rc) rc = hip_err(e);
    if (rc) return rc;
    if (!pin_o) memcpy(out, P->ho[0], 16 * n);
    return set_err(0);
  }
  size_t pend_lo[kPipeSlots] = {}, pend_cnt[kPipeSlots] = {};
  auto drain = [&](int s) -> int {  // the slot's previous chunk has left the device
    if (!pend_cnt[s]) return 0;
    hipError_t x = hipEventSynchronize(P->ev_out[s]);
    if (x != hipSuccess) return hip_err(x);
    if (!pin_o) memcpy(out + 2 * pend_lo[s], P->ho[s], pend_cnt[s] * 16);
    pend_cnt[s] = 0;
    return 0;
  };
  for (size_t c = 0; !rc && c + 1 < bounds.size(); c++) {
    const int s = (int)(c % slots);
    if ((rc = drain(s))) break;
    const size_t lo = bounds[c], cnt = bounds[c + 1] - lo;
    const uint64_t base = var ? offs[lo] : (uint64_t)lo * key_len;
    const size_t nbytes = var ? (size_t)(offs[lo + cnt] - base) : cnt * key_len;
    const uint8_t* src = keys + base;
    if (!pin_k && nbytes) { memcpy(P->hk[s], src, nbytes); src = P->hk[s]; }
    const uint64_t* fsrc = var ? offs + lo : nullptr;
    if (var && !pin_f) { memcpy(P->hoff[s], fsrc, 8 * (cnt + 1)); fsrc = P->hoff[s]; }
    uint64_t* dst = pin_o ? out + 2 * lo : P->ho[s];
    if ((nbytes && (e = hipMemcpyAsync(P->dk[s], src, nbytes, hipMemcpyHostToDevice, P->s_in)) != hipSuccess) ||
        (var && (e = hipMemcpyAsync(P->doff[s], fsrc, 8 * (cnt + 1), hipMemcpyHostToDevice, P->s_in)) != hipSuccess) ||
        (e = hipEventRecord(P->ev_in[s], P->s_in)) != hipSuccess ||
        (e = hipStreamWaitEvent(P->s_k, P->ev_in[s], 0)) != hipSuccess) {
      rc = hip_err(e); break;
    }
    // variable length: the chunk's offsets stay absolute (offs[lo] .. offs[hi]);
    // the key pointer handed to the kernel is biased by -offs[lo], so every
    // address it forms, keys + offs[i], lies inside this chunk's buffer
    rc = var ? kvh_meow128_var((const uint8_t*)((uintptr_t)P->dk[s] - (uintptr_t)base), P->doff[s], cnt, s1, s2,
                               P->dout[s], flags, P->s_k)
             : kvh_meow128_fixed(P->dk[s], key_len, cnt, s1, s2, P->dout[s], flags, P->s_k);
    if (rc) break;
    if ((e = hipEventRecord(P->ev_k[s], P->s_k)) != hipSuccess ||
        (e = hipStreamWaitEvent(P->s_out, P->ev_k[s], 0)) != hipSuccess ||
        (e = hipMemcpyAsync(dst, P->dout[s], cnt * 16, hipMemcpyDeviceToHost, P->s_out)) != hipSuccess ||
        (e = hipEventRecord(P->ev_out[s], P->s_out)) != hipSuccess) {
      rc = hip_err(e); break;
    }
    pend_lo[s] = lo; pend_cnt[s] = cnt;
  }
  for (int s = 0; s < slots; s++) {
    const int r2 = drain(s);
    if (!rc) rc = r2;
  }
  if (rc) {  // leave the pipeline idle for the next call
    (void)hipStreamSynchronize(P->s_in); (void)hipStreamSynchronize(P->s_k); (void)hipStreamSynchronize(P->s_out);
  }
  return rc ? rc : set_err(0);
}

// Shard d of n keys is [b[d], b[d+1]): equal index ranges (offs == nullptr)
// or, for variable length, ranges holding equal key bytes: b[d] = the first
// key whose start offset is >= offs[0] + total * d / ns (workload.py:
// shard_var).  b[0] = 0, b[ns] = n, non-decreasing.
void shard_bounds(const uint64_t* offs, size_t n, int ns, size_t* b) {
  for (int d = 0; d <= ns; d++) {
    if (!offs || n == 0) {
      b[d] = (size_t)((unsigned __int128)n * d / ns);
    } else {
      const uint64_t tot = offs[n] - offs[0];
      const uint64_t tgt = offs[0] + (uint64_t)((unsigned __int128)tot * d / ns);
      b[d] = d == 0 ? 0 : d == ns ? n : (size_t)(std::lower_bound(offs, offs + n + 1, tgt) - offs);
      if (b[d] > n) b[d] = n;
    }
  }
}

// Shards [lo_d, hi_d) of one host batch over ndev devices, one host thread
// each (SURVEY.md §8 e: independent keys, no collective; each device writes
// its disjoint slice of the caller's output, the same global layout as a
// one-device call).  Fixed length: equal index ranges; variable length:
// ranges of equal key BYTES (raikv_amd/workload.py: shard_var).
// Persistent host workers for the _multi entries: a job queue served by
// threads created on first use and kept for the process lifetime (grown to
// the largest device list seen), instead of one new std::thread per device
// per call.  Jobs are independent (a job never waits for another), so a
// pool smaller than the jobs in flight only serialises them.
struct WorkPool {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  int threads = 0;
  void run(std::vector<std::function<void()>>& jobs) {
    std::mutex dmu;
    std::condition_variable dcv;
    size_t left = jobs.size();
    {
      std::lock_guard<std::mutex> g(mu);
      while (threads < (int)jobs.size()) {
        std::thread([this]() { worker(); }).detach();
        threads++;
      }
      for (auto& j : jobs)
        q.push_back([&dmu, &dcv, &left, &j]() {
          j();
          std::lock_guard<std::mutex> g2(dmu);
          if (--left == 0) dcv.notify_all();
        });
    }
    cv.notify_all();
    std::unique_lock<std::mutex> lk(dmu);
    dcv.wait(lk, [&]() { return left == 0; });
  }
  void worker() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [this]() { return !q.empty(); });
        job = std::move(q.front());
        q.pop_front();
      }
      job();
    }
  }
};
WorkPool* g_pool = new WorkPool;  // never destroyed: its detached workers outlive static destructors

int host_multi(const uint8_t* keys, uint32_t key_len, const uint64_t* offs, size_t n, uint64_t s1, uint64_t s2,
               uint64_t* out, uint32_t flags, const int* devices, int ndev) {
  if (ndev < 1 || ndev > kMaxDev || !devices) return set_err(KVH_EINVAL);
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess) return hip_err(e);
  for (int d = 0; d < ndev; d++)
    if (devices[d] < 0 || devices[d] >= count || devices[d] >= kMaxDev) return set_err(KVH_EINVAL);
  std::vector<size_t> lo(ndev + 1);
  shard_bounds(offs, n, ndev, lo.data());
  std::vector<int> rcs(ndev, 0);
  std::vector<std::function<void()>> jobs;
  for (int d = 0; d < ndev; d++) {
    const size_t a = lo[d], b = std::max(lo[d], lo[d + 1]);
    if (b == a) continue;
    jobs.emplace_back([&, d, a, b]() {
      const hipError_t se = hipSetDevice(devices[d]);
      if (se != hipSuccess) { rcs[d] = hip_err(se); return; }
      // variable length: shard offsets stay absolute into `keys`;
      // fixed length: the shard's keys start at a * key_len
      rcs[d] = offs ? host_pipeline(keys, 0, offs + a, b - a, s1, s2, out + 2 * a, flags)
                    : host_pipeline(keys + (uint64_t)a * key_len, key_len, nullptr, b - a, s1, s2, out + 2 * a, flags);
    });
  }
  if (jobs.size() == 1) {  // one shard: on the calling thread, whose current device is restored
    int cur = 0;
    if ((e = hipGetDevice(&cur)) != hipSuccess) return hip_err(e);
    jobs[0]();
    (void)hipSetDevice(cur);
  } else if (!jobs.empty()) {
    g_pool->run(jobs);
  }
  for (int d = 0; d < ndev; d++)
    if (rcs[d]) return set_err(rcs[d]);
  return set_err(0);
}

}  // namespace

// =============================================================== C-ABI
extern "C" {

int kvh_meow128_fixed(const void* keys, uint32_t key_len, size_t n, uint64_t seed1, uint64_t seed2,
                      uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!keys || !out) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  return fixed_dispatch((const uint8_t*)keys, key_len, n, seed1, seed2, out, flags, (hipStream_t)stream, cus);
}

int kvh_meow128_var(const void* keys, const uint64_t* offsets, size_t n, uint64_t seed1, uint64_t seed2,
                    uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!keys || !offsets || !out) return set_err(KVH_EINVAL);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  return var_dispatch((const uint8_t*)keys, offsets, n, seed1, seed2, out, flags, (hipStream_t)stream, cus);
}

int kvh_meow128_multiseed(const void* keys, uint32_t key_len, size_t n, const uint64_t* seeds,
                          uint32_t arity, uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!keys || !out || !seeds || arity < 1 || arity > KVH_MAX_ARITY) return set_err(KVH_EINVAL);
  if (arity == 1) return kvh_meow128_fixed(keys, key_len, n, seeds[0], seeds[1], out, flags, stream);
  int cus = 0, rc = device_cus(&cus);
  if (rc) return rc;
  uint64_t s[16] = {0};
  for (uint32_t a = 0; a < arity; a++) { s[2 * a] = seeds[2 * a]; s[2 * a + 1] = seeds[2 * a + 1]; }
  return multiseed_dispatch((const uint8_t*)keys, key_len, n, s, arity, out, flags, (hipStream_t)stream, cus);
}

int kvh_meow128_batch(const void* keys, const uint64_t* offsets, uint32_t fixed_len, size_t n,
                      const uint64_t* seeds, uint32_t arity, uint64_t* out, uint32_t flags, void* stream) {
  if (!seeds) return set_err(KVH_EINVAL);
  if (offsets) {
    if (arity != 1) return set_err(KVH_EINVAL);
    return kvh_meow128_var(keys, offsets, n, seeds[0], seeds[1], out, flags, stream);
  }
  return kvh_meow128_multiseed(keys, fixed_len, n, seeds, arity, out, flags, stream);
}

int kvh_meow128_var_seeded(const void* keys, const uint64_t* offsets, size_t n, const uint64_t* seeds,
                           uint64_t* out, uint32_t flags, void* stream) {
  if (n == 0) return set_err(0);
  if (!keys || !offsets || !seeds || !out) return set_err(KVH_EINVAL);
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL(k_seeded, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)keys, offsets,
                     (uint64_t)n, seeds, out, flags);
  return launch_done();
}

int kvh_meow128_fixed_host(const void* keys, uint32_t key_len, size_t n, uint64_t seed1, uint64_t seed2,
                           uint64_t* out, uint32_t flags) {
  if (n == 0) return set_err(0);
  if (!keys || !out || key_len == 0) return set_err(KVH_EINVAL);
  return host_pipeline((const uint8_t*)keys, key_len, nullptr, n, seed1, seed2, out, flags);
}

int kvh_meow128_var_host(const void* keys, const uint64_t* offsets, size_t n, uint64_t seed1, uint64_t seed2,
                         uint64_t* out, uint32_t flags) {
  if (n == 0) return set_err(0);
  if (!keys || !offsets || !out) return set_err(KVH_EINVAL);
  return host_pipeline((const uint8_t*)keys, 0, offsets, n, seed1, seed2, out, flags);
}

int kvh_meow128_fixed_host_multi(const void* keys, uint32_t key_len, size_t n, uint64_t seed1, uint64_t seed2,
                                 uint64_t* out, uint32_t flags, const int* devices, int ndev) {
  if (n == 0) return set_err(0);
  if (!keys || !out || key_len == 0) return set_err(KVH_EINVAL);
  return host_multi((const uint8_t*)keys, key_len, nullptr, n, seed1, seed2, out, flags, devices, ndev);
}

int kvh_meow128_var_host_multi(const void* keys, const uint64_t* offsets, size_t n, uint64_t seed1, uint64_t seed2,
                               uint64_t* out, uint32_t flags, const int* devices, int ndev) {
  if (n == 0) return set_err(0);
  if (!keys || !offsets || !out) return set_err(KVH_EINVAL);
  return host_multi((const uint8_t*)keys, 0, offsets, n, seed1, seed2, out, flags, devices, ndev);
}

int kvh_shard_bounds(const uint64_t* offsets, size_t n, int nshards, size_t* bounds) {
  if (nshards < 1 || !bounds) return set_err(KVH_EINVAL);
  shard_bounds(offsets, n, nshards, bounds);
  return set_err(0);
}

int kvh_host_register(void* p, size_t bytes) {
  if (!p || !bytes) return set_err(KVH_EINVAL);
  const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterDefault);
  if (e == hipSuccess) pin_track(p, bytes);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_host_unregister(void* p) {
  if (!p) return set_err(KVH_EINVAL);
  pin_untrack(p);
  const hipError_t e = hipHostUnregister(p);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_host_alloc(void** p, size_t bytes) {
  if (!p) return set_err(KVH_EINVAL);
  *p = nullptr;
  const hipError_t e = hipHostMalloc(p, bytes ? bytes : 1, 0);
  if (e == hipSuccess) pin_track(*p, bytes ? bytes : 1);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_host_free(void* p) {
  if (!p) return set_err(0);
  pin_untrack(p);
  const hipError_t e = hipHostFree(p);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_device_alloc(void** p, size_t bytes) {
  if (!p) return set_err(KVH_EINVAL);
  *p = nullptr;
  const hipError_t e = hipMalloc(p, bytes ? bytes : 1);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_device_free(void* p) {
  if (!p) return set_err(0);
  const hipError_t e = hipFree(p);
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_hash_meow128(const void* p, size_t sz, uint64_t* h1, uint64_t* h2) {
  if (!h1 || !h2) return set_err(KVH_EINVAL);
  uint64_t s[2] = {*h1, *h2}, o[2];
  int rc = seeded_host(&p, &sz, 1, s, o, 0);
  if (rc) return rc;
  *h1 = o[0]; *h2 = o[1];
  return 0;
}

uint64_t kvh_hash_meow64(const void* p, size_t sz, uint64_t seed) {
  uint64_t h1 = seed, h2 = seed;
  kvh_hash_meow128(p, sz, &h1, &h2);
  return h1;
}

int kvh_hash_meow128_2_same_length(const void* p, const void* p2, size_t sz, uint64_t* x) {
  const void* ps[2] = {p, p2};
  return same_len_host(ps, 2, sz, x, false, x);
}
int kvh_hash_meow128_4_same_length(const void* p, const void* p2, const void* p3, const void* p4, size_t sz,
                                   uint64_t* x) {
  const void* ps[4] = {p, p2, p3, p4};
  return same_len_host(ps, 4, sz, x, false, x);
}
int kvh_hash_meow128_4_same_length_a(const void** p, size_t sz, uint64_t* x) {
  return same_len_host(p, 4, sz, x, false, x);
}
int kvh_hash_meow128_4_same_length_4_seed(const void* p, const void* p2, const void* p3, const void* p4,
                                          size_t sz, uint64_t* x) {
  const void* ps[4] = {p, p2, p3, p4};
  return same_len_host(ps, 4, sz, x, true, x);
}
int kvh_hash_meow128_8_same_length(const void* p, const void* p2, const void* p3, const void* p4,
                                   const void* p5, const void* p6, const void* p7, const void* p8, size_t sz,
                                   uint64_t* x) {
  const void* ps[8] = {p, p2, p3, p4, p5, p6, p7, p8};
  return same_len_host(ps, 8, sz, x, false, x);
}
int kvh_hash_meow128_8_same_length_a(const void** p, size_t sz, uint64_t* x) {
  return same_len_host(p, 8, sz, x, false, x);
}
int kvh_hash_meow128_2_diff_length(const void* p, size_t sz, const void* p2, size_t sz2, uint64_t* x) {
  const void* ps[2] = {p, p2};
  size_t ls[2] = {sz, sz2};
  uint64_t seeds[4] = {x[0], x[1], x[0], x[1]};
  return seeded_host(ps, ls, 2, seeds, x, 0);
}
int kvh_hash_meow128_4_diff_length(const void* p, size_t sz, const void* p2, size_t sz2, const void* p3,
                                   size_t sz3, const void* p4, size_t sz4, uint64_t* x) {
  const void* ps[4] = {p, p2, p3, p4};
  size_t ls[4] = {sz, sz2, sz3, sz4};
  uint64_t seeds[8] = {x[0], x[1], x[0], x[1], x[0], x[1], x[0], x[1]};
  return seeded_host(ps, ls, 4, seeds, x, 0);
}

int kvh_hash_meow128_vec(const kvh_meow_vec_t* vec, size_t vec_sz, uint64_t* h1, uint64_t* h2) {
  if (!h1 || !h2 || (vec_sz && !vec)) return set_err(KVH_EINVAL);
  size_t total = 0;
  for (size_t i = 0; i < vec_sz; i++) total += vec[i].sz;
  std::vector<uint8_t> cat(total ? total : 1);
  size_t o = 0;
  for (size_t i = 0; i < vec_sz; i++) {
    if (vec[i].sz) memcpy(cat.data() + o, vec[i].p, vec[i].sz);
    o += vec[i].sz;
  }
  return kvh_hash_meow128(cat.data(), total, h1, h2);
}

// Streaming: the 16-word Meow state lives in m->ctx (layout S0..S3 as
// little-endian 128-bit lanes, same as the reference's Meow_Save_Ctx).
static int stream_absorb_dev(kvh_meow_ctx_t* m, const uint8_t* data, size_t nblk) {
  std::lock_guard<std::mutex> g(g_stage.mu);
  int rc = stage_reserve(64 + nblk * 64);
  if (rc) return rc;
  uint8_t* d = g_stage.dev;
  hipError_t e = hipMemcpy(d, m->ctx, 64, hipMemcpyHostToDevice);
  if (e == hipSuccess && nblk) e = hipMemcpy(d + 64, data, nblk * 64, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_err(e);
  hipLaunchKernelGGL(k_stream_absorb, dim3(1), dim3(64), 0, 0, (uint32_t*)d, (const uint8_t*)(d + 64),
                     (uint64_t)nblk);
  if ((rc = launch_done())) return rc;
  e = hipMemcpy(m->ctx, d, 64, hipMemcpyDeviceToHost);
  return e == hipSuccess ? 0 : hip_err(e);
}

int kvh_meow128_init(kvh_meow_ctx_t* m, kvh_meow_block_t* b, uint64_t k1, uint64_t k2, size_t total) {
  if (!m || !b) return set_err(KVH_EINVAL);
  // Declare_Meow + Xor_Meow (key_hash.c:1509-1521): byte ramps ^ Mixer
  const uint64_t lo = k1 - total, hi = k2 + total + 1;
  for (int i = 0; i < 4; i++) {
    uint8_t r[16];
    for (int j = 0; j < 16; j++) r[j] = (uint8_t)(16 * i + j);
    uint64_t w0, w1;
    memcpy(&w0, r, 8); memcpy(&w1, r + 8, 8);
    m->ctx[2 * i] = w0 ^ lo;
    m->ctx[2 * i + 1] = w1 ^ hi;
  }
  b->off = 0;
  b->total_update_sz = total;
  return set_err(0);
}

int kvh_meow128_update(kvh_meow_ctx_t* m, kvh_meow_block_t* b, const void* p, size_t sz) {
  if (!m || !b || (sz && !p)) return set_err(KVH_EINVAL);
  const uint8_t* src = (const uint8_t*)p;
  size_t len = sz;
  int rc = 0;
  if (b->off > 0) {
    size_t fill = 64 - b->off;
    if (fill > len) fill = len;
    memcpy(&b->block[b->off], src, fill);
    b->off += fill; len -= fill; src += fill;
    if (b->off == 64) {
      if ((rc = stream_absorb_dev(m, b->block, 1))) return rc;
      b->off = 0;
    }
  }
  if (len > 0) {
    b->off = len & 63;
    if (len > b->off && (rc = stream_absorb_dev(m, src, (len - b->off) / 64))) return rc;
    memcpy(b->block, &src[len - b->off], b->off);
  }
  return set_err(0);
}

int kvh_meow128_final(kvh_meow_ctx_t* m, kvh_meow_block_t* b, uint64_t* k1, uint64_t* k2) {
  if (!m || !b || !k1 || !k2) return set_err(KVH_EINVAL);
  std::lock_guard<std::mutex> g(g_stage.mu);
  int rc = stage_reserve(64 + 64 + 16);
  if (rc) return rc;
  uint8_t* d = g_stage.dev;
  hipError_t e = hipMemcpy(d, m->ctx, 64, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d + 64, b->block, 64, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_err(e);
  hipLaunchKernelGGL(k_stream_final, dim3(1), dim3(64), 0, 0, (const uint32_t*)d, (const uint8_t*)(d + 64),
                     (uint64_t)b->off, *k1, *k2, (uint64_t)b->total_update_sz, (uint64_t*)(d + 128));
  if ((rc = launch_done())) return rc;
  uint64_t o[2];
  e = hipMemcpy(o, d + 128, 16, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_err(e);
  *k1 = o[0]; *k2 = o[1];
  return set_err(0);
}

int kvh_meow_test(const void* p, size_t sz, uint64_t* k1, uint64_t* k2) {
  kvh_meow_ctx_t m;
  kvh_meow_block_t b;
  int rc = kvh_meow128_init(&m, &b, *k1, *k2, sz);
  if (!rc) rc = kvh_meow128_update(&m, &b, p, sz);
  if (!rc) rc = kvh_meow128_final(&m, &b, k1, k2);
  return rc;
}

int kvh_hash_key_frag(const uint64_t seed[2], const kvh_key_frag_t* frag, uint64_t* k, uint64_t* k2) {
  if (!seed || !frag || !k || !k2) return set_err(KVH_EINVAL);
  const void* p = frag->buf;
  size_t len = frag->keylen;
  uint64_t o[2];
  int rc = seeded_host(&p, &len, 1, seed, o, KVH_FIXUP);
  if (rc) return rc;
  *k = o[0]; *k2 = o[1];
  return 0;
}

int kvh_hash_key_frags(const uint64_t seed[2], const kvh_key_frag_t* const* frags, size_t n, uint64_t* out) {
  if (!seed || (n && (!frags || !out))) return set_err(KVH_EINVAL);
  std::vector<const void*> ps(n);
  std::vector<size_t> ls(n);
  std::vector<uint64_t> seeds(2 * n);
  for (size_t i = 0; i < n; i++) {
    ps[i] = frags[i]->buf; ls[i] = frags[i]->keylen;
    seeds[2 * i] = seed[0]; seeds[2 * i + 1] = seed[1];
  }
  return seeded_host(ps.data(), ls.data(), n, seeds.data(), out, KVH_FIXUP);
}


int kvh_last_error(void) { return t_last_err; }

const char* kvh_strerror(int err) {
  if (err == 0) return "ok";
  if (err == KVH_EINVAL) return "invalid argument";
  if (err == KVH_ENOMEM) return "out of memory";
  if (err == KVH_ENODEV) return "no device";
  if (err <= KVH_EHIP_BASE) return hipGetErrorString((hipError_t)(KVH_EHIP_BASE - err));
  return "unknown error";
}

const char* kvh_version(void) { return KVH_VERSION; }

int kvh_stream_release(void* stream) { return stream_release((hipStream_t)stream); }

int kvh_device_synchronize(void) {
  hipError_t e = hipDeviceSynchronize();
  return e == hipSuccess ? set_err(0) : hip_err(e);
}

int kvh_debug_checks(uint64_t out[4]) {
  if (!out) return set_err(KVH_EINVAL);
  unsigned long long a[4], b[4];
  if (int rc = chk_take_refsort(a)) return rc;
  if (int rc = chk_take_ingest(b)) return rc;
  const unsigned long long* f = a[0] ? a : b;  // the sort's first failure, else the ingest's
  out[0] = a[0] + b[0];
  for (int i = 1; i < 4; i++) out[i] = f[i];
  set_err(0);
  return KVH_CHECKED_ON;
}

// Every knob selects among kernels whose outputs are the same hashes (or
// sizes the host pipeline); the ablation and research knobs exist only in
// the experiments build.  Atomic exchange: safe against concurrent calls.
#ifdef KVH_EXPERIMENTS
constexpr bool kExperiments = true;   // tools/libkvh_exp.so: the product sources with the losing variants
#else
constexpr bool kExperiments = false;
#endif
int kvh_set_tuning(int k, int value) {
  auto set = [](Knob& g, int v) { return g.exchange(v, std::memory_order_relaxed); };
  switch (k) {
    case 0: if (value != 0 && !(kExperiments && (value == 2 || value == 4))) return KVH_EINVAL; return set(g_tune_nt, value);
    case 1: if (value < 1 || value > 8) return KVH_EINVAL; return set(g_tune_wgmul, value);
    case 2: return set(g_tune_generic, value ? 1 : 0);
    case 3: if (value != 0 && !(kExperiments && value > 0 && value <= 8 && value != 5 && value != 6 && value != 7))
              return KVH_EINVAL;
            return set(g_tune_kpl, value);
    case 7: if (value != 0 && value != 23 && value != 46 && !(g_exp.var_knob && g_exp.var_knob(value)))
              return KVH_EINVAL;
            return set(g_tune_var, value);
    case 8: return set(g_tune_ms_lanes, value ? 1 : 0);
    case 14: if (value != 0 && value != 6 && !(kExperiments && value > 0 && value <= 7)) return KVH_EINVAL;
             return set(g_tune_crc_var, value);
    case 15: if (value < 1 || value > 1024) return KVH_EINVAL; return set(g_tune_pipe_mib, value);
    case 16: if (value < 2 || value > 16) return KVH_EINVAL; return set(g_tune_pipe_slots, value);
    case 17: if (value < 0 || value > 64) return KVH_EINVAL; return set(g_tune_sort_bits, value);
    case 18: if (value < 0 || value > (kExperiments ? 6 : 2)) return KVH_EINVAL; return set(g_tune_spans, value);
    case 19: if (value < 0 || value > 1) return KVH_EINVAL; return set(g_tune_tok, value);
    case 20: if (value < 0 || value > 2) return KVH_EINVAL; return set(g_tune_sort_engine, value);
    case 21: if (value < 0 || value > (1 << 20)) return KVH_EINVAL; return set(g_tune_tiny, value);
    case 22: if (value < 0 || value > 1) return KVH_EINVAL; return set(g_tune_sort_cap, value);
    case 23: if (value != 0 && value != 3 && !(kExperiments && (value == 1 || value == 2 || (value >= 5 && value <= 15) || value == 17))) return KVH_EINVAL;
             return set(g_tune_sort_b3, value);
    case 24: if (value < 0 || value > (kExperiments ? 5 : 2)) return KVH_EINVAL; return set(g_tune_order, value);
    case 25: if (value != 0 && value != 10 && value != 11 && value != 12) return KVH_EINVAL; return set(g_tune_sort_hd, value);
    case 26: if (value < 0 || value > 0xffff) return KVH_EINVAL; return g_tune_tkdbg.exchange(value);
    case 27: if (!kExperiments || (value != 0 && value != 128 && value != 256)) return KVH_EINVAL; return set(g_tune_refwg, value);
    default: return g_exp.set_tuning ? g_exp.set_tuning(k, value) : KVH_EINVAL;
  }
}

}  // extern "C"
