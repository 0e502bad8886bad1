// kvh_internal.hpp -- shared by the translation units of libkvh.so
// (kvh.hip: hash kernels + C-ABI; ht_pos.hip: table positions, SURVEY.md
// §8 f1): the fixed-length key loaders/stores and the host runtime helpers
// (error state, device properties).  Not installed, not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include "meow_dev.hpp"
#include "../../include/kvh.h"

namespace kvh {

constexpr int kBlock = 1024;  // threads per workgroup of the streaming kernels (16 waves)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));


// Key i of a fixed-length batch as NC 16-byte chunks (zero padded past L).
// NTM: non-temporal (streamed-once) loads.
template <int L, bool A16, bool NTM = false>
__device__ __forceinline__ void load_fixed(const uint8_t* __restrict__ p, Blk* D) {
  constexpr int NC = Plan<L>::NC;
  if constexpr (A16 && (L % 16) == 0) {
#pragma unroll
    for (int j = 0; j < NC; j++) {
      const v4u* q = (const v4u*)(p + 16 * j);
      const v4u v = NTM ? __builtin_nontemporal_load(q) : *q;
      D[j].w[0] = v.x; D[j].w[1] = v.y; D[j].w[2] = v.z; D[j].w[3] = v.w;
    }
  } else {
    // L % 8 == 0 and 8-byte aligned rows
#pragma unroll
    for (int j = 0; j < L / 8; j++) {
      const v2u* q = (const v2u*)(p + 8 * j);
      const v2u v = NTM ? __builtin_nontemporal_load(q) : *q;
      D[j / 2].w[(j & 1) * 2 + 0] = v.x;
      D[j / 2].w[(j & 1) * 2 + 1] = v.y;
    }
    if constexpr ((L % 16) == 8) { D[NC - 1].w[2] = 0; D[NC - 1].w[3] = 0; }
  }
}

// 64-byte keys at 16-byte aligned bases, by lane pairs:
// in a group of 64 keys, lanes 2i and 2i+1 own keys i and 32+i.  Loading
// key k in lane k reads a 16-byte piece of each of 64 keys per instruction,
// 64 B apart: 32 cache lines a quarter used each, and the kernel ran 15 %
// slower than with the pair form (tools/load_ab.py).  Here each instruction
// reads 32 contiguous bytes of each of 32 keys (16 lines, half each): the
// even lane loads pieces 0, 2 of key i and 1, 3 of key 32+i, the odd lane
// pieces 1, 3 of key i and 0, 2 of key 32+i, and each lane passes the two it
// loaded for its partner across the pair with one DPP move per dword.
// `last` clamps past-the-end keys to key n-1 (a benign duplicate, as in
// load_fixed's callers).
__device__ __forceinline__ uint32_t pair64_key(uint32_t lane) { return (lane & 1) ? 32 + (lane >> 1) : lane >> 1; }
__device__ __forceinline__ void load_pair64(const uint8_t* __restrict__ keys, uint64_t g, uint64_t last,
                                            uint32_t lane, Blk* D) {
  const uint64_t i = lane >> 1;
  const bool odd = (lane & 1) != 0;
  const uint64_t klo = g + i < last ? g + i : last, khi = g + 32 + i < last ? g + 32 + i : last;
  const uint32_t o = odd ? 16u : 0u, e = 16u - o;
  const uint8_t* src[4] = {keys + klo * 64 + o, keys + klo * 64 + 32 + o, keys + khi * 64 + e,
                           keys + khi * 64 + 32 + e};
  Blk R[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const v4u v = __builtin_nontemporal_load((const v4u*)src[c]);
    R[c].w[0] = v.x; R[c].w[1] = v.y; R[c].w[2] = v.z; R[c].w[3] = v.w;
  }
#pragma unroll
  for (int w = 0; w < 4; w++) {
    // sent: the even lane's R2/R3 (key 32+i), the odd lane's R0/R1 (key i);
    // quad_perm [1,0,3,2] swaps the lanes of each pair
    const uint32_t X = odd ? R[0].w[w] : R[2].w[w], Y = odd ? R[1].w[w] : R[3].w[w];
    D[0].w[w] = odd ? R[2].w[w] : R[0].w[w];
    D[1].w[w] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)X, 0xB1, 0xF, 0xF, false);
    D[2].w[w] = odd ? R[3].w[w] : R[1].w[w];
    D[3].w[w] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)Y, 0xB1, 0xF, 0xF, false);
  }
}

// 56-byte keys (8-byte aligned) by the same lane pairs: pieces 0-2 are 16
// bytes, piece 3 the last 8.  The even lane loads A.p0 and the odd lane A.p1
// in one instruction (32 contiguous bytes of key A = i), then B.p1 / B.p0
// (key B = 32+i), then each its own key's p2 (16 B) and p3 (8 B); the one
// piece each lane lacks (A.p1 on the even lane, B.p1 on the odd one) crosses
// the pair by DPP.  Per-key loads would read 8 bytes of each of 64 keys per
// instruction, 56 B apart: 28 lines for 512 bytes.
__device__ __forceinline__ void load_pair56(const uint8_t* __restrict__ keys, uint64_t g, uint64_t last,
                                            uint32_t lane, Blk* D) {
  const uint64_t i = lane >> 1;
  const bool odd = (lane & 1) != 0;
  const uint64_t ka = g + i < last ? g + i : last, kb = g + 32 + i < last ? g + 32 + i : last;
  const uint8_t* pa = keys + ka * 56;
  const uint8_t* pb = keys + kb * 56;
  const uint8_t* own = odd ? pb : pa;
  const v4u r0 = __builtin_nontemporal_load((const v4u*)(pa + (odd ? 16 : 0)));
  const v4u r1 = __builtin_nontemporal_load((const v4u*)(pb + (odd ? 0 : 16)));
  const v4u r2 = __builtin_nontemporal_load((const v4u*)(own + 32));
  const v2u r3 = __builtin_nontemporal_load((const v2u*)(own + 48));
  const uint32_t R0[4] = {r0.x, r0.y, r0.z, r0.w}, R1[4] = {r1.x, r1.y, r1.z, r1.w};
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const uint32_t X = odd ? R0[w] : R1[w];  // sent: the partner's p1
    D[0].w[w] = odd ? R1[w] : R0[w];
    D[1].w[w] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)X, 0xB1, 0xF, 0xF, false);
  }
  D[2].w[0] = r2.x; D[2].w[1] = r2.y; D[2].w[2] = r2.z; D[2].w[3] = r2.w;
  D[3].w[0] = r3.x; D[3].w[1] = r3.y; D[3].w[2] = 0; D[3].w[3] = 0;
}

template <bool NTM = false>
__device__ __forceinline__ void store_h(uint64_t* __restrict__ out, uint64_t idx, Blk h, bool fix) {
  if (fix) h = fixup(h);
  v4u v;
  v.x = h.w[0]; v.y = h.w[1]; v.z = h.w[2]; v.w = h.w[3];
  v4u* q = (v4u*)(out + 2 * idx);
  if constexpr (NTM) __builtin_nontemporal_store(v, q); else *q = v;
}

constexpr int kLT = 64;   // full per-length constant records (L < 64)
constexpr int kNF = 256;  // F-only records for 64 <= L < 64 + kNF

// MeowConst padded to 13 blocks, for LDS arrays read at a per-lane length: a
// 52-dword stride puts one field of 16 consecutive lengths on 16 distinct
// 16-byte bank slots (MeowConst's own 48-dword stride repeats every 4
// lengths: 4-way conflicts on every ds_read_b128 of a chunk of short spans).
struct MeowConstL : MeowConst {
  Blk pad;
};

// Per-length folding constants of a variable-length batch from LDS tables
// (k_generic, k_keysrc): full records for L < kLT, first-absorb folds for
// kLT <= L < kLT + kNF, in-lane folds beyond.  LenT = uint64_t for keys of
// 4 GiB and more (the Mixer takes the full length, key_hash.c:1418).
template <class Tab, class LenT = uint32_t, class KRec = MeowConst>
struct LdsK {
  const KRec* full;        // [kLT]
  const Blk* ftab;         // [kNF][4], or null: folds in-lane
  LenT L;
  Blk m;
  const Tab& T;
  __device__ __forceinline__ LdsK(const KRec* f, const Blk* ft, LenT len, uint64_t s1,
                                  uint64_t s2, const Tab& t)
      : full(f), ftab(ft), L(len), m(mixer(s1, s2, len)), T(t) {}
  __device__ __forceinline__ uint32_t li() const { return L < (LenT)kLT ? (uint32_t)L : (uint32_t)kLT - 1; }
  __device__ __forceinline__ Blk M() const { return m; }
  __device__ __forceinline__ Blk F(int i) const {
    if (L < (LenT)kLT) return full[L].F[i];
    if (ftab && L < (LenT)(kLT + kNF)) return ftab[(L - kLT) * 4 + i];
    return aesT(bxor(ramp(i), m), T);
  }
  __device__ __forceinline__ Blk G(int i) const { return full[li()].G[i]; }
  __device__ __forceinline__ Blk TG2() const { return full[li()].TG2; }
  __device__ __forceinline__ Blk CS2b() const { return full[li()].CS2b; }
  __device__ __forceinline__ Blk TCS0a() const { return full[li()].TCS0a; }
};

// Cross-lane LDS ordering inside one wave (its lanes' LDS writes visible to
// its later LDS reads), without a workgroup barrier.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave counting-sorts a window of k <= WIN consecutive keys (u64 offsets
// offs[i0 .. i0+k]) by length bucket min(len, 255), stably by index: LDS
// atomics rank each key inside its bucket, one wave-wide scan of the 256
// counts (hist[256], the wave's own) gives the bucket starts.  Writes the
// records in length order: r_off (u32 offset from the window's first byte),
// r_len (u16, 65535 = "re-read the offsets"), r_idx (u16 index in window).
// Returns the window's first byte offset.  Used by the length-sorted
// variable-length kernels (k_crc_var_sorted; k_var6 inlines the same steps).
// The offsets of a window (raw, as loaded), so that a kernel can load the
// next window's while it hashes the current one.
template <int WIN>
struct WinOffs {
  uint64_t ws, a[WIN / 64], e[WIN / 64];
};

template <int WIN>
__device__ __forceinline__ WinOffs<WIN> win_load(const uint64_t* __restrict__ offs, uint64_t i0, uint32_t k) {
  WinOffs<WIN> w;
  const uint32_t lane = threadIdx.x & 63;
  w.ws = offs[i0];
#pragma unroll
  for (int m = 0; m < WIN / 64; m++) {
    const uint32_t j = lane + 64 * m;
    const uint32_t jj = j < k ? j : k - 1;
    w.a[m] = offs[i0 + jj];
    w.e[m] = offs[i0 + jj + 1];
  }
  return w;
}

// SH: bucket = min(len >> SH, 255).  SH = 0 sorts by exact length; SH = 4 by
// 16-byte class (same full-block count, so the same trip counts), which keeps
// a class in address order (the counting sort is stable) and so coalesces
// the chunk's key gathers.  SUB sub-counters per bucket (by lane % SUB; hist
// holds 256 * SUB words) divide the same-address LDS atomics of one
// instruction -- a bucket's keys in one instruction serialise -- by SUB.
template <int WIN, int SH = 0, int SUB = 1>
__device__ __forceinline__ uint64_t wave_sort_from(const WinOffs<WIN>& W, uint32_t k, uint32_t* hist,
                                                   uint32_t* r_off, uint16_t* r_len, uint16_t* r_idx) {
  constexpr int M = WIN / 64, HQ = 4 * SUB;  // hist words per lane
  static_assert(SUB == 1 || SUB == 2 || SUB == 4, "sub-counters");
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t ws = W.ws;
  uint32_t o[M], L[M], r[M];
#pragma unroll
  for (int m = 0; m < M; m++) {
    o[m] = (uint32_t)(W.a[m] - ws);
    L[m] = W.e[m] - W.a[m] < 65535 ? (uint32_t)(W.e[m] - W.a[m]) : 65535u;
  }
  uint32_t bk[M];
#pragma unroll
  for (int m = 0; m < M; m++) bk[m] = ((L[m] >> SH) < 255u ? (L[m] >> SH) : 255u) * SUB + (lane % SUB);
#pragma unroll
  for (int q = 0; q < HQ; q++) hist[lane * HQ + q] = 0;
  wave_lds_sync();
#pragma unroll
  for (int m = 0; m < M; m++) {
    const uint32_t j = lane + 64 * m;
    r[m] = j < k ? atomicAdd(&hist[bk[m]], 1u) : 0u;
  }
  wave_lds_sync();
  {
    uint32_t v[HQ], sum = 0;
#pragma unroll
    for (int q = 0; q < HQ; q++) { v[q] = hist[lane * HQ + q]; sum += v[q]; }
    uint32_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (lane >= (uint32_t)d) inc += y;
    }
    uint32_t run = inc - sum;
#pragma unroll
    for (int q = 0; q < HQ; q++) { hist[lane * HQ + q] = run; run += v[q]; }
  }
  wave_lds_sync();
#pragma unroll
  for (int m = 0; m < M; m++) {
    const uint32_t j = lane + 64 * m;
    if (j < k) {
      const uint32_t pos = hist[bk[m]] + r[m];
      r_off[pos] = o[m];
      r_len[pos] = (uint16_t)L[m];
      r_idx[pos] = (uint16_t)j;
    }
  }
  wave_lds_sync();
  return ws;
}

template <int WIN, int SH = 0>
__device__ __forceinline__ uint64_t wave_sort_window(const uint64_t* __restrict__ offs, uint64_t i0, uint32_t k,
                                                     uint32_t* hist, uint32_t* r_off, uint16_t* r_len,
                                                     uint16_t* r_idx) {
  return wave_sort_from<WIN, SH>(win_load<WIN>(offs, i0, k), k, hist, r_off, r_len, r_idx);
}

// Bounds-checked build (`make checked` -> tools/libkvh_checked.so, compiled
// with -DKVH_CHECKED).  KVH_CHK(cond, site, value, limit)
// records the first failed check of its translation unit -- (count, site,
// value, limit) in that unit's device words g_chk[4], read back by
// kvh_debug_checks -- and never faults; the caller clamps the access it
// guards.  The product build compiles every check away.  A unit that checks
// puts KVH_CHK_DECL at namespace scope once.
#ifdef KVH_CHECKED
#define KVH_CHK_DECL static __device__ unsigned long long g_chk[4];
__device__ __forceinline__ void kvh_chk_fail(unsigned long long* g, unsigned long long site, unsigned long long v,
                                             unsigned long long l) {
  if (atomicAdd(&g[0], 1ull) == 0) { g[1] = site; g[2] = v; g[3] = l; }
}
#define KVH_CHK(cond, site, val, lim)                                                                       \
  do {                                                                                                      \
    if (!(cond)) kvh_chk_fail(g_chk, (site), (unsigned long long)(val), (unsigned long long)(lim));         \
  } while (0)
#define KVH_CHECKED_ON 1
#else
#define KVH_CHK_DECL
#define KVH_CHK(cond, site, val, lim) \
  do {                                \
  } while (0)
#define KVH_CHECKED_ON 0
#endif

namespace rt {
// checked build: the unit's (count, site, value, limit) words, then cleared (zeros in the product build)
int chk_take_refsort(unsigned long long out[4]);
int chk_take_ingest(unsigned long long out[4]);
// thread-local last error (kvh_last_error); returns e
int set_err(int e);
// HIP error -> KVH_EHIP_BASE - e, recorded
int hip_err(hipError_t e);
// compute units of the current device (cached)
int device_cus(int* cus);
// hipGetLastError after a launch -> 0 or the recorded error
int launch_done();
// the (device, stream)'s ticket words for the in-order streaming kernels (kvh.hip, tickets.hpp);
// *tk = nullptr (and 0 returned) for a stream being captured into a graph: the caller then launches the
// static-order form of its kernel
int stream_tickets(hipStream_t st, unsigned long long** tk);
// kvh_stream_release: synchronise `st` and hand its ticket words back
int stream_release(hipStream_t st);
// kv_ht_radix_sort's exact order on the device, n <= 64K (ht_refsort.hip)
size_t refsort_segments_scratch_bytes(size_t nseg, uint32_t max_seg);
int refsort_segments_launch(const uint64_t* hashes, const uint64_t* items, size_t n, const uint64_t* seg_offs,
                            size_t nseg, uint32_t max_seg, const kvh_ht_geom_t* geom, uint64_t* h_out, uint64_t* items_out,
                            uint64_t* dup_counts, bool dedup, void* scratch, size_t scratch_bytes, hipStream_t st);
size_t refsort_batched_scratch_bytes(size_t n, uint32_t batch);
int refsort_batched_launch(const uint64_t* hashes, const uint64_t* items, size_t n, uint32_t batch,
                           const kvh_ht_geom_t* geom, uint64_t* h_out, uint64_t* items_out, uint64_t* dup_counts,
                           bool dedup, void* scratch, size_t scratch_bytes, hipStream_t st);
size_t refsort_scratch_bytes(size_t n);
int refsort_launch(const uint64_t* hashes, const uint64_t* items, size_t n, const kvh_ht_geom_t* geom,
                   uint64_t* h_out, uint64_t* items_out, uint64_t* dup_count, bool dedup, void* scratch,
                   size_t scratch_bytes, hipStream_t st);
// variable-length CRC32C kernel: 3 = length-sorted windows on 16-copy tables (default), 1 = on 32-copy
// tables, 0 = lane per key in input order
// (tuning knobs are atomics: kvh_set_tuning may run concurrently with launches)
extern std::atomic<int> g_tune_crc_var;
// table-order sort: h1 bits sorted below the slot bits (0 = by batch size; 64 = the full key)
extern std::atomic<int> g_tune_sort_bits;
// table-order sort engine: 0 = two-pass bucketed when the batch fits it (else radix), 1 = radix (rocPRIM)
// always, 2 = one-pass bucketed when the batch fits it
extern std::atomic<int> g_tune_sort_engine;
// bucket sort: 0 = two workgroups per CU (capacity 8000) when the buckets are small enough, 1 = always the
// one-per-CU kernel (capacity 12288)
extern std::atomic<int> g_tune_sort_cap;
extern std::atomic<int> g_tune_refwg;    // knob 27 (experiments build): exact-order batched form A/B
extern std::atomic<int> g_tune_sort_hd;  // knob 25: counting-sort bits of the half-size bucket sort (0 = 12, 10, 11)
extern std::atomic<int> g_tune_sort_b3;  // knob 23: two-pass bucket sort 0 = k_bk_sort, 1 = k_bk_sortr, 2 = k_bk_sortr2, 3 = half-size buckets (up to 15 bits) and k_bk_sortr at two 512-thread workgroups per CU (default)
// span hashing: 2 / 1 = wave-chunked kernel with the short-key path, two / one spans per lane
// (default 2), 0 = lane per span
extern std::atomic<int> g_tune_spans;
// tokenizer: 1 = wave-chunked (default), 0 = workgroup-chunked
extern std::atomic<int> g_tune_tok;

// The kernel-selection knobs (defined in kvh.hip, read by kvh_fixed.hip and
// kvh_varlen.hip; kvh_set_tuning sets them): NT, workgroups per CU, force
// the generic kernel, keys per lane, multi-seed lanes per key,
// variable-length kernel.
extern std::atomic<int> g_tune_nt, g_tune_wgmul, g_tune_generic, g_tune_kpl, g_tune_ms_lanes, g_tune_var;
extern std::atomic<int> g_tune_order;  // knob 24: fixed-length chunk order (0 per-length default, 1 static, 2 wave tickets, 3-5 workgroup tickets)
inline int knob(const std::atomic<int>& k) { return k.load(std::memory_order_relaxed); }
// workgroups of kBlock threads for n items: wg_per_cu per CU (times knob 1), at most one per kBlock items
inline uint32_t grid_for(uint64_t n, int cus, int wg_per_cu) {
  const uint64_t need = (n + kBlock - 1) / kBlock;
  const int m = wg_per_cu * knob(g_tune_wgmul);
  uint64_t g = (uint64_t)cus * (uint64_t)(m > 1 ? m : 1);
  if (need < g) g = need;
  return (uint32_t)(g > 1 ? g : 1);
}
// the kernels of kvh_fixed.hip / kvh_varlen.hip behind the C-ABI entry points
// (arguments already checked; n > 0): everything kvh_meow128_fixed,
// kvh_meow128_multiseed (s = 8 seed pairs, arity 2..8) and kvh_meow128_var launch
int fixed_dispatch(const uint8_t* k, uint32_t key_len, uint64_t n, uint64_t seed1, uint64_t seed2, uint64_t* out,
                   uint32_t flags, hipStream_t st, int cus);
int multiseed_dispatch(const uint8_t* k, uint32_t key_len, uint64_t n, const uint64_t* s, uint32_t arity,
                       uint64_t* out, uint32_t flags, hipStream_t st, int cus);
int var_dispatch(const uint8_t* kp, const uint64_t* offsets, uint64_t n, uint64_t seed1, uint64_t seed2,
                 uint64_t* out, uint32_t flags, hipStream_t st, int cus);
int generic_launch(bool var, const uint8_t* keys, const uint64_t* offs, uint32_t fixed_len, uint64_t n,
                   const uint64_t* s, uint32_t arity, uint64_t* out, uint32_t flags, hipStream_t st, int cus);

// Research-build hook table.  libkvh.so leaves it empty.  The experiments
// library (`make experiments` -> tools/libkvh_exp.so: these objects plus
// tools/exp/*.o) fills it from a static initialiser, so the research kernels
// stay reachable through the same C-ABI calls and kvh_set_tuning knobs
// without living in the product sources.  Each launcher returns false when
// the knob value is not one of its own (the product path then runs).
struct ExpHooks {
  int (*set_tuning)(int k, int value);  // previous value, or KVH_EINVAL: not a research knob
  bool (*var_knob)(int value);          // a research value of knob 7
  bool (*fixed)(int L, const uint8_t* keys, uint64_t n, uint64_t s1, uint64_t s2, uint64_t* out, uint32_t flags,
                hipStream_t st, int cus, int tune_nt, int tune_kpl, int* rc);
  bool (*var)(int knob7, const uint8_t* keys, const uint64_t* offs, uint64_t n, uint64_t s1, uint64_t s2,
              uint64_t* out, uint32_t flags, hipStream_t st, int cus, int* rc);
};
extern ExpHooks g_exp;
}  // namespace rt

}  // namespace kvh
