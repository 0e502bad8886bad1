// ht_refsort.hip -- kv_ht_radix_sort's exact element order on the device
// (VERDICT r4 item 5): kvh_ht_sort with KVH_REF_ORDER, and
// kvh_ht_radix_sort for batches of up to 64K elements (ctest sorts 16K frags
// per batch, test/ctest.c:34, :92).
//
// The reference (src/radix_sort.cpp:31-41 -> include/raikv/radix_sort.h:
// 89-298) is an in-place MSD radix sort of the slots ht_mod(key): 8-bit
// American-flag permutations down to nodes of < 32 elements, a 1-bit Hoare
// pass when one bit is left, bubble / shell-sort tails on less(), and no
// order at all among equal slots.  Its tie order is whatever that sequence
// of swaps leaves, and ctest's duplicate count depends on it (ctest.c:96-104),
// so it is reproduced step for step:
//   - a node is (off, count, shift); nodes are disjoint ranges and each step
//     touches only its own range, so the nodes of one round run in parallel
//     (the reference's LIFO stack order does not change the result);
//   - a node above kWaveCap elements is one step of the whole workgroup:
//     digits and bucket counts in LDS (parallel), then ONE lane walks the
//     American-flag chains (inherently sequential: each swap decides the next
//     one) over the LDS digits and writes each element's final position, then
//     the workgroup moves the elements;
//   - smaller nodes go one per wave, the same with the wave's own LDS slice;
//     tails of < 32 elements are sorted by lane 0 with the reference's
//     compare-exchange sequences and gapped insertion passes.
// One workgroup does it all (n <= 64K); element slots and indices live in
// the caller's scratch.  The restatement it must equal word for word is
// oracle/sort_oracle.c, itself pinned to the reference's outputs
// (tests/golden/sort_*.npz).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include "kvh_internal.hpp"
#include "ht_pos.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

namespace {

KVH_CHK_DECL  // checked build: the first failed bounds check of this unit
// check sites (kvh_debug_checks' out[1])
enum : unsigned { kChkScratch = 2, kChkHashes, kChkElem, kChkList, kChkDig, kChkFin, kChkOut };

constexpr uint32_t kRefMax = 65536;  // elements per call
constexpr uint32_t kWaveCap = 2048;  // nodes up to this size: one wave each
constexpr uint32_t kSmallMax = 16384;  // batches up to this size: the small-workgroup form

// node = off | count << 17 | shift << 34 (off < 2^16 + 1, count <= 2^16, shift <= 64)
__device__ __forceinline__ uint64_t pack(uint32_t off, uint32_t cnt, uint32_t sh) {
  return (uint64_t)off | ((uint64_t)cnt << 17) | ((uint64_t)sh << 34);
}

template <uint32_t WCAP>
struct WaveArea {
  uint8_t dig[WCAP];
  uint16_t fin[WCAP];
  uint32_t c[256], o[256];
  uint64_t ls[32];
  uint8_t li[32];
};

// One sort per workgroup of RT threads, batches of up to MAXN elements;
// workgroup nodes of up to FINLDS elements keep fin[] in LDS (u16), larger
// ones in global scratch.  The single-call form (kvh_ht_sort KVH_REF_ORDER):
// 1024 threads, 64K elements, fin in LDS up to 32K -- one workgroup per CU.
// The many-batch form for batches of <= 16K (RefMany): 256 threads, fin
// always global (the walk's stores are off its dependency chain: digit, then
// bucket slot), wave nodes up to 512 elements, 18 KiB of LDS, so seven or
// eight sorts share a CU and their chain walks interleave.
// scratch of one sort of n elements: slot, slotT (u64), four node lists of n/2 + 2, idx, idxT, fin (u32)
__host__ __device__ inline uint64_t refsort_need(uint64_t n) {
  const uint64_t cap = n / 2 + 2;
  return 16 * n + 32 * cap + 12 * n + 256;
}

template <int RT_, uint32_t MAXN_, uint32_t FINLDS_, uint32_t WCAP_ = kWaveCap>
struct RefCfg {
  static constexpr int RT = RT_, RW = RT_ / 64;
  static constexpr uint32_t MAXN = MAXN_, FINLDS = FINLDS_, WCAP = WCAP_;  // WCAP: nodes up to this size: one wave
};
using RefBig = RefCfg<1024, kRefMax, 32768>;
// Many batches: 256 threads, fin always global, nodes of <= 512 elements to
// one wave (ctest's ~8K batches split into ~34-element nodes below the
// root): 18 KiB of LDS, seven or eight sorts per CU
using RefMany = RefCfg<256, kSmallMax, 1, 512>;
#ifdef KVH_EXPERIMENTS  // the forms RefMany replaced (round 5 A/B, knob 27)
using RefSmall = RefCfg<256, kSmallMax, 1>;  // 36 KiB: four sorts per CU
using RefTiny = RefCfg<128, kSmallMax, 1>;   // 19 KiB: eight two-wave sorts per CU
#endif

template <class Cf>
struct RefSmem {
  using C = Cf;
  // first, at LDS addresses below 64 KiB: the walk's bucket words fold their
  // base into the ds_read / ds_write offset field
  uint32_t bc[256], bo[256];
  uint32_t nl[2][2];  // node counts [list][0 big, 1 small]
  unsigned long long dups;
  union {
    struct {
      uint8_t bdig[C::MAXN];   // digits of a workgroup node (the first FINLDS bytes when fin is in LDS)
    };
    struct {
      uint8_t bdig_s[C::FINLDS];
      uint16_t bfin[C::FINLDS];  // fin of a workgroup node of <= FINLDS elements
    };
    WaveArea<C::WCAP> w[C::RW];  // per-wave slices (the two phases of a round never overlap)
  };
  uint8_t tail[4];  // dig[cnt] may be read (a head past its region): in the allocation
};

struct RefPtrs {  // no arrays: a dynamically indexed member would put the struct in scratch (flat accesses)
  uint64_t *slot, *slotT;
  uint32_t *idx, *idxT, *fin;
  uint64_t* lists;  // list (parity, big = 0 / small = 1) at lists + (2 parity + small) cap
  uint32_t cap;
  uint32_t n;  // elements of this sort (the extent of slot, idx, fin)
  __device__ __forceinline__ uint64_t* list(int parity, int small) const {
    return lists + (size_t)(2 * parity + small) * cap;
  }
};

template <class Sm>
__device__ __forceinline__ void push(Sm& S, const RefPtrs& P, int nx, uint32_t off, uint32_t cnt, uint32_t sh) {
  // a node of < 2 elements, or with no bits left (the reference sorts equal
  // slots by nothing: no sub key), is already in place
  if (cnt < 2 || sh == 0) return;
  const int big = cnt > Sm::C::WCAP ? 0 : 1;
  const uint32_t k = atomicAdd(&S.nl[nx][big], 1u);
  KVH_CHK(k < P.cap && off + cnt <= P.n, kChkList, k, P.cap);
  P.list(nx, big)[k] = pack(off, cnt, sh);
}

// Global scratch written by some waves of the workgroup and read by others:
// workgroup scope is enough (the workgroup's waves share one CU and its L1;
// no device-scope write-back per exchange).
__device__ __forceinline__ void gsync() { __syncthreads(); }

__device__ __forceinline__ void wsync() {  // the same within one wave
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The American-flag chains of one node (radix_sort.h:231-250), by one wave:
// the bucket starts (exclusive scan of the counts c, in LDS) in o (LDS),
// buckets of > 1 element pushed as nodes, then lane 0 walks the chains over
// the LDS digits: position p's element ends at fin(p) (node-relative).  The
// first unplaced slot of bucket b holds its original element (a slot is
// rewritten only when it is placed), so a chain is: take the element at the
// slot, send it to the first unplaced slot o[d] of its bucket d, take that
// slot's element, ... until one of bucket b comes back to the leader's slot.
// The walk is sequential by nature, each swap decides the next.  Each bucket
// head is kept with the digit of the element it holds (o[d] | dig[o[d]] <<
// 17, one LDS word), so a step is ONE LDS round trip: the word of the
// element's bucket gives the slot and the next digit; the next bucket's word
// and the digit behind the slot (for the head's new word) are read together.
// (Node-relative positions are <= 65536: 17 bits.  A head past its region
// reads a digit beyond it, never used: the counts are exact.)
template <class Sm, class Fin>
__device__ __forceinline__ void chains(Sm& S, const RefPtrs& P, int nx, uint32_t off, uint32_t sh2,
                                       const uint8_t* dig, uint32_t dcap, uint32_t* c, uint32_t* o, uint32_t nb,
                                       Fin fin) {
  // dcap: bytes of LDS behind dig that belong to the digit array and what follows it in the same
  // struct; the walk reads at most one digit past its node (checked build: against dcap)
  const uint32_t lane = threadIdx.x & 63;
  uint32_t base = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {  // exclusive scan of the counts in bucket order 64 q + lane
    const uint32_t b = 64u * q + lane;
    const uint32_t v = b < nb ? c[b] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (lane >= (uint32_t)d) inc += y;
    }
    const uint32_t st = base + inc - v;
    o[b] = st | (uint32_t)dig[st] << 17;  // o has 256 entries
    if (v > 1) push(S, P, nx, off + st, v, sh2);
    base += __shfl(inc, 63, 64);
  }
  wave_lds_sync();
  if (lane == 0) {
    uint32_t end = 0;
    for (uint32_t b = 0; b < nb; b++) {
      end += c[b];
      uint32_t q = o[b] & 0x1ffffu;  // o[b] as chains from buckets < b left it
      // The leaders' digits are read one ahead: bucket b's unplaced slots are
      // not written while its own chains run (those fill other buckets).
      uint32_t dq = q < end ? (uint32_t)dig[q] : 0u;
      for (; q < end; q++) {
        KVH_CHK(q + 1 < dcap, kChkDig, q + 1, dcap);
        const uint32_t dnext = dig[q + 1];  // past the region: read, never used
        uint32_t xp = q, d = dq;
        dq = dnext;
        if (d != b) {
          // the word is decoded before the loop and at the end of each step, so
          // the loop head waits for nothing: a step's only wait is for its own
          // two reads (LDS completes in order, the previous step's writes with them)
          const uint32_t w0 = __builtin_amdgcn_readfirstlane(o[d]);  // waited for here, not at the loop head
          uint32_t dst = w0 & 0x1ffffu, nd = w0 >> 17;
          for (;;) {
            KVH_CHK(dst + 1 < dcap, kChkDig, dst + 1, dcap);
            const uint32_t wn = o[nd];  // stale if nd == d: replaced below
            const uint32_t upd = (dst + 1) | (uint32_t)dig[dst + 1] << 17;
            o[d] = upd;
            fin(xp, dst);
            xp = dst;
            if (nd == b) break;
            const uint32_t w = nd == d ? upd : wn;
            d = nd;
            dst = w & 0x1ffffu;
            nd = w >> 17;
          }
        }
        fin(xp, q);
      }
    }
  }
}

// the 1-bit pass (radix_sort.h:251-285) on bit 0 (shift 1): Hoare
// partition; fin must start as the identity
template <class Fin>
__device__ __forceinline__ void hoare(const uint8_t* bit, uint32_t cnt, Fin fin) {
  uint32_t i = 0, j = cnt;
  for (;;) {
    while (i < j && bit[i] == 0) i++;
    while (i < j && bit[j - 1] != 0) j--;
    if (i == j) break;
    fin(i, j - 1);
    fin(j - 1, i);
    i++;
    j--;
  }
}

// count < 32 with bits left (radix_sort.h:121-177): compare-exchange
// sequences for 2-4 elements, gapped insertion passes (48, 21, 7, 3, 1)
// above; on (slot, local index) pairs in LDS, by one lane
__device__ __forceinline__ void leaf(uint64_t* ls, uint8_t* li, uint32_t cnt) {
  auto cx = [&](int a, int b) {
    if (ls[b] < ls[a]) {
      const uint64_t t = ls[a]; ls[a] = ls[b]; ls[b] = t;
      const uint8_t u = li[a]; li[a] = li[b]; li[b] = u;
    }
  };
  if (cnt == 4) { cx(0, 3); cx(1, 3); cx(2, 3); cx(1, 2); }
  if (cnt >= 2 && cnt <= 4) {
    if (cnt >= 3) { cx(0, 2); cx(1, 2); }
    cx(0, 1);
    return;
  }
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint32_t h = k == 0 ? 48u : k == 1 ? 21u : k == 2 ? 7u : k == 3 ? 3u : 1u;
    for (uint32_t i = h; i < cnt; i++) {
      if (!(ls[i] < ls[i - h])) continue;
      const uint64_t xs = ls[i];
      const uint8_t xi = li[i];
      uint32_t j = i;
      do {
        ls[j] = ls[j - h];
        li[j] = li[j - h];
        j -= h;
      } while (j >= h && xs < ls[j - h]);
      ls[j] = xs;
      li[j] = xi;
    }
  }
}

// one node above kWaveCap elements, the whole workgroup (uniform control flow)
template <class Sm>
__device__ __forceinline__ void wg_step(Sm& S, const RefPtrs& P, int nx, uint64_t node) {
  constexpr int kRT = Sm::C::RT;
  const uint32_t off = (uint32_t)(node & 0x1ffff), cnt = (uint32_t)((node >> 17) & 0x1ffff),
                 sh = (uint32_t)(node >> 34);
  const uint32_t tid = threadIdx.x;
  const bool lf = cnt <= Sm::C::FINLDS;  // fin in LDS (u16), else in global scratch
  uint32_t* gfin = P.fin + off;
  uint16_t* lfin = S.bfin;
  KVH_CHK(off + cnt <= P.n && cnt <= Sm::C::MAXN, kChkElem, off + cnt, P.n);
  auto setfin = [&](uint32_t from, uint32_t to) {
    KVH_CHK(from < cnt && to < cnt, kChkFin, from, cnt);
    if (lf) lfin[from] = (uint16_t)to; else gfin[from] = to;
  };
  auto getfin = [&](uint32_t p) -> uint32_t { return lf ? (uint32_t)lfin[p] : gfin[p]; };
  if (sh > 1) {
    const uint32_t k = sh > 8 ? 8 : sh, sh2 = sh - k, nb = 1u << k;
    for (uint32_t b = tid; b < 256; b += kRT) S.bc[b] = 0;
    __syncthreads();
#pragma unroll 4
    for (uint32_t p = tid; p < cnt; p += kRT) {
      const uint32_t d = (uint32_t)(P.slot[off + p] >> sh2) & (nb - 1);
      S.bdig[p] = (uint8_t)d;
      atomicAdd(&S.bc[d], 1u);
    }
    __syncthreads();
    if (S.bc[S.bdig[cnt - 1]] == cnt) {  // one bucket: the same node on the next bits
      if (tid == 0) push(S, P, nx, off, cnt, sh2);
      __syncthreads();
      return;
    }
    if (tid < 64) {  // the walk specialised on where fin lives (no branch per step)
      constexpr uint32_t dcap = sizeof(S.bdig) + sizeof(S.tail);
      if (lf)
        chains(S, P, nx, off, sh2, S.bdig, dcap, S.bc, S.bo, nb, [&](uint32_t f, uint32_t t) {
          KVH_CHK(f < cnt && t < cnt, kChkFin, f, cnt);
          lfin[f] = (uint16_t)t;
        });
      else
        chains(S, P, nx, off, sh2, S.bdig, dcap, S.bc, S.bo, nb, [&](uint32_t f, uint32_t t) {
          KVH_CHK(f < cnt && t < cnt, kChkFin, f, cnt);
          gfin[f] = t;
        });
    }
  } else {  // sh == 1
    for (uint32_t p = tid; p < cnt; p += kRT) {
      S.bdig[p] = (uint8_t)(P.slot[off + p] & 1);
      setfin(p, p);
    }
    gsync();
    if (tid == 0) hoare(S.bdig, cnt, setfin);
    // children have no bits left: in place
  }
  gsync();
#pragma unroll 4
  for (uint32_t p = tid; p < cnt; p += kRT) {
    const uint32_t t = getfin(p);
    P.slotT[off + t] = P.slot[off + p];
    P.idxT[off + t] = P.idx[off + p];
  }
  gsync();
#pragma unroll 4
  for (uint32_t p = tid; p < cnt; p += kRT) {
    P.slot[off + p] = P.slotT[off + p];
    P.idx[off + p] = P.idxT[off + p];
  }
  gsync();
}

// one node of <= kWaveCap elements, one wave
template <class Sm, class WA>
__device__ __forceinline__ void wave_step(Sm& S, const RefPtrs& P, int nx, uint64_t node, WA& W) {
  const uint32_t off = (uint32_t)(node & 0x1ffff), cnt = (uint32_t)((node >> 17) & 0x1ffff),
                 sh = (uint32_t)(node >> 34);
  const uint32_t lane = threadIdx.x & 63;
  KVH_CHK(off + cnt <= P.n && cnt <= Sm::C::WCAP, kChkElem, off + cnt, P.n);
  if (cnt < 32) {  // a tail: sorted on less() by lane 0 (sh >= 1 here)
    if (lane < cnt) { W.ls[lane] = P.slot[off + lane]; W.li[lane] = (uint8_t)lane; }
    wave_lds_sync();
    if (lane == 0) leaf(W.ls, W.li, cnt);
    wave_lds_sync();
    uint64_t s = 0;
    uint32_t ix = 0;
    if (lane < cnt) {
      s = W.ls[lane];
      ix = P.idx[off + W.li[lane]];
    }
    wsync();
    if (lane < cnt) {
      P.slot[off + lane] = s;
      P.idx[off + lane] = ix;
    }
    wsync();
    return;
  }
  auto setfin = [&](uint32_t from, uint32_t to) {
    KVH_CHK(from < cnt && to < cnt, kChkFin, from, cnt);
    W.fin[from] = (uint16_t)to;
  };
  if (sh > 1) {
    const uint32_t k = sh > 8 ? 8 : sh, sh2 = sh - k, nb = 1u << k;
    for (uint32_t b = lane; b < 256; b += 64) W.c[b] = 0;
    wave_lds_sync();
    for (uint32_t p = lane; p < cnt; p += 64) {
      const uint32_t d = (uint32_t)(P.slot[off + p] >> sh2) & (nb - 1);
      W.dig[p] = (uint8_t)d;
      atomicAdd(&W.c[d], 1u);
    }
    wave_lds_sync();
    if (W.c[W.dig[cnt - 1]] == cnt) {
      if (lane == 0) push(S, P, nx, off, cnt, sh2);
      wave_lds_sync();
      return;
    }
    chains(S, P, nx, off, sh2, W.dig, (uint32_t)(sizeof(W.dig) + sizeof(W.fin)), W.c, W.o, nb, setfin);
  } else {  // sh == 1
    for (uint32_t p = lane; p < cnt; p += 64) {
      W.dig[p] = (uint8_t)(P.slot[off + p] & 1);
      W.fin[p] = (uint16_t)p;
    }
    wave_lds_sync();
    if (lane == 0) hoare(W.dig, cnt, setfin);
  }
  wave_lds_sync();
  for (uint32_t p = lane; p < cnt; p += 64) {
    const uint32_t t = W.fin[p];
    P.slotT[off + t] = P.slot[off + p];
    P.idxT[off + t] = P.idx[off + p];
  }
  wsync();
  for (uint32_t p = lane; p < cnt; p += 64) {
    P.slot[off + p] = P.slotT[off + p];
    P.idx[off + p] = P.idxT[off + p];
  }
  wsync();
}

template <class Cf>
__global__ void __launch_bounds__(Cf::RT)
k_refsort(const uint64_t* __restrict__ hashes, const uint64_t* __restrict__ items, uint64_t ntot, uint32_t B,
          const uint64_t* __restrict__ segs, HtGeom g, uint32_t bits, uint64_t* __restrict__ h_out,
          uint64_t* __restrict__ items_out, unsigned long long* __restrict__ dup_count, uint32_t dedup,
          uint8_t* __restrict__ scratch, uint64_t sstride, uint64_t sbytes) {
  // workgroup b sorts batch b: elements [b * B, min(ntot, (b + 1) * B)), or with segs the
  // segment [segs[b], segs[b + 1]) of at most B elements, on its own scratch slice (one batch,
  // the kvh_ht_sort form: B = ntot, one workgroup).  dup_count[b], when given, gets the batch's
  // duplicate count (0 without dedup).  A segment is checked against ntot here, where the offsets
  // are read: reversed or ending past ntot -> flagged ~0, nothing written; longer than B ->
  // copied through in input order, unmarked, and flagged ~0.
  uint64_t b0 = (uint64_t)blockIdx.x * B, nb64 = ntot - b0 < B ? ntot - b0 : B;
  if (segs) {
    b0 = segs[blockIdx.x];
    const uint64_t e = segs[blockIdx.x + 1];
    if (e < b0 || e > ntot) {  // workgroup-uniform (a caller's bad offsets: flagged, not a failed check)
      if (threadIdx.x == 0 && dup_count) dup_count[blockIdx.x] = ~0ull;
      return;
    }
    nb64 = e - b0;
    if (nb64 > B) {
      for (uint64_t k = threadIdx.x; k < nb64; k += Cf::RT) {
        h_out[2 * (b0 + k)] = hashes[2 * (b0 + k)];
        h_out[2 * (b0 + k) + 1] = hashes[2 * (b0 + k) + 1];
        if (items_out) items_out[b0 + k] = items ? items[b0 + k] : b0 + k;
      }
      if (threadIdx.x == 0 && dup_count) dup_count[blockIdx.x] = ~0ull;
      return;
    }
  }
  const uint32_t n = (uint32_t)nb64;
  KVH_CHK(blockIdx.x * sstride + refsort_need(n) <= sbytes, kChkScratch, blockIdx.x * sstride + refsort_need(n),
          sbytes);
  hashes += 2 * b0;
  if (items) items += b0;
  h_out += 2 * b0;
  if (items_out) items_out += b0;
  if (dup_count) dup_count += blockIdx.x;
  scratch += blockIdx.x * sstride;
  constexpr int kRT = Cf::RT, kRW = Cf::RW;
  __shared__ RefSmem<Cf> S;
  const uint32_t tid = threadIdx.x, wv = tid >> 6;
  RefPtrs P;
  {
    uint8_t* s = scratch;
    const uint32_t cap = n / 2 + 2;
    P.cap = cap;
    P.n = n;
    P.slot = (uint64_t*)s; s += 8 * (size_t)n;
    P.slotT = (uint64_t*)s; s += 8 * (size_t)n;
    P.lists = (uint64_t*)s; s += 4 * 8 * (size_t)cap;
    P.idx = (uint32_t*)s; s += 4 * (size_t)n;
    P.idxT = (uint32_t*)s; s += 4 * (size_t)n;
    P.fin = (uint32_t*)s;
  }
  for (uint32_t i = tid; i < n; i += kRT) {
    KVH_CHK(b0 + i < ntot, kChkHashes, b0 + i, ntot);
    P.slot[i] = ht_mod(g, hashes[2 * (size_t)i]);  // FileHdr::ht_mod, shm_ht.h:181-184
    P.idx[i] = i;
  }
  if (tid < 4) S.nl[tid >> 1][tid & 1] = 0;
  if (tid == 0) S.dups = 0;
  __syncthreads();
  if (tid == 0) {  // the root (radix_sort.h:104-118): shift = bit_count
    if (n >= 32)
      push(S, P, 0, 0, n, bits);
    else if (n >= 2)  // a root of < 32 elements is one tail (even the shift-0 case cannot occur: bits >= 1)
      S.nl[0][1] = 1, P.list(0, 1)[0] = pack(0, n, bits);
  }
  gsync();
  for (int cur = 0;; cur ^= 1) {
    const int nx = cur ^ 1;
    const uint32_t nbig = S.nl[cur][0], nsmall = S.nl[cur][1];
    if (nbig + nsmall == 0) break;
    __syncthreads();
    if (tid < 2) S.nl[nx][tid] = 0;
    __syncthreads();
    for (uint32_t k = 0; k < nbig; k++) wg_step(S, P, nx, P.list(cur, 0)[k]);
    for (uint32_t k = wv; k < nsmall; k += kRW) wave_step(S, P, nx, P.list(cur, 1)[k], S.w[wv]);
    gsync();
  }
  // out: the sorted elements; ctest's marking (ctest.c:96-104): an element
  // equal (h1, h2) to its successor gets h1 = 0
  uint32_t local = 0;
  for (uint32_t k = tid; k < n; k += kRT) {
    const uint32_t i = P.idx[k];
    KVH_CHK(i < n && b0 + k < ntot, kChkOut, i, n);
    uint64_t h1 = hashes[2 * (size_t)i];
    const uint64_t h2 = hashes[2 * (size_t)i + 1];
    if (dedup && k + 1 < n) {
      const uint32_t j = P.idx[k + 1];
      if (hashes[2 * (size_t)j] == h1 && hashes[2 * (size_t)j + 1] == h2) {
        h1 = 0;
        local++;
      }
    }
    h_out[2 * (size_t)k] = h1;
    h_out[2 * (size_t)k + 1] = h2;
    if (items_out) items_out[k] = items ? items[i] : b0 + i;
  }
  if (dedup && local) atomicAdd(&S.dups, (unsigned long long)local);
  __syncthreads();
  if (tid == 0 && dup_count) *dup_count = dedup ? S.dups : 0ull;
}

}  // namespace

namespace kvh {
namespace rt {

size_t refsort_scratch_bytes(size_t n) { return refsort_need(n); }

namespace {
HtGeom ref_geom(const kvh_ht_geom_t* geom, uint32_t* bits) {
  HtGeom g;
  g.size = geom->ht_size;
  g.mask = geom->ht_mod_mask;
  g.frac = (uint32_t)geom->ht_mod_fraction;
  g.shift = geom->ht_mod_shift;
  g.buckets = geom->cuckoo_buckets;
  uint32_t b = 1;  // radix_sort.h:75-77: 1 + floor(log2 ht_size)
  for (uint64_t m = geom->ht_size; m > 1; m >>= 1) b++;
  *bits = b;
  return g;
}
}  // namespace

int refsort_launch(const uint64_t* hashes, const uint64_t* items, size_t n, const kvh_ht_geom_t* geom,
                   uint64_t* h_out, uint64_t* items_out, uint64_t* dup_count, bool dedup, void* scratch,
                   size_t scratch_bytes, hipStream_t st) {
  if (n > kRefMax || scratch_bytes < refsort_scratch_bytes(n)) return set_err(KVH_EINVAL);
  uint32_t bits;
  const HtGeom g = ref_geom(geom, &bits);
  hipLaunchKernelGGL(k_refsort<RefBig>, dim3(1), dim3(RefBig::RT), 0, st, hashes, items, (uint64_t)n, (uint32_t)n,
                     (const uint64_t*)nullptr, g, bits, h_out, items_out,
                     (unsigned long long*)(dedup ? dup_count : nullptr), dedup ? 1u : 0u, (uint8_t*)scratch,
                     (uint64_t)0, (uint64_t)scratch_bytes);
  return launch_done();
}

// per-batch scratch slices, 256-byte aligned
static size_t batch_stride(uint32_t batch) { return (refsort_scratch_bytes(batch) + 255) & ~(size_t)255; }

size_t refsort_batched_scratch_bytes(size_t n, uint32_t batch) {
  if (batch == 0 || batch > kRefMax) return 0;
  const size_t nb = (n + batch - 1) / batch;
  return (nb ? nb : 1) * batch_stride(batch);  // nonzero for every valid batch size, n = 0 included
}

// one workgroup per batch: up to one batch per CU the 1024-thread form is faster per batch; beyond
// that seven or eight RefMany sorts per CU interleave their chain walks
static int launch_many(const uint64_t* hashes, const uint64_t* items, uint64_t ntot, uint32_t B,
                       const uint64_t* segs, uint64_t nb, const kvh_ht_geom_t* geom, uint64_t* h_out,
                       uint64_t* items_out, uint64_t* dup_counts, bool dedup, void* scratch, size_t sbytes,
                       hipStream_t st) {
  uint32_t bits;
  const HtGeom g = ref_geom(geom, &bits);
  int cus = 0;
  if (int rc = device_cus(&cus)) return rc;
#ifdef KVH_EXPERIMENTS
  const int form = knob(g_tune_refwg);
  if (B <= kSmallMax && nb > (uint64_t)cus && form == 128)
    hipLaunchKernelGGL(k_refsort<RefTiny>, dim3((uint32_t)nb), dim3(RefTiny::RT), 0, st, hashes, items, ntot, B,
                       segs, g, bits, h_out, items_out, (unsigned long long*)dup_counts, dedup ? 1u : 0u,
                       (uint8_t*)scratch, (uint64_t)batch_stride(B), (uint64_t)sbytes);
  else if (B <= kSmallMax && nb > (uint64_t)cus && form == 256)
    hipLaunchKernelGGL(k_refsort<RefSmall>, dim3((uint32_t)nb), dim3(RefSmall::RT), 0, st, hashes, items, ntot, B,
                       segs, g, bits, h_out, items_out, (unsigned long long*)dup_counts, dedup ? 1u : 0u,
                       (uint8_t*)scratch, (uint64_t)batch_stride(B), (uint64_t)sbytes);
  else
#endif
  if (B <= kSmallMax && nb > (uint64_t)cus)
    hipLaunchKernelGGL(k_refsort<RefMany>, dim3((uint32_t)nb), dim3(RefMany::RT), 0, st, hashes, items, ntot, B,
                       segs, g, bits, h_out, items_out, (unsigned long long*)dup_counts, dedup ? 1u : 0u,
                       (uint8_t*)scratch, (uint64_t)batch_stride(B), (uint64_t)sbytes);
  else
    hipLaunchKernelGGL(k_refsort<RefBig>, dim3((uint32_t)nb), dim3(RefBig::RT), 0, st, hashes, items, ntot, B,
                       segs, g, bits, h_out, items_out, (unsigned long long*)dup_counts, dedup ? 1u : 0u,
                       (uint8_t*)scratch, (uint64_t)batch_stride(B), (uint64_t)sbytes);
  return launch_done();
}

int refsort_batched_launch(const uint64_t* hashes, const uint64_t* items, size_t n, uint32_t batch,
                           const kvh_ht_geom_t* geom, uint64_t* h_out, uint64_t* items_out, uint64_t* dup_counts,
                           bool dedup, void* scratch, size_t scratch_bytes, hipStream_t st) {
  if (batch == 0 || batch > kRefMax || n >= (1ull << 40)) return set_err(KVH_EINVAL);
  if (n == 0) return set_err(0);
  if (scratch_bytes < refsort_batched_scratch_bytes(n, batch)) return set_err(KVH_EINVAL);
  const uint64_t nb = (n + batch - 1) / batch;
  if (nb > 0x7fffffffull) return set_err(KVH_EINVAL);
  return launch_many(hashes, items, n, batch, nullptr, nb, geom, h_out, items_out, dup_counts, dedup, scratch,
                     scratch_bytes, st);
}

size_t refsort_segments_scratch_bytes(size_t nseg, uint32_t max_seg) {
  if (max_seg == 0 || max_seg > kRefMax) return 0;
  return (nseg ? nseg : 1) * batch_stride(max_seg);
}

int refsort_segments_launch(const uint64_t* hashes, const uint64_t* items, size_t n, const uint64_t* seg_offs,
                            size_t nseg, uint32_t max_seg, const kvh_ht_geom_t* geom, uint64_t* h_out,
                            uint64_t* items_out, uint64_t* dup_counts, bool dedup, void* scratch, size_t scratch_bytes,
                            hipStream_t st) {
  if (max_seg == 0 || max_seg > kRefMax || nseg > 0x7fffffffull) return set_err(KVH_EINVAL);
  if (nseg == 0) return set_err(0);
  if (!seg_offs || scratch_bytes < refsort_segments_scratch_bytes(nseg, max_seg)) return set_err(KVH_EINVAL);
  // n bounds every segment on the device (the offsets are device memory): an empty batch list (n = 0)
  // still flags each non-empty segment instead of reading past the pairs
  return launch_many(hashes, items, (uint64_t)n, max_seg, seg_offs, nseg, geom, h_out, items_out, dup_counts, dedup,
                     scratch, scratch_bytes, st);
}

int chk_take_refsort(unsigned long long out[4]) {
#if KVH_CHECKED_ON
  if (hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chk), 32)) return hip_err(e);
  const unsigned long long z[4] = {0, 0, 0, 0};
  if (hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_chk), z, 32)) return hip_err(e);
#else
  for (int i = 0; i < 4; i++) out[i] = 0;
#endif
  return 0;
}

}  // namespace rt
}  // namespace kvh
