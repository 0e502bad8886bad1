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

constexpr uint32_t kRefMax = 65536;  // elements per call
constexpr uint32_t kWaveCap = 2048;  // nodes up to this size: one wave each
constexpr int kRT = 1024, kRW = kRT / 64;

// node = off | count << 17 | shift << 34 (off < 2^16 + 1, count <= 2^16, shift <= 64)
__device__ __forceinline__ uint64_t pack(uint32_t off, uint32_t cnt, uint32_t sh) {
  return (uint64_t)off | ((uint64_t)cnt << 17) | ((uint64_t)sh << 34);
}

struct WaveArea {
  uint8_t dig[kWaveCap];
  uint16_t fin[kWaveCap];
  uint32_t c[256], o[256];
  uint64_t ls[32];
  uint8_t li[32];
};

struct RefSmem {
  union {
    uint8_t bdig[kRefMax];  // digits of a workgroup node
    WaveArea w[kRW];        // per-wave slices (the two phases of a round never overlap)
  };
  uint32_t bc[256], bo[256];
  uint32_t nl[2][2];  // node counts [list][0 big, 1 small]
  unsigned long long dups;
};

struct RefPtrs {
  uint64_t *slot, *slotT;
  uint32_t *idx, *idxT, *fin;
  uint64_t* list[2][2];  // [round parity][big, small], capacity cap each
  uint32_t cap;
};

__device__ __forceinline__ void push(RefSmem& S, const RefPtrs& P, int nx, uint32_t off, uint32_t cnt, uint32_t sh) {
  // a node of < 2 elements, or with no bits left (the reference sorts equal
  // slots by nothing: no sub key), is already in place
  if (cnt < 2 || sh == 0) return;
  const int big = cnt > kWaveCap ? 0 : 1;
  const uint32_t k = atomicAdd(&S.nl[nx][big], 1u);
  P.list[nx][big][k] = pack(off, cnt, sh);
}

__device__ __forceinline__ void gsync() {  // global scratch written before, read after, across the workgroup
  __threadfence();
  __syncthreads();
}

__device__ __forceinline__ void wsync() {  // the same within one wave
  __threadfence();
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// The American-flag chains of one node (radix_sort.h:231-250), walked by one
// lane over the node's digits: c[b] counts, o[b] bucket starts on entry.
// Position p's element ends at fin[p] (node-relative).  The first unplaced
// slot of bucket b holds its original element (a slot is rewritten only
// when it is placed), so a chain is: take the element at the slot, send it
// to the first unplaced slot of its bucket, take that slot's element, ...
// until one of bucket b comes back to the leader's slot.
template <class Fin>
__device__ void chains(const uint8_t* dig, uint32_t* c, uint32_t* o, uint32_t nb, Fin fin) {
  for (uint32_t b = 0; b < nb; b++) {
    while (c[b] > 0) {
      const uint32_t q = o[b];
      uint32_t xp = q, d = dig[q];
      while (d != b) {
        const uint32_t dst = o[d];
        o[d] = dst + 1;
        c[d]--;
        fin(xp, dst);
        xp = dst;
        d = dig[dst];
      }
      fin(xp, q);
      o[b] = q + 1;
      c[b]--;
    }
  }
}

// the 1-bit pass (radix_sort.h:251-285) on bit 0 (shift 1): Hoare
// partition; fin must start as the identity
template <class Fin>
__device__ void hoare(const uint8_t* bit, uint32_t cnt, Fin fin) {
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
__device__ void leaf(uint64_t* ls, uint8_t* li, uint32_t cnt) {
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
  const uint32_t gaps[5] = {48, 21, 7, 3, 1};
  for (int k = 0; k < 5; k++) {
    const uint32_t h = gaps[k];
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
__device__ void wg_step(RefSmem& S, const RefPtrs& P, int nx, uint64_t node) {
  const uint32_t off = (uint32_t)(node & 0x1ffff), cnt = (uint32_t)((node >> 17) & 0x1ffff),
                 sh = (uint32_t)(node >> 34);
  const uint32_t tid = threadIdx.x;
  uint32_t* fin = P.fin + off;
  if (sh > 1) {
    const uint32_t k = sh > 8 ? 8 : sh, sh2 = sh - k, nb = 1u << k;
    for (uint32_t b = tid; b < 256; b += kRT) S.bc[b] = 0;
    __syncthreads();
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
    if (tid == 0) {
      uint32_t base = 0;
      for (uint32_t b = 0; b < nb; b++) {
        S.bo[b] = base;
        if (S.bc[b] > 1) push(S, P, nx, off + base, S.bc[b], sh2);
        base += S.bc[b];
      }
      chains(S.bdig, S.bc, S.bo, nb, [&](uint32_t from, uint32_t to) { fin[from] = to; });
    }
  } else {  // sh == 1
    for (uint32_t p = tid; p < cnt; p += kRT) {
      S.bdig[p] = (uint8_t)(P.slot[off + p] & 1);
      fin[p] = p;
    }
    gsync();
    if (tid == 0) hoare(S.bdig, cnt, [&](uint32_t from, uint32_t to) { fin[from] = to; });
    // children have no bits left: in place
  }
  gsync();
  for (uint32_t p = tid; p < cnt; p += kRT) {
    const uint32_t t = fin[p];
    P.slotT[off + t] = P.slot[off + p];
    P.idxT[off + t] = P.idx[off + p];
  }
  gsync();
  for (uint32_t p = tid; p < cnt; p += kRT) {
    P.slot[off + p] = P.slotT[off + p];
    P.idx[off + p] = P.idxT[off + p];
  }
  gsync();
}

// one node of <= kWaveCap elements, one wave
__device__ void wave_step(RefSmem& S, const RefPtrs& P, int nx, uint64_t node, WaveArea& W) {
  const uint32_t off = (uint32_t)(node & 0x1ffff), cnt = (uint32_t)((node >> 17) & 0x1ffff),
                 sh = (uint32_t)(node >> 34);
  const uint32_t lane = threadIdx.x & 63;
  if (cnt < 32) {  // a tail: sorted on less() by lane 0 (sh >= 1 here)
    if (lane == 0) {
      for (uint32_t p = 0; p < cnt; p++) { W.ls[p] = P.slot[off + p]; W.li[p] = (uint8_t)p; }
      leaf(W.ls, W.li, cnt);
    }
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
    if (lane == 0) {
      uint32_t base = 0;
      for (uint32_t b = 0; b < nb; b++) {
        W.o[b] = base;
        if (W.c[b] > 1) push(S, P, nx, off + base, W.c[b], sh2);
        base += W.c[b];
      }
      chains(W.dig, W.c, W.o, nb, [&](uint32_t from, uint32_t to) { W.fin[from] = (uint16_t)to; });
    }
  } else {  // sh == 1
    for (uint32_t p = lane; p < cnt; p += 64) {
      W.dig[p] = (uint8_t)(P.slot[off + p] & 1);
      W.fin[p] = (uint16_t)p;
    }
    wave_lds_sync();
    if (lane == 0) hoare(W.dig, cnt, [&](uint32_t from, uint32_t to) { W.fin[from] = (uint16_t)to; });
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

__global__ void __launch_bounds__(kRT)
k_refsort(const uint64_t* __restrict__ hashes, const uint64_t* __restrict__ items, uint32_t n, HtGeom g,
          uint32_t bits, uint64_t* __restrict__ h_out, uint64_t* __restrict__ items_out,
          unsigned long long* __restrict__ dup_count, uint32_t dedup, uint8_t* __restrict__ scratch) {
  __shared__ RefSmem S;
  const uint32_t tid = threadIdx.x, wv = tid >> 6;
  RefPtrs P;
  {
    uint8_t* s = scratch;
    const uint32_t cap = n / 2 + 2;
    P.cap = cap;
    P.slot = (uint64_t*)s; s += 8 * (size_t)n;
    P.slotT = (uint64_t*)s; s += 8 * (size_t)n;
    for (int a = 0; a < 2; a++)
      for (int b = 0; b < 2; b++) { P.list[a][b] = (uint64_t*)s; s += 8 * (size_t)cap; }
    P.idx = (uint32_t*)s; s += 4 * (size_t)n;
    P.idxT = (uint32_t*)s; s += 4 * (size_t)n;
    P.fin = (uint32_t*)s;
  }
  for (uint32_t i = tid; i < n; i += kRT) {
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
      S.nl[0][1] = 1, P.list[0][1][0] = pack(0, n, bits);
  }
  gsync();
  for (int cur = 0;; cur ^= 1) {
    const int nx = cur ^ 1;
    const uint32_t nbig = S.nl[cur][0], nsmall = S.nl[cur][1];
    if (nbig + nsmall == 0) break;
    __syncthreads();
    if (tid < 2) S.nl[nx][tid] = 0;
    __syncthreads();
    for (uint32_t k = 0; k < nbig; k++) wg_step(S, P, nx, P.list[cur][0][k]);
    for (uint32_t k = wv; k < nsmall; k += kRW) wave_step(S, P, nx, P.list[cur][1][k], S.w[wv]);
    gsync();
  }
  // out: the sorted elements; ctest's marking (ctest.c:96-104): an element
  // equal (h1, h2) to its successor gets h1 = 0
  uint32_t local = 0;
  for (uint32_t k = tid; k < n; k += kRT) {
    const uint32_t i = P.idx[k];
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
    if (items_out) items_out[k] = items ? items[i] : (uint64_t)i;
  }
  if (dedup) {
    if (local) atomicAdd(&S.dups, (unsigned long long)local);
    __syncthreads();
    if (tid == 0 && dup_count) *dup_count = S.dups;
  }
}

}  // namespace

namespace kvh {
namespace rt {

size_t refsort_scratch_bytes(size_t n) {
  const size_t cap = n / 2 + 2;
  return 16 * n + 32 * cap + 12 * n + 256;
}

int refsort_launch(const uint64_t* hashes, const uint64_t* items, size_t n, const kvh_ht_geom_t* geom,
                   uint64_t* h_out, uint64_t* items_out, uint64_t* dup_count, bool dedup, void* scratch,
                   size_t scratch_bytes, hipStream_t st) {
  if (n > kRefMax || scratch_bytes < refsort_scratch_bytes(n)) return set_err(KVH_EINVAL);
  HtGeom g;
  g.size = geom->ht_size;
  g.mask = geom->ht_mod_mask;
  g.frac = (uint32_t)geom->ht_mod_fraction;
  g.shift = geom->ht_mod_shift;
  g.buckets = geom->cuckoo_buckets;
  uint32_t bits = 1;  // radix_sort.h:75-77: 1 + floor(log2 ht_size)
  for (uint64_t m = geom->ht_size; m > 1; m >>= 1) bits++;
  hipLaunchKernelGGL(k_refsort, dim3(1), dim3(kRT), 0, st, hashes, items, (uint32_t)n, g, bits, h_out, items_out,
                     (unsigned long long*)(dedup ? dup_count : nullptr), dedup ? 1u : 0u, (uint8_t*)scratch);
  return launch_done();
}

}  // namespace rt
}  // namespace kvh
