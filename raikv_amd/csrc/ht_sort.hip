// ht_sort.hip -- SURVEY.md §8 row f2: order a hashed batch by hash-table
// position and mark duplicates, on the device.
//
// Reference: kv_ht_radix_sort (src/radix_sort.cpp:31-41) sorts kv_ht_sort_t
// {key, key2, item} by ht_mod(key) with an in-place MSD radix sort over the
// bits of ht_size (include/raikv/radix_sort.h:29-316); elements whose slots
// are equal keep an unspecified order.  ctest.c:96-104 then zeroes the
// `hash` of every element equal (hash, hash2) to its successor and counts it.
//
// Here the order is total and deterministic: by slot, then by h1 (bit 63
// ignored first, as the key below does), then h1, then h2 -- a refinement of
// the reference's order, so every adjacent-equal pair the reference could
// find is adjacent here, and all duplicates of a key are contiguous.
//   1. k_sort_keys   key64 = slot << (64 - sbits) | (h1 << 1) >> sbits,
//                    kept: that prefix, as u32 when it fits 31 bits; idx = i
//                    (u32); with items, (h1, h2, item) -> 32-byte records in
//                    the same pass over the hashes
//   2. radix sort of (key, idx) pairs over a prefix of key64 only: the
//      slot bits and max(1, log2(n) + 5 - sbits) bits of h1, at most 31 with
//      u32 keys (100M keys, 64 GiB table: 31 bits in 4 onesweep passes of
//      u32 keys instead of 8 of u64): rocPRIM's rocprim::radix_sort_pairs
//      (the library primitive; ROCm's own), stable
//   4. k_sort_place  hashes_out / items_out[j] = record idx[j] (one random
//                    read per element)
//   5. k_sort_fixup  runs of equal sorted prefix (equal slot and equal top
//                    h1 bits: ≈3 % of the elements, and duplicates) of at
//                    most kShortRun elements insertion-sorted in the outputs
//                    by the full comparator: the order is a full 64-bit
//                    sort's; with KVH_DEDUP the h1 of an element equal to its
//                    successor set to 0 and counted.  Longer runs (only
//                    non-uniform "hashes" or mass duplicates make them) are
//                    listed for
//   6. k_sort_long   one workgroup per listed run: a bitonic sort network
//                    over the run's records (O(R log² R) work, R / 256-way
//                    parallel, instead of one thread's O(R²) insertion sort),
//                    the input order as the last tie-break so it stays the
//                    stable order insertion sort gives; same dedup
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <mutex>
#include <vector>
#include <rocprim/device/device_radix_sort.hpp>
#include "kvh_internal.hpp"
#include "ht_pos.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

namespace {

constexpr int kSB = 256;
// runs longer than this go to k_sort_long (insertion sort is O(R²) per thread)
constexpr uint64_t kShortRun = 64;

// (h1, h2, item) padded to 32 bytes: one aligned random read per record
struct __attribute__((aligned(16))) Rec {
  uint64_t h1, h2, item, pad;
};

__device__ __forceinline__ bool rec_less(uint64_t a1, uint64_t a2, uint64_t b1, uint64_t b2) {
  const uint64_t a0 = a1 << 1, b0 = b1 << 1;
  if (a0 != b0) return a0 < b0;
  if (a1 != b1) return a1 < b1;
  return a2 < b2;
}

// key = the top (64 - lo) bits of slot << (64 - sbits) | (h1 << 1) >> sbits,
// shifted down to bit 0: the radix sort then runs over bits [0, 64 - lo).
// (Not [lo, 64) in place: rocPRIM's merge-sort path, taken for n <= 1M,
// builds its mask as (1 << (begin_bit + bits)) - 1, undefined at 64.)
template <class K, bool PACK>
__global__ void __launch_bounds__(kSB)
k_sort_keys(const uint64_t* __restrict__ h, const uint64_t* __restrict__ items, uint64_t n, HtGeom g,
            uint32_t sbits, uint32_t lo, K* __restrict__ key, uint32_t* __restrict__ idx, Rec* __restrict__ rec,
            uint32_t* __restrict__ nlong) {
  const uint64_t i = (uint64_t)blockIdx.x * kSB + threadIdx.x;
  if (i == 0) *nlong = 0;  // k_sort_fixup's long-run list, empty per call
  if (i >= n) return;
  const uint64_t h1 = h[2 * i];
  const uint64_t slot = ht_mod(g, h1);
  const uint64_t k64 = sbits >= 64 ? slot : (slot << (64 - sbits)) | ((h1 << 1) >> sbits);
  key[i] = (K)(k64 >> lo);
  idx[i] = (uint32_t)i;
  if constexpr (PACK) {  // (h1, h2, item) -> 32-byte record, in the same pass over the hashes
    Rec r;
    r.h1 = h1;
    r.h2 = h[2 * i + 1];
    r.item = items[i];
    r.pad = 0;
    rec[i] = r;
  }
}

// sorted position j <- record idx[j]: one random read (a packed record, or
// the hash pair when the items are the indices), coalesced writes
__global__ void __launch_bounds__(kSB)
k_sort_place(const uint64_t* __restrict__ h, const Rec* __restrict__ rec, const uint32_t* __restrict__ idx,
             uint64_t n, uint64_t* __restrict__ h_out, uint64_t* __restrict__ items_out) {
  const uint64_t j = (uint64_t)blockIdx.x * kSB + threadIdx.x;
  if (j >= n) return;
  const uint32_t s = idx[j];
  uint64_t h1, h2, it;
  if (rec) {
    const Rec r = rec[s];
    h1 = r.h1; h2 = r.h2; it = r.item;
  } else {
    h1 = h[2 * (uint64_t)s]; h2 = h[2 * (uint64_t)s + 1]; it = s;
  }
  h_out[2 * j] = h1;
  h_out[2 * j + 1] = h2;
  if (items_out) items_out[j] = it;
}

__device__ __forceinline__ uint32_t block_sum(uint32_t d, uint32_t* wsum) {
  for (int o = 32; o >= 1; o >>= 1) d += __shfl_xor(d, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = d;
  __syncthreads();
  uint32_t t = 0;
  for (int w = 0; w < kSB / 64; w++) t += wsum[w];
  __syncthreads();
  return t;
}

// Runs of equal sorted prefix (equal slot and top h1 bits) of at most
// kShortRun elements are put in the full order (h1 << 1, h1, h2) by
// insertion sort -- stable, so exact duplicates keep the input order the
// radix sort left them in -- and, with dedup, every element equal (h1, h2)
// to its successor gets h1 = 0 (ctest.c:96-104).  Equal pairs share a
// prefix, so runs are the only place duplicates occur.  A longer run's start
// is appended to runs[] for k_sort_long (at most kShortRun + 1 key reads per
// thread here).  Grid-stride; one atomic per workgroup.
template <class K>
__global__ void __launch_bounds__(kSB)
k_sort_fixup(const K* __restrict__ key, uint64_t n, uint64_t* __restrict__ h, uint64_t* __restrict__ items,
             uint32_t dedup, unsigned long long* __restrict__ dups, uint32_t* __restrict__ nlong,
             uint32_t* __restrict__ runs) {
  __shared__ uint32_t wsum[kSB / 64];
  uint32_t d = 0;
  const uint64_t stride = (uint64_t)gridDim.x * kSB;
  for (uint64_t j = (uint64_t)blockIdx.x * kSB + threadIdx.x; j + 1 < n; j += stride) {
    if (key[j + 1] != key[j] || (j > 0 && key[j - 1] == key[j])) continue;  // run starts only
    uint64_t e = j + 2;
    while (e < n && e - j <= kShortRun && key[e] == key[j]) e++;
    if (e - j > kShortRun) {
      runs[atomicAdd(nlong, 1u)] = (uint32_t)j;
      continue;
    }
    for (uint64_t a = j + 1; a < e; a++) {  // insertion sort of [j, e)
      const uint64_t v1 = h[2 * a], v2 = h[2 * a + 1], vi = items ? items[a] : 0;
      uint64_t b = a;
      while (b > j && rec_less(v1, v2, h[2 * (b - 1)], h[2 * (b - 1) + 1])) {
        h[2 * b] = h[2 * (b - 1)];
        h[2 * b + 1] = h[2 * (b - 1) + 1];
        if (items) items[b] = items[b - 1];
        b--;
      }
      if (b != a) {
        h[2 * b] = v1;
        h[2 * b + 1] = v2;
        if (items) items[b] = vi;
      }
    }
    if (dedup) {
      for (uint64_t a = j; a + 1 < e; a++)
        if (h[2 * a] == h[2 * (a + 1)] && h[2 * a + 1] == h[2 * (a + 1) + 1]) { h[2 * a] = 0; d++; }
    }
  }
  if (dedup && dups) {
    const uint32_t t = block_sum(d, wsum);
    if (threadIdx.x == 0 && t) atomicAdd(dups, (unsigned long long)t);
  }
}

// record order within a long run: the full comparator, then the position the
// radix sort left the element at (the stable tie-break), kept in Rec::pad
__device__ __forceinline__ bool run_less(const Rec& a, const Rec& b) {
  if (a.h1 != b.h1 || a.h2 != b.h2) return rec_less(a.h1, a.h2, b.h1, b.h2);
  return a.pad < b.pad;
}

// One workgroup per long run (grid-stride over the list): find the run's end
// (256 keys per step), copy it to rec[j, e) with its positions (the records
// k_sort_place read are consumed by then; stream order), sort that in place
// with an all-ascending bitonic network -- every compare-exchange puts the
// smaller record at the lower index, so the pad to a power of two is virtual:
// a comparator whose upper index is past the run is a no-op -- then write it
// back with the dedup marks.  Already-ordered runs (e.g. all duplicates) skip
// the network.
template <class K>
__global__ void __launch_bounds__(kSB)
k_sort_long(const K* __restrict__ key, uint64_t n, uint64_t* __restrict__ h, uint64_t* __restrict__ items,
            Rec* __restrict__ rec, uint32_t dedup, unsigned long long* __restrict__ dups,
            const uint32_t* __restrict__ nlong, const uint32_t* __restrict__ runs) {
  __shared__ uint32_t wsum[kSB / 64];
  __shared__ uint64_t s_end;
  const uint32_t count = *nlong;
  const uint32_t tid = threadIdx.x;
  uint32_t d = 0;
  for (uint32_t r = blockIdx.x; r < count; r += gridDim.x) {
    const uint64_t j = runs[r];
    const K kj = key[j];
    if (tid == 0) s_end = n;
    __syncthreads();
    for (uint64_t base = j + 1 + kShortRun; base < n; base += kSB) {
      const uint64_t x = base + tid;
      const bool stop = x < n && key[x] != kj;
      if (stop) atomicMin((unsigned long long*)&s_end, (unsigned long long)x);
      __syncthreads();
      const bool done = s_end < n;
      __syncthreads();
      if (done) break;
    }
    const uint64_t len = s_end - j;
    Rec* R = rec + j;
    uint32_t unordered = 0;
    for (uint64_t t = tid; t < len; t += kSB) {
      Rec v;
      v.h1 = h[2 * (j + t)];
      v.h2 = h[2 * (j + t) + 1];
      v.item = items ? items[j + t] : 0;
      v.pad = t;
      R[t] = v;
      if (t + 1 < len) unordered |= rec_less(h[2 * (j + t + 1)], h[2 * (j + t + 1) + 1], v.h1, v.h2);
    }
    if (block_sum(unordered, wsum)) {
      uint64_t P = 1;
      while (P < len) P <<= 1;
      for (uint64_t k = 2; k <= P; k <<= 1) {
        for (uint64_t jj = k >> 1; jj > 0; jj >>= 1) {
          for (uint64_t t = tid; t < P / 2; t += kSB) {
            const uint64_t off = t & (jj - 1);
            uint64_t a, b;
            if (jj == (k >> 1)) {  // first step of the merge: the mirror comparator
              a = (t / jj) * k + off;
              b = (t / jj) * k + k - 1 - off;
            } else {
              a = (t / jj) * 2 * jj + off;
              b = a + jj;
            }
            if (b >= len) continue;
            const Rec x = R[a], y = R[b];
            if (run_less(y, x)) { R[a] = y; R[b] = x; }
          }
          __syncthreads();
        }
      }
    }
    __syncthreads();
    for (uint64_t t = tid; t < len; t += kSB) {
      const Rec v = R[t];
      bool dup = false;
      if (dedup && t + 1 < len) {
        const Rec w = R[t + 1];
        dup = v.h1 == w.h1 && v.h2 == w.h2;
      }
      d += dup;
      h[2 * (j + t)] = dup ? 0 : v.h1;
      h[2 * (j + t) + 1] = v.h2;
      if (items) items[j + t] = v.item;
    }
    __syncthreads();
  }
  if (dedup && dups) {
    const uint32_t t = block_sum(d, wsum);
    if (tid == 0 && t) atomicAdd(dups, (unsigned long long)t);
  }
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct SortLayout {
  size_t key_in, key_out, idx_in, idx_out, rec, runs, tmp, tmp_bytes, total;
};

int sort_layout(size_t n, SortLayout* L) {
  size_t tmp = 0, tmp32 = 0;  // either key width (sort_impl picks one)
  hipError_t e = rocprim::radix_sort_pairs((void*)nullptr, tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0u, 64u,
                                           (hipStream_t)0);
  if (e != hipSuccess) return hip_err(e);
  e = rocprim::radix_sort_pairs((void*)nullptr, tmp32, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0u, 31u, (hipStream_t)0);
  if (e != hipSuccess) return hip_err(e);
  tmp = std::max(tmp, tmp32);
  size_t o = 0;
  L->key_in = o; o += al256(8 * n);
  L->key_out = o; o += al256(8 * n);
  L->idx_in = o; o += al256(4 * n);
  L->idx_out = o; o += al256(4 * n);
  L->rec = o; o += al256(sizeof(Rec) * n);
  L->runs = o; o += al256(4 * (n / (kShortRun + 1) + 2));  // count, then run starts
  L->tmp = o; o += al256(tmp);
  L->tmp_bytes = tmp;
  L->total = o;
  return 0;
}

uint32_t slot_bits(uint64_t ht_size) {
  uint32_t b = 1;
  while (b < 64 && (ht_size >> b) != 0) b++;
  return b;
}

int sort_impl(const uint64_t* hashes, const uint64_t* items, size_t n, const kvh_ht_geom_t* geom, uint64_t* h_out,
              uint64_t* items_out, uint64_t* dup_count, uint32_t flags, void* scratch, size_t scratch_bytes,
              hipStream_t st) {
  if (!geom || geom->ht_size == 0 || geom->ht_mod_shift >= 64 || geom->ht_mod_fraction >= (1ull << 32))
    return set_err(KVH_EINVAL);
  const bool dedup = (flags & KVH_DEDUP) != 0;
  if (dedup && dup_count) {
    hipError_t e = hipMemsetAsync(dup_count, 0, 8, st);
    if (e != hipSuccess) return hip_err(e);
  }
  if (n == 0) return set_err(0);
  if (n >= (1ull << 32) || !hashes || !h_out || !scratch) return set_err(KVH_EINVAL);
  SortLayout L;
  int rc = sort_layout(n, &L);
  if (rc) return rc;
  if (scratch_bytes < L.total) return set_err(KVH_EINVAL);
  uint8_t* s = (uint8_t*)scratch;
  uint64_t* kin = (uint64_t*)(s + L.key_in);
  uint64_t* kout = (uint64_t*)(s + L.key_out);
  uint32_t* iin = (uint32_t*)(s + L.idx_in);
  uint32_t* iout = (uint32_t*)(s + L.idx_out);
  Rec* rec = (Rec*)(s + L.rec);
  uint32_t* nlong = (uint32_t*)(s + L.runs);
  uint32_t* runs = nlong + 1;
  HtGeom g;
  g.size = geom->ht_size;
  g.mask = geom->ht_mod_mask;
  g.frac = (uint32_t)geom->ht_mod_fraction;
  g.shift = geom->ht_mod_shift;
  g.buckets = geom->cuckoo_buckets;
  const uint32_t grid = (uint32_t)((n + kSB - 1) / kSB);
  // Sort a prefix of key64 (shifted down to bits [0, nb)): all slot bits
  // plus enough h1 bits that the prefix space holds >= 32x n values, so
  // equal-prefix runs stay rare (≈3 % of the elements, mostly pairs);
  // k_sort_fixup orders them by the full comparator.  100M keys into a
  // 64 GiB table: 32 bits, 4 radix passes instead of 8.
  const uint32_t sb = slot_bits(geom->ht_size);
  uint32_t lg = 0;
  while (lg < 63 && (1ull << lg) < (uint64_t)n) lg++;
  const int tsb = g_tune_sort_bits.load(std::memory_order_relaxed);
  uint32_t nb = tsb ? sb + (uint32_t)tsb : std::max(sb + 1, lg + 5);
  if (nb > 64) nb = 64;
  // u32 keys halve the key bytes every radix pass moves (16 instead of 24 per
  // element with the index): used when the prefix fits 31 bits -- all slot
  // bits and as many h1 bits as fit (rocPRIM's merge path, taken for small n,
  // builds its mask as (T(1) << end_bit) - 1: undefined at the type's width)
  const bool k32 = !tsb && sb <= 31;
  if (k32) nb = std::min(nb, 31u);
  const uint32_t lo = 64u - nb;
  int cus = 0;
  if ((rc = device_cus(&cus))) return rc;
  // grid-stride, one duplicate-count atomic per workgroup (one element per
  // lane made 390K same-address atomics at 100M keys: 11.5 ms for the whole
  // sort against 7.9; 8 or 32 workgroups per CU measure the same)
  const uint32_t fgrid = (uint32_t)std::min<uint64_t>(grid, (uint64_t)cus * 8);
  const uint32_t lgrid = (uint32_t)cus * 2;  // long runs: one workgroup each, grid-stride
  size_t tb = L.tmp_bytes;
  hipError_t e;
  if (k32) {
    uint32_t* k32in = (uint32_t*)kin;
    uint32_t* k32out = (uint32_t*)kout;
    if (items)
      hipLaunchKernelGGL((k_sort_keys<uint32_t, true>), dim3(grid), dim3(kSB), 0, st, hashes, items, (uint64_t)n, g,
                         sb, lo, k32in, iin, rec, nlong);
    else
      hipLaunchKernelGGL((k_sort_keys<uint32_t, false>), dim3(grid), dim3(kSB), 0, st, hashes, items, (uint64_t)n, g,
                         sb, lo, k32in, iin, rec, nlong);
    if ((rc = launch_done())) return rc;
    e = rocprim::radix_sort_pairs((void*)(s + L.tmp), tb, k32in, k32out, iin, iout, n, 0u, nb, st);
    if (e != hipSuccess) return hip_err(e);
    hipLaunchKernelGGL(k_sort_place, dim3(grid), dim3(kSB), 0, st, hashes, items ? rec : (const Rec*)nullptr, iout,
                       (uint64_t)n, h_out, items_out);
    if ((rc = launch_done())) return rc;
    hipLaunchKernelGGL((k_sort_fixup<uint32_t>), dim3(fgrid), dim3(kSB), 0, st, (const uint32_t*)k32out, (uint64_t)n,
                       h_out, items_out, dedup ? 1u : 0u, (unsigned long long*)dup_count, nlong, runs);
    if ((rc = launch_done())) return rc;
    hipLaunchKernelGGL((k_sort_long<uint32_t>), dim3(lgrid), dim3(kSB), 0, st, (const uint32_t*)k32out, (uint64_t)n,
                       h_out, items_out, rec, dedup ? 1u : 0u, (unsigned long long*)dup_count, nlong, runs);
    return launch_done();
  }
  if (items)
    hipLaunchKernelGGL((k_sort_keys<uint64_t, true>), dim3(grid), dim3(kSB), 0, st, hashes, items, (uint64_t)n, g,
                       sb, lo, kin, iin, rec, nlong);
  else
    hipLaunchKernelGGL((k_sort_keys<uint64_t, false>), dim3(grid), dim3(kSB), 0, st, hashes, items, (uint64_t)n, g,
                       sb, lo, kin, iin, rec, nlong);
  if ((rc = launch_done())) return rc;
  e = rocprim::radix_sort_pairs((void*)(s + L.tmp), tb, kin, kout, iin, iout, n, 0u, 64u - lo, st);
  if (e != hipSuccess) return hip_err(e);
  hipLaunchKernelGGL(k_sort_place, dim3(grid), dim3(kSB), 0, st, hashes, items ? rec : (const Rec*)nullptr, iout,
                     (uint64_t)n, h_out, items_out);
  if ((rc = launch_done())) return rc;
  hipLaunchKernelGGL((k_sort_fixup<uint64_t>), dim3(fgrid), dim3(kSB), 0, st, (const uint64_t*)kout, (uint64_t)n,
                     h_out, items_out, dedup ? 1u : 0u, (unsigned long long*)dup_count, nlong, runs);
  if ((rc = launch_done())) return rc;
  hipLaunchKernelGGL((k_sort_long<uint64_t>), dim3(lgrid), dim3(kSB), 0, st, (const uint64_t*)kout, (uint64_t)n,
                     h_out, items_out, rec, dedup ? 1u : 0u, (unsigned long long*)dup_count, nlong, runs);
  return launch_done();
}

}  // namespace

namespace kvh { namespace rt { std::atomic<int> g_tune_sort_bits{0}; } }

extern "C" {

size_t kvh_ht_sort_scratch_bytes(size_t n) {
  SortLayout L;
  if (sort_layout(n, &L) != 0) return 0;
  return L.total;
}

int kvh_ht_sort(const uint64_t* hashes, const uint64_t* items, size_t n, const kvh_ht_geom_t* geom,
                uint64_t* hashes_out, uint64_t* items_out, uint64_t* dup_count, uint32_t flags, void* scratch,
                size_t scratch_bytes, void* stream) {
  return sort_impl(hashes, items, n, geom, hashes_out, items_out, dup_count, flags, scratch, scratch_bytes,
                   (hipStream_t)stream);
}

int kvh_ht_radix_sort(kvh_ht_sort_t* ar, uint32_t ar_size, const kvh_ht_geom_t* geom) {
  if (!geom) return set_err(KVH_EINVAL);
  if (ar_size <= 1) return set_err(0);
  if (!ar) return set_err(KVH_EINVAL);
  const size_t n = ar_size;
  std::vector<uint64_t> hv(2 * n), iv(n);
  for (size_t i = 0; i < n; i++) {
    hv[2 * i] = ar[i].key;
    hv[2 * i + 1] = ar[i].key2;
    iv[i] = (uint64_t)(uintptr_t)ar[i].item;
  }
  const size_t sb = kvh_ht_sort_scratch_bytes(n);
  if (sb == 0) return set_err(KVH_EINVAL);
  const size_t off_h = 0, off_i = al256(16 * n), off_ho = off_i + al256(8 * n), off_io = off_ho + al256(16 * n),
               off_s = off_io + al256(8 * n), total = off_s + sb;
  uint8_t* d = nullptr;
  hipError_t e = hipMalloc(&d, total);
  if (e != hipSuccess) return hip_err(e);
  int rc = 0;
  do {
    if ((e = hipMemcpy(d + off_h, hv.data(), 16 * n, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_err(e); break; }
    if ((e = hipMemcpy(d + off_i, iv.data(), 8 * n, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_err(e); break; }
    rc = sort_impl((const uint64_t*)(d + off_h), (const uint64_t*)(d + off_i), n, geom, (uint64_t*)(d + off_ho),
                   (uint64_t*)(d + off_io), nullptr, 0, d + off_s, sb, (hipStream_t)0);
    if (rc) break;
    if ((e = hipMemcpy(hv.data(), d + off_ho, 16 * n, hipMemcpyDeviceToHost)) != hipSuccess) { rc = hip_err(e); break; }
    if ((e = hipMemcpy(iv.data(), d + off_io, 8 * n, hipMemcpyDeviceToHost)) != hipSuccess) { rc = hip_err(e); break; }
  } while (0);
  (void)hipFree(d);
  if (rc) return rc;
  for (size_t i = 0; i < n; i++) {
    ar[i].key = hv[2 * i];
    ar[i].key2 = hv[2 * i + 1];
    ar[i].item = (void*)(uintptr_t)iv[i];
  }
  return set_err(0);
}

}  // extern "C"
