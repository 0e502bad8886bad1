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
#include <cmath>
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
// (h1, h2, item) without the input index: the two-pass bucketed path, whose
// tile-stable scatters deliver every bucket in input order, so a record's
// position in its bucket is its tie-break (a quarter less to move per pass)
struct R24 {
  uint64_t h1, h2, item;
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

template <int NT = kSB>
__device__ __forceinline__ uint32_t block_sum(uint32_t d, uint32_t* wsum) {
  for (int o = 32; o >= 1; o >>= 1) d += __shfl_xor(d, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = d;
  __syncthreads();
  uint32_t t = 0;
  for (int w = 0; w < NT / 64; w++) t += wsum[w];
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

// ---------------------------------------------------------------------
// Bucketed path (the default when the batch fits it): slot order without a
// library sort and without the random gather of k_sort_place.
//   B0. k_bk_hist     per 64K-element tile, a histogram of the top B bits of
//                     key64 (B <= 14: ~6K elements per bucket), tile-major
//   B1. k_bk_colsum / k_bk_colscan / k_bk_scan / k_bk_tileoff
//                     column scans of the tile x bucket table -> each tile's
//                     first output position in each bucket
//   B2. k_bk_scatter  (h1, h2, item, index) records to their bucket, ranked
//                     by LDS atomics (a tile's elements of one bucket land
//                     together: ~4 per bucket per tile, 128-byte runs)
//   B3. k_bk_sort     one workgroup per bucket, in LDS: a counting sort on
//                     the next 13 bits of key64, runs of equal bits put in
//                     the full order (key64, h1 << 1, h1, h2, input index) by
//                     insertion sort, then the records gathered into the
//                     outputs with the dedup marks -- the order of the radix
//                     path exactly (the input index is its stable tie-break)
//   B4. k_bk_long     buckets over the LDS capacity or with a run over 64
//                     (non-uniform input) sorted by a bitonic network in
//                     global memory, one workgroup each (as k_sort_long)
constexpr int kBkMaxB = 14;
constexpr uint32_t kBkTile = 65536;  // elements per B0/B2 tile
constexpr uint32_t kBkChunk = 64;    // tiles per column-scan chunk
constexpr uint32_t kBkCap = 12288;   // B3 bucket capacity (LDS)
constexpr int kBkD = 13;             // B3 counting-sort bits
constexpr uint32_t kBkRun = 64;      // B3 longest run of equal bits
constexpr int kBkT = 1024;           // threads per workgroup

__device__ __forceinline__ uint64_t sort_key64(const HtGeom& g, uint32_t sb, uint64_t h1) {
  const uint64_t slot = ht_mod(g, h1);
  return sb >= 64 ? slot : (slot << (64 - sb)) | ((h1 << 1) >> sb);
}
__device__ __forceinline__ uint32_t bk_of(uint64_t k64, uint32_t B) { return B ? (uint32_t)(k64 >> (64 - B)) : 0u; }

// the full order: key64, then (h1 << 1, h1, h2), then the input index
__device__ __forceinline__ bool bk_less(const HtGeom& g, uint32_t sb, const Rec& a, const Rec& b) {
  const uint64_t ka = sort_key64(g, sb, a.h1), kb = sort_key64(g, sb, b.h1);
  if (ka != kb) return ka < kb;
  if (a.h1 != b.h1 || a.h2 != b.h2) return rec_less(a.h1, a.h2, b.h1, b.h2);
  return a.pad < b.pad;
}
// the same for records at bucket positions ia, ib: a Rec carries its input
// index; an R24 bucket is in input order, so the position stands in for it
__device__ __forceinline__ bool bk_less_at(const HtGeom& g, uint32_t sb, const Rec& a, const Rec& b, uint32_t,
                                           uint32_t) {
  return bk_less(g, sb, a, b);
}
__device__ __forceinline__ bool bk_less_at(const HtGeom& g, uint32_t sb, const R24& a, const R24& b, uint32_t ia,
                                           uint32_t ib) {
  const uint64_t ka = sort_key64(g, sb, a.h1), kb = sort_key64(g, sb, b.h1);
  if (ka != kb) return ka < kb;
  if (a.h1 != b.h1 || a.h2 != b.h2) return rec_less(a.h1, a.h2, b.h1, b.h2);
  return ia < ib;
}

// Tile of workgroup `bid` in a grid of G: the tiles of each XCD consecutive.
// Workgroups are dispatched to the 8 XCDs round-robin (bid % 8, speed only:
// correctness never depends on it), and each XCD has its own L2.  With tile
// = bid, neighbouring tiles ran on different XCDs, so the 128-byte lines
// where one tile's run of a bucket ends and the next tile's begins were
// written back partially from two L2s (k_tw_scatter2 wrote 6.4 GB for 3.2 GB
// of records); here XCD x takes tiles [x q + min(x, r), ...), q = G / 8,
// r = G % 8 -- a bijection on [0, G).
__device__ __forceinline__ uint32_t xcd_tile(uint32_t bid, uint32_t G) {
  const uint32_t q = G >> 3, r = G & 7u, x = bid & 7u, k = bid >> 3;
  return x * q + (x < r ? x : r) + k;
}

__global__ void __launch_bounds__(kBkT)
k_bk_hist(const uint64_t* __restrict__ h, uint64_t n, HtGeom g, uint32_t sb, uint32_t B, uint32_t* __restrict__ H,
          uint32_t* __restrict__ novf) {
  __shared__ uint32_t hist[1u << kBkMaxB];
  const uint32_t nb = 1u << B, tile = blockIdx.x;
  if (tile == 0 && threadIdx.x == 0) *novf = 0;  // B3's overflow list, empty per call
  for (uint32_t b = threadIdx.x; b < nb; b += kBkT) hist[b] = 0;
  __syncthreads();
  const uint64_t i0 = (uint64_t)tile * kBkTile;
  for (uint32_t t = threadIdx.x; t < kBkTile; t += kBkT) {
    const uint64_t i = i0 + t;
    if (i < n) atomicAdd(&hist[bk_of(sort_key64(g, sb, h[2 * i]), B)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += kBkT) H[(uint64_t)tile * nb + b] = hist[b];
}

// S[c][b] = sum of H[t][b] over the tiles t of chunk c
__global__ void __launch_bounds__(256)
k_bk_colsum(const uint32_t* __restrict__ H, uint32_t ntiles, uint32_t nb, uint32_t* __restrict__ S) {
  const uint64_t x = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t nch = (ntiles + kBkChunk - 1) / kBkChunk;
  if (x >= (uint64_t)nch * nb) return;
  const uint32_t c = (uint32_t)(x / nb), b = (uint32_t)(x % nb);
  const uint32_t t1 = min(ntiles, (c + 1) * kBkChunk);
  uint32_t s = 0;
  for (uint32_t t = c * kBkChunk; t < t1; t++) s += H[(uint64_t)t * nb + b];
  S[x] = s;
}

// per bucket: S[c][b] -> exclusive prefix over chunks, cnt[b] = the total
__global__ void __launch_bounds__(256)
k_bk_colscan(uint32_t* __restrict__ S, uint32_t nch, uint32_t nb, uint32_t* __restrict__ cnt) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nb) return;
  uint32_t run = 0;
  for (uint32_t c = 0; c < nch; c++) {
    const uint32_t v = S[(uint64_t)c * nb + b];
    S[(uint64_t)c * nb + b] = run;
    run += v;
  }
  cnt[b] = run;
}

// exclusive scan of the bucket sizes (nb <= 16384, one workgroup)
__global__ void __launch_bounds__(kBkT)
k_bk_scan(const uint32_t* __restrict__ cnt, uint32_t nb, uint32_t* __restrict__ start) {
  __shared__ uint32_t wsum[kBkT / 64];
  constexpr uint32_t per = (1u << kBkMaxB) / kBkT;  // 16 buckets per thread
  uint32_t v[per], s = 0;
#pragma unroll
  for (uint32_t j = 0; j < per; j++) {
    const uint32_t b = threadIdx.x * per + j;
    v[j] = b < nb ? cnt[b] : 0u;
    s += v[j];
  }
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t wo = 0;
  for (uint32_t q = 0; q < w; q++) wo += wsum[q];
  uint32_t run = wo + inc - s;
#pragma unroll
  for (uint32_t j = 0; j < per; j++) {
    const uint32_t b = threadIdx.x * per + j;
    if (b < nb) start[b] = run;
    run += v[j];
  }
}

// H[t][b] -> the absolute output position of tile t's first element of bucket b
__global__ void __launch_bounds__(256)
k_bk_tileoff(uint32_t* __restrict__ H, const uint32_t* __restrict__ S, const uint32_t* __restrict__ start,
             uint32_t ntiles, uint32_t nb) {
  const uint64_t x = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t nch = (ntiles + kBkChunk - 1) / kBkChunk;
  if (x >= (uint64_t)nch * nb) return;
  const uint32_t c = (uint32_t)(x / nb), b = (uint32_t)(x % nb);
  const uint32_t t1 = min(ntiles, (c + 1) * kBkChunk);
  uint32_t run = start[b] + S[x];
  for (uint32_t t = c * kBkChunk; t < t1; t++) {
    const uint32_t v = H[(uint64_t)t * nb + b];
    H[(uint64_t)t * nb + b] = run;
    run += v;
  }
}

__global__ void __launch_bounds__(kBkT)
k_bk_scatter(const uint64_t* __restrict__ h, const uint64_t* __restrict__ items, uint64_t n, HtGeom g, uint32_t sb,
             uint32_t B, const uint32_t* __restrict__ H, Rec* __restrict__ recs) {
  __shared__ uint32_t pos[1u << kBkMaxB];
  const uint32_t nb = 1u << B, tile = xcd_tile(blockIdx.x, gridDim.x);
  for (uint32_t b = threadIdx.x; b < nb; b += kBkT) pos[b] = H[(uint64_t)tile * nb + b];
  __syncthreads();
  const uint64_t i0 = (uint64_t)tile * kBkTile;
  for (uint32_t t = threadIdx.x; t < kBkTile; t += kBkT) {
    const uint64_t i = i0 + t;
    if (i >= n) break;
    Rec r;
    r.h1 = h[2 * i];
    r.h2 = h[2 * i + 1];
    r.item = items ? items[i] : i;
    r.pad = i;
    recs[atomicAdd(&pos[bk_of(sort_key64(g, sb, r.h1), B)], 1u)] = r;
  }
}

// outputs for sorted position p of a bucket whose record for p is r, next
// the record at p + 1 (when has_next): dedup marks as ctest.c:96-104
template <class RT>
__device__ __forceinline__ uint32_t bk_emit(uint64_t j, const RT& r, bool has_next, uint64_t n1, uint64_t n2,
                                            uint32_t dedup, uint64_t* __restrict__ h_out,
                                            uint64_t* __restrict__ items_out) {
  const bool dup = dedup && has_next && r.h1 == n1 && r.h2 == n2;
  h_out[2 * j] = dup ? 0 : r.h1;
  h_out[2 * j + 1] = r.h2;
  if (items_out) items_out[j] = r.item;
  return dup ? 1u : 0u;
}

// CAP / D: bucket capacity and counting-sort bits.  <12288, 13> needs
// 128 KiB of LDS (one workgroup per CU); <8000, 12> fits two per CU (78.6
// KiB), so one workgroup's loads overlap the other's LDS phases -- used when
// the mean bucket leaves the largest far below 8000.
template <uint32_t CAP, int D, class RT = Rec>
__global__ void __launch_bounds__(kBkT, CAP <= 8192 ? 8 : 1)
k_bk_sort(const RT* __restrict__ recs, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ start,
          uint32_t nb, uint32_t B, HtGeom g, uint32_t sb, uint64_t* __restrict__ h_out,
          uint64_t* __restrict__ items_out, uint32_t dedup, unsigned long long* __restrict__ dups,
          uint32_t* __restrict__ novf, uint32_t* __restrict__ ovf) {
  constexpr uint32_t kBkCap = CAP;
  constexpr int kBkD = D;
  __shared__ uint32_t K[kBkCap];         // key64 bits [B, B + 32) of each record
  __shared__ uint16_t dig[kBkCap];       // its top kBkD bits
  __shared__ uint16_t ord[kBkCap];       // sorted position -> record
  __shared__ uint32_t hist[1u << kBkD];  // digit counts -> starts -> ends
  __shared__ uint32_t wsum[kBkT / 64], wmax[kBkT / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr uint32_t nd = 1u << kBkD, per = nd / kBkT;  // 4-8 digits per thread
  uint32_t d_total = 0;
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t R = cnt[b], base = start[b];
    if (R == 0) continue;
    if (R > kBkCap) {
      if (tid == 0) ovf[atomicAdd(novf, 1u)] = b;
      continue;
    }
    const RT* rb = recs + base;
#pragma unroll
    for (uint32_t j = 0; j < per; j++) hist[tid * per + j] = 0;
    __syncthreads();
    for (uint32_t t = tid; t < R; t += kBkT) {
      const uint32_t k32 = (uint32_t)((sort_key64(g, sb, rb[t].h1) << B) >> 32);
      K[t] = k32;
      dig[t] = (uint16_t)(k32 >> (32 - kBkD));
      atomicAdd(&hist[k32 >> (32 - kBkD)], 1u);
    }
    __syncthreads();
    {  // exclusive scan of the digit counts, and the longest run
      uint32_t v[per], s = 0, mx = 0;
#pragma unroll
      for (uint32_t j = 0; j < per; j++) { v[j] = hist[tid * per + j]; s += v[j]; mx = max(mx, v[j]); }
      uint32_t inc = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
      if (lane == 63) wsum[w] = inc;
      if (lane == 0) wmax[w] = mx;
      __syncthreads();
      uint32_t wo = 0, bm = 0;
      for (uint32_t q = 0; q < kBkT / 64; q++) {
        if (q < w) wo += wsum[q];
        bm = max(bm, wmax[q]);
      }
      if (bm > kBkRun) {  // a run too long for insertion sort: the bitonic path
        if (tid == 0) ovf[atomicAdd(novf, 1u)] = b;
        __syncthreads();
        continue;
      }
      uint32_t run = wo + inc - s;
#pragma unroll
      for (uint32_t j = 0; j < per; j++) { hist[tid * per + j] = run; run += v[j]; }
    }
    __syncthreads();
    for (uint32_t t = tid; t < R; t += kBkT) ord[atomicAdd(&hist[dig[t]], 1u)] = (uint16_t)t;
    __syncthreads();
    // runs of equal digit (hist[d] is now the end of digit d): full order
#pragma unroll
    for (uint32_t j = 0; j < per; j++) {
      const uint32_t d = tid * per + j;
      const uint32_t e = hist[d], s0 = d ? hist[d - 1] : 0u;
      for (uint32_t a = s0 + 1; a < e; a++) {
        const uint16_t x = ord[a];
        const uint32_t kx = K[x];
        uint32_t c = a;
        while (c > s0) {
          const uint16_t y = ord[c - 1];
          const uint32_t ky = K[y];
          const bool lt = kx != ky ? kx < ky : bk_less_at(g, sb, rb[x], rb[y], x, y);
          if (!lt) break;
          ord[c] = y;
          c--;
        }
        ord[c] = x;
      }
    }
    __syncthreads();
    for (uint32_t p0 = 0; p0 < R; p0 += kBkT) {
      const uint32_t p = p0 + tid;
      RT r;
      if (p < R) r = rb[ord[p]];
      // the successor's pair: the next lane's record, or a load at a wave's edge
      uint64_t n1 = (uint64_t)__shfl_down((unsigned long long)r.h1, 1, 64),
               n2 = (uint64_t)__shfl_down((unsigned long long)r.h2, 1, 64);
      const bool has_next = p + 1 < R;
      if (lane == 63 && has_next) {
        const RT& q = rb[ord[p + 1]];
        n1 = q.h1;
        n2 = q.h2;
      }
      if (p < R) d_total += bk_emit((uint64_t)base + p, r, has_next, n1, n2, dedup, h_out, items_out);
    }
    __syncthreads();
  }
  if (dedup && dups) {
    const uint32_t t = block_sum<kBkT>(d_total, wsum);
    if (tid == 0 && t) atomicAdd(dups, (unsigned long long)t);
  }
}

// B3r (round 4): k_bk_sort's order and marks, with the bucket's records
// read ONCE and kept in registers.  k_bk_sort reads each record twice -- its
// key field first, the whole record in sorted order at the end -- and that
// final gather misses L2 (≈9 MB of buckets in flight per XCD against 4 MB:
// FETCH 4.0 GB raw for 2.4 GB of records).  Here thread t owns records
// t, t + 1024, ... (their three words in 3 x PER registers: the three loads
// of a record slot fetch the same lines, so every byte a line brings is
// used), files their sort keys, the LDS counting sort runs as in k_bk_sort,
// and the records leave in three rounds, one field per round: the owners
// write the field into LDS (aliasing the sort arrays), each thread reads it
// for its sorted positions and stores it coalesced.  The duplicate test takes
// the successor's field from the same LDS round.  Runs of equal digit still
// compare ties through global memory (rare, and those lines are L2-hot).
// (Its barriers do not wait for global accesses on gfx950 -- workgroup scope
// orders LDS only, s_waitcnt lgkmcnt -- so a bucket's output stores already
// drain under the next bucket's phases.  Touching the next bucket's lines at
// the start of this one's LDS phases, so its loads would hit L2 / MALL, was
// 4 % slower: profiles/r04/s12/; so was taking the buckets in address
// order from a ticket counter, 2 %: s19/.)
// W2 (round 5): h1 and h2 leave in ONE field round (16-byte LDS records, one
// random ds_read_b128 per record and a 16-byte output store) and the item in
// a second, instead of three 8-byte rounds: two barriers and one ord[] read
// fewer per record.  The union then holds 56 KiB, 63 KiB per workgroup.
// RK (round 5): the histogram atomic returns each record's rank within its
// digit, kept in a register, so the records are placed with one read of the
// digit's start: no digit array and no second (returning) atomic pass --
// two LDS accesses and one random atomic fewer per record.  hist[] then
// holds the starts, and a run ends at the next digit's start.
// AB (experiments build, knob 23 = 7-10: phase ablations, outputs not sorted):
// 1 no run insertion sort, 2 no output field rounds (linear stores of the
// loaded records), 3 no counting sort (ord = identity), 4 no record loads
// (records made from their index).
template <uint32_t CAP, int D, int T = kBkT, bool W2 = false, bool RK = false, int AB = 0>
__global__ void __launch_bounds__(T, 4)  // 4 waves per SIMD (512 threads x 2 per CU spill: 87 VGPRs)
k_bk_sortr(const R24* __restrict__ recs, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ start,
           uint32_t nb, uint32_t B, HtGeom g, uint32_t sb, uint64_t* __restrict__ h_out,
           uint64_t* __restrict__ items_out, uint32_t dedup, unsigned long long* __restrict__ dups,
           uint32_t* __restrict__ novf, uint32_t* __restrict__ ovf) {
  static_assert(CAP % T == 0, "records per thread");
  constexpr uint32_t PER = CAP / T;
  constexpr uint32_t nd = 1u << D, per = nd / T;
  struct SortArrays {
    uint32_t K[CAP];       // key64 bits [B, B + 32) of each record
    uint16_t dig[CAP];     // its top D bits
    uint32_t hist[nd];     // digit counts -> starts -> ends
  };
  union Lds {
    SortArrays s;
    uint64_t X[CAP];  // one field of every record, in record order
    ulonglong2 X2[W2 ? CAP : 1];  // W2: h1 and h2 of every record
  };
  __shared__ Lds u;
  __shared__ uint16_t ord[CAP];  // sorted position -> record
  __shared__ uint32_t wsum[T / 64], wmax[T / 64];
  uint32_t* K = u.s.K;
  uint16_t* dig = u.s.dig;
  uint32_t* hist = u.s.hist;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t d_total = 0;
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t R = cnt[b], base = start[b];
    if (R == 0) continue;
    if (R > CAP) {
      if (tid == 0) ovf[atomicAdd(novf, 1u)] = b;
      continue;
    }
    const R24* rb = recs + base;
    uint64_t f0[PER], f1[PER], f2[PER];  // h1, h2, item of records tid + j * T
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t r = tid + j * T;
      f0[j] = f1[j] = f2[j] = 0;
      if (r < R) {  // non-temporal: read once, and they must not push the outputs out of L2
        if constexpr (AB == 4) {
          const uint64_t x = (uint64_t)(base + r) * 0x9E3779B97F4A7C15ull;
          f0[j] = x; f1[j] = x ^ 0x5555; f2[j] = base + r;
        } else {
          const uint64_t* q = (const uint64_t*)(rb + r);
          f0[j] = __builtin_nontemporal_load(q);
          f1[j] = __builtin_nontemporal_load(q + 1);
          f2[j] = __builtin_nontemporal_load(q + 2);
        }
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < per; j++) hist[tid * per + j] = 0;
    __syncthreads();
    uint32_t rk[RK ? PER : 1];  // RK: digit << 16 | rank within the digit
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t r = tid + j * T;
      if (r < R) {
        const uint32_t k32 = (uint32_t)((sort_key64(g, sb, f0[j]) << B) >> 32);
        K[r] = k32;
        if constexpr (RK) {
          rk[j] = (k32 >> (32 - D)) << 16 | atomicAdd(&hist[k32 >> (32 - D)], 1u);
        } else {
          dig[r] = (uint16_t)(k32 >> (32 - D));
          atomicAdd(&hist[k32 >> (32 - D)], 1u);
        }
      }
    }
    __syncthreads();
    {  // exclusive scan of the digit counts, and the longest run
      uint32_t v[per], s = 0, mx = 0;
#pragma unroll
      for (uint32_t j = 0; j < per; j++) { v[j] = hist[tid * per + j]; s += v[j]; mx = max(mx, v[j]); }
      uint32_t inc = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
      if (lane == 63) wsum[w] = inc;
      if (lane == 0) wmax[w] = mx;
      __syncthreads();
      uint32_t wo = 0, bm = 0;
      for (uint32_t q = 0; q < T / 64; q++) {
        if (q < w) wo += wsum[q];
        bm = max(bm, wmax[q]);
      }
      if (bm > kBkRun) {  // a run too long for insertion sort: the bitonic path
        if (tid == 0) ovf[atomicAdd(novf, 1u)] = b;
        __syncthreads();
        continue;
      }
      uint32_t run = wo + inc - s;
#pragma unroll
      for (uint32_t j = 0; j < per; j++) { hist[tid * per + j] = run; run += v[j]; }
    }
    __syncthreads();
    if constexpr (AB == 3) {
      for (uint32_t t = tid; t < R; t += T) ord[t] = (uint16_t)t;
    } else if constexpr (RK) {
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t r = tid + j * T;
        if (r < R) ord[hist[rk[j] >> 16] + (rk[j] & 0xffffu)] = (uint16_t)r;
      }
    } else {
      for (uint32_t t = tid; t < R; t += T) ord[atomicAdd(&hist[dig[t]], 1u)] = (uint16_t)t;
    }
    __syncthreads();
    // runs of equal digit (RK: hist[d] is the start of digit d, else its end): full order
#pragma unroll
    for (uint32_t j = 0; j < (AB == 1 || AB == 3 ? 0u : per); j++) {
      const uint32_t d = tid * per + j;
      const uint32_t e = RK ? (d + 1 < nd ? hist[d + 1] : R) : hist[d];
      const uint32_t s0 = RK ? hist[d] : d ? hist[d - 1] : 0u;
      for (uint32_t a = s0 + 1; a < e; a++) {
        const uint16_t x = ord[a];
        const uint32_t kx = K[x];
        uint32_t c = a;
        while (c > s0) {
          const uint16_t y = ord[c - 1];
          const uint32_t ky = K[y];
          const bool lt = kx != ky ? kx < ky : bk_less_at(g, sb, rb[x], rb[y], x, y);
          if (!lt) break;
          ord[c] = y;
          c--;
        }
        ord[c] = x;
      }
    }
    __syncthreads();  // ord final; the sort arrays are free for the field rounds
    if constexpr (AB == 2) {  // linear stores of the loaded records, no LDS rounds
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t p = tid + j * T;
        if (p < R) {
          *(ulonglong2*)(h_out + 2 * ((uint64_t)base + p)) = make_ulonglong2(f0[j], f1[j]);
          if (items_out) items_out[(uint64_t)base + p] = f2[j];
        }
      }
      __syncthreads();
      continue;
    }
    if constexpr (W2) {
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t r = tid + j * T;
        if (r < R) u.X2[r] = make_ulonglong2(f0[j], f1[j]);
      }
      __syncthreads();
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t p = tid + j * T;
        ulonglong2 v = make_ulonglong2(0ull, 0ull);
        if (p < R) v = u.X2[ord[p]];
        // the successor's pair: the next lane's, a gather only at a wave's last lane
        uint64_t n1 = (uint64_t)__shfl_down((unsigned long long)v.x, 1, 64),
                 n2 = (uint64_t)__shfl_down((unsigned long long)v.y, 1, 64);
        if (lane == 63 && dedup && p + 1 < R) {
          const ulonglong2 w = u.X2[ord[p + 1]];
          n1 = w.x;
          n2 = w.y;
        }
        if (p < R) {
          const bool dup = dedup && p + 1 < R && n1 == v.x && n2 == v.y;
          d_total += dup ? 1u : 0u;
          *(ulonglong2*)(h_out + 2 * ((uint64_t)base + p)) = make_ulonglong2(dup ? 0ull : v.x, v.y);
        }
      }
      __syncthreads();
      if (items_out) {
#pragma unroll
        for (uint32_t j = 0; j < PER; j++) {
          const uint32_t r = tid + j * T;
          if (r < R) u.X[r] = f2[j];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < PER; j++) {
          const uint32_t p = tid + j * T;
          if (p < R) items_out[(uint64_t)base + p] = u.X[ord[p]];
        }
        __syncthreads();
      }
      continue;
    }
    uint64_t h1v[PER];
    uint32_t eq1 = 0;  // bit j: sorted position tid + j * T has the same h1 as its successor
#pragma unroll
    for (uint32_t f = 0; f < 3; f++) {
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t r = tid + j * T;
        if (r < R) u.X[r] = f == 0 ? f0[j] : f == 1 ? f1[j] : f2[j];
      }
      __syncthreads();
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t p = tid + j * T;
        const uint64_t v = p < R ? u.X[ord[p]] : 0ull;
        // the successor's field: the next lane's (one random LDS gather per
        // record instead of two), a gather only at a wave's last lane
        uint64_t nv = (uint64_t)__shfl_down((unsigned long long)v, 1, 64);
        if (lane == 63 && f < 2 && dedup && p + 1 < R) nv = u.X[ord[p + 1]];
        if (p < R) {
          const bool eq = f < 2 && dedup && p + 1 < R && nv == v;
          if (f == 0) {
            h1v[j] = v;
            eq1 |= (eq ? 1u : 0u) << j;
          } else if (f == 1) {
            const bool dup = eq && ((eq1 >> j) & 1u);
            d_total += dup ? 1u : 0u;
            uint64_t* o = h_out + 2 * ((uint64_t)base + p);
            o[0] = dup ? 0ull : h1v[j];
            o[1] = v;
          } else if (items_out) {
            items_out[(uint64_t)base + p] = v;
          }
        }
      }
      __syncthreads();
    }
  }
  if (dedup && dups) {
    const uint32_t t = block_sum<T>(d_total, wsum);
    if (tid == 0 && t) atomicAdd(dups, (unsigned long long)t);
  }
}

// B3x (round 5): k_bk_sortr with every record's (h1, h2) in LDS from the
// start.  The phase ablations (profiles/r05/s21/) put 0.74 of the bucket
// sort's 1.73 ms in its run insertion sort (per-thread chains of dependent
// LDS reads over a wave's longest runs, and ties of the 32 key bits -- f2's
// 1 % duplicate pairs -- through global loads).  Here each record ranks
// itself in its run with independent comparisons against the pairs in LDS
// (the 64-bit key recomputed from h1: a multiply), so nothing is chained
// and no tie leaves the CU.  The 32-bit key array is gone (the
// pairs replace it) and the rank comes from the histogram atomic (RK), so
// the LDS is 56 KiB of pairs + 8 KiB of counts + 7 KiB of ranks: two
// workgroups per CU as before.  The h1/h2 output round reads the pairs
// already there; the items round reuses their space.
// AB (experiments build, knob 23 = 12-15: phase ablations, outputs not
// sorted): 1 no run ranking, 2 no output rounds (the records stored back
// linearly), 3 no counting sort and no ranking (identity order), 4 no record
// loads (records made from their index).
template <uint32_t CAP, int D, int T = 512, int AB = 0>
__global__ void __launch_bounds__(T, 4)
k_bk_sortx(const R24* __restrict__ recs, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ start,
           uint32_t nb, uint32_t B, HtGeom g, uint32_t sb, uint64_t* __restrict__ h_out,
           uint64_t* __restrict__ items_out, uint32_t dedup, unsigned long long* __restrict__ dups,
           uint32_t* __restrict__ novf, uint32_t* __restrict__ ovf) {
  static_assert(CAP % T == 0, "records per thread");
  constexpr uint32_t PER = CAP / T;
  constexpr uint32_t nd = 1u << D, per = nd / T;
  union Pairs {
    ulonglong2 X2[CAP];  // (h1, h2) of every record, in record order
    uint64_t X[CAP];     // then the items, for their output round
  };
  __shared__ Pairs u;
  __shared__ uint32_t hist[nd];   // digit counts -> starts
  __shared__ uint16_t ord[CAP];   // sorted position -> record
  __shared__ uint32_t wsum[T / 64], wmax[T / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t d_total = 0;
  // the full order on records in LDS: key64, then (h1 << 1, h1, h2), then the position
  auto less_at = [&](uint32_t x, uint32_t y) {
    const ulonglong2 a = u.X2[x], b = u.X2[y];
    const uint64_t ka = sort_key64(g, sb, a.x), kb = sort_key64(g, sb, b.x);
    if (ka != kb) return ka < kb;
    if (a.x != b.x || a.y != b.y) return rec_less(a.x, a.y, b.x, b.y);
    return x < y;
  };
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t R = cnt[b], base = start[b];
    if (R == 0) continue;
    if (R > CAP) {
      if (tid == 0) ovf[atomicAdd(novf, 1u)] = b;
      continue;
    }
    const R24* rb = recs + base;
    uint64_t f2[PER];  // items stay in registers until their round
    uint32_t rk[PER];  // digit << 16 | rank within the digit
#pragma unroll
    for (uint32_t j = 0; j < per; j++) hist[tid * per + j] = 0;
    __syncthreads();
    // every record load of the bucket in flight before the first use (clamped
    // indices, not a branch per record: a branch made each of the PER loads
    // its own memory round trip)
    uint64_t la[PER], lb[PER];
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t r = tid + j * T, rc = r < R ? r : R - 1;
      if constexpr (AB == 4) {
        la[j] = (uint64_t)(base + r) * 0x9E3779B97F4A7C15ull;
        lb[j] = la[j] ^ 0x5555;
        f2[j] = base + r;
      } else {  // non-temporal: read once, and they must not push the outputs out of L2
        const uint64_t* q = (const uint64_t*)(rb + rc);
        la[j] = __builtin_nontemporal_load(q);
        lb[j] = __builtin_nontemporal_load(q + 1);
        f2[j] = __builtin_nontemporal_load(q + 2);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t r = tid + j * T;
      // stored on every lane (r < CAP; slots past R are never read), so the
      // compiler cannot sink a load into the branch below
      u.X2[r] = make_ulonglong2(la[j], lb[j]);
      if (r < R) {
        const uint64_t h1 = la[j];
        const uint32_t k32 = (uint32_t)((sort_key64(g, sb, h1) << B) >> 32);
        rk[j] = (k32 >> (32 - D)) << 16 | atomicAdd(&hist[k32 >> (32 - D)], 1u);
      }
    }
    __syncthreads();
    {  // exclusive scan of the digit counts, and the longest run
      uint32_t v[per], s = 0, mx = 0;
#pragma unroll
      for (uint32_t j = 0; j < per; j++) { v[j] = hist[tid * per + j]; s += v[j]; mx = max(mx, v[j]); }
      uint32_t inc = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
      if (lane == 63) wsum[w] = inc;
      if (lane == 0) wmax[w] = mx;
      __syncthreads();
      uint32_t wo = 0, bm = 0;
      for (uint32_t q = 0; q < T / 64; q++) {
        if (q < w) wo += wsum[q];
        bm = max(bm, wmax[q]);
      }
      if (bm > kBkRun) {  // a run too long for insertion sort: the bitonic path
        if (tid == 0) ovf[atomicAdd(novf, 1u)] = b;
        __syncthreads();
        continue;
      }
      uint32_t run = wo + inc - s;
#pragma unroll
      for (uint32_t j = 0; j < per; j++) { hist[tid * per + j] = run; run += v[j]; }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t r = tid + j * T;
      if (r < R) ord[AB == 3 ? r : hist[rk[j] >> 16] + (rk[j] & 0xffffu)] = (uint16_t)r;
    }
    __syncthreads();
    if constexpr (AB != 1 && AB != 3) {
    // Runs of equal digit (hist[d] is the start of digit d), in the full
    // order: each record counts the members of its run that precede it --
    // independent LDS reads, no per-thread insertion chain -- and takes that
    // rank as its place (the order is total: ranks are distinct).
    uint32_t pos[PER];
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t r = tid + j * T;
      pos[j] = 0;
      if (r < R) {
        const uint32_t d = rk[j] >> 16, s0 = hist[d], e = d + 1 < nd ? hist[d + 1] : R;
        uint32_t rank = 0;
        if (e - s0 > 1) {
          const ulonglong2 me = u.X2[r];
          const uint64_t km = sort_key64(g, sb, me.x);
          for (uint32_t a = s0; a < e; a++) {
            const uint32_t y = ord[a];
            const ulonglong2 o = u.X2[y];
            const uint64_t ko = sort_key64(g, sb, o.x);
            const bool lt = ko != km ? ko < km
                                     : (o.x != me.x || o.y != me.y) ? rec_less(o.x, o.y, me.x, me.y) : y < r;
            rank += (y != r && lt) ? 1u : 0u;
          }
        }
        pos[j] = s0 + rank;
      }
    }
    __syncthreads();  // every run read before any place is written
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t r = tid + j * T;
      if (r < R) ord[pos[j]] = (uint16_t)r;
    }
    __syncthreads();
    }  // AB
    if constexpr (AB == 2) {  // linear stores of the records, no output rounds
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t p = tid + j * T;
        if (p < R) {
          *(ulonglong2*)(h_out + 2 * ((uint64_t)base + p)) = u.X2[p];
          if (items_out) items_out[(uint64_t)base + p] = f2[j];
        }
      }
      __syncthreads();
      continue;
    }
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {  // h1, h2 out, from the pairs already in LDS
      const uint32_t p = tid + j * T;
      ulonglong2 v = make_ulonglong2(0ull, 0ull);
      if (p < R) v = u.X2[ord[p]];
      // the successor's pair: the next lane's, a gather only at a wave's last lane
      uint64_t n1 = (uint64_t)__shfl_down((unsigned long long)v.x, 1, 64),
               n2 = (uint64_t)__shfl_down((unsigned long long)v.y, 1, 64);
      if (lane == 63 && dedup && p + 1 < R) {
        const ulonglong2 nx = u.X2[ord[p + 1]];
        n1 = nx.x;
        n2 = nx.y;
      }
      if (p < R) {
        const bool dup = dedup && p + 1 < R && n1 == v.x && n2 == v.y;
        d_total += dup ? 1u : 0u;
        *(ulonglong2*)(h_out + 2 * ((uint64_t)base + p)) = make_ulonglong2(dup ? 0ull : v.x, v.y);
      }
    }
    __syncthreads();
    if (items_out) {
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t r = tid + j * T;
        if (r < R) u.X[r] = f2[j];
      }
      __syncthreads();
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t p = tid + j * T;
        if (p < R) items_out[(uint64_t)base + p] = u.X[ord[p]];
      }
      __syncthreads();
    }
  }
  if (dedup && dups) {
    const uint32_t t = block_sum<T>(d_total, wsum);
    if (tid == 0 && t) atomicAdd(dups, (unsigned long long)t);
  }
}

// B3r2: k_bk_sortr at two workgroups per CU, so one workgroup's loads run
// under the other's LDS phases (k_bk_sortr at one per CU serialises them:
// 1.75 ms, no better than k_bk_sort's re-fetching gather).  To fit two
// 1024-thread workgroups (≤ 64 VGPRs, ≤ 80 KiB of LDS each) the h1 words go
// straight into the LDS field array X, where the sort reads them (its key
// and digit recomputed from h1 instead of kept: ht_mod is a multiply and a
// shift), D = 11 digit bits (8 KiB of counts), and only h2 and the item
// stay in registers until their rounds.
template <uint32_t CAP, int D>
__global__ void __launch_bounds__(kBkT, 8)  // 8 waves per SIMD: two 1024-thread workgroups per CU
k_bk_sortr2(const R24* __restrict__ recs, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ start,
            uint32_t nb, uint32_t B, HtGeom g, uint32_t sb, uint64_t* __restrict__ h_out,
            uint64_t* __restrict__ items_out, uint32_t dedup, unsigned long long* __restrict__ dups,
            uint32_t* __restrict__ novf, uint32_t* __restrict__ ovf) {
  static_assert(CAP % kBkT == 0, "records per thread");
  constexpr uint32_t PER = CAP / kBkT;
  constexpr uint32_t nd = 1u << D, per = nd / kBkT;
  __shared__ uint64_t X[CAP];      // h1 of every record (the sort's input), then h2, then the item
  __shared__ uint32_t hist[nd];    // digit counts -> starts -> ends
  __shared__ uint16_t ord[CAP];    // sorted position -> record
  __shared__ uint32_t wsum[kBkT / 64], wmax[kBkT / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  auto k32_of = [&](uint64_t h1) { return (uint32_t)((sort_key64(g, sb, h1) << B) >> 32); };
  uint32_t d_total = 0;
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t R = cnt[b], base = start[b];
    if (R == 0) continue;
    if (R > CAP) {
      if (tid == 0) ovf[atomicAdd(novf, 1u)] = b;
      continue;
    }
    const R24* rb = recs + base;
    // the thread index laundered per bucket: otherwise the compiler hoists
    // every per-slot address out of the bucket loop and spills them
    uint32_t tl = tid;
    asm volatile("" : "+v"(tl));
    uint64_t f1[PER], f2[PER];  // h2 and item of records tid + j * kBkT
#pragma unroll
    for (uint32_t j = 0; j < per; j++) hist[tid * per + j] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t r = tl + j * kBkT;
      f1[j] = f2[j] = 0;
      if (r < R) {  // non-temporal: the record lines are not reused (and must not evict the outputs)
        const uint64_t* q = (const uint64_t*)(rb + r);
        const uint64_t h1 = __builtin_nontemporal_load(q);
        f1[j] = __builtin_nontemporal_load(q + 1);
        f2[j] = __builtin_nontemporal_load(q + 2);
        X[r] = h1;
        atomicAdd(&hist[k32_of(h1) >> (32 - D)], 1u);
      }
    }
    __syncthreads();
    {  // exclusive scan of the digit counts, and the longest run
      uint32_t v[per], s = 0, mx = 0;
#pragma unroll
      for (uint32_t j = 0; j < per; j++) { v[j] = hist[tid * per + j]; s += v[j]; mx = max(mx, v[j]); }
      uint32_t inc = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
      if (lane == 63) wsum[w] = inc;
      if (lane == 0) wmax[w] = mx;
      __syncthreads();
      uint32_t wo = 0, bm = 0;
      for (uint32_t q = 0; q < kBkT / 64; q++) {
        if (q < w) wo += wsum[q];
        bm = max(bm, wmax[q]);
      }
      if (bm > kBkRun) {  // a run too long for insertion sort: the bitonic path
        if (tid == 0) ovf[atomicAdd(novf, 1u)] = b;
        __syncthreads();
        continue;
      }
      uint32_t run = wo + inc - s;
#pragma unroll
      for (uint32_t j = 0; j < per; j++) { hist[tid * per + j] = run; run += v[j]; }
    }
    __syncthreads();
    for (uint32_t t = tid; t < R; t += kBkT) ord[atomicAdd(&hist[k32_of(X[t]) >> (32 - D)], 1u)] = (uint16_t)t;
    __syncthreads();
    // runs of equal digit (hist[d] is now the end of digit d): full order
#pragma unroll
    for (uint32_t j = 0; j < per; j++) {
      const uint32_t d = tid * per + j;
      const uint32_t e = hist[d], s0 = d ? hist[d - 1] : 0u;
      for (uint32_t a = s0 + 1; a < e; a++) {
        const uint16_t x = ord[a];
        const uint32_t kx = k32_of(X[x]);
        uint32_t c = a;
        while (c > s0) {
          const uint16_t y = ord[c - 1];
          const uint32_t ky = k32_of(X[y]);
          const bool lt = kx != ky ? kx < ky : bk_less_at(g, sb, rb[x], rb[y], x, y);
          if (!lt) break;
          ord[c] = y;
          c--;
        }
        ord[c] = x;
      }
    }
    __syncthreads();
    // field rounds: h1 (already in X), h2, item.  The h1 word of each output
    // pair is stored in the first round and zeroed in the second for a marked
    // duplicate (ctest.c:96-104), so no h1 stays in a register
    uint32_t eq1 = 0;  // bit j: sorted position tid + j * kBkT has the same h1 as its successor
#pragma unroll
    for (uint32_t f = 0; f < 3; f++) {
      if (f > 0) {
#pragma unroll
        for (uint32_t j = 0; j < PER; j++) {
          const uint32_t r = tl + j * kBkT;
          if (r < R) X[r] = f == 1 ? f1[j] : f2[j];
        }
        __syncthreads();
      }
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t p = tl + j * kBkT;
        if (p < R) {
          const uint64_t v = X[ord[p]];
          const bool eq = f < 2 && dedup && p + 1 < R && X[ord[p + 1 < R ? p + 1 : p]] == v;
          uint64_t* o = h_out + 2 * ((uint64_t)base + p);
          if (f == 0) {
            o[0] = v;
            eq1 |= (eq ? 1u : 0u) << j;
          } else if (f == 1) {
            const bool dup = eq && ((eq1 >> j) & 1u);
            d_total += dup ? 1u : 0u;
            if (dup) o[0] = 0ull;
            o[1] = v;
          } else if (items_out) {
            items_out[(uint64_t)base + p] = v;
          }
        }
      }
      __syncthreads();
    }
  }
  if (dedup && dups) {
    const uint32_t t = block_sum<kBkT>(d_total, wsum);
    if (tid == 0 && t) atomicAdd(dups, (unsigned long long)t);
  }
}

// all-ascending bitonic network over R[0, len) by the full order (every
// comparator puts the smaller record at the lower index, so the pad to a
// power of two is virtual); one workgroup
__device__ __forceinline__ void bk_bitonic(Rec* __restrict__ R, uint64_t len, const HtGeom& g, uint32_t sb) {
  const uint32_t tid = threadIdx.x;
  uint64_t P = 1;
  while (P < len) P <<= 1;
  for (uint64_t k = 2; k <= P; k <<= 1) {
    for (uint64_t jj = k >> 1; jj > 0; jj >>= 1) {
      for (uint64_t t = tid; t < P / 2; t += kSB) {
        const uint64_t off = t & (jj - 1);
        uint64_t a, c;
        if (jj == (k >> 1)) {
          a = (t / jj) * k + off;
          c = (t / jj) * k + k - 1 - off;
        } else {
          a = (t / jj) * 2 * jj + off;
          c = a + jj;
        }
        if (c >= len) continue;
        const Rec x = R[a], y = R[c];
        if (bk_less(g, sb, y, x)) { R[a] = y; R[c] = x; }
      }
      __syncthreads();
    }
  }
}

// Stable three-way partition of R[0, len) around the key of q (key64, h1,
// h2) into T: T = [less | equal | greater], each part in its input order.
// One workgroup, blocks of kSB records in order: per block, each class's
// wave ballots and the wave counts give the positions; the running totals
// are kept in every thread's registers (all threads sum the same counts),
// and the counts alternate between two LDS buffers, so a block costs one
// barrier.  Returns the sizes of the less and equal parts.
__device__ __forceinline__ void bk_partition3(const Rec* __restrict__ R, Rec* __restrict__ T, uint64_t len,
                                              const Rec& q, const HtGeom& g, uint32_t sb, uint64_t* n_less,
                                              uint64_t* n_eq, uint32_t (&wc)[2][3][kSB / 64]) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t qk = sort_key64(g, sb, q.h1);
  auto cls = [&](const Rec& x) -> uint32_t {  // 0 less, 1 equal, 2 greater than q's key
    const uint64_t k = sort_key64(g, sb, x.h1);
    if (k != qk) return k < qk ? 0u : 2u;
    if (x.h1 == q.h1 && x.h2 == q.h2) return 1u;
    return rec_less(x.h1, x.h2, q.h1, q.h2) ? 0u : 2u;
  };
  // pass 1: the part sizes
  uint32_t c0 = 0, c1 = 0;
  for (uint64_t t = tid; t < len; t += kSB) {
    const uint32_t c = cls(R[t]);
    c0 += c == 0; c1 += c == 1;
  }
  __shared__ uint32_t ws0[kSB / 64], ws1[kSB / 64];
  for (int o = 32; o >= 1; o >>= 1) { c0 += __shfl_xor(c0, o, 64); c1 += __shfl_xor(c1, o, 64); }
  if (lane == 0) { ws0[w] = c0; ws1[w] = c1; }
  __syncthreads();
  uint64_t L0 = 0, L1 = 0;
  for (int q2 = 0; q2 < kSB / 64; q2++) { L0 += ws0[q2]; L1 += ws1[q2]; }
  *n_less = L0;
  *n_eq = L1;
  uint64_t tot[3] = {0, L0, L0 + L1};
  // pass 2: stable scatter
  uint32_t p = 0;
  for (uint64_t b0 = 0; b0 < len; b0 += kSB, p ^= 1u) {
    const uint64_t t = b0 + tid;
    const bool v = t < len;
    Rec x;
    uint32_t c = 3;
    if (v) { x = R[t]; c = cls(x); }
    uint32_t below = 0;
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
      const uint64_t m = __ballot(c == k);
      if (c == k) below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (lane == 0) wc[p][k][w] = (uint32_t)__popcll(m);
    }
    // one barrier: the next block writes the other buffer, and no thread can
    // reach the block after that before every thread has passed this one's reads
    __syncthreads();
    uint32_t before[3] = {0, 0, 0}, all[3] = {0, 0, 0};
#pragma unroll
    for (uint32_t q2 = 0; q2 < kSB / 64; q2++) {
#pragma unroll
      for (uint32_t k = 0; k < 3; k++) {
        const uint32_t x2 = wc[p][k][q2];
        before[k] += q2 < w ? x2 : 0u;
        all[k] += x2;
      }
    }
    if (v) {
      const uint64_t at = c == 0 ? tot[0] + before[0] : c == 1 ? tot[1] + before[1] : tot[2] + before[2];
      T[at + below] = x;
    }
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) tot[k] += all[k];
  }
  __syncthreads();
}

// The pivot of a k_bk_long partition: wave 0 samples 64 records spread over
// R[0, len) and takes the (h1, h2) that occurs most often among them (ties:
// the lowest lane; with no repeat, the middle sample).  A key holding a
// share p of the range is the pivot unless it shows up in fewer samples than
// some other key, which for p >= 10 % of a bucket is vanishingly rare
// (64 draws), so a hot key goes to the equal part -- already ordered -- in
// the first partition whatever its share (the middle record was
// the hot key only with probability p).  Written to *q; ends with a barrier.
__device__ __forceinline__ void bk_mode_pivot(const Rec* __restrict__ R, uint64_t len, Rec* q) {
  const uint32_t tid = threadIdx.x;
  if (tid < 64) {
    const Rec s = R[(len * tid) >> 6];
    uint32_t c = 0;
    for (int j = 0; j < 64; j++) {
      const uint64_t o1 = (uint64_t)__shfl((unsigned long long)s.h1, j, 64);
      const uint64_t o2 = (uint64_t)__shfl((unsigned long long)s.h2, j, 64);
      c += (o1 == s.h1 && o2 == s.h2) ? 1u : 0u;
    }
    uint32_t best = c;
    for (int o = 32; o >= 1; o >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, o, 64));
    const uint64_t m = __ballot(c == best);
    const uint32_t pick = best > 1 ? (uint32_t)__builtin_ctzll(m) : 32u;
    if (tid == pick) *q = s;
  }
  __syncthreads();
}

// Buckets B3 could not sort in LDS, one workgroup each.  A bucket already in
// the full order (with the tile-stable two-pass scatter a bucket's records
// arrive in input order, so a bucket holding one repeated key) skips the
// network.  Otherwise, when `tmp` is given (the two-pass path: its first
// record buffer is free by now), a quicksort of stable three-way partitions
// around the sampled-mode pivot (bk_mode_pivot): each equal part is final
// (one key, input order), the less and greater parts are partitioned again
// while longer than kBkNet records, and the parts at or below it go through
// the bitonic network.  A hot key repeated millions of times (the KVH_DEDUP
// case) among a bucket's ordinary keys, or several of them,
// costs a few passes instead of O(R log^2 R) network steps on one
// workgroup.  The smaller part is taken first (stack depth <= log2 R) and a
// bucket gets at most kBkParts partitions before the network takes the
// rest, so the loop ends on any input.  Without `tmp`, the whole bucket
// through the network.
constexpr uint64_t kBkNet = 2048;   // parts at or below this size: bitonic network in LDS (64 KiB)
constexpr int kBkStack = 40;        // > log2 of any bucket length
constexpr int kBkParts = 256;       // partitions per bucket before the (global) network takes over

__global__ void __launch_bounds__(kSB)
k_bk_long(Rec* __restrict__ recs, Rec* __restrict__ tmp, const uint32_t* __restrict__ cnt,
          const uint32_t* __restrict__ start, HtGeom g, uint32_t sb, uint64_t* __restrict__ h_out,
          uint64_t* __restrict__ items_out, uint32_t dedup, unsigned long long* __restrict__ dups,
          const uint32_t* __restrict__ novf, const uint32_t* __restrict__ ovf) {
  __shared__ uint32_t wsum[kSB / 64];
  __shared__ uint32_t wc[2][3][kSB / 64];
  __shared__ Rec pivot;
  __shared__ uint64_t st_lo[kBkStack], st_len[kBkStack];
  __shared__ Rec S[kBkNet];
  const uint32_t count = *novf, tid = threadIdx.x;
  uint32_t d = 0;
  for (uint32_t r = blockIdx.x; r < count; r += gridDim.x) {
    const uint32_t b = ovf[r];
    const uint64_t len = cnt[b];
    Rec* R = recs + start[b];
    uint32_t unordered = 0;
    for (uint64_t t = tid; t + 1 < len; t += kSB) unordered |= bk_less(g, sb, R[t + 1], R[t]) ? 1u : 0u;
    if (block_sum(unordered, wsum)) {
      if (tmp) {
        Rec* Tm = tmp + start[b];
        // workgroup-uniform stack of parts (offset, length); thread 0 writes,
        // every thread reads after the barrier that follows
        int sp = 1, parts = 0;
        if (tid == 0) { st_lo[0] = 0; st_len[0] = len; }
        __syncthreads();
        while (sp > 0) {
          sp--;
          const uint64_t lo = st_lo[sp], l = st_len[sp];
          __syncthreads();
          if (l <= kBkNet) {  // the part in LDS, the network there, back
            for (uint64_t t = tid; t < l; t += kSB) S[t] = R[lo + t];
            __syncthreads();
            bk_bitonic(S, l, g, sb);
            for (uint64_t t = tid; t < l; t += kSB) R[lo + t] = S[t];
            __syncthreads();
            continue;
          }
          if (parts >= kBkParts || sp + 2 > kBkStack) {
            bk_bitonic(R + lo, l, g, sb);
            __syncthreads();
            continue;
          }
          parts++;
          bk_mode_pivot(R + lo, l, &pivot);
          const Rec q = pivot;
          uint64_t nl = 0, ne = 0;
          bk_partition3(R + lo, Tm + lo, l, q, g, sb, &nl, &ne, wc);
          for (uint64_t t = tid; t < l; t += kSB) R[lo + t] = Tm[lo + t];
          const uint64_t ng = l - nl - ne;
          // push the larger part first, so the smaller one is taken next
          const bool less_first = nl >= ng;
          const uint64_t a_lo = less_first ? lo : lo + nl + ne, a_len = less_first ? nl : ng;
          const uint64_t b_lo = less_first ? lo + nl + ne : lo, b_len = less_first ? ng : nl;
          if (tid == 0) {
            int s = sp;
            if (a_len > 1) { st_lo[s] = a_lo; st_len[s] = a_len; s++; }
            if (b_len > 1) { st_lo[s] = b_lo; st_len[s] = b_len; s++; }
          }
          sp += (a_len > 1) + (b_len > 1);
          __syncthreads();
        }
      } else {
        bk_bitonic(R, len, g, sb);
      }
    }
    for (uint64_t t = tid; t < len; t += kSB) {
      const Rec v = R[t];
      const bool has_next = t + 1 < len;
      uint64_t n1 = 0, n2 = 0;
      if (has_next) { n1 = R[t + 1].h1; n2 = R[t + 1].h2; }
      d += bk_emit(start[b] + t, v, has_next, n1, n2, dedup, h_out, items_out);
    }
    __syncthreads();
  }
  if (dedup && dups) {
    const uint32_t t = block_sum(d, wsum);
    if (tid == 0 && t) atomicAdd(dups, (unsigned long long)t);
  }
}

// Two-pass path, before k_bk_long: each overflowing bucket (R24 records in
// input order) copied as 32-byte records whose `pad` is the bucket position
// (the input order's stand-in) into the first-pass buffer, free by now; the
// second-pass buffer then serves as k_bk_long's partition space.
__global__ void __launch_bounds__(kSB)
k_bk_cvt(const R24* __restrict__ src, Rec* __restrict__ dst, const uint32_t* __restrict__ cnt,
         const uint32_t* __restrict__ start, const uint32_t* __restrict__ novf, const uint32_t* __restrict__ ovf) {
  const uint32_t count = *novf;
  for (uint32_t r = blockIdx.x; r < count; r += gridDim.x) {
    const uint32_t b = ovf[r];
    const uint64_t len = cnt[b], base = start[b];
    for (uint64_t t = threadIdx.x; t < len; t += kSB) {
      const R24 x = src[base + t];
      Rec y;
      y.h1 = x.h1; y.h2 = x.h2; y.item = x.item; y.pad = t;
      dst[base + t] = y;
    }
  }
}


// ---------------------------------------------------------------------
// Two-pass bucketed path (round 3): the B bucket bits of B2 (k_bk_scatter's
// one pass into 2^B <= 16K bucket streams) split into a pass over the top
// B1 = ceil(B / 2) bits and one over the low B2 = B - B1 bits, each <= 7
// bits (<= 128 streams), each a TILE-STABLE, LDS-staged scatter: a tile of
// kTwTile elements is ranked by digit in input order (wave ballots "match
// any" on the 7 digit bits + per (round, wave, digit) counts), staged in LDS
// in digit order and written out from there, so a store instruction's lanes
// write one digit's consecutive records (16 per digit per tile on average)
// instead of 64 different bucket streams (tools/scatter_probe.hip prices the
// 16K-stream scatter at 2.4-4.5x a copy).  Tiles keep input order, so every
// bucket's records arrive in input order: k_bk_sort's order is unchanged
// (its comparator ends in the input index) and a bucket of one repeated key
// is already ordered for k_bk_long.
//   T0. k_tw_hist1     per tile, the counts of the top-B1 digit
//   T1. k_bk_colsum / k_tw_scan1 / k_bk_scan / k_bk_tileoff (as B1 above,
//                      over 2^B1 columns; the chunk scan one parallel
//                      workgroup) -> each tile's first position per digit
//   T2. k_tw_scatter1  records (h1, h2, item, index) -> recA by top digit,
//                      with their full bucket id (u16) -> bA
//   T3. k_tw_tiles     pass-2 tiles: each top-digit region cut into kTwTile runs
//   T4. k_tw_hist2     per pass-2 tile, the counts of the low digit
//   T5. k_tw_scan2 / k_tw_start2   per bucket: running offsets over its
//                      region's tiles, the bucket sizes and starts
//   T6. k_tw_scatter2  recA -> rec by low digit (stable)
//   then B3 k_bk_sort / B4 k_bk_long as the one-pass path.
constexpr uint32_t kTwTile = 2048;             // elements per tile
constexpr int kTwT = 512;                      // threads per workgroup
constexpr int kTwW = kTwT / 64;                // waves
constexpr int kTwPer = (int)(kTwTile / kTwT);  // elements per thread
constexpr int kTwD = 128;                      // digit values (<= 7 bits)
constexpr int kTwD8 = 256;                     // pass 2 of the 15-bit split (knob 23 = 3): 8 bits
constexpr int kTwMaxB = 15;                    // bucket bits of the two-pass path

template <uint32_t ND>
struct TwSh {
  R24 stage[kTwTile];                // the tile in digit order
  uint16_t cnt[kTwPer][kTwW][ND];    // per (round, wave, digit) counts -> offsets in the digit
  uint16_t bkt[kTwTile];             // the full bucket id of each staged record
  uint8_t dig[kTwTile];              // its digit
  uint32_t lstart[ND], gofs[ND], wtot[ND / 64];
};
using TwShared = TwSh<kTwD>;

// Stable rank of the tile's elements by digit (element k*kTwT + tid holds
// dg[k], valid v[k]): pos[k] = its position in the digit-sorted tile;
// S.lstart[d] = digit d's first position.  Ends with a barrier.  ND = 128
// or 256 digit values.
template <uint32_t ND = kTwD>
__device__ __forceinline__ void tw_rank(const uint32_t (&dg)[kTwPer], const bool (&v)[kTwPer], TwSh<ND>& S,
                                        uint32_t (&pos)[kTwPer]) {
  constexpr int DB = ND == 256 ? 8 : 7;
  static_assert(ND == 128 || ND == 256, "digit values");
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint16_t* c = &S.cnt[0][0][0];
  for (uint32_t i = tid; i < (uint32_t)(kTwPer * kTwW * ND); i += kTwT) c[i] = 0;
  __syncthreads();
  uint32_t below[kTwPer];
#pragma unroll
  for (int k = 0; k < kTwPer; k++) {
    uint64_t eq = __ballot(v[k]);
#pragma unroll
    for (int bit = 0; bit < DB; bit++) {
      const uint64_t B = __ballot((dg[k] >> bit) & 1u);
      eq &= ((dg[k] >> bit) & 1u) ? B : ~B;
    }
    below[k] = __builtin_amdgcn_mbcnt_hi((uint32_t)(eq >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)eq, 0u));
    if (v[k] && below[k] == 0) S.cnt[k][w][dg[k]] = (uint16_t)__popcll(eq);
  }
  __syncthreads();
  if (tid < ND) {  // per digit: running offsets over (round, wave), then the digit starts
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < kTwPer; k++)
#pragma unroll
      for (int q = 0; q < kTwW; q++) {
        const uint32_t x = S.cnt[k][q][tid];
        S.cnt[k][q][tid] = (uint16_t)run;
        run += x;
      }
    uint32_t inc = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (lane >= (uint32_t)d) inc += y;
    }
    if (lane == 63) S.wtot[w] = inc;
    S.lstart[tid] = inc - run;  // within this wave's 64 digits
  }
  __syncthreads();
  if (tid >= 64 && tid < ND) {
    uint32_t add = 0;
    for (uint32_t q = 0; q < w; q++) add += S.wtot[q];
    S.lstart[tid] += add;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kTwPer; k++)
    pos[k] = v[k] ? S.lstart[dg[k]] + S.cnt[k][w][dg[k]] + below[k] : 0u;
}

__global__ void __launch_bounds__(kTwT)
k_tw_hist1(const uint64_t* __restrict__ h, uint64_t n, HtGeom g, uint32_t sb, uint32_t B, uint32_t B2,
           uint32_t* __restrict__ H, uint32_t* __restrict__ novf) {
  __shared__ uint32_t hist[kTwD];
  const uint32_t tid = threadIdx.x, tile = blockIdx.x, nb1 = 1u << (B - B2);
  if (tile == 0 && tid == 0) *novf = 0;  // B4's overflow list, empty per call
  if (tid < (uint32_t)kTwD) hist[tid] = 0;
  __syncthreads();
  const uint64_t i0 = (uint64_t)tile * kTwTile;
  // every load issued before the first use (indices clamped, not branched
  // around: a branch made each one its own memory round trip)
  uint64_t hv[kTwPer];
#pragma unroll
  for (int k = 0; k < kTwPer; k++) hv[k] = h[2 * min<uint64_t>(i0 + (uint64_t)k * kTwT + tid, n - 1)];
#pragma unroll
  for (int k = 0; k < kTwPer; k++)
    if (i0 + (uint64_t)k * kTwT + tid < n) atomicAdd(&hist[bk_of(sort_key64(g, sb, hv[k]), B) >> B2], 1u);
  __syncthreads();
  if (tid < nb1) H[(uint64_t)tile * nb1 + tid] = hist[tid];
}

__global__ void __launch_bounds__(kTwT)
k_tw_scatter1(const uint64_t* __restrict__ h, const uint64_t* __restrict__ items, uint64_t n, HtGeom g, uint32_t sb,
              uint32_t B, uint32_t B2, const uint32_t* __restrict__ H, R24* __restrict__ recA,
              uint16_t* __restrict__ bA) {
  __shared__ TwShared S;
  const uint32_t tid = threadIdx.x, tile = xcd_tile(blockIdx.x, gridDim.x), nb1 = 1u << (B - B2);
  const uint64_t i0 = (uint64_t)tile * kTwTile;
  R24 r[kTwPer];
  uint32_t dg[kTwPer], bk[kTwPer], pos[kTwPer];
  bool v[kTwPer];
  // all the tile's loads in flight together (clamped indices; a branch
  // around each element's loads made them four memory round trips)
#pragma unroll
  for (int k = 0; k < kTwPer; k++) {
    const uint64_t i = i0 + (uint64_t)k * kTwT + tid, ic = min<uint64_t>(i, n - 1);
    v[k] = i < n;
    r[k].h1 = h[2 * ic];
    r[k].h2 = h[2 * ic + 1];
    r[k].item = items ? items[ic] : i;
  }
  const uint32_t go = tid < nb1 ? H[(uint64_t)tile * nb1 + tid] : 0u;
#pragma unroll
  for (int k = 0; k < kTwPer; k++) {
    bk[k] = v[k] ? bk_of(sort_key64(g, sb, r[k].h1), B) : 0u;
    dg[k] = bk[k] >> B2;
  }
  if (tid < nb1) S.gofs[tid] = go;
  tw_rank(dg, v, S, pos);
#pragma unroll
  for (int k = 0; k < kTwPer; k++)
    if (v[k]) {
      S.stage[pos[k]] = r[k];
      S.dig[pos[k]] = (uint8_t)dg[k];
      S.bkt[pos[k]] = (uint16_t)bk[k];
    }
  __syncthreads();
  const uint32_t total = (uint32_t)min<uint64_t>(kTwTile, n - i0);
  // one 8-byte word per lane: a store instruction covers ~21 whole
  // consecutive records (512 B)
  const uint64_t* sw = (const uint64_t*)S.stage;
  for (uint32_t w = tid; w < 3 * total; w += kTwT) {
    const uint32_t p = w / 3, part = w - 3 * p;
    const uint32_t d = S.dig[p];
    const uint64_t q = (uint64_t)S.gofs[d] + (p - S.lstart[d]);
    ((uint64_t*)(recA + q))[part] = sw[w];
    if (part == 0) bA[q] = S.bkt[p];
  }
}

// pass-2 tiles: top digit d's records [start1[d], start1[d] + cnt1[d]) cut
// into kTwTile runs; tbs[d] = the first tile of digit d, tbs[nb1] = all tiles
__global__ void __launch_bounds__(kTwD)
k_tw_tiles(const uint32_t* __restrict__ cnt1, uint32_t nb1, uint32_t* __restrict__ tbs) {
  __shared__ uint32_t w0;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t t = tid < nb1 ? (cnt1[tid] + kTwTile - 1) / kTwTile : 0u;
  uint32_t inc = t;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += y;
  }
  if (tid == 63) w0 = inc;
  __syncthreads();
  if (tid >= 64) inc += w0;
  if (tid < nb1) tbs[tid + 1] = inc;
  if (tid == 0) tbs[0] = 0;
}

// pass-2 tile j -> its top digit and record range [*p0, *p1); false past the last tile
__device__ __forceinline__ bool tw_tile2(uint32_t j, const uint32_t* __restrict__ tbs, uint32_t nb1,
                                         const uint32_t* __restrict__ cnt1, const uint32_t* __restrict__ start1,
                                         uint32_t* d1, uint32_t* p0, uint32_t* p1) {
  if (j >= tbs[nb1]) return false;
  uint32_t lo = 0, hi = nb1;  // the last d with tbs[d] <= j
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (tbs[mid] <= j) lo = mid; else hi = mid;
  }
  *d1 = lo;
  *p0 = start1[lo] + (j - tbs[lo]) * kTwTile;
  *p1 = min(*p0 + kTwTile, start1[lo] + cnt1[lo]);
  return true;
}

template <uint32_t ND = kTwD>
__global__ void __launch_bounds__(kTwT)
k_tw_hist2(const uint16_t* __restrict__ bA, const uint32_t* __restrict__ tbs, const uint32_t* __restrict__ cnt1,
           const uint32_t* __restrict__ start1, uint32_t nb1, uint32_t B2, uint32_t* __restrict__ H2) {
  __shared__ uint32_t hist[ND];
  const uint32_t tid = threadIdx.x, nb2 = 1u << B2;
  uint32_t d1, p0, p1;
  if (!tw_tile2(blockIdx.x, tbs, nb1, cnt1, start1, &d1, &p0, &p1)) return;  // workgroup-uniform
  if (tid < ND) hist[tid] = 0;
  __syncthreads();
  // a tile is <= kTwTile = kTwPer x kTwT records: every load before the first atomic
  uint32_t bv[kTwPer];
#pragma unroll
  for (int k = 0; k < kTwPer; k++) bv[k] = bA[min(p0 + (uint32_t)k * kTwT + tid, p1 - 1)];
#pragma unroll
  for (int k = 0; k < kTwPer; k++)
    if (p0 + (uint32_t)k * kTwT + tid < p1) atomicAdd(&hist[bv[k] & (nb2 - 1)], 1u);
  __syncthreads();
  if (tid < nb2) H2[(uint64_t)blockIdx.x * nb2 + tid] = hist[tid];
}

// Exclusive scan, in place, of the columns c < ncols (<= NC = 128 or 256)
// of rows [r0, r1) of a row-major table with `ncols` words per row, by one
// 1024-thread workgroup: 1024 / NC groups of NC threads, group g scans a
// contiguous share of the rows (the NC threads of a group read one row's
// words together: coalesced), group sums combined in LDS.  *total[c] gets
// the column sum when total != nullptr.
template <uint32_t NC = kTwD>
__device__ __forceinline__ void tw_colscan(uint32_t* __restrict__ Tb, uint32_t r0, uint32_t r1, uint32_t ncols,
                                           uint32_t* __restrict__ total, uint32_t (&part)[1024 / NC][NC]) {
  constexpr uint32_t NG = 1024 / NC;
  const uint32_t c = threadIdx.x & (NC - 1), grp = threadIdx.x / NC;
  const uint32_t rows = r1 - r0, per = (rows + NG - 1) / NG;
  const uint32_t a = r0 + min(rows, grp * per), b = r0 + min(rows, (grp + 1) * per);
  uint32_t sum = 0;
  if (c < ncols) {
    uint32_t r = a;
    for (; r + 8 <= b; r += 8) {
      uint32_t v[8];
#pragma unroll
      for (int q = 0; q < 8; q++) v[q] = Tb[(uint64_t)(r + q) * ncols + c];
#pragma unroll
      for (int q = 0; q < 8; q++) sum += v[q];
    }
    for (; r < b; r++) sum += Tb[(uint64_t)r * ncols + c];
  }
  part[grp][c] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t g = 0; g < grp; g++) run += part[g][c];
  if (c < ncols) {
    if (grp == 0 && total) {
      uint32_t t = 0;
      for (uint32_t g = 0; g < NG; g++) t += part[g][c];
      total[c] = t;
    }
    uint32_t r = a;
    for (; r + 8 <= b; r += 8) {
      uint32_t v[8];
#pragma unroll
      for (int q = 0; q < 8; q++) v[q] = Tb[(uint64_t)(r + q) * ncols + c];
#pragma unroll
      for (int q = 0; q < 8; q++) { Tb[(uint64_t)(r + q) * ncols + c] = run; run += v[q]; }
    }
    for (; r < b; r++) {
      const uint32_t v = Tb[(uint64_t)r * ncols + c];
      Tb[(uint64_t)r * ncols + c] = run;
      run += v;
    }
  }
}

// pass 1: the chunk sums S[nch][nb1] -> exclusive prefix per column, cnt1 = the column sums
__global__ void __launch_bounds__(1024)
k_tw_scan1(uint32_t* __restrict__ S, uint32_t nch, uint32_t nb1, uint32_t* __restrict__ cnt1) {
  __shared__ uint32_t part[8][kTwD];
  tw_colscan(S, 0, nch, nb1, cnt1, part);
}

// pass 2, one workgroup per top digit d1: H2 over d1's tiles -> running
// offsets within each bucket (d1, d2); cnt[(d1, d2)] = the bucket's size
template <uint32_t ND = kTwD>
__global__ void __launch_bounds__(1024)
k_tw_scan2(uint32_t* __restrict__ H2, const uint32_t* __restrict__ tbs, uint32_t B2, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t part[1024 / ND][ND];
  const uint32_t d1 = blockIdx.x;
  tw_colscan<ND>(H2, tbs[d1], tbs[d1 + 1], 1u << B2, cnt + (d1 << B2), part);
}

// start[b] = start1[d1] + the sizes of d1's earlier buckets: one workgroup
// per top digit d1, an exclusive scan of its 2^B2 <= 256 bucket sizes (round
// 5: one thread per d1 walking them serially took ~50 us per sort)
__global__ void __launch_bounds__(256)
k_tw_start2(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ start1, uint32_t nb1, uint32_t B2,
            uint32_t* __restrict__ start) {
  __shared__ uint32_t wsum[4];
  const uint32_t d1 = blockIdx.x, d2 = threadIdx.x, nb2 = 1u << B2, lane = d2 & 63, w = d2 >> 6;
  const uint32_t v = d2 < nb2 ? cnt[(d1 << B2) | d2] : 0u;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t wo = 0;
  for (uint32_t q = 0; q < w; q++) wo += wsum[q];
  if (d2 < nb2) start[(d1 << B2) | d2] = start1[d1] + wo + inc - v;
}

// MODE selects how a tile's records are read; the library launches MODE 7
// (MODE 3 with the digit recomputed from h1 instead of loaded from bA).
// tools/scatter2_real.hip ran every mode on the real
// pass-2 inputs (profiles/r04/s1/s2real*.json): with plain 24-byte record
// loads (MODE 0, the round-3 kernel) the stride-24 load instructions pull
// their lines through L2 and push out the tile runs' partially written
// lines before their neighbours complete them, so each boundary line is
// written back twice: WRITE_SIZE 4.72 GB for 2.4 GB of records, 1.75 ms.
// Non-temporal loads (3) or coalesced 8-byte word loads (5) leave the dirty
// lines in place: 2.34 / 2.35 GB and 1.03 / 1.07 ms, bit-exact.  1 stores to
// `dummy` (same offsets; still 4.7 GB: not the destination), 2 makes records
// from the position without loading (2.17 GB, 0.90 ms: the floor), 4 stores
// non-temporally (5.06 GB), 6 = 5 with non-temporal loads.  Only 0, 3, 5, 6
// give the product's output; 1, 2, 4 are attribution probes.
template <int MODE, uint32_t ND = kTwD>
__global__ void __launch_bounds__(kTwT)
k_tw_scatter2(const R24* __restrict__ recA, const uint16_t* __restrict__ bA, const uint32_t* __restrict__ tbs,
              const uint32_t* __restrict__ cnt1, const uint32_t* __restrict__ start1, uint32_t nb1, uint32_t B2,
              const uint32_t* __restrict__ H2, const uint32_t* __restrict__ start, R24* __restrict__ rec,
              R24* __restrict__ dummy, HtGeom g, uint32_t sb, uint32_t B) {
  __shared__ TwSh<ND> S;
  const uint32_t tid = threadIdx.x, nb2 = 1u << B2, j = xcd_tile(blockIdx.x, gridDim.x);
  uint32_t d1, p0, p1;
  if (!tw_tile2(j, tbs, nb1, cnt1, start1, &d1, &p0, &p1)) return;  // workgroup-uniform
  R24 r[kTwPer];
  uint32_t dg[kTwPer], pos[kTwPer];
  bool v[kTwPer];
  // MODE 5: the tile's records read as 8-byte words, word w = tid + m * kTwT
  // (every load instruction a contiguous 512 B), placed by the record
  // positions the rank publishes in LDS
  constexpr int kW = 3 * kTwPer;
  uint64_t wd[MODE == 5 || MODE == 6 ? kW : 1];
  const uint32_t nwords = 3 * (p1 - p0);
  if constexpr (MODE == 5 || MODE == 6) {
    const uint64_t* src = (const uint64_t*)(recA + p0);
#pragma unroll
    for (int m = 0; m < kW; m++) {
      const uint32_t w = tid + (uint32_t)m * kTwT;
      if constexpr (MODE == 6)
        wd[m] = w < nwords ? __builtin_nontemporal_load(src + w) : 0ull;
      else
        wd[m] = w < nwords ? src[w] : 0ull;
    }
  }
#pragma unroll
  for (int k = 0; k < kTwPer; k++) {
    const uint32_t p = p0 + (uint32_t)k * kTwT + tid;
    v[k] = p < p1;
    dg[k] = 0;
    if (v[k]) {
      if constexpr (MODE == 5 || MODE == 6) {
        dg[k] = (MODE == 6 ? __builtin_nontemporal_load(bA + p) : bA[p]) & (nb2 - 1);
      } else if constexpr (MODE == 2) {
        r[k].h1 = p; r[k].h2 = ~(uint64_t)p; r[k].item = p;
        dg[k] = (p * 2654435761u >> 9) & (nb2 - 1);
      } else if constexpr (MODE == 3 || MODE == 7) {
        // (loaded below, outside the branch)
      } else {
        r[k] = recA[p];
        dg[k] = bA[p] & (nb2 - 1);
      }
    }
  }
  if constexpr (MODE == 3 || MODE == 7) {  // every load of the tile in flight together: clamped, not branched around
    uint32_t bv[kTwPer];
#pragma unroll
    for (int k = 0; k < kTwPer; k++) {
      const uint32_t pc = min(p0 + (uint32_t)k * kTwT + tid, p1 - 1);
      const uint64_t* q = (const uint64_t*)(recA + pc);
      r[k].h1 = __builtin_nontemporal_load(q);
      r[k].h2 = __builtin_nontemporal_load(q + 1);
      r[k].item = __builtin_nontemporal_load(q + 2);
      if constexpr (MODE == 3) bv[k] = __builtin_nontemporal_load(bA + pc);
    }
    // MODE 7 (the library's, round 6): the low digit recomputed from h1
    // (ht_mod is a multiply and a shift) instead of read from bA: 2 B less
    // per record, 3.80 -> 3.75 ms for f2 (profiles/r06/f2_ab/)
#pragma unroll
    for (int k = 0; k < kTwPer; k++)
      dg[k] = v[k] ? (MODE == 7 ? bk_of(sort_key64(g, sb, r[k].h1), B) : bv[k]) & (nb2 - 1) : 0u;
  }
  if (tid < nb2) S.gofs[tid] = start[(d1 << B2) | tid] + H2[(uint64_t)j * nb2 + tid];
  tw_rank<ND>(dg, v, S, pos);
  if constexpr (MODE == 5 || MODE == 6) {
#pragma unroll
    for (int k = 0; k < kTwPer; k++)
      if (v[k]) {
        S.bkt[(uint32_t)k * kTwT + tid] = (uint16_t)pos[k];  // record -> its staged position
        S.dig[pos[k]] = (uint8_t)dg[k];
      }
    __syncthreads();
    uint64_t* sw5 = (uint64_t*)S.stage;
#pragma unroll
    for (int m = 0; m < kW; m++) {
      const uint32_t w = tid + (uint32_t)m * kTwT, q = w / 3u;
      if (w < nwords) sw5[3u * S.bkt[q] + (w - 3u * q)] = wd[m];
    }
  } else {
#pragma unroll
    for (int k = 0; k < kTwPer; k++)
      if (v[k]) {
        S.stage[pos[k]] = r[k];
        S.dig[pos[k]] = (uint8_t)dg[k];
      }
  }
  __syncthreads();
  // one 8-byte word per lane: a store instruction covers ~21 whole
  // consecutive records (512 B) instead of the same third of 64 records
  const uint64_t* sw = (const uint64_t*)S.stage;
  R24* dst = MODE == 1 ? dummy : rec;
  for (uint32_t w = tid; w < 3 * (p1 - p0); w += kTwT) {
    const uint32_t p = w / 3, part = w - 3 * p;
    const uint32_t d = S.dig[p];
    uint64_t* a = ((uint64_t*)(dst + (uint64_t)S.gofs[d] + (p - S.lstart[d]))) + part;
    if constexpr (MODE == 4)
      __builtin_nontemporal_store(sw[w], a);
    else
      *a = sw[w];
  }
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct SortLayout {
  size_t key_in, key_out, idx_in, idx_out, rec, runs, tmp, tmp_bytes;
  // the two-pass bucketed path (its own offsets from 0)
  size_t tw_recA, tw_rec, tw_bA, tw_H1, tw_S1, tw_small, tw_H2, tw_bk;
  size_t total;
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
  const size_t radix_total = o;
  const size_t ntiles = (n + kTwTile - 1) / kTwTile, nch = (ntiles + kBkChunk - 1) / kBkChunk;
  o = 0;
  L->tw_recA = o; o += al256(sizeof(Rec) * n);
  L->tw_rec = o; o += al256(sizeof(Rec) * n);
  L->tw_bA = o; o += al256(2 * n);
  L->tw_H1 = o; o += al256(4 * ntiles * kTwD);
  L->tw_S1 = o; o += al256(4 * nch * kTwD);
  L->tw_small = o; o += al256(4 * (3 * kTwD + 2));  // cnt1, start1, tbs
  L->tw_H2 = o; o += al256(4 * (ntiles + kTwD8) * kTwD8);  // pass-2 counts, up to 8-bit digits
  L->tw_bk = o; o += al256(4 * (3 * (1u << kTwMaxB) + 1));   // cnt, start, ovf, novf
  L->total = std::max(radix_total, o);
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
  if (flags & KVH_REF_ORDER)  // the reference's exact element order, n <= 64K (ht_refsort.hip)
    return refsort_launch(hashes, items, n, geom, h_out, items_out, dup_count, dedup, scratch, scratch_bytes, st);
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
  const int tsb = g_tune_sort_bits.load(std::memory_order_relaxed);
  int cus = 0;
  if ((rc = device_cus(&cus))) return rc;
  const int engine = g_tune_sort_engine.load(std::memory_order_relaxed);
  if (!tsb && engine != 1) {
    // the bucketed paths: ~6K elements per bucket over the buckets the
    // table's slots reach (slot < ht_size: a share ht_size / 2^sb of the 2^B
    // top-bit buckets, 1/2 to 1), B <= 14 bucket bits, so up to
    // ~75-147M elements per call (a mean bucket of <= 9000 under the 12288
    // LDS capacity); larger batches take the radix path below
    const double reach = (double)geom->ht_size / std::ldexp(1.0, (int)std::min<uint32_t>(sb, 64));
    auto mean_of = [&](uint32_t B) { return (double)n / (reach * std::ldexp(1.0, (int)B)); };
    // knob 23 = 3: half-size buckets (mean <= 3072, up to 15 bits: pass 2 of
    // 8 bits) for the bucket sort at two 512-thread workgroups per CU
    const int b3 = g_tune_sort_b3.load(std::memory_order_relaxed);
    const bool half = (b3 == 3 || b3 >= 5) && engine != 2;
    uint32_t B = 0;
    while (B < (uint32_t)(half ? kTwMaxB : kBkMaxB) && mean_of(B) > (half ? 3072.0 : 6144.0)) B++;
    // buckets then hold ~mean +- sqrt(mean): the two-per-CU bucket sort (capacity
    // 8000) when the mean leaves a wide margin (knob 22 = 1 forces the 12288 one)
    const bool small_b = mean_of(B) <= (half ? 3200.0 : 6400.0) && g_tune_sort_cap.load(std::memory_order_relaxed) == 0;
    if (mean_of(B) <= 9000.0 && engine != 2 && B >= 2) {
      // two passes of <= 7 bits (the 15-bit split: 7 + 8), tile-stable LDS-staged scatters
      const uint32_t B2 = half ? std::min<uint32_t>(8, B - B / 2) : B / 2, B1 = B - B2, nb1 = 1u << B1,
                     nb = 1u << B;
      const bool d8 = B2 == 8;
      const uint32_t ntiles = (uint32_t)((n + kTwTile - 1) / kTwTile);
      const uint32_t nch = (ntiles + kBkChunk - 1) / kBkChunk;
      R24* recA = (R24*)(s + L.tw_recA);
      R24* recB = (R24*)(s + L.tw_rec);
      uint16_t* bA = (uint16_t*)(s + L.tw_bA);
      uint32_t* H1 = (uint32_t*)(s + L.tw_H1);
      uint32_t* S1 = (uint32_t*)(s + L.tw_S1);
      uint32_t* cnt1 = (uint32_t*)(s + L.tw_small);
      uint32_t* start1 = cnt1 + kTwD;
      uint32_t* tbs = start1 + kTwD;
      uint32_t* H2 = (uint32_t*)(s + L.tw_H2);
      uint32_t* cnt = (uint32_t*)(s + L.tw_bk);
      uint32_t* start = cnt + nb;
      uint32_t* ovf = start + nb;
      uint32_t* novf = ovf + nb;
      const uint32_t cgrid = (uint32_t)(((uint64_t)nch * nb1 + 255) / 256);
      hipLaunchKernelGGL(k_tw_hist1, dim3(ntiles), dim3(kTwT), 0, st, hashes, (uint64_t)n, g, sb, B, B2, H1, novf);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_colsum, dim3(cgrid), dim3(256), 0, st, (const uint32_t*)H1, ntiles, nb1, S1);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_tw_scan1, dim3(1), dim3(1024), 0, st, S1, nch, nb1, cnt1);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(kBkT), 0, st, (const uint32_t*)cnt1, nb1, start1);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_tileoff, dim3(cgrid), dim3(256), 0, st, H1, (const uint32_t*)S1,
                         (const uint32_t*)start1, ntiles, nb1);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_tw_scatter1, dim3(ntiles), dim3(kTwT), 0, st, hashes, items, (uint64_t)n, g, sb, B, B2,
                         (const uint32_t*)H1, recA, bA);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_tw_tiles, dim3(1), dim3(kTwD), 0, st, (const uint32_t*)cnt1, nb1, tbs);
      if ((rc = launch_done())) return rc;
      const uint32_t ntB = ntiles + nb1;  // an upper bound: the tiles past tbs[nb1] return at once
      if (d8)
        hipLaunchKernelGGL(k_tw_hist2<kTwD8>, dim3(ntB), dim3(kTwT), 0, st, (const uint16_t*)bA, (const uint32_t*)tbs,
                           (const uint32_t*)cnt1, (const uint32_t*)start1, nb1, B2, H2);
      else
        hipLaunchKernelGGL(k_tw_hist2<kTwD>, dim3(ntB), dim3(kTwT), 0, st, (const uint16_t*)bA, (const uint32_t*)tbs,
                           (const uint32_t*)cnt1, (const uint32_t*)start1, nb1, B2, H2);
      if ((rc = launch_done())) return rc;
      if (d8)
        hipLaunchKernelGGL(k_tw_scan2<kTwD8>, dim3(nb1), dim3(1024), 0, st, H2, (const uint32_t*)tbs, B2, cnt);
      else
        hipLaunchKernelGGL(k_tw_scan2<kTwD>, dim3(nb1), dim3(1024), 0, st, H2, (const uint32_t*)tbs, B2, cnt);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_tw_start2, dim3(nb1), dim3(256), 0, st, (const uint32_t*)cnt, (const uint32_t*)start1,
                         nb1, B2, start);
      if ((rc = launch_done())) return rc;
#define KVH_TWS2(M, NDv)                                                                                             \
  hipLaunchKernelGGL((k_tw_scatter2<M, NDv>), dim3(ntB), dim3(kTwT), 0, st, (const R24*)recA, (const uint16_t*)bA,     \
                     (const uint32_t*)tbs, (const uint32_t*)cnt1, (const uint32_t*)start1, nb1, B2, (const uint32_t*)H2,  \
                     (const uint32_t*)start, recB, (R24*)nullptr, g, sb, B)
#ifdef KVH_EXPERIMENTS
      if (b3 == 17) {  // A/B: the round-5 pass 2, low digit loaded from bA
        if (d8) KVH_TWS2(3, kTwD8); else KVH_TWS2(3, kTwD);
      } else
#endif
      if (d8) KVH_TWS2(7, kTwD8); else KVH_TWS2(7, kTwD);
#undef KVH_TWS2
      if ((rc = launch_done())) return rc;
      if (small_b && half) {  // half-size buckets: two 512-thread workgroups per CU
        const uint32_t hg = std::min<uint32_t>(nb, 2u * (uint32_t)cus);
        const int hd = g_tune_sort_hd.load(std::memory_order_relaxed);  // knob 25: counting-sort bits
#define KVH_BKH(Dv, W2v)                                                                                             \
  hipLaunchKernelGGL((k_bk_sortr<3584, Dv, 512, W2v>), dim3(hg), dim3(512), 0, st, (const R24*)recB,                  \
                     (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out, items_out, dedup ? 1u : 0u,   \
                     (unsigned long long*)dup_count, novf, ovf)
#define KVH_BKX(Dv)                                                                                                  \
  hipLaunchKernelGGL((k_bk_sortx<3584, Dv, 512>), dim3(hg), dim3(512), 0, st, (const R24*)recB, (const uint32_t*)cnt, \
                     (const uint32_t*)start, nb, B, g, sb, h_out, items_out, dedup ? 1u : 0u,                         \
                     (unsigned long long*)dup_count, novf, ovf)
#define KVH_BKH2(Dv)                                                                                                 \
  hipLaunchKernelGGL((k_bk_sortr<3584, Dv, 512, true, true>), dim3(hg), dim3(512), 0, st, (const R24*)recB,          \
                     (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out, items_out, dedup ? 1u : 0u,   \
                     (unsigned long long*)dup_count, novf, ovf)
#ifdef KVH_EXPERIMENTS
#define KVH_BKAB(Dv, A)                                                                                              \
  hipLaunchKernelGGL((k_bk_sortr<3584, Dv, 512, true, true, A>), dim3(hg), dim3(512), 0, st, (const R24*)recB,       \
                     (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out, items_out, dedup ? 1u : 0u,   \
                     (unsigned long long*)dup_count, novf, ovf)
        if (b3 >= 7 && b3 <= 10) {  // phase ablations, outputs not sorted
          if (b3 == 7) KVH_BKAB(11, 1); else if (b3 == 8) KVH_BKAB(11, 2); else if (b3 == 9) KVH_BKAB(11, 3); else KVH_BKAB(11, 4);
        } else
#undef KVH_BKAB
        if (b3 == 5) {  // the round-4 three 8-byte field rounds (A/B)
          if (hd == 10) KVH_BKH(10, false); else if (hd == 12) KVH_BKH(12, false); else KVH_BKH(11, false);
        } else if (b3 == 6) {  // the round-5 W2 form before RK (A/B)
          if (hd == 10) KVH_BKH(10, true); else if (hd == 12) KVH_BKH(12, true); else KVH_BKH(11, true);
        } else if (b3 >= 12 && b3 <= 15) {  // k_bk_sortx phase ablations, outputs not sorted
#define KVH_BKXAB(A)                                                                                                 \
  hipLaunchKernelGGL((k_bk_sortx<3584, 12, 512, A>), dim3(hg), dim3(512), 0, st, (const R24*)recB, (const uint32_t*)cnt, \
                     (const uint32_t*)start, nb, B, g, sb, h_out, items_out, dedup ? 1u : 0u,                         \
                     (unsigned long long*)dup_count, novf, ovf)
          if (b3 == 12) KVH_BKXAB(1); else if (b3 == 13) KVH_BKXAB(2); else if (b3 == 14) KVH_BKXAB(3); else KVH_BKXAB(4);
#undef KVH_BKXAB
        } else if (b3 == 11) {  // the W2 + RK form before the pairs stayed in LDS (A/B)
          if (hd == 10) KVH_BKH2(10); else if (hd == 12) KVH_BKH2(12); else KVH_BKH2(11);
        } else
#endif
        // 12 digit bits by default: shorter runs to rank (4.12 vs 4.24 ms with 11, profiles/r05/finalE/);
        // 81 KiB of LDS, still two workgroups per CU
        if (hd == 10) KVH_BKX(10); else if (hd == 11) KVH_BKX(11); else KVH_BKX(12);
#undef KVH_BKH2
#undef KVH_BKX
#undef KVH_BKH
      }
#ifdef KVH_EXPERIMENTS  // knob 23 = 1 / 2 lost their A/B (round 4): experiments build only
      else if (small_b && b3 == 2)
        hipLaunchKernelGGL((k_bk_sortr2<7168, 11>), dim3(std::min<uint32_t>(nb, 2u * (uint32_t)cus)), dim3(kBkT), 0,
                           st, (const R24*)recB, (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out,
                           items_out, dedup ? 1u : 0u, (unsigned long long*)dup_count, novf, ovf);
      else if (small_b && b3 == 1)
        hipLaunchKernelGGL((k_bk_sortr<7168, 12>), dim3(std::min<uint32_t>(nb, (uint32_t)cus)), dim3(kBkT), 0, st,
                           (const R24*)recB, (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out,
                           items_out, dedup ? 1u : 0u, (unsigned long long*)dup_count, novf, ovf);
#endif
      else if (small_b)
        hipLaunchKernelGGL((k_bk_sort<8000, 12, R24>), dim3(std::min<uint32_t>(nb, 2u * (uint32_t)cus)), dim3(kBkT), 0, st,
                           (const R24*)recB, (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out,
                           items_out, dedup ? 1u : 0u, (unsigned long long*)dup_count, novf, ovf);
      else
      hipLaunchKernelGGL((k_bk_sort<12288, 13, R24>), dim3(std::min<uint32_t>(nb, (uint32_t)cus)), dim3(kBkT), 0, st,
                         (const R24*)recB, (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out,
                         items_out, dedup ? 1u : 0u, (unsigned long long*)dup_count, novf, ovf);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_cvt, dim3(std::min<uint32_t>(nb, (uint32_t)cus * 2)), dim3(kSB), 0, st, (const R24*)recB,
                         (Rec*)(s + L.tw_recA), (const uint32_t*)cnt, (const uint32_t*)start, (const uint32_t*)novf,
                         (const uint32_t*)ovf);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_long, dim3(std::min<uint32_t>(nb, (uint32_t)cus * 2)), dim3(kSB), 0, st,
                         (Rec*)(s + L.tw_recA), (Rec*)(s + L.tw_rec),
                         (const uint32_t*)cnt, (const uint32_t*)start, g, sb, h_out, items_out, dedup ? 1u : 0u,
                         (unsigned long long*)dup_count, (const uint32_t*)novf, (const uint32_t*)ovf);
      return launch_done();
    }
    if (mean_of(B) <= 9000.0) {
      // one pass: LDS-atomic-ranked scatter into 2^B bucket streams (knob 20 = 2; small B)
      const uint32_t nb = 1u << B;
      const uint32_t ntiles = (uint32_t)((n + kBkTile - 1) / kBkTile);
      const uint32_t nch = (ntiles + kBkChunk - 1) / kBkChunk;
      // scratch: records in L.rec; the tile x bucket table in the key areas;
      // chunk sums, bucket sizes, starts and the overflow list in the index areas
      if ((uint64_t)ntiles * nb * 4 > L.idx_in - L.key_in || (uint64_t)nch * nb * 4 > L.idx_out - L.idx_in ||
          (uint64_t)(3 * nb + 1) * 4 > L.rec - L.idx_out)
        return set_err(KVH_EINVAL);  // cannot happen for the B chosen above
      uint32_t* H = (uint32_t*)(s + L.key_in);
      uint32_t* S = (uint32_t*)(s + L.idx_in);
      uint32_t* cnt = (uint32_t*)(s + L.idx_out);
      uint32_t* start = cnt + nb;
      uint32_t* ovf = start + nb;
      uint32_t* novf = ovf + nb;
      const uint32_t cgrid = (uint32_t)(((uint64_t)nch * nb + 255) / 256);
      hipLaunchKernelGGL(k_bk_hist, dim3(ntiles), dim3(kBkT), 0, st, hashes, (uint64_t)n, g, sb, B, H, novf);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_colsum, dim3(cgrid), dim3(256), 0, st, (const uint32_t*)H, ntiles, nb, S);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_colscan, dim3((nb + 255) / 256), dim3(256), 0, st, S, nch, nb, cnt);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(kBkT), 0, st, (const uint32_t*)cnt, nb, start);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_tileoff, dim3(cgrid), dim3(256), 0, st, H, (const uint32_t*)S, (const uint32_t*)start,
                         ntiles, nb);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_scatter, dim3(ntiles), dim3(kBkT), 0, st, hashes, items, (uint64_t)n, g, sb, B,
                         (const uint32_t*)H, rec);
      if ((rc = launch_done())) return rc;
      if (small_b)
        hipLaunchKernelGGL((k_bk_sort<8000, 12>), dim3(std::min<uint32_t>(nb, 2u * (uint32_t)cus)), dim3(kBkT), 0, st,
                           (const Rec*)rec, (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out, items_out,
                           dedup ? 1u : 0u, (unsigned long long*)dup_count, novf, ovf);
      else
      hipLaunchKernelGGL((k_bk_sort<12288, 13>), dim3(std::min<uint32_t>(nb, (uint32_t)cus)), dim3(kBkT), 0, st, (const Rec*)rec,
                         (const uint32_t*)cnt, (const uint32_t*)start, nb, B, g, sb, h_out, items_out,
                         dedup ? 1u : 0u, (unsigned long long*)dup_count, novf, ovf);
      if ((rc = launch_done())) return rc;
      hipLaunchKernelGGL(k_bk_long, dim3(std::min<uint32_t>(nb, (uint32_t)cus * 2)), dim3(kSB), 0, st, rec,
                         (Rec*)nullptr, (const uint32_t*)cnt, (const uint32_t*)start, g, sb, h_out, items_out, dedup ? 1u : 0u,
                         (unsigned long long*)dup_count, (const uint32_t*)novf, (const uint32_t*)ovf);
      return launch_done();
    }
  }
  uint32_t lg = 0;
  while (lg < 63 && (1ull << lg) < (uint64_t)n) lg++;
  uint32_t nb = tsb ? sb + (uint32_t)tsb : std::max(sb + 1, lg + 5);
  if (nb > 64) nb = 64;
  // u32 keys halve the key bytes every radix pass moves (16 instead of 24 per
  // element with the index): used when the prefix fits 31 bits -- all slot
  // bits and as many h1 bits as fit (rocPRIM's merge path, taken for small n,
  // builds its mask as (T(1) << end_bit) - 1: undefined at the type's width)
  const bool k32 = !tsb && sb <= 31;
  if (k32) nb = std::min(nb, 31u);
  const uint32_t lo = 64u - nb;
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

namespace kvh { namespace rt { std::atomic<int> g_tune_sort_bits{0}; std::atomic<int> g_tune_sort_engine{0}; std::atomic<int> g_tune_sort_cap{0}; std::atomic<int> g_tune_sort_b3{3}; std::atomic<int> g_tune_sort_hd{0}; } }

extern "C" {

size_t kvh_ht_sort_scratch_bytes(size_t n) {
  SortLayout L;
  if (sort_layout(n, &L) != 0) return 0;
  return n <= 65536 ? std::max(L.total, refsort_scratch_bytes(n)) : L.total;  // either order
}

int kvh_ht_sort(const uint64_t* hashes, const uint64_t* items, size_t n, const kvh_ht_geom_t* geom,
                uint64_t* hashes_out, uint64_t* items_out, uint64_t* dup_count, uint32_t flags, void* scratch,
                size_t scratch_bytes, void* stream) {
  return sort_impl(hashes, items, n, geom, hashes_out, items_out, dup_count, flags, scratch, scratch_bytes,
                   (hipStream_t)stream);
}

size_t kvh_ht_sort_batched_scratch_bytes(size_t n, uint32_t batch) { return refsort_batched_scratch_bytes(n, batch); }

int kvh_ht_sort_batched(const uint64_t* hashes, const uint64_t* items, size_t n, uint32_t batch,
                        const kvh_ht_geom_t* geom, uint64_t* hashes_out, uint64_t* items_out, uint64_t* dup_counts,
                        uint32_t flags, void* scratch, size_t scratch_bytes, void* stream) {
  if (!geom || (flags & ~(KVH_DEDUP | KVH_REF_ORDER)) || (n && (!hashes || !hashes_out || !scratch)))
    return set_err(KVH_EINVAL);
  return refsort_batched_launch(hashes, items, n, batch, geom, hashes_out, items_out, dup_counts,
                                (flags & KVH_DEDUP) != 0, scratch, scratch_bytes, (hipStream_t)stream);
}

size_t kvh_ht_sort_segments_scratch_bytes(size_t nseg, uint32_t max_seg) {
  return refsort_segments_scratch_bytes(nseg, max_seg);
}

int kvh_ht_sort_segments(const uint64_t* hashes, const uint64_t* items, size_t n, const uint64_t* seg_offs,
                         size_t nseg, uint32_t max_seg, const kvh_ht_geom_t* geom, uint64_t* hashes_out,
                         uint64_t* items_out, uint64_t* dup_counts, uint32_t flags, void* scratch,
                         size_t scratch_bytes, void* stream) {
  if (!geom || (flags & ~(KVH_DEDUP | KVH_REF_ORDER)) || (nseg && n && (!hashes || !hashes_out || !scratch)))
    return set_err(KVH_EINVAL);
  return refsort_segments_launch(hashes, items, n, seg_offs, nseg, max_seg, geom, hashes_out, items_out, dup_counts,
                                 (flags & KVH_DEDUP) != 0, scratch, scratch_bytes, (hipStream_t)stream);
}

// Many kv_ht_radix_sort calls in one launch from host arrays: the batching front end a
// raikv process with several ctest threads would use.  The batches are packed into one pinned staging
// buffer, moved in one H2D copy, sorted by one kvh_ht_sort_segments launch (one workgroup per batch, each
// in the reference's exact element order) and moved back in one D2H copy; each array is then rewritten in
// place.  Staging and device buffers persist per process (grown on demand, under a lock).
namespace {
struct BatchStage {
  std::mutex mu;
  uint8_t *host = nullptr, *dev = nullptr;
  size_t hcap = 0, dcap = 0;
  int device = -1;
};
BatchStage g_bstage;
}  // namespace

int kvh_ht_radix_sort_batch(kvh_ht_sort_t* const* ars, const uint32_t* sizes, uint32_t nbatch,
                            const kvh_ht_geom_t* geom) {
  if (!geom || (nbatch && (!ars || !sizes))) return set_err(KVH_EINVAL);
  size_t n = 0;
  uint32_t maxb = 1;
  for (uint32_t b = 0; b < nbatch; b++) {
    if (sizes[b] > 65536 || (sizes[b] && !ars[b])) return set_err(KVH_EINVAL);
    n += sizes[b];
    maxb = std::max(maxb, sizes[b]);
  }
  if (n == 0) return set_err(0);
  // one layout for host staging and device: pairs, items, segment offsets (the host copy's region),
  // then on the device only the outputs and the sort's scratch
  const size_t off_h = 0, off_i = al256(16 * n), off_g = off_i + al256(8 * n), in_bytes = off_g + al256(8 * (nbatch + 1));
  const size_t sb = kvh_ht_sort_segments_scratch_bytes(nbatch, maxb);
  if (sb == 0) return set_err(KVH_EINVAL);
  const size_t off_ho = in_bytes, off_io = off_ho + al256(16 * n), off_s = off_io + al256(8 * n), dev_bytes = off_s + sb;
  const size_t out_bytes = off_s - off_ho;  // hashes_out + items_out, contiguous
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e);
  std::lock_guard<std::mutex> g(g_bstage.mu);
  if (g_bstage.device != dev) {  // buffers belong to one device
    if (g_bstage.host) (void)hipHostFree(g_bstage.host);
    if (g_bstage.dev) (void)hipFree(g_bstage.dev);
    g_bstage.host = g_bstage.dev = nullptr;
    g_bstage.hcap = g_bstage.dcap = 0;
    g_bstage.device = dev;
  }
  const size_t hneed = std::max(in_bytes, out_bytes);
  if (g_bstage.hcap < hneed) {
    if (g_bstage.host) (void)hipHostFree(g_bstage.host);
    g_bstage.host = nullptr;
    g_bstage.hcap = 0;
    if ((e = hipHostMalloc((void**)&g_bstage.host, hneed, hipHostMallocDefault)) != hipSuccess) return hip_err(e);
    g_bstage.hcap = hneed;
  }
  if (g_bstage.dcap < dev_bytes) {
    if (g_bstage.dev) (void)hipFree(g_bstage.dev);
    g_bstage.dev = nullptr;
    g_bstage.dcap = 0;
    if ((e = hipMalloc((void**)&g_bstage.dev, dev_bytes)) != hipSuccess) return hip_err(e);
    g_bstage.dcap = dev_bytes;
  }
  uint8_t *hs = g_bstage.host, *d = g_bstage.dev;
  uint64_t *hv = (uint64_t*)(hs + off_h), *iv = (uint64_t*)(hs + off_i), *sg = (uint64_t*)(hs + off_g);
  size_t k = 0;
  for (uint32_t b = 0; b < nbatch; b++) {
    sg[b] = k;
    for (uint32_t i = 0; i < sizes[b]; i++, k++) {
      hv[2 * k] = ars[b][i].key;
      hv[2 * k + 1] = ars[b][i].key2;
      iv[k] = (uint64_t)(uintptr_t)ars[b][i].item;
    }
  }
  sg[nbatch] = k;
  hipStream_t st = hipStreamPerThread;
  if ((e = hipMemcpyAsync(d, hs, in_bytes, hipMemcpyHostToDevice, st)) != hipSuccess) return hip_err(e);
  int rc = refsort_segments_launch((const uint64_t*)(d + off_h), (const uint64_t*)(d + off_i), n,
                                   (const uint64_t*)(d + off_g), nbatch, maxb, geom, (uint64_t*)(d + off_ho),
                                   (uint64_t*)(d + off_io), nullptr, false, d + off_s, sb, st);
  if (rc) {
    (void)hipStreamSynchronize(st);
    return rc;
  }
  if ((e = hipMemcpyAsync(hs, d + off_ho, out_bytes, hipMemcpyDeviceToHost, st)) != hipSuccess) return hip_err(e);
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_err(e);
  const uint64_t *ho = (const uint64_t*)hs, *io = (const uint64_t*)(hs + (off_io - off_ho));
  k = 0;
  for (uint32_t b = 0; b < nbatch; b++)
    for (uint32_t i = 0; i < sizes[b]; i++, k++) {
      ars[b][i].key = ho[2 * k];
      ars[b][i].key2 = ho[2 * k + 1];
      ars[b][i].item = (void*)(uintptr_t)io[k];
    }
  return set_err(0);
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
    // up to 64K elements (ctest's batches) in the reference's exact order
    rc = sort_impl((const uint64_t*)(d + off_h), (const uint64_t*)(d + off_i), n, geom, (uint64_t*)(d + off_ho),
                   (uint64_t*)(d + off_io), nullptr, n <= 65536 ? KVH_REF_ORDER : 0u, d + off_s, sb, (hipStream_t)0);
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
