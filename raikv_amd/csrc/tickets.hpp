// tickets.hpp -- in-address-order work assignment for the persistent
// streaming kernels (round 4; fetch order round 5, §4.3.1).
//
// A persistent kernel that hands each wave a static sequence of chunks lets
// the waves drift apart over a launch, and the chip's active address set
// spreads: on MI355X a static-order copy streams 5.2-5.4 TB/s where the same
// copy taking its chunks in address order streams 6.7 (profiles/r04/s4-s5).
// WaveTickets keeps the order without a workgroup barrier per step: the
// workgroup's waves take items one at a time from an LDS counter; the global
// ticket covering items [wpb j, wpb (j + 1)) of the workgroup (wpb = waves per
// workgroup) is fetched from the launch's counter by the wave that takes
// item wpb (j - 2), and published in a 16-slot LDS ring with j + 1 as its tag;
// a slot is rewritten (with ticket j + 16) only after all wpb takers of
// ticket j have read it (per-slot read counts), so a wave that stalls between
// taking its item and reading the ring still reads its own ticket.
//
// Fetch order.  The fetch of ticket j + 2 waits until ticket j + 1 is
// published: the fetches of one workgroup are then issued one after another
// on one address, so the workgroup's global tickets strictly increase with j,
// and so does the item sequence of every wave.  The kernels rely on that: a
// wave whose item lies past the end exits, and every later item of the
// workgroup lies past the end too.  (Round 4 let the fetches of j + 2 and
// j + 3 race: a later ticket could come back below an earlier one, and if the
// earlier one lay past the end, all wpb waves took one of its items and
// exited, leaving the later, in-range chunk unhashed.)  The wait costs nothing
// in steady state: the fetch of j + 1 was issued one whole ticket (wpb chunks)
// earlier.
//
// Ticket words (4 x u64 per (device, stream), rt::stream_tickets):
//   [0] the launch's counter, [1] workgroups done, both zero at launch -- the
//   last workgroup to finish puts them back to zero; [2] test-only delay
//   (kvh_set_tuning knob 26, host-written when the words are made; 0 in
//   production): the fetchers of even tickets in even workgroups sleep
//   (value & 0xffff) x ~4 us before fetching, which reorders unordered fetches
//   deterministically; [3] unused.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kvh {

struct WaveTickets {
  static constexpr int kRing = 16;
  unsigned long long ring[kRing];
  uint32_t tag[kRing];  // ticket index + 1 of the slot's ticket (0: none yet); only grows
  uint32_t rd[kRing];   // reads of the slot so far (wpb per ticket it has held)
  uint32_t lk;          // next item of this workgroup
  uint32_t dbg;         // ticket word 2 (test-only fetch delay)
};

// every thread of the workgroup; ends with a barrier
__device__ __forceinline__ void wt_init(WaveTickets& W, unsigned long long* tk) {
  if (threadIdx.x < WaveTickets::kRing) { W.tag[threadIdx.x] = 0; W.rd[threadIdx.x] = 0; }
  if (threadIdx.x == 0) W.lk = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    W.dbg = (uint32_t)tk[2];
    W.ring[0] = atomicAdd(tk, 1ull);  // one thread, one address: in order
    W.ring[1] = atomicAdd(tk, 1ull);
    W.tag[0] = 1;
    W.tag[1] = 2;
  }
  __syncthreads();
}

// the wave's next global item index (wave-uniform); items are handed out in
// address order across the whole launch, `wpb` per ticket, and each wave's
// items strictly increase
__device__ __forceinline__ uint64_t wt_next(WaveTickets& W, unsigned long long* tk, uint32_t wpb) {
  constexpr int R = WaveTickets::kRing;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t k = 0;
  if (lane == 0) k = atomicAdd(&W.lk, 1u);
  k = __builtin_amdgcn_readfirstlane(k);
  const uint32_t j = k / wpb, s = k - j * wpb;
  if (s == 0 && lane == 0) {  // this ticket's first taker fetches the one two ahead
    const uint32_t jn = j + 2, sl = jn % R;
    const uint32_t dbg = W.dbg;
    if (dbg && !(jn & 1u) && !(blockIdx.x & 1u))  // test-only (knob 26): delay this fetch
      for (uint32_t d = 0; d < (dbg & 0xffffu); d++) __builtin_amdgcn_s_sleep(127);
#ifndef KVH_TICKETS_UNORDERED  // (the unordered form only in a probe build: tools/Makefile target)
    // ticket jn - 1 published first (its fetcher took item wpb (jn - 3), before
    // ours, and waits on nothing later): the fetches of this workgroup are
    // issued in ticket order
    while (__hip_atomic_load(&W.tag[(jn - 1) % R], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < jn)
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
    const unsigned long long g = atomicAdd(tk, 1ull);
    // the slot's previous ticket (jn - R) read by all its takers first; they
    // wait on nothing later than their own ticket, so this wait ends
    if (jn >= (uint32_t)R)
      while (__hip_atomic_load(&W.rd[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (jn / R) * wpb)
        __builtin_amdgcn_s_sleep(1);
    W.ring[sl] = g;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __hip_atomic_store(&W.tag[sl], jn + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  // tags only grow, and the slot keeps ticket j until this wave has read it
  while (__hip_atomic_load(&W.tag[j % R], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < j + 1)
    __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const unsigned long long t = W.ring[j % R];
  if (lane == 0) __hip_atomic_fetch_add(&W.rd[j % R], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  return t * wpb + s;
}

// every thread of the workgroup, after its last wt_next: the last workgroup
// to get here resets the launch's counter pair
__device__ __forceinline__ void wt_done(unsigned long long* tk) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(tk + 1, 1ull) == (unsigned long long)gridDim.x - 1) {
      atomicExch(tk, 0ull);
      atomicExch(tk + 1, 0ull);
    }
  }
}

}  // namespace kvh
