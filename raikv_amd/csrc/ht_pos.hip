// ht_pos.hip -- SURVEY.md §8 row f1: hash-table positions on gfx950.
//
//   k_positions<A,P32,U>        (h1,h2) pairs resident in HBM -> A slots
//                               per key (kvh_ht_positions)
//   k_fixed_pos<L,NT,A,P32,U>   fused: fixed-length keys -> Meow128 ->
//                               KeyFragment fixup -> A slots, optionally
//                               also storing the hashes
//                               (kvh_meow128_fixed_positions)
//
// Both stream their inputs once: per key 16 B in + 8A (or 4A) B out for
// k_positions; L B in + 8A (+16) B out for the fused kernel, which also
// carries the Meow128 LDS T-table work of k_fixed.  The positions math is
// ~40 VALU ops per slot (64-bit multiply, ring distances) and sits far
// below the HBM roofline.  Same wave-chunked access shape as k_fixed (see
// kvh.hip): wave w owns chunks of 64*U consecutive keys, lane l key
// base + 64u + l, so every load and store instruction moves one contiguous
// run; tail indices are clamped to n-1 (benign duplicate stores).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <algorithm>
#include "kvh_internal.hpp"
#include "ht_pos.hpp"
#include "tickets.hpp"
#include "../../include/kvh.h"

using namespace kvh;
using namespace kvh::rt;

namespace {

constexpr int kPosBlock = 256;  // no LDS: small groups, many waves per CU
constexpr int kFusedBlock = 1024;

template <int A, bool P32, typename W>
__device__ __forceinline__ void store_pos(void* __restrict__ pos, uint64_t idx, const W (&q)[A]) {
  if constexpr (P32) {
    uint32_t* p = (uint32_t*)pos + idx * A;
    if constexpr (A % 4 == 0) {
#pragma unroll
      for (int i = 0; i < A; i += 4) {
        v4u v;
        v.x = (uint32_t)q[i]; v.y = (uint32_t)q[i + 1]; v.z = (uint32_t)q[i + 2]; v.w = (uint32_t)q[i + 3];
        __builtin_nontemporal_store(v, (v4u*)(p + i));
      }
    } else if constexpr (A % 2 == 0) {
#pragma unroll
      for (int i = 0; i < A; i += 2) {
        v2u v;
        v.x = (uint32_t)q[i]; v.y = (uint32_t)q[i + 1];
        __builtin_nontemporal_store(v, (v2u*)(p + i));
      }
    } else {
#pragma unroll
      for (int i = 0; i < A; i++) __builtin_nontemporal_store((uint32_t)q[i], p + i);
    }
  } else {
    uint32_t* p = (uint32_t*)((uint64_t*)pos + idx * A);
    if constexpr (A % 2 == 0) {
#pragma unroll
      for (int i = 0; i < A; i += 2) {
        v4u v;
        v.x = (uint32_t)q[i]; v.y = (uint32_t)((uint64_t)q[i] >> 32);
        v.z = (uint32_t)q[i + 1]; v.w = (uint32_t)((uint64_t)q[i + 1] >> 32);
        __builtin_nontemporal_store(v, (v4u*)(p + 2 * i));
      }
    } else {
#pragma unroll
      for (int i = 0; i < A; i++) {
        v2u v;
        v.x = (uint32_t)q[i]; v.y = (uint32_t)((uint64_t)q[i] >> 32);
        __builtin_nontemporal_store(v, (v2u*)(p + 2 * i));
      }
    }
  }
}

// 32-byte position records (A = 4 u64, or A = 8 u32): one lane per key
// would store each record as two 16-byte pieces 32 bytes apart, so every
// store instruction half-fills the lines it touches (the write traffic
// inflates, as measured for the multi-seed kernel).  Instead lane 2m owns
// key m and lane 2m+1 key 32+m of the 64-key chunk; adjacent lanes swap one
// half through a DPP quad permute, after which store 0 writes keys 0..31
// and store 1 keys 32..63, each one contiguous 1 KiB run.
template <int A, bool P32>
constexpr bool kPairRec = A * (P32 ? 4 : 8) == 32;

__device__ __forceinline__ uint64_t chunk_key(uint64_t lane, bool pair) {
  return pair ? (lane >> 1) + 32 * (lane & 1) : lane;
}

template <int A, bool P32, typename W>
__device__ __forceinline__ void store_pos_pair(void* __restrict__ pos, uint64_t base, uint64_t lane, uint64_t last,
                                               const W (&q)[A]) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < A; i++) {
    if constexpr (P32) {
      w[i] = (uint32_t)q[i];
    } else {
      w[2 * i] = (uint32_t)q[i];
      w[2 * i + 1] = (uint32_t)((uint64_t)q[i] >> 32);
    }
  }
  const bool even = (lane & 1) == 0;
  uint32_t y[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t x = even ? w[4 + c] : w[c];
    y[c] = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  }
  v4u s0, s1;
  s0.x = even ? w[0] : y[0]; s0.y = even ? w[1] : y[1]; s0.z = even ? w[2] : y[2]; s0.w = even ? w[3] : y[3];
  s1.x = even ? y[0] : w[4]; s1.y = even ? y[1] : w[5]; s1.z = even ? y[2] : w[6]; s1.w = even ? y[3] : w[7];
  v4u* p = (v4u*)((uint8_t*)pos + base * 32) + lane;
  if (base + (lane >> 1) <= last) __builtin_nontemporal_store(s0, p);
  if (base + 32 + (lane >> 1) <= last) __builtin_nontemporal_store(s1, p + 64);
}

template <int A, bool P32, typename W, int U>
__global__ void __launch_bounds__(kPosBlock)
k_positions(const uint64_t* __restrict__ hashes, uint64_t n, HtGeom g, void* __restrict__ pos) {
  constexpr bool PAIR = kPairRec<A, P32>;
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t step = (((uint64_t)gridDim.x * blockDim.x) >> 6) * 64 * U;
  const uint64_t last = n - 1;
  const uint64_t kofs = chunk_key(lane, PAIR);
  for (uint64_t b = wave * 64 * U; b < n; b += step) {
    v4u h[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = std::min<uint64_t>(b + 64 * u + kofs, last);
      h[u] = __builtin_nontemporal_load((const v4u*)(hashes + 2 * j));
    }
    __builtin_amdgcn_sched_barrier(0);  // keep all U loads in flight before the first use
#pragma unroll
    for (int u = 0; u < U; u++) {
      W q[A];
      cuckoo_positions<A, W>(g, (uint64_t)h[u].x | ((uint64_t)h[u].y << 32),
                             (uint64_t)h[u].z | ((uint64_t)h[u].w << 32), q);
      if constexpr (PAIR)
        store_pos_pair<A, P32, W>(pos, b + 64 * u, lane, last, q);
      else
        store_pos<A, P32, W>(pos, std::min<uint64_t>(b + 64 * u + kofs, last), q);
    }
  }
}

// Fused epilogue on k_fixed's body (kvh.hip): the hash is fixed up
// (KeyFragment::hash, hash_entry.h:84-85) because KeyCtx::set_key_hash
// feeds the fixed-up h1 to ht_mod (key_ctx.cpp:97-105).
template <int L, int NT, int A, bool P32, typename W, int U, bool Q = false>
__global__ void __launch_bounds__(kFusedBlock)
k_fixed_pos(const uint8_t* __restrict__ keys, uint64_t n, uint64_t s1, uint64_t s2, HtGeom g,
            uint64_t* __restrict__ out, void* __restrict__ pos, unsigned long long* __restrict__ tk = nullptr) {
  constexpr int NC = Plan<L>::NC;
  // one LDS object, tables first; Q: chunks in address order through wave tickets (knob 24, tickets.hpp)
  struct Smem { uint32_t tab[LdsTab<NT>::kWords]; WaveTickets Wt; };
  __shared__ Smem sm;
  uint32_t* lds = sm.tab;
  fill_tables<NT>(lds);
  __syncthreads();
  if constexpr (Q) wt_init(sm.Wt, tk);
  const LdsTab<NT> T(lds);
  const MeowConst K = uniform(make_const(s1, s2, (uint64_t)L, T));
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t step = (((uint64_t)gridDim.x * blockDim.x) >> 6) * 64 * U;
  const uint64_t last = n - 1;
  const bool keep = out != nullptr;
  constexpr bool PAIR = kPairRec<A, P32>;
  const uint64_t kofs = chunk_key(lane, PAIR);
  for (uint64_t b = Q ? wt_next(sm.Wt, tk, blockDim.x >> 6) * (64 * U) : wave * 64 * U; b < n;
       b = Q ? wt_next(sm.Wt, tk, blockDim.x >> 6) * (64 * U) : b + step) {
    Blk D[U][NC];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = std::min<uint64_t>(b + 64 * u + kofs, last);
      load_fixed<L, true, true>(keys + j * L, D[u]);
    }
    Blk h[U];
#pragma unroll
    for (int u = 0; u < U; u++) h[u] = fixup(meow_ct<L>(D[u], K, T));
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = std::min<uint64_t>(b + 64 * u + kofs, last);
      if (keep) store_h<true>(out, j, h[u], false);
      W q[A];
      cuckoo_positions<A, W>(g, (uint64_t)h[u].w[0] | ((uint64_t)h[u].w[1] << 32),
                             (uint64_t)h[u].w[2] | ((uint64_t)h[u].w[3] << 32), q);
      if constexpr (PAIR)
        store_pos_pair<A, P32, W>(pos, b + 64 * u, lane, last, q);
      else
        store_pos<A, P32, W>(pos, j, q);
    }
  }
  if constexpr (Q) wt_done(tk);
}

// ------------------------------------------------------------ host side
uint32_t per_key(const kvh_ht_geom_t* g) {
  return (g->cuckoo_arity > 1 && g->cuckoo_buckets > 1) ? g->cuckoo_arity : 1;
}

// A geometry the kernels can serve: the ht_mod range covers more than half
// the table (ht_init.cpp:139-150 guarantees it), and the slots left after
// A-1 earlier picks (each excluding a 2*buckets-1 ring window and its
// 13-bit index class) are non-empty, so the rejection loop terminates.
int check_geom(const kvh_ht_geom_t* g, bool p32) {
  if (!g || g->ht_size == 0 || g->ht_mod_shift >= 64 || g->ht_mod_fraction == 0 ||
      g->ht_mod_fraction >= (1ull << 32))
    return KVH_EINVAL;
  const uint64_t top = (g->ht_mod_mask * g->ht_mod_fraction) >> g->ht_mod_shift;
  if (top >= g->ht_size) return KVH_EINVAL;  // ht_mod must stay inside ht[]
  if (p32 && g->ht_size > (1ull << 32)) return KVH_EINVAL;
  const uint32_t a = per_key(g);
  if (a > KVH_MAX_ARITY) return KVH_EINVAL;
  if (a > 1) {
    const double reach = (double)top / 2.0;
    const double bar = (double)(a - 1) * ((2.0 * g->cuckoo_buckets - 1.0) + (double)g->ht_size / 8192.0 + 1.0);
    if (!(reach > bar)) return KVH_EINVAL;
  }
  return 0;
}

HtGeom dev_geom(const kvh_ht_geom_t* g) {
  HtGeom d;
  d.size = g->ht_size;
  d.mask = g->ht_mod_mask;
  d.frac = (uint32_t)g->ht_mod_fraction;
  d.shift = g->ht_mod_shift;
  d.buckets = g->cuckoo_buckets;
  return d;
}

bool narrow(const HtGeom& g) { return g.mask < (1ull << 32) && g.size < (1ull << 32); }

template <int A, bool P32>
void launch_positions(const uint64_t* h, uint64_t n, HtGeom g, void* pos, hipStream_t st, int cus) {
  constexpr int U = 4;
  const uint64_t need = (n + kPosBlock * U - 1) / (kPosBlock * U);
  // no LDS to fill, so the in-address-order form is simply a one-shot grid
  // (the dispatcher hands blocks out in order); knob 24 = 1
  // restores the persistent grid of 8 blocks per CU
  const uint64_t grid = std::max<uint64_t>(
      1, knob(g_tune_order) == 1 ? std::min<uint64_t>(need, (uint64_t)cus * 8) : std::min<uint64_t>(need, 1u << 30));
  if (narrow(g))
    hipLaunchKernelGGL((k_positions<A, P32, uint32_t, U>), dim3((uint32_t)grid), dim3(kPosBlock), 0, st, h, n, g,
                       pos);
  else if constexpr (!P32)  // wide tables have no u32 output (check_geom)
    hipLaunchKernelGGL((k_positions<A, P32, uint64_t, U>), dim3((uint32_t)grid), dim3(kPosBlock), 0, st, h, n, g,
                       pos);
}

template <bool P32>
int positions_a(uint32_t a, const uint64_t* h, uint64_t n, HtGeom g, void* pos, hipStream_t st, int cus) {
  switch (a) {
    case 1: launch_positions<1, P32>(h, n, g, pos, st, cus); break;
    case 2: launch_positions<2, P32>(h, n, g, pos, st, cus); break;
    case 3: launch_positions<3, P32>(h, n, g, pos, st, cus); break;
    case 4: launch_positions<4, P32>(h, n, g, pos, st, cus); break;
    case 5: launch_positions<5, P32>(h, n, g, pos, st, cus); break;
    case 6: launch_positions<6, P32>(h, n, g, pos, st, cus); break;
    case 7: launch_positions<7, P32>(h, n, g, pos, st, cus); break;
    case 8: launch_positions<8, P32>(h, n, g, pos, st, cus); break;
    default: return set_err(KVH_EINVAL);
  }
  return launch_done();
}

template <int L, int A, bool P32>
int launch_fused(const uint8_t* k, uint64_t n, uint64_t s1, uint64_t s2, HtGeom g, uint64_t* out, void* pos,
                 hipStream_t st, int cus) {
  constexpr int NT = 2, U = 2;
  const uint64_t need = (n + kFusedBlock - 1) / kFusedBlock;
  const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(need, (uint64_t)cus * 2));
  // chunk order (knob 24): wave tickets (in address order) unless 1 = static
  unsigned long long* tk = nullptr;
  if (knob(g_tune_order) != 1)
    if (int rc = stream_tickets(st, &tk)) return rc;
  const bool q = tk != nullptr;  // no words for a captured launch: the static order
#define KVH_FP(Wt, Qv) hipLaunchKernelGGL((k_fixed_pos<L, NT, A, P32, Wt, U, Qv>), dim3((uint32_t)grid), \
                                          dim3(kFusedBlock), 0, st, k, n, s1, s2, g, out, pos, tk)
  if (narrow(g)) {
    if (q) KVH_FP(uint32_t, true); else KVH_FP(uint32_t, false);
  } else if constexpr (!P32) {
    if (q) KVH_FP(uint64_t, true); else KVH_FP(uint64_t, false);
  }
#undef KVH_FP
  return 0;
}

template <int L, bool P32>
int fused_a(uint32_t a, const uint8_t* k, uint64_t n, uint64_t s1, uint64_t s2, HtGeom g, uint64_t* out,
            void* pos, hipStream_t st, int cus) {
  int rc = 0;
  switch (a) {
    case 1: rc = launch_fused<L, 1, P32>(k, n, s1, s2, g, out, pos, st, cus); break;
    case 2: rc = launch_fused<L, 2, P32>(k, n, s1, s2, g, out, pos, st, cus); break;
    case 4: rc = launch_fused<L, 4, P32>(k, n, s1, s2, g, out, pos, st, cus); break;
    case 8: rc = launch_fused<L, 8, P32>(k, n, s1, s2, g, out, pos, st, cus); break;
    default: return set_err(KVH_EINVAL);
  }
  if (rc) return rc;
  return launch_done();
}

bool fused_ok(uint32_t key_len, uint32_t a, const void* keys) {
  return (key_len == 16 || key_len == 32) && (a == 1 || a == 2 || a == 4 || a == 8) &&
         ((uintptr_t)keys & 15) == 0;
}

}  // namespace

extern "C" {

int kvh_ht_geom_init(uint64_t map_size, uint32_t hash_entry_size, float hash_value_ratio,
                     uint16_t cuckoo_buckets, uint8_t cuckoo_arity, kvh_ht_geom_t* geom) {
  // HashTab::initialize, src/ht_init.cpp:117-156 (header regions:
  // include/raikv/shm_ht.h:59-69, 192K + 128K + 128K)
  const uint64_t hdr = (192ull + 128ull + 128ull) * 1024ull;
  if (!geom || map_size <= hdr || hash_entry_size == 0 || !(hash_value_ratio > 0.0f))
    return set_err(KVH_EINVAL);
  const uint64_t area = map_size - hdr;
  const uint64_t entries = (uint64_t)((double)hash_value_ratio * (double)area) / (uint64_t)hash_entry_size;
  if (entries == 0) return set_err(KVH_EINVAL);
  uint32_t bits = 1;
  while (bits < 63 && (1ull << bits) < entries) bits++;
  const uint64_t mask = (1ull << bits) - 1;
  uint64_t frac = 0, top = 0;
  uint32_t shift = 30;
  for (; shift > 1; shift--) {
    frac = (uint64_t)(((double)entries / (double)mask) * (double)(1ull << shift));
    top = (mask * frac) >> shift;
    if (top > entries / 2) {
      if (top == entries) frac--;
      break;
    }
  }
  geom->ht_size = entries;
  geom->ht_mod_mask = mask;
  geom->ht_mod_fraction = frac;
  geom->ht_mod_shift = shift;
  geom->cuckoo_buckets = cuckoo_buckets;
  geom->cuckoo_arity = cuckoo_arity;
  geom->pad = 0;
  return set_err(0);
}

uint32_t kvh_positions_per_key(const kvh_ht_geom_t* geom) { return geom ? per_key(geom) : 0; }

int kvh_ht_positions(const uint64_t* hashes, size_t n, const kvh_ht_geom_t* geom, void* pos, uint32_t flags,
                     void* stream) {
  const bool p32 = (flags & KVH_POS32) != 0;
  int rc = check_geom(geom, p32);
  if (rc) return set_err(rc);
  if (n == 0) return set_err(0);
  if (!hashes || !pos || ((uintptr_t)hashes & 15) || ((uintptr_t)pos & 15)) return set_err(KVH_EINVAL);
  int cus = 0;
  rc = device_cus(&cus);
  if (rc) return rc;
  const HtGeom g = dev_geom(geom);
  const uint32_t a = per_key(geom);
  hipStream_t st = (hipStream_t)stream;
  return p32 ? positions_a<true>(a, hashes, n, g, pos, st, cus) : positions_a<false>(a, hashes, n, g, pos, st, cus);
}

int kvh_meow128_fixed_positions(const void* keys, uint32_t key_len, size_t n, uint64_t seed1, uint64_t seed2,
                                const kvh_ht_geom_t* geom, uint64_t* hashes, void* pos, uint32_t flags,
                                void* stream) {
  const bool p32 = (flags & KVH_POS32) != 0;
  int rc = check_geom(geom, p32);
  if (rc) return set_err(rc);
  if (n == 0) return set_err(0);
  if (!keys || !pos || ((uintptr_t)pos & 15) || (hashes && ((uintptr_t)hashes & 15))) return set_err(KVH_EINVAL);
  int cus = 0;
  rc = device_cus(&cus);
  if (rc) return rc;
  const HtGeom g = dev_geom(geom);
  const uint32_t a = per_key(geom);
  hipStream_t st = (hipStream_t)stream;
  const uint8_t* k = (const uint8_t*)keys;
  if (fused_ok(key_len, a, keys)) {
    if (key_len == 16)
      return p32 ? fused_a<16, true>(a, k, n, seed1, seed2, g, hashes, pos, st, cus)
                 : fused_a<16, false>(a, k, n, seed1, seed2, g, hashes, pos, st, cus);
    return p32 ? fused_a<32, true>(a, k, n, seed1, seed2, g, hashes, pos, st, cus)
               : fused_a<32, false>(a, k, n, seed1, seed2, g, hashes, pos, st, cus);
  }
  // two passes: hash kernel (any length), then the positions kernel
  uint64_t* h = hashes;
  if (!h) {
    hipError_t e = hipMallocAsync((void**)&h, 16 * n, st);
    if (e != hipSuccess) return hip_err(e);
  }
  rc = kvh_meow128_fixed(keys, key_len, n, seed1, seed2, h, KVH_FIXUP, stream);
  if (rc == 0)
    rc = p32 ? positions_a<true>(a, h, n, g, pos, st, cus) : positions_a<false>(a, h, n, g, pos, st, cus);
  if (!hashes) {
    hipError_t e = hipFreeAsync(h, st);
    if (rc == 0 && e != hipSuccess) rc = hip_err(e);
  }
  return rc ? rc : set_err(0);
}

}  // extern "C"
