/*
 * kvh.h -- C-ABI of the MI355X (gfx950) batched key-hash engine: raikv's
 * 128-bit Meow-derived AES-round key hash (kv_hash_meow128 and family) as
 * hand-written HIP kernels.
 *
 * Plain C: no HIP, torch or C++ types in any signature.  `stream` is a
 * hipStream_t passed as void* (NULL = the null stream).  Device entry points
 * are asynchronous on `stream`; caller owns every buffer; nothing is
 * allocated in a hot call.
 *
 * Semantics follow the reference (/root/reference):
 *   - (h1,h2) are "the seed and the hash result" (include/raikv/key_hash.h:41)
 *   - batch outputs interleave (h1,h2) per key exactly like the reference's
 *     x[] arrays of the x2/x4/x8 variants (key_hash.c:1657-2020)
 *   - KVH_FIXUP applies KeyFragment::hash's epilogue to h1
 *     (include/raikv/hash_entry.h:84-85): clear bit 63, 0/1 -> 2.
 *
 * Error convention (new: the reference has no error path, key_hash.h
 * functions are void): 0 on success, negative on failure; HIP runtime
 * errors are returned as KVH_EHIP_BASE - hipError_t.
 */
#ifndef KVH_H
#define KVH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KVH_OK          0
#define KVH_EINVAL    (-22)
#define KVH_ENOMEM    (-12)
#define KVH_ENODEV    (-19)
#define KVH_EHIP_BASE (-1000)

/* flags */
#define KVH_FIXUP     0x1u  /* KeyFragment::hash epilogue on h1 (hash_entry.h:84-85) */

#define KVH_MAX_ARITY 8

/* ---------------------------------------------------------------------
 * Batched device entry points (the hot path).  keys/offsets/out are device
 * pointers (hipMalloc'd or host-registered).  Output layout is
 * out[(i*arity + a)*2 + 0] = h1, [.. + 1] = h2.
 * ------------------------------------------------------------------- */

/* n keys of key_len bytes packed at stride key_len.  Replaces n calls of
 * kv_hash_meow128(p + i*key_len, key_len, &h1, &h2) with h1,h2 = seed1,seed2
 * (reference key_hash.c:1413-1429, key_hash.h:61) and generalises
 * kv_hash_meow128_{2,4,8}_same_length (key_hash.c:1657, :1846, :1946). */
int kvh_meow128_fixed(const void *keys, uint32_t key_len, size_t n,
                      uint64_t seed1, uint64_t seed2, uint64_t *out,
                      uint32_t flags, void *stream);

/* n variable-length keys, key i = keys[offsets[i] .. offsets[i+1]) with
 * 64-bit offsets (n+1 entries, non-decreasing).  Generalises
 * kv_hash_meow128_{2,4}_diff_length (key_hash.c:1685, :1740). */
int kvh_meow128_var(const void *keys, const uint64_t *offsets, size_t n,
                    uint64_t seed1, uint64_t seed2, uint64_t *out,
                    uint32_t flags, void *stream);

/* Each key hashed under `arity` seeds (seeds = HOST array of 2*arity
 * words, seed k = (seeds[2k], seeds[2k+1])).  With arity 4 this is the
 * reference's kv_hash_meow128_4_same_length_4_seed with one key in all four
 * slots (key_hash.c:1891-1937); it feeds cuckoo slotting (config C3). */
int kvh_meow128_multiseed(const void *keys, uint32_t key_len, size_t n,
                          const uint64_t *seeds, uint32_t arity,
                          uint64_t *out, uint32_t flags, void *stream);

/* One entry point for all of the above (SURVEY.md §8 b): offsets == NULL
 * selects fixed length `fixed_len`; arity > 1 requires offsets == NULL. */
int kvh_meow128_batch(const void *keys, const uint64_t *offsets,
                      uint32_t fixed_len, size_t n, const uint64_t *seeds,
                      uint32_t arity, uint64_t *out, uint32_t flags,
                      void *stream);

/* Device-resident batch through the straight-line (unfolded) restatement
 * with per-key seeds (seeds = DEVICE array, 2 words per key); this is the
 * kernel behind the host drop-ins below and the x2/x4/x8 variants. */
int kvh_meow128_var_seeded(const void *keys, const uint64_t *offsets,
                           size_t n, const uint64_t *seeds, uint64_t *out,
                           uint32_t flags, void *stream);

/* ---------------------------------------------------------------------
 * Host-buffer pipeline: keys and out in (pageable or pinned) host memory;
 * chunked H2D -> kernel -> D2H on the current device, one stream per
 * direction so both PCIe directions run at once.  Synchronous.  This is the
 * PCIe-inclusive path (keys arrive from a socket / shm segment, hashes feed
 * the cuckoo probe).  Pinned buffers from kvh_host_alloc (or a range
 * page-locked by kvh_host_register whose first and last byte are) are
 * DMA'd directly; pageable ones go through pinned bounce buffers (about
 * half the rate).  Batches of <= 16384 keys and 512 KiB (knob 21) are
 * copied into a coherent pinned buffer that one kernel reads and writes
 * across PCIe (no DMA, ~15 us per call).  Below ~16-32K 16-byte keys per call one CPU core
 * running the reference hash is faster.
 * ------------------------------------------------------------------- */
int kvh_meow128_fixed_host(const void *keys, uint32_t key_len, size_t n,
                           uint64_t seed1, uint64_t seed2, uint64_t *out,
                           uint32_t flags);
/* Variable-length keys in host memory (socket / shm-segment keys: EvKeyCtx
 * key buffers, include/raikv/ev_key.h:83-114; ctest's frag stream,
 * test/ctest.c:202-233): key i = keys[offsets[i] .. offsets[i+1]), n+1 host
 * u64 offsets (offsets[0] need not be 0).  Chunks of at most 16 MiB of key
 * bytes (knob 15; a longer key is a chunk of its own), offsets and hashes
 * DMA'd with them; out[2n] receives the hashes (global layout).  Same
 * result as kvh_meow128_var on device copies of the buffers. */
int kvh_meow128_var_host(const void *keys, const uint64_t *offsets, size_t n,
                         uint64_t seed1, uint64_t seed2, uint64_t *out,
                         uint32_t flags);
/* The two above sharded over ndev GPUs of this process, one host thread
 * per entry of devices[] (a device may be listed more than once): equal
 * index ranges (fixed) or ranges of equal key bytes (variable), each
 * device writing its disjoint slice of out.  Keys are independent: no
 * device-to-device traffic (the one-process shape of raikv's threads,
 * test/test.cpp:682, test/ctest.c:395).  Synchronous; 0 or the first
 * error of any shard. */
int kvh_meow128_fixed_host_multi(const void *keys, uint32_t key_len, size_t n,
                                 uint64_t seed1, uint64_t seed2, uint64_t *out,
                                 uint32_t flags, const int *devices, int ndev);
int kvh_meow128_var_host_multi(const void *keys, const uint64_t *offsets,
                               size_t n, uint64_t seed1, uint64_t seed2,
                               uint64_t *out, uint32_t flags,
                               const int *devices, int ndev);
/* The shard arithmetic of the _multi entries (host only, no device call):
 * bounds[0..nshards], shard d = keys [bounds[d], bounds[d+1]).  offsets ==
 * NULL: equal index ranges; else n+1 offsets and ranges of equal key bytes
 * (each shard starts at the first key whose offset is >= offsets[0] +
 * total * d / nshards).  For callers that drive their own devices. */
int kvh_shard_bounds(const uint64_t *offsets, size_t n, int nshards,
                     size_t *bounds);
/* Page-lock an existing host range (e.g. raikv's shared-memory segment,
 * include/raikv/shm_ht.h:23-29) so the pipelines above DMA it directly.
 * RULE (a HIP runtime defect on this ROCm stack, reproduced without this
 * library: DESIGN.md §4.4, tools/copy_fault_stress.py,
 * tools/heap_reuse_probe.py): register long-lived memory (the shm segment,
 * a mapping of your own) and keep it mapped after kvh_host_unregister until
 * the process ends.  Do NOT register and unregister transient heap
 * (malloc / numpy) buffers in a process that also makes its own pageable
 * hipMemcpy calls of more than ~1 MiB: once those pages come back from the
 * heap as the buffer of such a copy, the runtime's locked-user-page copy
 * can raise hipErrorIllegalAddress (about 1 in 1,500 such copies in the
 * reproduction).  And do not hand the runtime a pageable copy whose range is
 * registered only in part: it can return wrong bytes with no error.  The
 * pipelines of this library never do either (a range that is not pinned
 * from its first to its last byte goes through their own pinned bounce
 * buffers). */
int kvh_host_register(void *p, size_t bytes);
int kvh_host_unregister(void *p);
/* pinned (page-locked, DMA-able) host memory for kvh_meow128_fixed_host's
 * key and hash buffers -- the role of raikv's shared-memory segment on the
 * GPU side; 0 or a negative error.  Free with kvh_host_free. */
int kvh_host_alloc(void **p, size_t bytes);
int kvh_host_free(void *p);
/* Device memory on the current GPU (scratch for kvh_ht_sort / kvh_tokenize
 * from hosts that do not link the HIP runtime themselves); 0 or a negative
 * error.  Free with kvh_device_free. */
int kvh_device_alloc(void **p, size_t bytes);
int kvh_device_free(void *p);

/* ---------------------------------------------------------------------
 * Drop-ins for include/raikv/key_hash.h (host pointers, synchronous).  They
 * execute on the current GPU through kvh_meow128_var_seeded; results are
 * bit-identical to the reference.  Return 0 or a negative error.
 *
 * LATENCY: each call is a host->device copy, a kernel and a device->host
 * copy, serialised behind one staging buffer: tens of microseconds per call
 * against the reference CPU's 5-20 ns per key.  They exist for API
 * completeness and for tests; never call them per key in a hot loop (e.g.
 * KeyCtx::set_key_hash, key_ctx.cpp:98-105).  Batch instead: hash a socket
 * or shm batch with kvh_meow128_fixed_host / kvh_meow128_var_host (or the
 * device entries) and hand each (h1, h2) to KeyCtx::set_hash
 * (key_ctx.h:188-192), INTEGRATION.md §3.
 * ------------------------------------------------------------------- */
/* key_hash.h:61 kv_hash_meow128 */
int kvh_hash_meow128(const void *p, size_t sz, uint64_t *h1, uint64_t *h2);
/* key_hash.h:60 kv_hash_meow64 (returns h1; errors via kvh_last_error) */
uint64_t kvh_hash_meow64(const void *p, size_t sz, uint64_t seed);
/* key_hash.h:104-105 */
int kvh_hash_meow128_2_same_length(const void *p, const void *p2, size_t sz,
                                   uint64_t *x4);
/* key_hash.h:106 */
int kvh_hash_meow128_4_same_length_a(const void **p, size_t sz, uint64_t *x);
/* key_hash.h:107 */
int kvh_hash_meow128_8_same_length_a(const void **p, size_t sz, uint64_t *x);
/* key_hash.h:108-110 */
int kvh_hash_meow128_4_same_length(const void *p, const void *p2,
                                   const void *p3, const void *p4, size_t sz,
                                   uint64_t *x);
/* key_hash.h:112-114 */
int kvh_hash_meow128_4_same_length_4_seed(const void *p, const void *p2,
                                          const void *p3, const void *p4,
                                          size_t sz, uint64_t *x);
/* key_hash.h:115-119 */
int kvh_hash_meow128_8_same_length(const void *p, const void *p2,
                                   const void *p3, const void *p4,
                                   const void *p5, const void *p6,
                                   const void *p7, const void *p8, size_t sz,
                                   uint64_t *x);
/* key_hash.h:120-121 */
int kvh_hash_meow128_2_diff_length(const void *p, size_t sz, const void *p2,
                                   size_t sz2, uint64_t *x);
/* key_hash.h:122-124 */
int kvh_hash_meow128_4_diff_length(const void *p, size_t sz, const void *p2,
                                   size_t sz2, const void *p3, size_t sz3,
                                   const void *p4, size_t sz4, uint64_t *x);

/* key_hash.h:85-92 meow_vec_t / kv_hash_meow128_vec */
typedef struct {
  const void *p;
  size_t      sz;
} kvh_meow_vec_t;
int kvh_hash_meow128_vec(const kvh_meow_vec_t *vec, size_t vec_sz,
                         uint64_t *h1, uint64_t *h2);

/* key_hash.h:67-83, :93-99 streaming hash; same layout as meow_ctx_t /
 * meow_block_t.  total_update_sz must be known at init (the Mixer uses it). */
typedef struct {
  uint64_t ctx[8];
} kvh_meow_ctx_t __attribute__((__aligned__(64)));
typedef struct {
  uint8_t block[64];
  size_t  off, total_update_sz;
} kvh_meow_block_t __attribute__((__aligned__(64)));

int kvh_meow128_init(kvh_meow_ctx_t *m, kvh_meow_block_t *b, uint64_t k1,
                     uint64_t k2, size_t total_update_sz);
int kvh_meow128_update(kvh_meow_ctx_t *m, kvh_meow_block_t *b, const void *p,
                       size_t sz);
int kvh_meow128_final(kvh_meow_ctx_t *m, kvh_meow_block_t *b, uint64_t *k1,
                      uint64_t *k2);
/* key_hash.c:1570-1579 kv_meow_test: streaming == one-shot */
int kvh_meow_test(const void *p, size_t sz, uint64_t *k1, uint64_t *k2);

/* ---------------------------------------------------------------------
 * Key fragments (include/raikv/hash_entry.h:28-36, key_ctx.cpp:1737-1783).
 * kvh_key_frag_t is layout-identical to kv_key_frag_t (u16 keylen + bytes).
 * ------------------------------------------------------------------- */
typedef struct {
  uint16_t keylen;
  char     buf[4]; /* keylen bytes follow in place, like kv_key_frag_s */
} kvh_key_frag_t;

/* KeyFragment::hash with a HashSeed (shm_ht.h:338-341, hash_entry.h:80-86):
 * seed in (seed[0], seed[1]) -> fixed-up (k, k2).  kv_hash_key_frag
 * (key_ctx.cpp:1774-1783) is this with the db-0 seed of the table. */
int kvh_hash_key_frag(const uint64_t seed[2], const kvh_key_frag_t *frag,
                      uint64_t *k, uint64_t *k2);
/* Batch form for a ctest-style pipeline (test/ctest.c:76-104): n fragments
 * (host pointers) hashed with one seed, fixed-up, into out[2n]. */
int kvh_hash_key_frags(const uint64_t seed[2], const kvh_key_frag_t *const *frags,
                       size_t n, uint64_t *out);

/* ---------------------------------------------------------------------
 * Table positions: what KeyCtx probes for a key hash.
 *   home slot  FileHdr::ht_mod, include/raikv/shm_ht.h:181-184
 *   cuckoo     CuckooAltHash::calc_hash, src/ht_cuckoo.cpp:38-79
 *              (called with start = ht_mod(h1), ht_cuckoo.cpp:374-398,
 *              key_ctx.cpp:89-94)
 * kvh_ht_geom_t carries the FileHdr fields those read (shm_ht.h:143-157);
 * a maintainer fills it from ht->hdr directly or via kvh_ht_geom_init.
 * Positions per key: cuckoo_arity when cuckoo_buckets > 1 and arity > 1
 * (pos[0] = home slot, pos[k] = CuckooAltHash::pos[k]), else 1 (the
 * linear-probe start slot, key_ctx.cpp:130).  Output layout
 * pos[i * per_key + k], u64 (u32 with KVH_POS32).  hashes are (h1,h2)
 * pairs already fixed up as KeyFragment::hash leaves them.
 * ------------------------------------------------------------------- */
#define KVH_POS32     0x2u  /* store positions as u32 (ht_size <= 2^32) */

typedef struct {
  uint64_t ht_size;         /* FileHdr::ht_size          shm_ht.h:143 */
  uint64_t ht_mod_mask;     /* FileHdr::ht_mod_mask      shm_ht.h:146 */
  uint64_t ht_mod_fraction; /* FileHdr::ht_mod_fraction  shm_ht.h:147 */
  uint32_t ht_mod_shift;    /* FileHdr::ht_mod_shift     shm_ht.h:156 */
  uint16_t cuckoo_buckets;  /* FileHdr::cuckoo_buckets   shm_ht.h:153 */
  uint8_t  cuckoo_arity;    /* FileHdr::cuckoo_arity     shm_ht.h:157 */
  uint8_t  pad;
} kvh_ht_geom_t;

/* HashTab::initialize's geometry (src/ht_init.cpp:117-156) for a map of
 * map_size bytes: same ht_size / mask / fraction / shift as the reference
 * (kv_geom_t fields, shm_ht.h:14-21).  Host only. */
int kvh_ht_geom_init(uint64_t map_size, uint32_t hash_entry_size,
                     float hash_value_ratio, uint16_t cuckoo_buckets,
                     uint8_t cuckoo_arity, kvh_ht_geom_t *geom);
/* positions stored per key for this geometry (0 for NULL) */
uint32_t kvh_positions_per_key(const kvh_ht_geom_t *geom);

/* n device-resident hash pairs (16-byte aligned) -> positions (16-byte
 * aligned device buffer).  Replaces, per key, ht_mod(key) and
 * CuckooAltHash::calc_hash(kctx, key, key2, ht_mod(key)).  KVH_EINVAL for a
 * geometry whose ht_mod leaves ht[] or whose table is too small to place
 * per_key non-clashing slots; a slot the rejection loop could not place
 * within 2^20 steps (unreachable for an accepted geometry) is ~0. */
int kvh_ht_positions(const uint64_t *hashes, size_t n,
                     const kvh_ht_geom_t *geom, void *pos, uint32_t flags,
                     void *stream);

/* Fused: n fixed-length keys -> kv_hash_meow128 with (seed1, seed2) ->
 * KeyFragment fixup -> positions, one pass (KeyCtx::set_key_hash then the
 * probe positions, key_ctx.cpp:97-105).  `hashes` (2n u64, may be NULL)
 * receives the fixed-up hashes.  One kernel for key_len 16/32 with 16-byte
 * aligned keys and 1/2/4/8 positions per key; other shapes run the hash
 * kernel then kvh_ht_positions. */
int kvh_meow128_fixed_positions(const void *keys, uint32_t key_len, size_t n,
                                uint64_t seed1, uint64_t seed2,
                                const kvh_ht_geom_t *geom, uint64_t *hashes,
                                void *pos, uint32_t flags, void *stream);

/* ---------------------------------------------------------------------
 * Batch order by table position: the role of
 * kv_ht_radix_sort (src/radix_sort.cpp:31-41) + ctest.c:96-104's duplicate
 * marking.  CONTRACT: the slot sequence equals kv_ht_radix_sort's (ht_mod(h1)
 * ascending) and every slot holds the same rows; the order WITHIN a slot and
 * the duplicate count differ.  The reference's in-place bit-pivot sort
 * (include/raikv/radix_sort.h:31-33) leaves equal slots in an input-dependent
 * order, so ctest's adjacent-pair scan finds only the duplicates that land
 * next to each other; here equal slots are ordered by (h1 << 1, h1, h2) and
 * then input order, all duplicates are adjacent and the count is the true
 * one (reference fixtures:
 * 99 vs 500 on the 600-entry table, 992 vs 1000 on a 64 MiB one; tests/golden/
 * sort_*.npz).  That default is not a bit-identical drop-in for
 * kv_ht_radix_sort.  KVH_REF_ORDER (n <= 65536, ctest's batch sizes) and
 * kvh_ht_sort_batched ARE: they step RadixSort::sort's own algorithm
 * (radix_sort.h:89-298) on the device and leave the reference's exact
 * element order, so the duplicate count is the reference's too (99 on the
 * 600-entry fixture).
 * ------------------------------------------------------------------- */
#define KVH_DEDUP     0x8u  /* zero h1 of an element equal (h1,h2) to its successor, count it */
#define KVH_REF_ORDER 0x10u /* kvh_ht_sort: the reference's exact element order, n <= 65536 */

/* layout of kv_ht_sort_t (include/raikv/radix_sort.h:8-11) */
typedef struct {
  uint64_t key, key2;
  void    *item;
} kvh_ht_sort_t;

/* device scratch for n elements (0 on error) */
size_t kvh_ht_sort_scratch_bytes(size_t n);
/* n < 2^32 device (h1,h2) pairs (+ optional u64 items, NULL = carry the
 * input index) -> hashes_out / items_out in table order; with KVH_DEDUP
 * the duplicate count is written to *dup_count (device u64, optional).
 * Asynchronous on stream.  Two engines give the same output word for word
 * (kvh_set_tuning knob 20): a bucketed one (~6K-element buckets filled by
 * two tile-stable LDS-staged scatter passes of <= 7 bucket bits each, an
 * LDS sort per bucket; the default up to ~75-147M elements per call, the
 * bound scaled by the share of bucket ids the table's slots reach) and a
 * radix one (rocPRIM onesweep on a key prefix + gather; beyond that size).
 * Non-uniform input (many pairs sharing a slot and h1) is bounded at
 * O(R log^2 R) per such group; a bucket of one repeated pair (the
 * KVH_DEDUP hot key) arrives in order and costs one pass. */
int kvh_ht_sort(const uint64_t *hashes, const uint64_t *items, size_t n,
                const kvh_ht_geom_t *geom, uint64_t *hashes_out,
                uint64_t *items_out, uint64_t *dup_count, uint32_t flags,
                void *scratch, size_t scratch_bytes, void *stream);
/* Many kv_ht_radix_sort calls in one launch (ctest sorts its fragments in
 * batches, test/ctest.c:34, :90, then marks duplicates, :96-104): the n
 * pairs are cut into batches of `batch` (1..65536; the last may be
 * shorter), and each batch is sorted on its own workgroup in the
 * reference's exact element order (KVH_REF_ORDER's algorithm), as a
 * separate kv_ht_radix_sort call on it would leave it.  flags: KVH_DEDUP
 * marks and counts duplicates per batch: dup_counts[b] (device u64,
 * ceil(n / batch) entries; NULL: not written) gets batch b's count (0
 * without KVH_DEDUP).  items NULL: the global input index.  Asynchronous
 * on stream.  scratch: a device buffer of
 * kvh_ht_sort_batched_scratch_bytes(n, batch) (0: batch out of range). */
size_t kvh_ht_sort_batched_scratch_bytes(size_t n, uint32_t batch);
int kvh_ht_sort_batched(const uint64_t *hashes, const uint64_t *items,
                        size_t n, uint32_t batch, const kvh_ht_geom_t *geom,
                        uint64_t *hashes_out, uint64_t *items_out,
                        uint64_t *dup_counts, uint32_t flags, void *scratch,
                        size_t scratch_bytes, void *stream);
/* The same over batches of any sizes: batch b is elements [seg_offs[b],
 * seg_offs[b+1]) of the n pairs (device u64, nseg + 1 entries,
 * non-decreasing, last <= n), each of at most max_seg (1..65536) elements --
 * ctest's batches end when 16K frags or its 64 KiB frag buffer fill
 * (ctest.c:31-34, :214-222).  The offsets are read on the device, so they
 * are checked there: a batch longer than max_seg is copied through in input
 * order, unmarked, and flagged dup_counts[b] = ~0; a batch that is reversed
 * or ends past n is flagged ~0 and its output is NOT written (it may not
 * even exist).  scratch: kvh_ht_sort_segments_scratch_bytes(nseg, max_seg). */
size_t kvh_ht_sort_segments_scratch_bytes(size_t nseg, uint32_t max_seg);
int kvh_ht_sort_segments(const uint64_t *hashes, const uint64_t *items,
                         size_t n, const uint64_t *seg_offs, size_t nseg,
                         uint32_t max_seg, const kvh_ht_geom_t *geom,
                         uint64_t *hashes_out, uint64_t *items_out,
                         uint64_t *dup_counts, uint32_t flags, void *scratch,
                         size_t scratch_bytes, void *stream);
/* host form of kv_ht_radix_sort(ar, ar_size, ht) (radix_sort.h:19-20):
 * sorts ar[] in place (synchronous, on the current GPU); the table is
 * given by its geometry.  Up to 65536 elements (ctest's batches) in the
 * reference's exact order (KVH_REF_ORDER); beyond that the same slot order
 * with the tie order described above. */
int kvh_ht_radix_sort(kvh_ht_sort_t *ar, uint32_t ar_size,
                      const kvh_ht_geom_t *geom);
/* Batching front end of the drop-in (ctest's threads each sort a batch,
 * test/ctest.c:89-104, :395): nbatch host arrays ars[b] of sizes[b] <=
 * 65536 elements, each sorted in place in kv_ht_radix_sort's exact order,
 * all in ONE device launch (one pinned H2D copy, kvh_ht_sort_segments, one
 * D2H copy).  Synchronous, on the calling thread's hipStreamPerThread; the
 * staging buffers persist per process.  Per batch it costs the launch /
 * nbatch: the way a device pays for the exact order at ctest's batch sizes
 * (DESIGN.md §3.5).  No duplicate marking (the caller's loop, as ctest's). */
int kvh_ht_radix_sort_batch(kvh_ht_sort_t *const *ars, const uint32_t *sizes,
                            uint32_t nbatch, const kvh_ht_geom_t *geom);

/* ---------------------------------------------------------------------
 * Key ingest: the key formats raikv produces, hashed on
 * the device without host repacking.
 * ------------------------------------------------------------------- */
#define KVH_NULTERM   0x4u  /* hash span + one 0 byte (kv_set_key_frag_string, key_ctx.cpp:1764-1772) */

/* Whitespace tokenizer of test/ctest.c:202-233: tokens are maximal runs of
 * bytes other than ' ', '\n', '\t' in text[0, nbytes) (device buffer);
 * a token of i bytes is kept when i < max_token (MAX_TOKEN_SIZE 256,
 * ctest.c:23).  Writes the first min(count, cap) kept tokens' byte offsets
 * and lengths in text order and the kept count to *count (all device
 * memory).  scratch: device buffer of kvh_tokenize_scratch_bytes(nbytes). */
size_t kvh_tokenize_scratch_bytes(size_t nbytes);
int kvh_tokenize(const void *text, size_t nbytes, uint32_t max_token,
                 uint64_t *tok_offs, uint32_t *tok_lens, size_t cap,
                 uint64_t *count, void *scratch, size_t scratch_bytes,
                 void *stream);

/* Tokenize and hash in one asynchronous call: ctest's ingest loop
 * (ctest.c:202-233, a kv_hash_key_frag of every kept token,
 * key_ctx.cpp:1774-1783) as kvh_tokenize followed by kvh_meow128_spans over
 * its tokens, the span hash reading the token count from the device (no
 * host round trip between the two).  out: cap x 2 u64, hashes of the first
 * min(count, cap) tokens in text order; flags as kvh_meow128_spans
 * (KVH_NULTERM | KVH_FIXUP for kv_hash_key_frag).  Same scratch as
 * kvh_tokenize. */
int kvh_tokenize_hash(const void *text, size_t nbytes, uint32_t max_token,
                      uint64_t seed1, uint64_t seed2, uint32_t flags,
                      uint64_t *tok_offs, uint32_t *tok_lens, uint64_t *out,
                      size_t cap, uint64_t *count, void *scratch,
                      size_t scratch_bytes, void *stream);

/* Meow128 of n keys given as (offset, length) spans into buf (device).
 * With KVH_NULTERM the hashed key is the span followed by one 0 byte that
 * need not be in buf: a token becomes the kv_key_frag_t "token\0" of
 * ctest.c:223 (keylen = len + 1).  KVH_FIXUP as elsewhere; with the
 * table's db-0 seed this is kv_hash_key_frag (key_ctx.cpp:1774-1783). */
int kvh_meow128_spans(const void *buf, const uint64_t *offs,
                      const uint32_t *lens, size_t n, uint64_t seed1,
                      uint64_t seed2, uint64_t *out, uint32_t flags,
                      void *stream);

/* Record offsets of a packed kv_key_frag_t stream: buf
 * holds records {u16 keylen, keylen bytes, pad to 2} back to back from byte
 * 0 (kv_make_key_frag, key_ctx.cpp:1737-1745, ctest.c:223); writes the byte
 * offsets of the first min(count, cap) records and the record count to
 * *count (device), found on the device by list ranking.  A record running
 * past nbytes ends the stream.  nbytes < 8 GiB.  scratch: device buffer of
 * kvh_frag_offsets_scratch_bytes(nbytes). */
size_t kvh_frag_offsets_scratch_bytes(size_t nbytes);
int kvh_frag_offsets(const void *buf, size_t nbytes, uint64_t *rec_offs,
                     size_t cap, uint64_t *count, void *scratch,
                     size_t scratch_bytes, void *stream);
/* kvh_frag_offsets, then kvh_meow128_frags over those records reading the
 * count on the device (one asynchronous call): the hashes of a packed frag
 * stream, out cap x 2 u64. */
int kvh_frags_hash(const void *buf, size_t nbytes, uint64_t seed1,
                   uint64_t seed2, uint32_t flags, uint64_t *rec_offs,
                   uint64_t *out, size_t cap, uint64_t *count, void *scratch,
                   size_t scratch_bytes, void *stream);

/* Meow128 of n packed kv_key_frag_t records {u16 keylen, keylen bytes,
 * pad to 2} (hash_entry.h:28-36, kv_make_key_frag key_ctx.cpp:1737-1745):
 * rec_offs[i] is the byte offset of record i in buf (ctest.c's xh[].frag
 * pointers relative to its buffer).  Same result as kv_hash_key_frag. */
int kvh_meow128_frags(const void *buf, const uint64_t *rec_offs, size_t n,
                      uint64_t seed1, uint64_t seed2, uint64_t *out,
                      uint32_t flags, void *stream);

/* ---------------------------------------------------------------------
 * CRC32C: raikv's kv_crc_c family (key_hash.c:27-179),
 * the SSE4.2 crc32 chain from `seed`, no pre/post inversion.
 * ------------------------------------------------------------------- */
/* Device batches: out[i] = kv_crc_c(key_i, len_i, seeds ? seeds[i] : seed).
 * seeds (optional, device) may equal out (kv_crc_c_array's in/out seeds). */
int kvh_crc_c_fixed(const void *keys, uint32_t key_len, size_t n,
                    const uint32_t *seeds, uint32_t seed, uint32_t *out,
                    void *stream);
int kvh_crc_c_var(const void *keys, const uint64_t *offsets, size_t n,
                  const uint32_t *seeds, uint32_t seed, uint32_t *out,
                  void *stream);
/* Host drop-ins (synchronous, executed on the current GPU). */
/* key_hash.c:53-63 kv_crc_c (returns the crc; errors via kvh_last_error) */
uint32_t kvh_crc_c(const void *p, size_t sz, uint32_t seed);
/* key_hash.c:27-37 kv_hash_uint / kv_hash_uint2 */
uint32_t kvh_hash_uint(uint32_t i);
uint32_t kvh_hash_uint2(uint32_t r, uint32_t i);
/* key_hash.c:65-84, :86-120 */
int kvh_crc_c_2_diff(const void *p, size_t sz, uint32_t *seed,
                     const void *p2, size_t sz2, uint32_t *seed2);
int kvh_crc_c_4_diff(const void *p, size_t sz, uint32_t *seed,
                     const void *p2, size_t sz2, uint32_t *seed2,
                     const void *p3, size_t sz3, uint32_t *seed3,
                     const void *p4, size_t sz4, uint32_t *seed4);
/* key_hash.c:122-142: seed[i] = kv_crc_c(p[i], psz[i], seed[i]) */
int kvh_crc_c_array(const void **p, size_t *psz, uint32_t *seed, size_t count);
/* key_hash.c:168-179: seed[i] = kv_crc_c(p, psz[i], seed[i]) -- prefixes
 * of ONE buffer p (every entry reads from the same start) */
int kvh_crc_c_key_array(const void *p, size_t *psz, uint32_t *seed,
                        size_t count);

/* ---------------------------------------------------------------------
 * Runtime / diagnostics
 * ------------------------------------------------------------------- */
int         kvh_last_error(void);
const char *kvh_strerror(int err);
/* engine version string */
const char *kvh_version(void);
/* synchronise the current device (host wall-clock timing helpers) */
int         kvh_device_synchronize(void);
/* Bounds-checked build (`make checked`, tools/libkvh_checked.so, a debug
 * build of these same sources): out[0..3] = (failed checks, site, value,
 * limit) of the first failed device-side index check since the last call
 * (exact-order sort and ingest kernels), then cleared.  Returns 1 from the
 * checked build, 0 from the product build (which checks nothing: out is all
 * zero), or a negative error. */
int         kvh_debug_checks(uint64_t out[4]);
/* Streams.  The in-order streaming kernels (fixed and variable length,
 * multi-seed, fused positions, CRC32C, span hashing) take their chunks in
 * address order through ticket words kept per (device, stream), taken on a
 * stream's first call from a per-device pool of 1024 sets (allocated once,
 * on the device's first such call, and zeroed asynchronously on that call's
 * stream: nothing on a launch synchronises the device or another stream;
 * while the pool is dry a call takes the static chunk order, with the same
 * results), reset by each launch's last workgroup, so launches on one
 * stream need nothing else.  hipStreamPerThread gets words per calling
 * thread, returned when the thread exits.  That one hipMalloc per device is
 * the only allocation: make the first call on each device before another
 * thread starts a hipStreamCaptureModeGlobal capture.  A call on a stream
 * that is being captured into a graph launches
 * the static-order form of its kernel (no shared words: the graph may be
 * replayed on any stream, and concurrently).  kvh_stream_release
 * synchronises `stream` and hands its words back; call it before destroying
 * a stream that called this library (not needed for the null stream or
 * hipStreamPerThread).  0 or a negative error. */
int         kvh_stream_release(void *stream);
/* Tuning knobs: each selects among kernels that return the same hashes, or
 * sizes the host pipeline.  Process-wide; atomic (a call already running
 * keeps the value it read).
 *   1 = workgroups per CU multiplier (1-8), 2 = force the generic kernel (0/1),
 *   7 = variable-length kernel (46 default: per-wave windows sorted by
 *       16-byte length class, keys read as dwordx4 groups, one straight-line
 *       variant per chunk shape, windows taken in address order through wave
 *       tickets; 23 the same in the static window order; 0 lane per key in
 *       input order),
 *   8 = multi-seed kernel (1 lanes per key, 0 one lane per key),
 *  14 = variable-length CRC32C kernel (6 default: length-sorted windows, 16
 *       waves on 16-copy tables, keys read as dwordx4 groups, the next key's
 *       first groups in flight; 0 input order),
 *  15 / 16 = host pipeline chunk MiB / slots, 17 = ht_sort radix key bits
 *       (0 auto; nonzero also selects the radix engine),
 *  18 = span-hash kernel (2 / 1 short spans in place + per-wave medium and
 *       long queues, two / one spans per lane per step; 0 lane per span),
 *  19 = tokenizer (1 wave-chunked, 0 workgroup-chunked),
 *  20 = ht_sort engine (0 two-pass bucketed when the batch fits it, else
 *       radix; 1 radix always; 2 one-pass bucketed when the batch fits it),
 *  21 = host batches of at most this many keys (and 512 KiB of key bytes)
 *       take the zero-copy tiny path (default 16384; 0 off),
 *  22 = ht_sort bucket sort (0 two workgroups per CU when the buckets are
 *       small enough; 1 always one per CU),
 *  23 = ht_sort two-pass bucket sort (3 default: buckets of <= 3K records,
 *       up to 15 bucket bits with an 8-bit second pass, each bucket's
 *       records read once into registers by one of two 512-thread
 *       workgroups per CU; 0 k_bk_sort),
 *  24 = chunk order of the streaming kernels (0 default and 2: every
 *       fixed-length, runtime-length, multi-seed, fused-positions,
 *       variable-length, CRC32C and span kernel takes its chunks in address
 *       order through per-stream wave tickets; 1 the static per-wave order
 *       everywhere),
 *  25 = counting-sort bits of the knob-23 = 3 bucket sort (0 default = 12,
 *       10, 11),
 *  26 = TEST ONLY: the first takers of every other wave ticket sleep
 *       value x ~4 us before fetching the next one (0 default, up to 65535);
 *       slows the in-order kernels, never changes their output.
 * Returns the previous value or KVH_EINVAL.  The kernels that lost their A/B
 * (knobs 0 and 3: tables per LDS and keys per lane other than the per-length
 * defaults; knob 7 = 7, 13, 24, 25, 44, 45, 47-50; knob 14 = 1-5; knob 23 =
 * 1, 2, 5, 6; knob 24 = 3-5; knob 27 = 128, 256: the exact-order batched
 * sort's earlier many-batch forms) and the ablation builds whose outputs are not
 * hashes exist only in the experiments build, tools/libkvh_exp.so, never in
 * libkvh.so, which rejects those values. */
int         kvh_set_tuning(int knob, int value);

#ifdef __cplusplus
}
#endif

#endif /* KVH_H */
