/*
 * oracle/sort_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker for
 * SURVEY.md §8 row f2 in the reference's exact element order).  Linked into
 * liboracle.so; nothing in the product links, loads or calls it.
 *
 * Clean-room restatement of kv_ht_radix_sort (src/radix_sort.cpp:31-41):
 * RadixSort<kv_ht_sort_t, uint64_t, HtSortCompare>::sort
 * (include/raikv/radix_sort.h:89-298) with key(e) = ht_mod(e.key), max_val =
 * ht_size, no sub key:
 *   bits     bit_count = 1 + floor(log2 ht_size)          (radix_sort.h:75-77)
 *   node     (off, count, shift), the remaining bits [0, shift)
 *   leaf     count < 32 or shift == 0: with shift != 0, bubble (2-4) or a
 *            shell sort with gaps 48, 21, 7, 3, 1 on less() (:121-177);
 *            shift == 0 leaves the node in place (no sub key)
 *   radix    shift > 1: k = min(8, shift) bits; all in one bucket -> the node
 *            again with shift - k; else its buckets of > 1 elements as nodes
 *            and the in-place American-flag permutation (:178-250)
 *   1 bit    shift == 1: a Hoare partition on bit 0 (:251-285)
 * Nodes are disjoint ranges, so the order in which they are taken (the
 * reference's LIFO stack) does not change the result; this restatement keeps
 * a LIFO stack too.  ctest's duplicate marking (test/ctest.c:96-104) follows
 * in orc_ht_mark_dups.
 *
 * Pinning: tests/golden/sort_*.npz are the reference's own kv_ht_radix_sort +
 * ctest marking compiled where they lie (oracle/ref_cuckoo.cpp ref_ht_sort);
 * tests/test_sort_oracle.py checks this restatement against them word for word.
 */
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t ht_size, ht_mod_mask, ht_mod_fraction;
  uint32_t ht_mod_shift;
  uint16_t cuckoo_buckets;
  uint8_t  cuckoo_arity, pad;
} orc_sgeom_t;  /* the layout of orc_geom_t (cuckoo_oracle.c) */

typedef struct { uint64_t key, key2, item; } orc_sort_el_t;  /* kv_ht_sort_t (radix_sort.h:8-11) */

static uint64_t slot_of(const orc_sgeom_t *g, const orc_sort_el_t *e)
{
  return ((e->key & g->ht_mod_mask) * g->ht_mod_fraction) >> g->ht_mod_shift;  /* shm_ht.h:181-184 */
}

static void el_swap(orc_sort_el_t *a, orc_sort_el_t *b)
{
  orc_sort_el_t t = *a; *a = *b; *b = t;
}

/* count < 32 with bits left: fixed compare-exchange sequences for 2-4
 * elements, else gapped insertion passes */
static void leaf_sort(const orc_sgeom_t *g, orc_sort_el_t *v, uint32_t count)
{
#define LT(a, b) (slot_of(g, &v[a]) < slot_of(g, &v[b]))
#define CX(a, b) do { if (LT(b, a)) el_swap(&v[a], &v[b]); } while (0)
  if (count == 4) { CX(0, 3); CX(1, 3); CX(2, 3); CX(1, 2); }
  if (count >= 2 && count <= 4) {
    if (count >= 3) { CX(0, 2); CX(1, 2); }
    CX(0, 1);
    return;
  }
  if (count < 2) return;
  static const uint32_t gaps[5] = { 48, 21, 7, 3, 1 };
  for (int k = 0; k < 5; k++) {
    const uint32_t h = gaps[k];
    for (uint32_t i = h; i < count; i++) {
      if (!LT(i, i - h)) continue;
      const orc_sort_el_t x = v[i];
      const uint64_t xs = slot_of(g, &x);
      uint32_t j = i;
      do {
        v[j] = v[j - h];
        j -= h;
      } while (j >= h && xs < slot_of(g, &v[j - h]));
      v[j] = x;
    }
  }
#undef CX
#undef LT
}

typedef struct { uint32_t off, count, shift; } node_t;

void orc_ht_radix_sort_ref(const orc_sgeom_t *g, orc_sort_el_t *v, uint32_t n)
{
  if (n <= 1 || g->ht_size == 0) return;
  uint32_t bits = 1;
  for (uint64_t m = g->ht_size; m != 1; m >>= 1) bits++;
  /* every push is a node of >= 2 elements on a range disjoint from the
   * others on the stack: at most n / 2 of them, + the re-pushed node */
  node_t *st = (node_t *) malloc(sizeof(node_t) * (n / 2 + 2));
  uint32_t top = 0;
  node_t cur = { 0, n, bits };
  for (;;) {
    const uint32_t off = cur.off, count = cur.count, shift = cur.shift;
    orc_sort_el_t *a = v + off;
    if (count < 32 || shift == 0) {
      if (shift != 0) leaf_sort(g, a, count);
    } else if (shift > 1) {
      const uint32_t k = shift > 8 ? 8 : shift, sh = shift - k, nb = 1u << k;
      const uint64_t m = (uint64_t) (nb - 1) << sh;
      uint32_t c[256], o[256], last = 0;
      memset(c, 0, sizeof c);
      for (uint32_t i = 0; i < count; i++) {
        last = (uint32_t) ((slot_of(g, &a[i]) & m) >> sh);
        c[last]++;
      }
      if (c[last] == count) {
        st[top].off = off; st[top].count = count; st[top].shift = sh; top++;
      } else {
        uint32_t base = 0;
        for (uint32_t b = 0; b < nb; b++) {
          o[b] = base;
          if (c[b] > 1) { st[top].off = off + base; st[top].count = c[b]; st[top].shift = sh; top++; }
          base += c[b];
        }
        /* American flag: the first unplaced slot of bucket b is o[b]; the
         * element there is examined until one of bucket b lands in it */
        for (uint32_t b = 0; b < nb; b++) {
          while (c[b] > 0) {
            const uint32_t d = (uint32_t) ((slot_of(g, &a[o[b]]) & m) >> sh);
            if (d != b) {
              el_swap(&a[o[b]], &a[o[d]]);
              o[d]++; c[d]--;
            } else {
              o[b]++; c[b]--;
            }
          }
        }
      }
    } else {
      uint32_t i = 0, j = count;
      for (;;) {
        while (i < j && (slot_of(g, &a[i]) & 1) == 0) i++;
        while (i < j && (slot_of(g, &a[j - 1]) & 1) != 0) j--;
        if (i == j) break;
        el_swap(&a[i], &a[j - 1]);
        i++; j--;
      }
      if (i > 1) { st[top].off = off; st[top].count = i; st[top].shift = 0; top++; }
      if (count - j > 1) { st[top].off = off + j; st[top].count = count - j; st[top].shift = 0; top++; }
    }
    if (top == 0) break;
    cur = st[--top];
  }
  free(st);
}

/* test/ctest.c:96-104: an element equal (key, key2) to its successor gets
 * key = 0; returns the count */
uint64_t orc_ht_mark_dups(orc_sort_el_t *v, uint32_t n)
{
  uint64_t d = 0;
  for (uint32_t k = 1; k < n; k++)
    if (v[k - 1].key == v[k].key && v[k - 1].key2 == v[k].key2) { v[k - 1].key = 0; d++; }
  return d;
}
