"""CPU: the table-order oracle (tests/oracle_lib.py np_ht_sort, SURVEY.md
§8 f2) against the reference's own kv_ht_radix_sort + ctest.c dedup
outputs (tests/golden/sort_*.npz): identical slot sequence, identical
element multiset within every slot, and a duplicate count at least the
reference's (all duplicates adjacent here; the reference's tie order can
separate them)."""
import numpy as np
import pytest

from oracle_lib import (load_oracle, load_ref_ht, np_ht_mod, np_ht_sort, orc_geom, orc_ht_radix_sort_ref,
                        ref_ht_sort, ref_order_cases, sort_fixtures)

FIX = sort_fixtures()
ORC = load_oracle()


@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_order_refines_reference(f):
    g = orc_geom(ORC, f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    h, items = f["hashes"], f["out_items"]
    ref_items = f["out_items"]
    # the reference order's slots (from the input rows it placed)
    ref_slots = np_ht_mod(g, h[ref_items.astype(np.int64), 0])
    assert np.all(np.diff(ref_slots.astype(np.int64)) >= 0)
    oh, oi, dups = np_ht_sort(g, h, dedup=True)
    ours_slots = np_ht_mod(g, h[oi.astype(np.int64), 0])
    np.testing.assert_array_equal(ours_slots, ref_slots)
    # same rows within each slot run
    bounds = np.flatnonzero(np.diff(ref_slots.astype(np.int64))) + 1
    for a, b in zip(np.r_[0, bounds], np.r_[bounds, len(ref_slots)]):
        assert sorted(ref_items[a:b].tolist()) == sorted(oi[a:b].tolist())
    # duplicates: all adjacent here -> n - #unique pairs; the reference finds a subset
    uniq = len(np.unique(h, axis=0))
    assert dups == len(h) - uniq
    assert f["dups"] <= dups
    # the reference's zeroed rows are duplicates
    ref_zero = f["out_hashes"][:, 0] == 0
    np.testing.assert_array_equal(f["out_hashes"][~ref_zero], h[ref_items[~ref_zero].astype(np.int64)])


@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_reference_order_restatement_word_for_word(f):
    """oracle/sort_oracle.c (RadixSort::sort restated, radix_sort.h:89-298)
    reproduces the reference's kv_ht_radix_sort output WORD FOR WORD on its
    own fixtures -- elements, tie order within every slot, ctest's zeroed
    duplicates and their count (99 on the 600-slot table)."""
    g = orc_geom(ORC, f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    oh, oi, dups = orc_ht_radix_sort_ref(ORC, g, f["hashes"], dedup=True)
    np.testing.assert_array_equal(oi, f["out_items"])
    np.testing.assert_array_equal(oh, f["out_hashes"])
    assert dups == f["dups"]


def test_reference_order_restatement_vs_compiled_reference():
    """The restatement against the reference's kv_ht_radix_sort compiled where
    it lies (oracle/_ref/libkvref_ht.so, this container only) on generated
    batches that reach every step of RadixSort::sort (oracle_lib.ref_order_cases)."""
    ref = load_ref_ht()
    if ref is None:
        pytest.skip("oracle/_ref/libkvref_ht.so not built (no /root/reference here)")
    for ms, h in ref_order_cases(seed=11):
        g = orc_geom(ORC, ms, 64, 1.0, 4, 4)
        want = ref_ht_sort(ref, ms, h)
        got = orc_ht_radix_sort_ref(ORC, g, h, dedup=True)
        np.testing.assert_array_equal(got[1], want[1], err_msg=f"map {ms} n {len(h)}")
        np.testing.assert_array_equal(got[0], want[0])
        assert got[2] == want[2]


def test_capi_sort_argument_checks_without_device():
    import ctypes
    import raikv_amd as kvh
    lib = kvh.lib
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    assert lib.kvh_ht_radix_sort(None, 0, None) == -22      # no geometry
    assert lib.kvh_ht_radix_sort(None, 1, ctypes.byref(g)) == 0  # 0/1 elements: nothing to sort
    assert lib.kvh_ht_radix_sort(None, 2, ctypes.byref(g)) == -22
