"""CPU: the table-order oracle (tests/oracle_lib.py np_ht_sort, SURVEY.md
§8 f2) against the reference's own kv_ht_radix_sort + ctest.c dedup
outputs (tests/golden/sort_*.npz): identical slot sequence, identical
element multiset within every slot, and a duplicate count at least the
reference's (all duplicates adjacent here; the reference's tie order can
separate them)."""
import numpy as np
import pytest

from oracle_lib import load_oracle, np_ht_mod, np_ht_sort, orc_geom, sort_fixtures

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


def test_capi_sort_argument_checks_without_device():
    import ctypes
    import raikv_amd as kvh
    lib = kvh.lib
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    assert lib.kvh_ht_radix_sort(None, 0, None) == -22      # no geometry
    assert lib.kvh_ht_radix_sort(None, 1, ctypes.byref(g)) == 0  # 0/1 elements: nothing to sort
    assert lib.kvh_ht_radix_sort(None, 2, ctypes.byref(g)) == -22
