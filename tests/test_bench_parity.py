"""CPU: bench.py's own parity field and its rank launcher.

- tests/bench_parity.py (the checker bench.py runs on the timed launch's
  output) reports 0 mismatches for correct hashes and counts every wrong one
  for hashes made under an off-by-one seed;
- `bench.py --gpus N` without WORLD_SIZE starts N rank processes itself with
  torch.distributed.run's environment, prints rank 0's JSON line and fails if
  any rank fails; a WORLD_SIZE that disagrees with --gpus is refused.
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import bench_parity as bp  # noqa: E402
from oracle_lib import load_oracle, orc_fixed, orc_var  # noqa: E402
from raikv_amd.workload import STATIC_SEED, zipf_lengths, offsets_from_lengths  # noqa: E402

SEED = STATIC_SEED
BAD_SEED = (STATIC_SEED[0] + 1, STATIC_SEED[1])


def test_sample_indices_hold_first_and_last():
    idx = bp.sample_indices(100_000_000, 20_000, seed=3)
    assert idx[0] == 0 and idx[-1] == 100_000_000 - 1
    assert np.all(np.diff(idx) > 0) and 19_000 < len(idx) <= 20_002
    assert np.array_equal(bp.sample_indices(5, 20_000), np.arange(5))
    assert bp.sample_indices(0).size == 0


def test_fixed_parity_passes_and_catches_off_by_one_seed():
    lib = load_oracle()
    keys = np.random.default_rng(1).integers(0, 256, 3000 * 16, dtype=np.uint8)
    good = orc_fixed(lib, keys, 16, SEED)
    r = bp.meow_fixed(keys.reshape(-1, 16), 16, good, [SEED])
    assert r["checked"] == 3000 and r["mismatches"] == 0
    bad = orc_fixed(lib, keys, 16, BAD_SEED)
    r = bp.meow_fixed(keys.reshape(-1, 16), 16, bad, [SEED])
    assert r["mismatches"] == 3000 and r["first_bad_sample_row"] == 0


def test_multiseed_parity():
    lib = load_oracle()
    keys = np.random.default_rng(2).integers(0, 256, 500 * 32, dtype=np.uint8)
    seeds = [(1, 2), (3, 4), (5, 6), (7, 8)]
    out = np.stack([orc_fixed(lib, keys, 32, s) for s in seeds], axis=1)
    assert bp.meow_fixed(keys.reshape(-1, 32), 32, out, seeds)["mismatches"] == 0
    out[7, 2, 1] ^= np.uint64(1)
    assert bp.meow_fixed(keys.reshape(-1, 32), 32, out, seeds)["mismatches"] == 1


def test_var_parity_passes_and_catches_off_by_one_seed():
    lib = load_oracle()
    offs = offsets_from_lengths(zipf_lengths(2000, 8, 256, seed=5))
    keys = np.random.default_rng(3).integers(0, 256, int(offs[-1]), dtype=np.uint8)
    assert bp.meow_var(keys, offs, orc_var(lib, keys, offs, SEED), SEED)["mismatches"] == 0
    assert bp.meow_var(keys, offs, orc_var(lib, keys, offs, BAD_SEED), SEED)["mismatches"] == 2000
    fx = orc_var(lib, keys, offs, SEED, fixup=True)
    assert bp.meow_var(keys, offs, fx, SEED, fixup=True)["mismatches"] == 0


def test_crc_parity():
    from oracle_lib import orc_crc_var
    lib = load_oracle()
    offs = offsets_from_lengths(zipf_lengths(1000, 8, 256, seed=6))
    keys = np.random.default_rng(4).integers(0, 256, int(offs[-1]), dtype=np.uint8)
    good = orc_crc_var(lib, keys, offs, seed=0)
    assert bp.crc_var(keys, offs, good, 0)["mismatches"] == 0
    assert bp.crc_var(keys, offs, orc_crc_var(lib, keys, offs, seed=1), 0)["mismatches"] > 990


def test_span_parity_checks_hashes_and_token_boundaries():
    from oracle_lib import orc_hash_spans
    lib = load_oracle()
    text = np.frombuffer(b"alpha beta\tgamma\ndelta", np.uint8)
    offs, lens = np.array([0, 6, 11, 17]), np.array([5, 4, 5, 5])
    out = orc_hash_spans(lib, text, offs, lens, SEED)
    toks = [text[o:o + l] for o, l in zip(offs, lens)]
    before = np.array([-1, 32, 9, 10])
    after = np.array([32, 9, 10, -1])
    assert bp.spans(toks, before, after, out, SEED)["mismatches"] == 0
    # a token cut short ("alph") is not a maximal run: counted even with its right hash
    short = [text[0:4]] + toks[1:]
    out2 = out.copy()
    out2[0] = orc_hash_spans(lib, text, [0], [4], SEED)[0]
    after2 = after.copy()
    after2[0] = ord("a")
    assert bp.spans(short, before, after2, out2, SEED)["mismatches"] == 1


def test_ht_order_properties():
    pi = np.array([[5, 1], [9, 2], [7, 3]], np.uint64)
    r = bp.ht_order(0, True, pi, pi, 0, 0)
    assert r["mismatches"] == 0
    po = pi.copy()
    po[1, 0] = 0  # a marked duplicate
    assert bp.ht_order(0, True, pi, po, 1, 1)["mismatches"] == 0
    assert bp.ht_order(0, True, pi, po, 0, 1)["mismatches"] == 1   # count disagrees
    assert bp.ht_order(2, True, pi, pi, 0, 0)["mismatches"] == 2   # slot descents
    assert bp.ht_order(0, False, pi, pi, 0, 0)["mismatches"] == 1  # not a permutation
    po[2, 1] = 4
    assert bp.ht_order(0, True, pi, po, 1, 1)["mismatches"] == 1   # pair changed


# ------------------------------------------------------------------ launcher
def test_rank_env_matches_torchrun_shape():
    env = bench.rank_env(3, 8, 29555, base={"PATH": "/bin"})
    assert env["RANK"] == env["LOCAL_RANK"] == "3" and env["WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555" and env["PATH"] == "/bin"


FAKE_RANK = r"""
import json, os, sys
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["MASTER_PORT"]) > 0
if r == int(os.environ.get("FAIL_RANK", "-1")):
    sys.exit(7)
if r == 0:
    print("log line")
    print(json.dumps({"n_gpus": w, "argv": sys.argv[1:]}))
"""


def test_launch_ranks_prints_rank0_line(tmp_path, capsys):
    f = tmp_path / "fake_rank.py"
    f.write_text(FAKE_RANK)
    rc = bench.launch_ranks(4, ["--gpus", "4", "--steps", "3"], exe=[sys.executable, str(f)])
    assert rc == 0
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line == {"n_gpus": 4, "argv": ["--gpus", "4", "--steps", "3"]}


def test_launch_ranks_fails_when_a_rank_fails(tmp_path, capsys, monkeypatch):
    f = tmp_path / "fake_rank.py"
    f.write_text(FAKE_RANK)
    monkeypatch.setenv("FAIL_RANK", "1")
    assert bench.launch_ranks(3, [], exe=[sys.executable, str(f)]) != 0
    assert "{" not in capsys.readouterr().out


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr and r.stdout == ""


# ------------------------------------------------------------ scaling anchor
def test_anchor_efficiency_fields():
    """an N-rank c4g line is read against the 1-GPU c4g
    anchor each rank measured alone on its GPU: aggregate / (N x anchor),
    and per rank its shard's kernel rate / its anchor's kernel rate."""
    anchors = [{"hashes_per_s": 100e9, "hashes_per_s_kernel": 110e9},
               {"hashes_per_s": 120e9, "hashes_per_s_kernel": 130e9}]
    per_gpu = [{"rank": 0, "hashes_per_s": 99e9}, {"rank": 1, "hashes_per_s": 117e9}]
    e = bench.anchor_efficiency(2, 198e9, per_gpu, anchors)
    assert abs(e["efficiency_vs_anchor"] - 198e9 / (2 * 110e9)) < 1e-12
    assert abs(e["anchor_hashes_per_s_mean"] - 110e9) < 1
    assert [p["rank"] for p in e["per_rank"]] == [0, 1]
    assert abs(e["per_rank"][0]["efficiency_vs_anchor"] - 0.9) < 1e-12
    assert abs(e["per_rank"][1]["efficiency_vs_anchor"] - 0.9) < 1e-12


def test_anchor_is_the_c4g_workload():
    """The anchor is the workload `--config c4g` runs at N > 1 (BASELINE
    configs[4], 1B x 32 B, one global batch), so the N = 1 line carries its
    1-GPU point; the default N > 1 lines are c1 per GPU (weak scaling)."""
    name, cfg, n_global = bench.resolve_config(bench.ANCHOR, 0, 2)
    assert cfg.get("global_batch") and n_global == bench.CONFIGS[bench.ANCHOR]["n"]
    assert bench.resolve_config(None, 0, 1)[0] == "c1" and bench.resolve_config(None, 0, 2)[0] == "c1"
