"""CPU: bench.py's workload selection (the driver runs `bench.py --gpus N`
with no --config): c1 (BASELINE configs[1]) per GPU at every N (weak
scaling); `--config c4g` is the north star's C4 as stated -- one global batch
of 1B 32-byte keys whose index ranges the ranks share exactly (strong
scaling)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_default_is_c1_at_one_gpu():
    name, cfg, n = bench.resolve_config(None, 0, 1)
    assert name == "c1" and cfg["n"] == n == 100_000_000 and cfg["key_len"] == 16
    assert not cfg.get("global_batch")


def test_default_is_c1_per_gpu_at_n_gpus():
    """Weak scaling: every rank its own 100M x 16 B shard, the N = 1 workload."""
    for world in (2, 4, 8):
        for r in range(world):
            name, cfg, n = bench.resolve_config(None, r, world)
            assert name == "c1" and cfg["n"] == n == 100_000_000 and cfg["key_len"] == 16
            assert not cfg.get("global_batch")


def test_c4g_is_one_global_batch_at_n_gpus():
    for world in (2, 4, 8, 3):
        shards = []
        for r in range(world):
            name, cfg, n = bench.resolve_config("c4g", r, world)
            assert name == "c4g" and n == 1_000_000_000 and cfg["key_len"] == 32 and cfg["global_batch"]
            lo, hi = cfg["shard"]
            assert hi - lo == cfg["n"]
            shards.append((lo, hi))
        shards.sort()
        assert shards[0][0] == 0 and shards[-1][1] == 1_000_000_000
        assert all(a[1] == b[0] for a, b in zip(shards, shards[1:]))  # disjoint, covering, in order
        assert max(h - l for l, h in shards) - min(h - l for l, h in shards) <= 1


def test_named_config_and_override():
    name, cfg, n = bench.resolve_config("c4g", 0, 1)
    assert cfg["n"] == n == 1_000_000_000 and cfg["shard"] == [0, 1_000_000_000]
    name, cfg, n = bench.resolve_config("c2", 1, 4, keys_override=1000)
    assert name == "c2" and cfg["n"] == n == 1000 and cfg["var"]
    name, cfg, n = bench.resolve_config("c64", 0, 1)
    assert cfg["key_len"] == 64 and n == 100_000_000


def test_committed_traffic_is_never_below_the_algorithmic_bytes():
    """the HBM traffic bench.py reports for a config
    (profiles/pmc_traffic.json, from rocprofv3 FETCH_SIZE / WRITE_SIZE) is
    at least the bytes the launch must move (the alg_bytes_per_launch of the
    bench line profiled beside it); the gather kernels carry their bracket."""
    import json
    import os
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t = json.load(open(os.path.join(root, "profiles", "pmc_traffic.json")))
    checked = 0
    for c, e in t.items():
        m = re.match(r"(profiles/\S+)/" + re.escape(c) + r"_pmc_summary\.json", e["source"])
        if not m:
            continue
        bj = os.path.join(root, m.group(1), f"{c}_bench_under_rocprof.json")
        if not os.path.exists(bj):
            continue
        line = [l for l in open(bj) if l.startswith("{")][-1]
        alg = json.loads(line)["roofline"]["alg_bytes_per_launch"]
        assert e["hbm_bytes_per_launch"] >= alg, (c, e["hbm_bytes_per_launch"], alg)
        if "traffic_bounds" in e:
            lo, hi = e["traffic_bounds"]
            assert abs(lo - alg) <= 1e-6 * alg and lo <= e["hbm_bytes_per_launch"] <= hi
        checked += 1
    assert checked >= 8
