# f2 kernel breakdown: kernel-trace of a short f2 bench, plus FETCH/WRITE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=${1:-gpurun_out/f2prof}; mkdir -p $O
B="python3 bench.py --config f2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-copy-peak --settle-ms 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/bench.json 2> $O/trace.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O/fetch $O/write > $O/pmc_summary.json || exit 1
python3 - $O <<'PY'
import csv, json, sys
o = sys.argv[1]
st = list(csv.DictReader(open(o + "/trace/run_kernel_stats.csv")))
pm = json.load(open(o + "/pmc_summary.json"))
for r in st:
    if "k_bk" in r["Name"] or "k_sort" in r["Name"] or "k_tw" in r["Name"]:
        k = [v for n, v in pm.items() if n[:60] == r["Name"][:60]]
        fw = ""
        if k and "FETCH_SIZE" in k[0]:
            # pmc_summary holds per-dispatch means (KB): x1024, FETCH x2 (gfx950 streaming rule)
            fw = "fetch %.2f GB write %.2f GB per dispatch" % (k[0]["FETCH_SIZE"] * 2048 / 1e9, k[0]["WRITE_SIZE"] * 1024 / 1e9)
        print("%-40s calls %4s avg %8.1f us  %s" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3, fw))
PY
