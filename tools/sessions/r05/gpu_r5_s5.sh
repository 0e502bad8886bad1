#!/bin/bash
# Round-5 session 5: (a) C2 load-path ablations (67 no key loads, 68
# coalesced key reads) and the stable window sort (69, hashes) against 46;
# (b) f2 / f3 after the bank-conflict changes (bucket sort successor by lane
# shuffle, span constants at a 52-dword stride): bench A/B against the
# previous library on the same box, then LDS counters of both.
set -o pipefail
O=${1:-gpurun_out/r5s5}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
KVH_LIB=$PWD/tools/libkvh_exp.so timeout -k 10 400 python3 tools/c2_ab.py --variants 46,69 --ablations 67,68 --rounds 6 > $O/c2_ab.json 2> $O/c2_ab.log || { tail $O/c2_ab.log; exit 1; }
cat $O/c2_ab.json
BF="--steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-copy-peak"
for r in 1 2; do
  for lib in prev new; do
    L=$PWD/raikv_amd/libkvh.so; [ $lib = prev ] && L=$PWD/tools/libkvh_prev.so
    for c in f2 f3; do
      KVH_LIB=$L timeout -k 10 300 python3 bench.py --config $c $BF > $O/bench_${c}_${lib}_$r.json 2> $O/bench_${c}_${lib}_$r.log || exit 1
      python3 -c "import json;d=json.load(open('$O/bench_${c}_${lib}_$r.json'));print('$c $lib $r', round(d['ms_per_step'],4), d['roofline']['kernel_ms'], d['parity'].get('mismatches'), d['parity'].get('full_compare'))"
    done
  done
done
for lib in prev new; do
  L=$PWD/raikv_amd/libkvh.so; [ $lib = prev ] && L=$PWD/tools/libkvh_prev.so
  for c in f2 f3; do
    R="python3 tools/run_kernel.py --config $c --reps 3"
    KVH_LIB=$L timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${c}_$lib -o run -- $R > $O/pmc_${c}_$lib.log 2>&1 || exit 1
    python3 tools/pmc_summary.py $O/pmc_${c}_$lib > $O/pmc_${c}_$lib.json || exit 1
  done
done
