#!/bin/bash
# Round-4 first GPU session: gpu suite, the streaming forms on one box,
# bench.py's own N-rank launcher (no external launcher), and the driver's
# protocol on C1/C2 with the new parity field.
# usage: tools/gpu_r4_s1.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/r4s1}
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.txt; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 tools/stream_forms 100000000 500 5 20 > $O/stream_forms.json 2> $O/stream_forms.log || exit 1
cat $O/stream_forms.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c1.json 2> $O/bench_c1.log || exit 1
cut -c1-300 $O/bench_c1.json; python3 -c "import json;print(json.load(open('$O/bench_c1.json'))['parity'])"
timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gpus2.json 2> $O/bench_gpus2.log || exit 1
cut -c1-300 $O/bench_gpus2.json
python3 -c "import json;d=json.load(open('$O/bench_gpus2.json'));print(d['n_gpus'],d['config']['config'],d['scaling'],d['parity'],d['per_gpu'])"
timeout -k 10 300 python3 bench.py --config c2 --steps 20 --warmup 5 --no-e2e > $O/bench_c2.json 2> $O/bench_c2.log || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity'])"
# C2: NT=2 x 32 copies (knob 7 = 23, the default) vs four tables x 16 copies (44), one process
KVH_LIB=raikv_amd/libkvh.so timeout -k 10 300 python3 tools/c2_ab.py --variants 23,44,45 --rounds 5 > $O/c2_nt5_ab.jsonl 2> $O/c2_nt5_ab.log || exit 1
cat $O/c2_nt5_ab.jsonl
# f2: the real k_tw_scatter2 under ablations, timings then one PMC pass per counter group
timeout -k 10 120 tools/scatter2_real 100000000 5 > $O/s2real.json 2> $O/s2real.log || exit 1
cat $O/s2real.json
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/s2real_w -o run -- tools/scatter2_real 100000000 1 > $O/s2real_w.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/s2real_f -o run -- tools/scatter2_real 100000000 1 > $O/s2real_f.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O/s2real_w $O/s2real_f > $O/s2real_pmc.json || exit 1
python3 -c "import json;d=json.load(open('$O/s2real_pmc.json'));[print(k[:50],v) for k,v in d.items() if 'scatter2' in k]"
# f2: bucket sort k_bk_sort (knob 23 = 0) vs the register-resident k_bk_sortr (1), outputs asserted equal
TUNE_KNOB=23 timeout -k 10 300 python3 tools/tune_sort.py 0,1 > $O/f2_sortr_ab.jsonl 2> $O/f2_sortr_ab.log || exit 1
cat $O/f2_sortr_ab.jsonl
