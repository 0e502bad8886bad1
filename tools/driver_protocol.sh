#!/bin/bash
# The driver's bench protocol (python bench.py --gpus 1 --steps 20 --warmup 5)
# against the long protocol (W = K = 100), under a per-dispatch kernel trace
# and with GRBM_GUI_ACTIVE per dispatch (engine clock = cycles / duration).
# usage (GPU box): tools/driver_protocol.sh <outdir> [config]
set -o pipefail
OUT=${1:-gpurun_out/drv}; CFG=${2:-c1}
export TMPDIR=/tmp
mkdir -p $OUT
B="python3 bench.py --gpus 1 --config $CFG --no-cpu-baseline"
timeout -k 10 150 $B --steps 20 --warmup 5 > $OUT/plain_w5_k20_a.json 2> $OUT/plain_a.log &&
timeout -k 10 150 $B --steps 100 --warmup 100 > $OUT/plain_w100_k100.json 2> $OUT/plain_b.log &&
timeout -k 10 150 $B --steps 20 --warmup 5 > $OUT/plain_w5_k20_b.json 2> $OUT/plain_c.log &&
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_w5 -o run -- $B --steps 20 --warmup 5 > $OUT/trace_w5.json 2> $OUT/trace_w5.log &&
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_w100 -o run -- $B --steps 100 --warmup 100 > $OUT/trace_w100.json 2> $OUT/trace_w100.log &&
timeout -k 10 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/clk_w5 -o run -- $B --steps 20 --warmup 5 > $OUT/clk_w5.json 2> $OUT/clk_w5.log
