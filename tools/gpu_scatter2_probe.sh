#!/bin/bash
# f2 pass-2 write amplification probe: time and WRITE_SIZE per mode
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
O=gpurun_out/s2probe; mkdir -p $O
MODES=${MODES:-1 2 3}
for m in $MODES; do
  timeout -k 10 60 tools/scatter2_probe $m 100 10 >> $O/time.jsonl || exit 1
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$m -o run -- tools/scatter2_probe $m 100 3 > $O/w$m.log 2>&1 || exit 1
done
cat $O/time.jsonl
for m in $MODES; do python3 tools/pmc_summary.py $O/w$m > $O/w$m.json || exit 1; done
python3 -c "
import json
for m in [int(x) for x in '$MODES'.split()]:
    d=json.load(open('$O/w%d.json'%m))
    for k,v in d.items():
        if 'probe' in k: print('mode', m, k[:40], 'WRITE GB per launch', round(v['WRITE_SIZE']*1024/1e9,3), 'alg GB', 2.4 if m<4 else 'see time.jsonl')
"
