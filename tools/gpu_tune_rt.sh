# runtime-length fixed kernel: (NT, U) sweep at a few lengths per chunk count
set -o pipefail
cd $GRAFT_REPO_ROOT; O=${1:-gpurun_out/tune_rt}; mkdir -p $O
for L in 12 20 28 36 44 52 60; do
  if [ $L -le 16 ]; then V="nt=4,2;kpl=2,4,8"; else V="nt=4,2;kpl=2,4"; fi
  timeout -k 10 300 python3 tools/tune.py --n 50000000 --L $L --variants "$V" --rounds 3 > $O/L$L.txt 2>&1 || exit 1
  echo "== L=$L"; grep variant $O/L$L.txt | head -3
done
