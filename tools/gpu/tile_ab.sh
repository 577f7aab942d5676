#!/bin/bash
# cc_bench base vs a variant build (tools/bin/cc_bench_$1), alternating, L = 8192 p 0.5 and 4096 p 0.6
mkdir -p gpurun_out
alt=${1:-flat}
for L in "8192 0.5" "4096 0.6"; do
  set -- $L $alt
  for b in base $3 base $3; do
    exe=./tools/bin/cc_bench; [ $b = $3 ] && exe=./tools/bin/cc_bench_$3
    timeout -k 10 200 $exe $1 $2 10 > gpurun_out/tab_$b.log 2>&1 || { echo "$b failed"; tail -5 gpurun_out/tab_$b.log; exit 1; }
    echo "== L $1 $b"; grep -E "tile 16 rows|mixed kind: D|site kind: D|ballots.*MISMATCH" gpurun_out/tab_$b.log
  done
done
