#!/bin/bash
# A/B of two cc_bench builds (tools/bin/cc_bench vs tools/bin/cc_bench_$1), twice each, L = 8192
mkdir -p gpurun_out
alt=${1:-pj}
for b in base $alt base $alt; do
  exe=./tools/bin/cc_bench; [ $b = $alt ] && exe=./tools/bin/cc_bench_$alt
  timeout -k 10 200 $exe 8192 0.5 10 > gpurun_out/abt_$b.log 2>&1 || { echo "$b failed"; tail -5 gpurun_out/abt_$b.log; exit 1; }
  echo "== $b"; grep -E "tile 16 rows|MISMATCH|chain wave 128 x 16 \(production\)|square merge  " gpurun_out/abt_$b.log | head -8
done
