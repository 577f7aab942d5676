#!/bin/bash
# round 5, call ab: the tile union-find's find returning a root found one hop
# up without a third read, against the old loop (two harness builds, twice each)
mkdir -p gpurun_out
for b in old new old new; do
  exe=./tools/bin/cc_bench; [ $b = old ] && exe=./tools/bin/cc_bench_old
  timeout -k 10 200 $exe 8192 0.5 10 > gpurun_out/r5ab_$b.log 2>&1 || { echo "$b failed"; exit 1; }
  echo "== $b"; grep -E "tile 16 rows|MISMATCH|chain wave 16 \(|production\)" gpurun_out/r5ab_$b.log | head -8
done
