#!/bin/bash
# cc_bench at L = 4096 / 8192 / 1000 (bond p = 0.6 / 0.5 / 0.6): the tile ring-depth sweep and the rest
mkdir -p gpurun_out
for c in "4096 0.6" "8192 0.5" "1000 0.6"; do
  set -- $c
  timeout -k 10 200 ./tools/bin/cc_bench $1 $2 10 > gpurun_out/ccd_$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/ccd_$1.log; exit 1; }
  echo "== L $1"; grep -E "tile depth|MISMATCH" gpurun_out/ccd_$1.log
done
