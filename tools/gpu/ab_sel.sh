#!/bin/bash
# occupancy draw + labels per realisation: the in-tree library against probe builds ($1, comma-separated),
# config 5 stated and bond L=4096, plus the select-window kernel under a kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
alts=${1:-v1}
for c in "c5 --L 8192 --kind sitebond --ps 0.593 --p 0.5" "bond --L 4096 --p 0.6"; do
  set -- $c; n=$1; shift
  timeout -k 10 300 python -u tools/lib_ab.py --what label "$@" --libs main,$alts > gpurun_out/abs_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abs_$n.log; exit 1; }
  echo "$n:"; grep -v "^\s*$" gpurun_out/abs_$n.log | tail -6 | cut -c1-200
done
