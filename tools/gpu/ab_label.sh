#!/bin/bash
# labels per realisation: the current build against a probe build ($1), config 5 stated and bond L=4096
mkdir -p gpurun_out
export TMPDIR=/tmp
alt=${1:-pageable}
for c in "c5 --L 8192 --kind sitebond --ps 0.593 --p 0.5" "bond --L 4096 --p 0.6"; do
  set -- $c; n=$1; shift
  timeout -k 10 300 python -u tools/lib_ab.py --what label "$@" --libs main,$alt > gpurun_out/abl_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abl_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/abl_$n.log | cut -c1-140)"
done
