#!/bin/bash
# kernel + memory-copy trace of per-realisation labeling (tools/lib_ab.py's label child), one realisation's timeline
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in "bond --L 4096 --p 0.6" "c5 --L 8192 --kind sitebond --ps 0.593 --p 0.5"; do
  set -- $c; n=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/lt_$n -o lt -- python3 -u tools/lib_ab.py --child --what label "$@" --reps 6 > gpurun_out/lt_$n.log 2>&1 || { tail -5 gpurun_out/lt_$n.log; exit 1; }
  echo "== $n"; python3 tools/label_timeline.py gpurun_out/lt_$n 4
done
