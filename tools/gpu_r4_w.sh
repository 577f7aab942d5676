#!/bin/bash
# round 4 end: rocprofv3 kernel-trace of a short default bench on the final tree
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_w -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r4w_bench_prof.json 2> gpurun_out/r4w_bench_prof.err
rc=$?; tail -c 800 gpurun_out/r4w_bench_prof.json; exit $rc
