#!/bin/bash
# the default bench line and the kernel trace summary of a 2-step bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/bp_bench.log 2>&1 || { tail -20 gpurun_out/bp_bench.log; exit 1; }
grep "^{" gpurun_out/bp_bench.log | tail -1 | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bp_prof -o bench -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --inflight 0 > gpurun_out/bp_prof.log 2>&1 || { tail -20 gpurun_out/bp_prof.log; exit 1; }
rm -f gpurun_out/bp_prof/bench_kernel_trace.csv
