#!/bin/bash
# the kernel trace summary of a 2-step bench (K = 1, no in-flight leg)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/po_prof -o bench -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --inflight 0 > gpurun_out/po_prof.log 2>&1 || { tail -20 gpurun_out/po_prof.log; exit 1; }
rm -f gpurun_out/po_prof/bench_kernel_trace.csv
