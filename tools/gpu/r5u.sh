#!/bin/bash
# round 5, call u: labeling tile height A/B (tools/cc_bench.hip) at L = 8192
mkdir -p gpurun_out
timeout -k 10 300 ./tools/bin/cc_bench 8192 0.5 10 > gpurun_out/r5u_cc8192.log 2>&1
rc=$?; cat gpurun_out/r5u_cc8192.log; exit $rc
