#!/bin/bash
# round 4: wave tiles with relaxed wavefront-scope LDS atomics instead of volatile accesses, and
# k_cc_tile_v (branch-free row loads, a prefetch ring, run nodes in registers): labeling harness
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 ./tools/cc_bench 4096 0.6 20 > gpurun_out/r4o_cc_bench.log 2>&1
rc=$?; cat gpurun_out/r4o_cc_bench.log; exit $rc
