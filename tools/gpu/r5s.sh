#!/bin/bash
# round 5, call s: grid all-reduction transports (tools/sync_bench.hip)
mkdir -p gpurun_out
timeout -k 10 120 ./tools/bin/sync_bench 2000 > gpurun_out/r5s_sync.log 2>&1
rc=$?; cat gpurun_out/r5s_sync.log; exit $rc
