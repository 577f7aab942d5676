#!/bin/bash
# round 5, call v: the wave tile with each site loaded once per row (SL)
mkdir -p gpurun_out
timeout -k 10 300 ./tools/bin/cc_bench 8192 0.5 10 > gpurun_out/r5v_cc8192.log 2>&1
rc=$?; grep -E "site loads|mismatch|MISMATCH|differ|tile 16" gpurun_out/r5v_cc8192.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./tools/bin/cc_bench 4096 0.6 20 > gpurun_out/r5v_cc4096.log 2>&1
rc=$?; grep -E "site loads|mismatch|MISMATCH|differ|tile 16" gpurun_out/r5v_cc4096.log; exit $rc
