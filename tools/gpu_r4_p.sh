#!/bin/bash
# round 4: the wave tiles with branch-free row loads, a prefetch ring and run nodes in registers
# (every kind of the open square lattice): labeling harness, the whole GPU suite, a default bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 ./tools/cc_bench 4096 0.6 20 > gpurun_out/r4p_cc_bench.log 2>&1
rc=$?; cat gpurun_out/r4p_cc_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4p_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r4p_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r4p_bench.json 2> gpurun_out/r4p_bench.err
rc=$?; tail -c 2500 gpurun_out/r4p_bench.json; exit $rc
