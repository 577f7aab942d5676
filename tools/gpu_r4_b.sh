#!/bin/bash
# round 4: full GPU suite, then the default bench (CPU anchors beside it)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4_pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/r4_pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err
rc=$?
tail -c 4000 gpurun_out/r4_bench.json; tail -8 gpurun_out/r4_bench.err
exit $rc
