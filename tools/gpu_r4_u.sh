#!/bin/bash
# round 4 end: the whole GPU suite and smoke on the final tree, then a default bench line
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4u_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r4u_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4u_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r4u_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r4u_bench.json 2> gpurun_out/r4u_bench.err
rc=$?; tail -c 1500 gpurun_out/r4u_bench.json; exit $rc
