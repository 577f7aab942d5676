#!/bin/bash
# round 4: wave-deduplicated merge (every lattice), CSR S one row per thread, LDS CSR tiles and the
# register-node tile variant removed: the whole GPU suite, the labeling harness, a default bench line
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/cc_bench 4096 0.6 20 > gpurun_out/r4n_cc_bench.log 2>&1
rc=$?; cat gpurun_out/r4n_cc_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4n_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r4n_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r4n_bench.json 2> gpurun_out/r4n_bench.err
rc=$?; tail -c 2500 gpurun_out/r4n_bench.json; exit $rc
