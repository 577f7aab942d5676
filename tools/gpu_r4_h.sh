#!/bin/bash
# round 4: the GPU suite on the one-row-per-thread CSR SpMV, the wave-per-block labeling of
# the open square lattice, ConductCalc weights from C, the bondocc.txt trace; labeling and
# SpMV harnesses; the split-solve bench with the Python loop over "nccl" (tensor placement fix)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4h_pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/r4h_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/cc_bench 4096 0.6 20 > gpurun_out/r4h_cc_bench.log 2>&1
rc=$?; cat gpurun_out/r4h_cc_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/spmv_bench 4096 20 > gpurun_out/r4h_spmv_bench.log 2>&1
rc=$?; cat gpurun_out/r4h_spmv_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/dslab_bench.py --L 4096 --iters 2000 --reps 2 --torch > gpurun_out/r4h_dslab_bench.json 2> gpurun_out/r4h_dslab_bench.err
rc=$?; cat gpurun_out/r4h_dslab_bench.json; tail -3 gpurun_out/r4h_dslab_bench.err; exit $rc
