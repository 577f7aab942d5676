#!/bin/bash
# the strip-major march's halo columns from the edge arrays against the
# neighbouring strips (probe build noedge): 20000-iteration solves and
# probes, then the march / literal parity tests
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/lib_ab.py --L 4096 --libs main,noedge --iters 20000 --reps 10 --rounds 2 > gpurun_out/abe_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -1 gpurun_out/abe_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_literal_dot.py tests/test_gpu_parity.py -m gpu -x -q -k "march or literal or nibble or tag or strip" --timeout 300 --timeout-method thread > gpurun_out/abe_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/abe_pytest.log; exit $rc
