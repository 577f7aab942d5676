#!/bin/bash
# the march's bitwise tests, then a same-box solve A/B of the in-tree library against probe builds ($1,
# comma-separated) at L = 4096 bond p = 0.6 (kernel probes + fixed-iteration solve slope)
mkdir -p gpurun_out
export TMPDIR=/tmp
alts=${1:-gc}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_literal_dot.py -m gpu -x -q --timeout 200 --timeout-method thread -k "tagged or march_modes or band_heights or oracle_linbcg" > gpurun_out/abv_tests.log 2>&1 || { tail -20 gpurun_out/abv_tests.log; exit 1; }
tail -1 gpurun_out/abv_tests.log
timeout -k 10 500 python -u tools/lib_ab.py --L 4096 --libs main,$alts --rounds ${ROUNDS:-3} > gpurun_out/abv_solve.log 2>&1 || { tail -5 gpurun_out/abv_solve.log; exit 1; }
grep -v "^\s*$" gpurun_out/abv_solve.log | tail -4 | cut -c1-600
