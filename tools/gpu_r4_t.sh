#!/bin/bash
# round 4: config 2 in the literal order at tol 1e-8 (LDS-broadcast folds, guarded table division)
# against the fixture, then the literal and division tests
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/literal_config.py c2_sq1024_bond_p50 1e-08 > gpurun_out/r4t_literal_c2.log 2>&1
rc=$?; grep -v "^\.\.\. " gpurun_out/r4t_literal_c2.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_literal_dot.py \
  tests/test_gpu_parity.py -k "division or literal" > gpurun_out/r4t_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4t_pytest.log; exit $rc
