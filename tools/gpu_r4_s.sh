#!/bin/bash
# round 4: the table division guarded near underflow: its self-test (now with subnormal-range
# numerators) and the literal tests, then config 2 in the literal order at tol 1e-8 against the fixture
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_literal_dot.py \
  tests/test_gpu_parity.py -k "division or literal" > gpurun_out/r4s_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4s_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 960 python -u tools/literal_config.py c2_sq1024_bond_p50 1e-08 > gpurun_out/r4s_literal_c2.log 2>&1
rc=$?; grep -v "^\.\.\. " gpurun_out/r4s_literal_c2.log | tail -2; exit $rc
