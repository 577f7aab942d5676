#!/usr/bin/env bash
# persistent march: bitwise parity test, then a same-box A/B against the
# launched kernels (one L = 4096 realisation per variant and round)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k persistent > gpurun_out/pm_test.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_march.py --L 4096 --rounds 2 --variants "PERSIST=0;PERSIST=1" \
  > gpurun_out/pm_ab.log 2>&1 || exit $?
