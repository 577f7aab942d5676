#!/usr/bin/env bash
# strip-major march (memory-path fix applied) vs row-major, full solve, one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_slabs.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "march or bitwise or boundary or conductance or slabs or resident" > gpurun_out/strips_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for mm in 10 26; do
    timeout -k 10 300 python bench.py --march-mode $mm --steps 2 --warmup 1 --no-cpu-baseline \
      > gpurun_out/ab_mm${mm}_$rep.log 2>&1 || exit 1
  done
done
