#!/usr/bin/env bash
# resident solve: tagged-granule all-gather reductions vs counter barrier
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
PERC_RES_GATHER=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_config_goldens.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "resident or config_fixture" > gpurun_out/gather_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for g in 0 1; do
    for L in 1024 2048; do
      PERC_RES_GATHER=$g timeout -k 10 300 python bench.py --L $L --p 0.6 --steps 4 --warmup 1 --no-cpu-baseline \
        > gpurun_out/gat_g${g}_L${L}_$rep.log 2>&1 || exit 1
    done
  done
done
