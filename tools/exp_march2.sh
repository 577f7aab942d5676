#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_slabs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "march or bitwise or boundary or conductance or slabs" > gpurun_out/march2_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/env_probe.py --rounds 2 --sets '[{}, {"PERC_MARCH_ROWS": 32}, {"PERC_MARCH_ROWS": 48}, {"PERC_MARCH_ROWS": 64}, {"PERC_MARCH_ROWS": 24}]' > gpurun_out/march2_probe.json 2> gpurun_out/march2_probe.log || exit 1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/march2_bench.log 2>&1
