#!/usr/bin/env bash
# L = 4096: q stored (strip-major 26) vs q rebuilt in a marching B (q-free strip-major 27 at
# prefetch depth 3 and 2), one realisation each (the same one: device occupancy, same seed)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --march-mode 26 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/abq_mm26.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --march-mode 27 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/abq_mm27.log 2>&1 || exit 1
PERC_MARCH_DEPTH=2 timeout -k 10 200 python bench.py --march-mode 27 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/abq_mm27d2.log 2>&1 || exit 1
