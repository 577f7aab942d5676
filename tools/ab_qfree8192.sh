#!/usr/bin/env bash
# L = 8192 (row-major march, past the Infinity Cache): q stored (10) vs q-free (11), one realisation each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for mm in 10 11; do
  timeout -k 10 300 python bench.py --L 8192 --p 0.6 --march-mode $mm --steps 1 --warmup 0 --itmax 100000 --no-cpu-baseline \
    > gpurun_out/abq8192_mm${mm}.log 2>&1 || exit 1
done
