#!/usr/bin/env bash
# L = 4096 default solve: the q-free march at 3 rows prefetched (P 162 / B 148
# VGPRs, 3 waves per SIMD, 43-row bands) vs 2 rows prefetched held to 128
# VGPRs (4 waves per SIMD, 32-row bands; one round of resident waves either way)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for d in 3 2 3 2; do
  PERC_MARCH_DEPTH=$d timeout -k 10 200 python bench.py --steps 1 --warmup 0 \
    --no-cpu-baseline >> gpurun_out/ab_depth4w_$d.log 2>&1 || exit 1
done
