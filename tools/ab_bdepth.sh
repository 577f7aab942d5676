#!/usr/bin/env bash
# L = 4096 default solve: q-free march B prefetching 3 vs 2 rows (PERC_MARCH_BDEPTH), same realisation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for bd in 3 2 3 2; do
  PERC_MARCH_BDEPTH=$bd timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    >> gpurun_out/ab_bdepth_$bd.log 2>&1 || exit 1
done
