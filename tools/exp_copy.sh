#!/usr/bin/env bash
# STREAM-copy variants (perc_bench_kernel 4, PERC_COPY_VARIANT) on one system
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python tools/env_probe.py --L 1024 --which 4 --reps 20 --rounds 3 --sets \
  '[{}, {"PERC_COPY_VARIANT": 1}, {"PERC_COPY_VARIANT": 2}, {"PERC_COPY_VARIANT": 4}, {"PERC_COPY_VARIANT": 8}, {"PERC_COPY_VARIANT": 17}, {"PERC_COPY_VARIANT": 18}, {"PERC_COPY_VARIANT": 20}, {"PERC_COPY_VARIANT": 24}]' \
  > gpurun_out/copy_probe.json 2> gpurun_out/copy_probe.log
