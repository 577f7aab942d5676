#!/usr/bin/env bash
# L = 8192: row-major march (default) vs strip-major (PERC_MARCH_LARGE=1)
# with the march B on its own short bands (PERC_MARCH_BROWS); same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 700 python tools/ab_march.py --L 8192 --rounds 1 --itmax 200000 \
  --variants "LARGE=0;LARGE=1,BROWS=8;LARGE=1,BROWS=16;LARGE=1,BROWS=32;LARGE=1,BROWS=64" > gpurun_out/large_ab3.log 2>&1
