#!/usr/bin/env bash
# resident solve: merged barrier+reduction vs separate (configs 2 and 4's shapes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for rep in 1 2; do
  for mg in 0 1; do
    for L in 1024 2048; do
      PERC_RES_MERGED=$mg timeout -k 10 300 python bench.py --L $L --p 0.6 --steps 4 --warmup 1 --no-cpu-baseline \
        > gpurun_out/res_m${mg}_L${L}_$rep.log 2>&1 || exit 1
    done
  done
done
