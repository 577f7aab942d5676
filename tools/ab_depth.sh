#!/usr/bin/env bash
# whole-solve A/B of the march prefetch depth on one box (bench.py twice each, interleaved)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for rep in 1 2; do
  for d in 3 2; do
    PERC_MARCH_DEPTH=$d timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      > gpurun_out/ab_d${d}_$rep.log 2>&1 || exit 1
  done
done
