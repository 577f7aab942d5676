#!/usr/bin/env bash
# phase probe of the resident solve (PERC_RES_TRACE): L = 1024 with
# and L = 2048; one realisation each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
rm -f gpurun_out/res_trace_*.csv
for cfg in "1024 1024" "2048 1024"; do
  set -- $cfg
  PERC_RES_TRACE=gpurun_out/res_trace_$1_$2.csv timeout -k 10 200 python bench.py --L $1 --p 0.6 \
    --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/res_trace_$1_$2.log 2>&1 || exit 1
done
