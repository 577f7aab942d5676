#!/usr/bin/env bash
# L = 4096 default solve: cache policies of the q-free march: last-use loads
# (PERC_MARCH_PAUX: P's p(k-1), PERC_MARCH_BAUX: B's r(k); 0 plain / 2 nt) and the
# p(k) / r(k+1) stores (PERC_MARCH_SAUX: 2 nt / 0 plain)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for cfg in "2 2 2" "2 2 0" "2 2 2" "2 2 0"; do
  set -- $cfg
  PERC_MARCH_PAUX=$1 PERC_MARCH_BAUX=$2 PERC_MARCH_SAUX=$3 timeout -k 10 200 python bench.py --steps 1 --warmup 0 \
    --no-cpu-baseline >> gpurun_out/ab_aux_$1_$2_$3.log 2>&1 || exit 1
done
