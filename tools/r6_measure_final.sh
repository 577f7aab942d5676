#!/usr/bin/env bash
# Round 6's final measurement set, one GPU call: the L = 4096 bench line with
# its rocprof / PMC evidence (tools/measure_round.sh), config 5's companion
# and its PMC reconciliation at L = 8192, config 5 as stated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6_24}
TAG=$TAG bash tools/measure_round.sh || exit 1
timeout -k 10 300 python3 bench.py --L 8192 --kind sitebond --ps 0.85 --p 0.85 --steps 1 --warmup 0 --itmax 300000 \
  --no-cpu-baseline > "gpurun_out/${TAG}_c5_companion.json" 2> "gpurun_out/${TAG}_c5_companion.err" || exit 1
timeout -k 10 300 python3 bench.py --L 8192 --kind sitebond --ps 0.593 --p 0.50 --steps 32 --warmup 1 \
  --no-cpu-baseline > "gpurun_out/${TAG}_c5_stated.json" 2> "gpurun_out/${TAG}_c5_stated.err" || exit 1
L=8192 PROBE_ARGS="--kind sitebond --ps 0.85 --p 0.85" TAG=mixed timeout -k 10 600 bash tools/pmc_r2.sh || exit 1
