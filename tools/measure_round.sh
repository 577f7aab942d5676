#!/usr/bin/env bash
# One GPU call's measurement set for the bench line's evidence (round 6):
# the default bench, a rocprofv3 --kernel-trace --stats pass over a short
# bench (without the in-flight leg, whose two concurrent solves would
# stretch every launch), and the PMC reconciliation at L = 4096
# (tools/pmc_r2.sh).  Every
# step under its own time limit; stops at the first failure.
#   TAG=r6_7 bash tools/measure_round.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${TAG:-rX}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err" || exit 1
rm -rf "gpurun_out/${TAG}_prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_prof" -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --inflight 1 > "gpurun_out/${TAG}_benchprof.json" \
  2> "gpurun_out/${TAG}_benchprof.err" || exit 1
TAG="" L=4096 timeout -k 10 600 bash tools/pmc_r2.sh || exit 1
