#!/usr/bin/env bash
# round-end check: whole GPU suite, config fixtures with their numbers,
# smoke, default bench, rocprofv3 stats of a short bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_config_goldens.py -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/config_goldens.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1 || exit $?
