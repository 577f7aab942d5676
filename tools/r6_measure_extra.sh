cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r6_8_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_8_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --inflight 1 > gpurun_out/r6_8_benchprof.json 2> gpurun_out/r6_8_benchprof.err || exit 1
timeout -k 10 400 python -u -m pytest tests/test_config_goldens.py -m gpu -s -v --timeout 300 --timeout-method thread -k test_config_fixture > gpurun_out/r6_8_config_distances.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --L 8192 --kind sitebond --ps 0.85 --p 0.85 --steps 1 --warmup 0 --itmax 300000 --no-cpu-baseline > gpurun_out/r6_8_c5_companion.json 2> gpurun_out/r6_8_c5_companion.err || exit 1
timeout -k 10 300 python3 bench.py --L 8192 --kind sitebond --ps 0.593 --p 0.50 --steps 32 --warmup 1 --no-cpu-baseline > gpurun_out/r6_8_c5_stated.json 2> gpurun_out/r6_8_c5_stated.err || exit 1
L=8192 PROBE_ARGS="--kind sitebond --ps 0.85 --p 0.85" TAG=mixed timeout -k 10 600 bash tools/pmc_r2.sh || exit 1
