set -o pipefail
mkdir -p gpurun_out/lab1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_labeling_oracle.py tests/test_gpu_parity.py > gpurun_out/lab1/tests.log 2>&1 && \
PERC_TILE_TRACE=1 timeout -k 10 300 python tools/label_probe.py --L 4096 --reps 8 > gpurun_out/lab1/probe.json 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/lab1/prof -o run -- python3 $R/tools/label_probe.py --L 4096 --reps 8 > $R/gpurun_out/lab1/prof.log 2>&1
