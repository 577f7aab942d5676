set -o pipefail
mkdir -p gpurun_out/lab1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/lab1/prof -o run -- python3 $R/tools/label_probe.py --L 4096 --reps 8 > $R/gpurun_out/lab1/prof.log 2>&1
