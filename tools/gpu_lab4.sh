set -o pipefail
mkdir -p gpurun_out/lab4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for x in 0 7; do
  PERC_ASM_EXP=$x timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/lab4/x$x -o run -- python3 $R/tools/label_probe.py --L 4096 --reps 4 > $R/gpurun_out/lab4/x$x.log 2>&1 || exit 1
done
