# SQ counters (wave cycles split: active / waiting / issue-stall; VALU, LDS
# and VMEM instruction counts) of the CG kernels under an env switch
# usage: bash tools/pmc_sq.sh "1 0"   (values of PERC_NT)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
for v in $1; do
  PERC_NT=$v timeout -k 10 300 rocprofv3 --kernel-trace \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES \
    -d gpurun_out/pmc_sq_$v -o run --output-format csv -- \
    python3 tools/ps_probe.py --sizes 4096 --itmax 3 --reps 20 > gpurun_out/pmc_sq_$v.log 2>&1 || exit 1
done
