# SQ counters of the CG kernels per march mode (tools/march_probe.py,
# whole iterations on the L = 4096 system); summary: tools/sq_summary.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in ${MODES:-2 6}; do
  timeout -k 10 300 rocprofv3 --kernel-trace \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES \
    -d gpurun_out/pmc_sq_m$mode -o run --output-format csv -- \
    python3 tools/march_probe.py --modes $mode --reps 10 --solve-L 0 > gpurun_out/pmc_sq_m$mode.log 2>&1 || exit 1
done
