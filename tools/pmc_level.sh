#!/usr/bin/env bash
# outstanding EA read/write requests (Little's law) of the CG kernels for the
# march band heights in $ROWS (tools/pmc_probe.py dispatch set)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in ${ROWS:-0}; do
  PERC_MARCH_ROWS=$r timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_cg_march|k_cg_b|k_copy" -f csv -d gpurun_out/pmc_level/rows$r -o run -- \
    python3 tools/pmc_probe.py >> gpurun_out/pmc_level.log 2>&1 || exit 1
  PERC_MARCH_ROWS=$r timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
    --kernel-include-regex "k_cg_march|k_cg_b|k_copy" -f csv -d gpurun_out/pmc_level/rows${r}_n -o run -- \
    python3 tools/pmc_probe.py >> gpurun_out/pmc_level.log 2>&1 || exit 1
done
