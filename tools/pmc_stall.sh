#!/usr/bin/env bash
# Memory-side queue occupancy of the march P+S vs the streaming B kernel
# (tools/pmc_probe.py dispatch set): outstanding EA read / write requests
# integrated over cycles (Little's law: level / requests = mean latency in
# cycles), DRAM credit stalls, TCC busy cycles.  One counter group per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
L=${L:-4096}
i=5
for ctrs in "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE" \
            "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum"; do
  i=$((i + 1))
  echo "== pass $i: $ctrs" >> gpurun_out/pmc_stall.log
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "k_cg_march|k_cg_b|k_copy" \
    -f csv -d gpurun_out/pmc_r2/p$i -o run -- python3 tools/pmc_probe.py --L $L \
    >> gpurun_out/pmc_stall.log 2>&1 || { echo "pass $i failed rc=$?" >> gpurun_out/pmc_stall.log; exit 1; }
done
