#!/usr/bin/env bash
# PMC passes over the labeling-side kernels (tools/label_probe.py), one
# counter group per run; rocprofv3 -f csv under gpurun_out/pmc_label/p<i>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/pmc_label
export TMPDIR=/tmp
timeout -k 10 300 python -c "import torch; torch.cuda.init()" || exit 1
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT" \
            "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  echo "== pass $i: $ctrs" >> gpurun_out/pmc_label.log
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "k_cc_tile|k_assemble|k_cc_merge|k_select|k_cc_compress" \
    -f csv -d gpurun_out/pmc_label/p$i -o run -- python3 tools/label_probe.py --L 4096 --reps 2 \
    >> gpurun_out/pmc_label.log 2>&1 || { echo "pass $i failed rc=$?" >> gpurun_out/pmc_label.log; exit 1; }
done
