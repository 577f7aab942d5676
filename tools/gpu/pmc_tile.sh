#!/bin/bash
# SQ counters of the labeling wave tiles (tools/cc_bench at L = 4096), one
# counter group per pass
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmct_list.txt 2>&1
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
            "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU"; do
  i=$((i + 1))
  rm -rf gpurun_out/pmct/p$i
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-include-regex "k_cc_tile_w" -f csv -d gpurun_out/pmct/p$i -o run \
    -- ./tools/bin/cc_bench 4096 0.6 3 > gpurun_out/pmct_p$i.log 2>&1
  echo "pass $i rc=$?"
done
