#!/bin/bash
# round 4 end: the BASELINE configs 2-5 on the final tree (tools/configs.sh)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/configs.log
bash tools/configs.sh || { tail -5 gpurun_out/configs.log; exit 1; }
tail -12 gpurun_out/configs.log
