#!/bin/bash
# the labeling GPU tests, then labels per realisation: in-tree library vs probe builds ($1)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_labeling_oracle.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "label or occupy or span or cluster or partition" > gpurun_out/abl_tests.log 2>&1 || { tail -20 gpurun_out/abl_tests.log; exit 1; }
tail -1 gpurun_out/abl_tests.log
bash tools/gpu/ab_sel.sh ${1:-d2}
