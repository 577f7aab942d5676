#!/bin/bash
# round 4 end: the §8(f) callers' throughput (threshold scans, bond_cond) on the final tree
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/scan_bench.py --L 256,1024 --trials 8 --cond-L 64,128 --cond-trials 2 \
  > gpurun_out/r4x_scan_bench.json 2> gpurun_out/r4x_scan_bench.err
rc=$?; cat gpurun_out/r4x_scan_bench.json; exit $rc
