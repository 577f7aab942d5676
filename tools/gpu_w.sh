#!/usr/bin/env bash
# fine slot-weight A/B of the march P (event times without the system fence)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_march.py --L 4096 --rounds 3 \
  --variants "SLOTW=100:75:50;SLOTW=100:78:52;SLOTW=100:73:48;SLOTW=100:76:54;SLOTW=100:74:52" > gpurun_out/w_ab.log 2>&1
