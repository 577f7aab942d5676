#!/usr/bin/env bash
# shorter tagged reduction tail: bitwise tests of the march modes, then a
# same-box A/B (PERC_MARCH_TAG=0: ticket reduction with drains) and the
# device-kernarg A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "deferred or persistent or band_heights or one_iteration or slot" > gpurun_out/tag_test.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_march.py --L 4096 --rounds 2 --variants "TAG=1;TAG=0" \
  > gpurun_out/tag_ab.log 2>&1 || exit $?
for v in 1 0; do
  echo "== HIP_FORCE_DEV_KERNARG=$v" >> gpurun_out/kernarg_ab.log
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python tools/ab_march.py --L 4096 --rounds 1 --variants "" >> gpurun_out/kernarg_ab.log 2>&1 || exit $?
done
