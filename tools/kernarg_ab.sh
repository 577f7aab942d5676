cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
for r in 1 2; do
for v in unset 1 0; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  echo "== KERNARG=$v round $r" >> gpurun_out/kernarg_ab.log
  timeout -k 10 120 python tools/ab_march.py --L 4096 --rounds 1 --variants "" >> gpurun_out/kernarg_ab.log 2>&1 || exit 1
done
done
