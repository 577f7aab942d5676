# BASELINE.json configs 2-5 on one GPU (config 4's per-GPU shape), one call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
run() {  # run NAME TIMEOUT ARGS...
  local name=$1 to=$2
  shift 2
  echo "== $name: $*" >> gpurun_out/configs.log
  timeout -k 10 "$to" python bench.py "$@" > "gpurun_out/cfg_$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> gpurun_out/configs.log
  [ "$rc" -eq 0 ] || exit "$rc"
}
run c2_sq1024_bond_p50 600 --L 1024 --p 0.50 --steps 64 --warmup 1 --no-cpu-baseline
run c3_tri1024_site_p50 600 --L 1024 --lattice tri --kind site --p 0.50 --steps 32 --warmup 1 --no-cpu-baseline
run c4_sq2048_bond_p50 600 --L 2048 --p 0.50 --steps 16 --warmup 1 --no-cpu-baseline
# config 5 as BASELINE.json states it (below the mixed threshold: labeling + spanning test, G = 0)
run c5_sq8192_mixed_stated 300 --L 8192 --kind sitebond --ps 0.593 --p 0.50 --steps 32 --warmup 1 --no-cpu-baseline
# ... with two realisations in flight (two contexts, each its own stream)
run c5_sq8192_mixed_stated_k2 300 --L 8192 --kind sitebond --ps 0.593 --p 0.50 --steps 64 --warmup 2 --concurrent 2 --no-cpu-baseline
run c5_sq8192_mixed_p85 650 --L 8192 --kind sitebond --ps 0.85 --p 0.85 --steps 1 --warmup 0 --itmax 300000 --no-cpu-baseline
