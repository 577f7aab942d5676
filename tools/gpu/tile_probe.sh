#!/bin/bash
# cost probes of the wave tile (cc_bench builds with PERC_TILE_PROBE_*: wrong partitions, timing only), L = 8192
mkdir -p gpurun_out
for b in "" _nounion _nofinal _nounion_nofinal; do
  timeout -k 10 200 ./tools/bin/cc_bench$b 8192 0.5 10 > gpurun_out/tp$b.log 2>&1 || { echo "$b failed"; tail -5 gpurun_out/tp$b.log; exit 1; }
  echo "== base$b"; grep -E "tile 16 rows|tile depth" gpurun_out/tp$b.log
done
