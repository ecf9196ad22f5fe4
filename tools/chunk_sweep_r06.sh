#!/bin/bash
# C2 headline at spp_chunks 8 / 12 / 16 / 32: bench.py's
# pipelined rate and the --no-pipeline kernel rate, alternating twice.
# Usage: bash tools/chunk_sweep_r06.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r06_chunks}
mkdir -p $OUT
for rep in 1 2; do
  for P in 32 16 12 8; do
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --chunks $P > $OUT/p${P}_r${rep}.json 2> $OUT/p${P}_r${rep}.err || exit 1
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --chunks $P --no-pipeline > $OUT/p${P}_np_r${rep}.json 2> $OUT/p${P}_np_r${rep}.err || exit 1
    echo "P=$P rep=$rep $(cut -c1-120 $OUT/p${P}_r${rep}.json)"
  done
done
