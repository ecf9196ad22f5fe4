#!/bin/bash
# spp_chunks P = 32 / 16 / 12 on every config: full-spp
# kernel rates of C3, C4, nature, C5 (tools/bench_configs.py) and rank 0's
# share of an N-way cyclic split of C2 (tools/rank_share_rate.py, 1-row
# tiles, two frames in flight).  Usage: bash tools/chunk_cfg_r06.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r06_chunkcfg}
mkdir -p $OUT
for P in 32 12 16; do
  timeout -k 10 300 python3 tools/bench_configs.py --only C3,C4,NATURE,C5 --full-spp --chunks $P > $OUT/cfg_p$P.jsonl 2> $OUT/cfg_p$P.err || exit 1
  timeout -k 10 300 python3 tools/rank_share_rate.py --chunks $P --pipeline --tile-rows 1 > $OUT/share_p$P.jsonl 2> $OUT/share_p$P.err || exit 1
  echo "P=$P done"
done
