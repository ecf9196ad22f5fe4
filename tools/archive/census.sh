#!/bin/bash
# Round census of render_kernel_q per scene with the diagnostic build
# tools/variants/qstats.so (-DRT_QSTATS=1 of the r03 e313b16 kernel, which
# still carried the census hooks).  Usage: bash tools/census.sh OUT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-census}
mkdir -p $OUT
for sc in c2 c3 c4 sweep; do
  spp=256; [ $sc = c4 ] && spp=64
  RT_HIP_LIB=tools/variants/qstats.so timeout -k 10 200 python3 tools/qstats.py $spp $sc >> $OUT/census.jsonl 2> $OUT/census_$sc.err || { echo "census $sc failed"; tail -5 $OUT/census_$sc.err; exit 1; }
done
cat $OUT/census.jsonl
