#!/bin/bash
# C4 / sweep counter passes (tools/pmc_c4.sh) of each library variant named in $VARS
# (tools/variants/<name>.so) -> gpurun_out/TAG/<name>/pmc
TAG=${1:-r05_pmcv}
for n in ${VARS:-a_base}; do
  echo "[$(date +%T)] pmc $n"
  RT_HIP_LIB=tools/variants/$n.so ONLY=${ONLY:-C4} SPP=${SPP:-256} bash tools/pmc_c4.sh $TAG/$n || exit 1
  grep -q "exit=0" gpurun_out/$TAG/$n/done.txt || { echo "pmc $n failed"; exit 1; }
done
