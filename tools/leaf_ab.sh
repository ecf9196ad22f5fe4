mkdir -p gpurun_out/r06_leaf
for L in 1 2 3 4; do
  RT_BVH_LEAF=$L timeout -k 10 300 python3 tools/probes/nonopq_scenes.py 128 > gpurun_out/r06_leaf/leaf$L.jsonl 2> gpurun_out/r06_leaf/leaf$L.err || exit 1
  sed "s/^/leaf $L /" gpurun_out/r06_leaf/leaf$L.jsonl
done
