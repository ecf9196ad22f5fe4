# bench.py kernel rate at N=1 for several spp_chunks values
for ch in 8 16 32 64; do
  RT_BENCH_CHUNKS=$ch timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cs.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/cs.json').read()); print('chunks', $ch, d['value'], d['roofline']['kernel_ms'])"
done
