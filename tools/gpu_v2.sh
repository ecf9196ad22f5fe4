set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02_v2; mkdir -p $OUT
timeout -k 10 120 ./tools/probes/op_rates2 > $OUT/op_rates2.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $OUT/kt.log 2>&1
echo "exit=$?" > $OUT/done.txt
