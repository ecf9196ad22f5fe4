#!/bin/bash
# GPU step: the whole GPU suite, smoke, the default bench line and a
# rocprofv3 kernel trace of the bench.  Usage: bash tools/final_check.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $OUT/kt.log 2>&1
