#!/bin/bash
# Round-4 gate call on the GPU box: the -m gpu suite, smoke() and the default
# bench.py line (configs, end_to_end, cpu_baseline).  Usage: bash tools/r04_gate.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_gate}
mkdir -p $O
step() { echo "[$(date +%T)] $1"; }
step tests
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
step bench
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json; echo
step done
