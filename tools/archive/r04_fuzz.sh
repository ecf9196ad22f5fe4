#!/bin/bash
# Round-4 fuzz call: the GPU fuzz tests (incl. the opaque-instantiation
# families) and a fuzz campaign on unused seeds.  Usage: bash tools/r04_fuzz.sh TAG [N] [SEED]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_fuzz}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_instantiations.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_fuzz.log 2>&1 || { tail -30 $O/pytest_fuzz.log; exit 1; }
tail -1 $O/pytest_fuzz.log
timeout -k 10 900 python3 -u tools/fuzz_campaign.py $O/fuzz.json ${2:-1000} ${3:-70000} > $O/fuzz.log 2>&1 || { tail -20 $O/fuzz.log; exit 1; }
tail -1 $O/fuzz.log
