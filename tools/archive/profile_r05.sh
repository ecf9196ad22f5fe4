#!/bin/bash
# Round-5 measurement pass on the GPU box (one call): parity suite, smoke,
# the full bench line (configs, end_to_end, cpu_baseline), a
# rocprofv3 kernel trace of the same bench command and of the configs, the
# HBM-traffic PMC passes at HEAD (FETCH_SIZE, WRITE_SIZE), SQ passes for C2,
# and the C4 counter passes.  Usage: bash tools/profile_r05.sh TAG
set -o pipefail
TAG=${1:-r05_final}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
step() { echo "[$(date +%T)] $1"; }
step tests
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
step smoke
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
step bench
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json; echo
step kernel-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-pipeline > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg -o run --output-format csv -- python3 tools/bench_configs.py > $OUT/kt_cfg.log 2>&1 || { tail -20 $OUT/kt_cfg.log; exit 1; }
step pmc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 || { tail -5 $OUT/write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1 || { tail -5 $OUT/sq2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH -d $OUT/mix -o run --output-format csv -- $B > $OUT/mix.log 2>&1 || { tail -5 $OUT/mix.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU -d $OUT/flops -o run --output-format csv -- $B > $OUT/flops.log 2>&1 || { tail -5 $OUT/flops.log; exit 1; }
step pmc-c4
ONLY=C4,SWEEP bash tools/pmc_c4.sh $TAG/pmc_bvh || exit 1
step pmc-c3
ONLY=C3 SPP=200 bash tools/pmc_c4.sh $TAG/pmc_c3 || exit 1
step done
