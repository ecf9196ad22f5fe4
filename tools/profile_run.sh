#!/bin/bash
# GPU measurement pass: parity tests, bench (+CPU baseline), rocprofv3 kernel
# trace + PMC passes, host-path rate, demo.  Usage: bash tools/profile_run.sh TAG
set -o pipefail
TAG=${1:-run}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err &&
ps -u "$(id -u)" -o pid,ppid,etimes,args > $OUT/ps_after_bench.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $OUT/kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg -o run --output-format csv -- python3 tools/bench_configs.py > $OUT/kt_cfg.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH -d $OUT/mix -o run --output-format csv -- $B > $OUT/mix.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU -d $OUT/flops -o run --output-format csv -- $B > $OUT/flops.log 2>&1 &&
ONLY=C4,SWEEP bash tools/pmc_c4.sh $TAG/pmc_bvh &&
timeout -k 10 200 python3 tools/host_path_rate.py > $OUT/host_path.json 2> $OUT/host_path.err &&
timeout -k 10 100 ./tipe-raytracer_amd/rt_demo -w 400 -s 100 -b 5 -o $OUT/demo.ppm > $OUT/demo.log 2>&1
echo "exit=$?" > $OUT/done.txt
