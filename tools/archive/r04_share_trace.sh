#!/bin/bash
# Kernel trace of the rank-share frames (N = 1, 2, 4, 8 on one GPU, two
# streams): where a frame's fixed cost goes.  Usage: bash tools/r04_share_trace.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_share_trace}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv \
   -- python3 $GRAFT_REPO_ROOT/tools/rank_share_rate.py --chunks 32 --pipeline --tile-rows 1 --reps 6 > $GRAFT_REPO_ROOT/$O/share.jsonl 2> $GRAFT_REPO_ROOT/$O/kt.log || { tail -5 $GRAFT_REPO_ROOT/$O/kt.log; exit 1; }
cat $GRAFT_REPO_ROOT/$O/share.jsonl
