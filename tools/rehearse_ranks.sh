#!/bin/bash
# Multi-rank rehearsal on ONE GPU (all ranks share cuda:0; gloo gathers through
# host copies): bench.py at N ranks with --verify (rank 0 re-renders the frame
# alone and compares the assembled colour bit for bit).  -> gpurun_out/rehearse/
mkdir -p gpurun_out/rehearse
for N in ${NS:-2 4}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29600 + N)) bench.py --gpus $N --steps 2 --warmup 1 --dist-backend gloo --verify \
      --no-cpu-baseline ${EXTRA} > gpurun_out/rehearse/n$N.json 2> gpurun_out/rehearse/n$N.err || { echo "N=$N failed"; tail -5 gpurun_out/rehearse/n$N.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rehearse/n$N.json').read().strip().splitlines()[-1]); print('N=$N', d['value'], d.get('verified_vs_single_device'), d['config'].get('gather_payload'))"
done
