#!/bin/bash
# 2-rank functional run of bench.py on ONE GPU (gloo; both ranks share cuda:0):
# exercises the cost-balanced cut, its broadcast and the key all-gather.
export TMPDIR=/tmp
mkdir -p gpurun_out/gloo2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --no-cpu > gpurun_out/gloo2/c4.log 2>&1
rc=$?; grep '"metric"' gpurun_out/gloo2/c4.log | cut -c1-400; exit $rc
