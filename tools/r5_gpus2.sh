#!/bin/bash
# Round 5: the N = 2 path on the one-GPU box (both ranks on its GPU, gloo).
export TMPDIR=/tmp
O=gpurun_out/r5g2; mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 2 --no-cpu --no-regimes > $O/bench2.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{' $O/bench2.log | cut -c1-400; tail -3 $O/bench2.log | cut -c1-300; exit $rc
