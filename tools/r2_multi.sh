#!/bin/bash
# Multi-rank paths on the one-GPU box: bench.py --gpus 2 launching its own
# ranks (gloo, both on cuda:0), and the 8-rank shard emulation of C4.
export TMPDIR=/tmp
O=gpurun_out/multi; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step gloo2 400 python bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo --no-cpu --no-regimes
TAILN=10 step shards 400 python tools/shard_emulate.py --config C4 --balance 0
echo done
