#!/bin/bash
# All bench lines of the round: C4 default (with CPU baseline and regimes),
# C3, C2, C5 (streaming).  Logs under gpurun_out/benchall/.
export TMPDIR=/tmp
O=gpurun_out/benchall; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step c4 400 python bench.py --steps 20
step c3 200 python bench.py --config C3 --no-cpu --no-regimes --steps 10
step c2 200 python bench.py --config C2 --no-cpu --no-regimes --steps 20
step c5 300 python bench.py --config C5 --steps 50
echo done
