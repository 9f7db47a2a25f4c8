#!/bin/bash
# Bench lines for the other configs (C2, C3, C5) plus the variance error at
# N = 8192 under the default budget.  Logs under gpurun_out/cfg/.
export TMPDIR=/tmp
O=gpurun_out/cfg; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step bench_c3 400 python bench.py --config C3
step bench_c2 300 python bench.py --config C2
step bench_c5 400 python bench.py --config C5
step acc_8192 400 python tools/variant_accuracy.py --n 8192 --variants 3 --budget 20
echo done
