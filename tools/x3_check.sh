#!/bin/bash
# Split-operand (bf16 x3) sweep: accuracy vs a host f64 sweep, A/B timing vs the f32 kernel.
mkdir -p gpurun_out/x3
O=gpurun_out/x3
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -8 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step acc_small 120 python tools/variant_accuracy.py --n 2048 --variants 0 2 3 --nq 1024
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 0 2 3 4 6 --rounds 2
