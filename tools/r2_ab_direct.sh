#!/bin/bash
# A/B: one- (42) and three-product (43) tiles accumulated straight into the
# outer sums vs the default per-tile chains (3); accuracy vs a host f64 sweep.
export TMPDIR=/tmp
O=gpurun_out/abd; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 3 42 43 22 --rounds 3
step ab_c3 300 python tools/ab_variants.py --config C3 --variants 3 42 43 --rounds 3
step acc 400 python tools/variant_accuracy.py --n 8192 16384 --variants 3 42 43 22 --nq 2048
echo done
