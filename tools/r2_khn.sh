#!/bin/bash
# A/B (diagnostic build): variant 55 = variant 3 with a kh-only K* split
# whenever a one-product step follows a one-product step.
export TMPDIR=/tmp
O=gpurun_out/khn; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep variant $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
SBO_LIB=$L/libsbo_diag.so step c4 300 python tools/ab_variants.py --config C4 --variants 3 55 56 3 55 56 --rounds 3
SBO_LIB=$L/libsbo_diag.so step c3 300 python tools/ab_variants.py --config C3 --variants 3 55 56 --rounds 3
SBO_LIB=$L/libsbo_diag.so step c2 300 python tools/ab_variants.py --config C2 --variants 3 55 56 --rounds 5
SBO_LIB=$L/libsbo_diag.so SBO_LVL_FORCE=2 step c4_lv2 300 python tools/ab_variants.py --config C4 --variants 3 55 56 --rounds 3
