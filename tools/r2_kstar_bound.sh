#!/bin/bash
# Timing bounds (diagnostic build, wrong results): variant 53 = one-multiply K*
# evaluation, 41 = K* split reduced to kh, 54 = both; C4 default plan and every
# tile forced to one product.
export TMPDIR=/tmp
O=gpurun_out/kbound; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-5} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
SBO_LIB=$L/libsbo_diag.so step c4 300 python tools/ab_variants.py --config C4 --variants 3 53 41 54 --rounds 3
SBO_LIB=$L/libsbo_diag.so SBO_LVL_FORCE=2 step c4_lv2 300 python tools/ab_variants.py --config C4 --variants 3 53 41 54 --rounds 3
SBO_LIB=$L/libsbo_diag.so SBO_LVL_FORCE=0 step c4_lv0 300 python tools/ab_variants.py --config C4 --variants 3 53 41 54 --rounds 3
