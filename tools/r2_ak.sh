#!/bin/bash
# A/B (diagnostic build): 57 = the default reading sf2 alpha only before the mean's row block.
export TMPDIR=/tmp
O=gpurun_out/ak; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep variant $O/$name.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
SBO_LIB=$L/libsbo_diag.so step c4 300 python tools/ab_variants.py --config C4 --variants 3 57 3 57 --rounds 3
SBO_LIB=$L/libsbo_diag.so step c3 300 python tools/ab_variants.py --config C3 --variants 3 57 --rounds 3
SBO_LIB=$L/libsbo_diag.so SBO_LVL_FORCE=2 step c4_lv2 300 python tools/ab_variants.py --config C4 --variants 3 57 --rounds 3
