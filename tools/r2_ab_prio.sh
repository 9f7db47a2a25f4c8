#!/bin/bash
# A/B: static issue priority for waves 4-7 (51) or 0-3 (52) vs the default (3).
export TMPDIR=/tmp
O=gpurun_out/abp; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep variant $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step c4 300 env SBO_LIB=$D python tools/ab_variants.py --config C4 --variants 3 51 52 --rounds 5
step c3 300 env SBO_LIB=$D python tools/ab_variants.py --config C3 --variants 3 51 52 --rounds 4
step f0 300 env SBO_LIB=$D SBO_LVL_FORCE=0 python tools/ab_variants.py --config C4 --variants 3 51 52 --rounds 3
echo done
