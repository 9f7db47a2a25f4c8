#!/bin/bash
# A/B: A stage loaded by all eight waves (3), by waves 0-3 (47: the older
# wave of each SIMD pair, which idles at the barrier) or 4-7 (48).
export TMPDIR=/tmp
O=gpurun_out/abl; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-4} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step c4 300 env SBO_LIB=$D python tools/ab_variants.py --config C4 --variants 3 47 48 --rounds 4
step c3 300 env SBO_LIB=$D python tools/ab_variants.py --config C3 --variants 3 47 48 --rounds 4
step c4f0 300 env SBO_LIB=$D SBO_LVL_FORCE=0 python tools/ab_variants.py --config C4 --variants 3 47 --rounds 3
step c4f2 300 env SBO_LIB=$D SBO_LVL_FORCE=2 python tools/ab_variants.py --config C4 --variants 3 47 --rounds 3
echo done
