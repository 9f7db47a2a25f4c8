#!/bin/bash
# Stress box (lpsc.yaml box, C4 N and grid): the default mixed-level plan vs
# every kept tile forced to one level (diagnostic build) and variant 22.
export TMPDIR=/tmp
O=gpurun_out/box; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step mix 300 env SBO_LIB=$D python tools/ab_variants.py --config C4 --box --variants 3 22 --rounds 1
for l in 0 1 2; do step force$l 300 env SBO_LIB=$D SBO_LVL_FORCE=$l python tools/ab_variants.py --config C4 --box --variants 3 --rounds 1; done
step span_mix 300 env SBO_LIB=$D python tools/x3_stamps.py --config C4 --box --variant 46
step span_f0 300 env SBO_LIB=$D SBO_LVL_FORCE=0 python tools/x3_stamps.py --config C4 --box --variant 46
echo done
