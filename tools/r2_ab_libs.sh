#!/bin/bash
# A/B of this tree's libsbo.so against lib/libsbo_base.so (alternating
# processes), C4 and C3 default sweep; bitwise comparison first.
export TMPDIR=/tmp
O=gpurun_out/abx; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-1} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 400 python tools/compare_libs.py $L/libsbo_base.so $L/libsbo.so --configs C4 C2 box > $O/cmp.log 2>&1; echo "cmp rc=$?"; tail -20 $O/cmp.log
for r in 1 2 3; do
  SBO_LIB=$L/libsbo_base.so step base_c4_$r 200 python tools/ab_variants.py --config C4 --variants 3 --rounds 3
  step new_c4_$r 200 python tools/ab_variants.py --config C4 --variants 3 --rounds 3
done
SBO_LIB=$L/libsbo_base.so step base_c3 200 python tools/ab_variants.py --config C3 --variants 3 --rounds 3
step new_c3 200 python tools/ab_variants.py --config C3 --variants 3 --rounds 3
echo done
