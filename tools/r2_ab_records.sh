#!/bin/bash
# A/B of the step-record staging (this tree's libsbo.so) against the previous
# build (lib/libsbo_base.so): bitwise outputs, sweep times, then the GPU tests.
export TMPDIR=/tmp
O=gpurun_out/abr; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-6} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
TAILN=20 step cmp 400 python tools/compare_libs.py $L/libsbo_base.so $L/libsbo.so --configs C4 C2 box
SBO_LIB=$L/libsbo_base.so step base1 200 python tools/ab_variants.py --config C4 --variants 3 22 --rounds 3
step new1 200 python tools/ab_variants.py --config C4 --variants 3 22 42 43 --rounds 3
SBO_LIB=$L/libsbo_base.so step base2 200 python tools/ab_variants.py --config C4 --variants 3 22 --rounds 3
step new2 200 python tools/ab_variants.py --config C4 --variants 3 22 --rounds 3
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo done
