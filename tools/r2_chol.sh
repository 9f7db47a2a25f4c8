#!/bin/bash
# Diagonal-block Cholesky (register panels): bitwise vs the previous build,
# fit timing at C3/C4, GPU tests.
export TMPDIR=/tmp
O=gpurun_out/chol; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
TAILN=2 step cmp 400 python tools/compare_libs.py $L/libsbo_base.so $L/libsbo.so --configs C4 C2 box
TAILN=4 step fit_base 300 env SBO_LIB=$L/libsbo_base.so python tools/fit_timing.py --n 8192 16384 --reps 3
TAILN=4 step fit_new 300 python tools/fit_timing.py --n 8192 16384 --reps 3 --chol 1 0
step prof_fit 300 rocprofv3 --kernel-trace --stats -d $O/prof_fit -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2
[ -n "$NOTESTS" ] || step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo done
