#!/bin/bash
# tile_norm_kernel on f64 MFMA: GPU tests (bounds, budgets, headline), fit
# timing, kernel stats of a C4 fit, and the outputs against the previous build.
export TMPDIR=/tmp
O=gpurun_out/tn; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=4 step fit 300 python tools/fit_timing.py --n 8192 16384 --reps 3
step prof_fit 300 rocprofv3 --kernel-trace --stats -d $O/prof_fit -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2
TAILN=25 step cmp 400 python tools/compare_libs.py $L/libsbo_base.so $L/libsbo.so --configs C4 C2 box
echo done
