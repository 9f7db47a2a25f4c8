#!/bin/bash
# Look-ahead blocked Cholesky (aux stream): GPU tests, fit timing, fit kernel stats.
export TMPDIR=/tmp
O=gpurun_out/la; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=6 step fit 300 python tools/fit_timing.py --n 8192 16384 --reps 3 --chol 1 0
step prof_fit 300 rocprofv3 --kernel-trace --stats -d $O/prof_fit -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2
step bench_c5 400 python bench.py --config C5 --steps 50 --no-cpu
echo done
