#!/bin/bash
# Inverse first half beside the Cholesky tail: inverse/Cholesky tests, fit
# timing (SBO_OPT_INVERSE 1 = overlapped recursion, 0 = rocSOLVER dtrtri),
# fit kernel stats, GPU suite, smoke, C4/C5 benches.
export TMPDIR=/tmp
O=gpurun_out/ovl; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step inv_test 300 python -u -m pytest tests/test_gpu_parity.py -k "cholesky or not_spd or jitter or inverse or append or c3" -v -s --timeout 200 --timeout-method thread
TAILN=6 step fit 300 python tools/fit_timing.py --n 8192 16384 --reps 3 --inv 1 0
step prof_fit 300 rocprofv3 --kernel-trace --stats -d $O/prof_fit -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
step bench_c4 400 python bench.py
step bench_c5 400 python bench.py --config C5 --steps 50 --no-cpu
echo done
