#!/bin/bash
# Jitter retry test, the GPU suite, C4 kernel stats (rocprofv3) and the default bench.
export TMPDIR=/tmp
O=gpurun_out/jit; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step jit_test 200 python -u -m pytest tests/test_gpu_parity.py -k "jitter or not_spd" -v -s --timeout 100 --timeout-method thread
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step prof_c4 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python bench.py --steps 12 --no-cpu --no-regimes
step bench_c4 400 python bench.py
echo done
