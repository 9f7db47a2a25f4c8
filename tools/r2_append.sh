#!/bin/bash
# Append path with two dgemms instead of in-place dtrmm: append tests, the C5
# headline test, C5 bench and its kernel stats.
export TMPDIR=/tmp
O=gpurun_out/app; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread -k "append or c5 or import or state or chol or spd"
step bench_c5 400 python bench.py --config C5 --steps 50 --no-cpu
step prof_c5 400 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python bench.py --config C5 --steps 50 --no-cpu
echo done
