#!/bin/bash
# Round 5 (end of round: adaptive digits, left-looking chain kernels): the whole -m gpu suite, smoke,
# the default bench line and its kernel-trace summary.
export TMPDIR=/tmp
O=gpurun_out/r5final5; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 560 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python -u bench.py
step prof 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-regimes
