#!/bin/bash
# Round 5: smoke, the default bench line (C4, CPU comparator and regimes),
# and the rocprofv3 kernel-trace summary of a bench run.
export TMPDIR=/tmp
O=gpurun_out/r5bench; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 600 python -u bench.py
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-regimes
