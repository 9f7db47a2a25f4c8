#!/bin/bash
# Round 4 final: the GPU suite, smoke, and the default bench line under a
# kernel trace (its summary goes to profiles/r4_bench_kernel_stats.csv).
export TMPDIR=/tmp
O=gpurun_out/r4final; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step suite 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 700 rocprofv3 --kernel-trace --stats -d $O/benchprof -o run --output-format csv -- python3 bench.py
echo done
