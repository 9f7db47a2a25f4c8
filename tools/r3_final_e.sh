#!/bin/bash
# Round-3 last check of HEAD (tile-norm layout changes, bitwise equal to r3_final_d's build):
# GPU tests, smoke, the C4 bench line.  gpurun_out/fine/.
export TMPDIR=/tmp
O=gpurun_out/fine; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_c4 420 python bench.py
echo done
