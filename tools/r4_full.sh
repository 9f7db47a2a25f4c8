#!/bin/bash
# Round 4: the whole GPU suite, smoke, the default bench line and its kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r4full; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step suite 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 600 python -u bench.py
echo done
