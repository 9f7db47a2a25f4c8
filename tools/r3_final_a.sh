#!/bin/bash
# Round-3 final validation, part 1: GPU tests, smoke, PMC HBM traffic of the C4 sweep
# (profiles/r3_pmc_C4.json, read by bench.py), the C4 bench line.  Logs under gpurun_out/fin/.
export TMPDIR=/tmp
O=gpurun_out/fin; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step pmc_c4 300 bash tools/collect_pmc.sh C4 r3
step bench_c4 400 python bench.py
echo done
