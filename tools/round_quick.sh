#!/bin/bash
# Quick GPU validation: parity tests, smoke, C4 bench, rocprofv3 kernel-trace stats (logs under gpurun_out/val/).
export TMPDIR=/tmp
mkdir -p gpurun_out/val
O=gpurun_out/val
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step pmc_c4 900 bash tools/collect_pmc.sh C4 r1
step bench_c4 400 python bench.py
step prof_c4 400 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python bench.py --no-cpu --steps 3
echo done
