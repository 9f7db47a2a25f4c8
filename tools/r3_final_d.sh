#!/bin/bash
# Round-3 final validation of the last build (fit tail on aux_stream, faster tile norms, probe
# reference at 2^-24): GPU tests, smoke, PMC HBM traffic of the C4 sweep (profiles/r3_pmc_C4.json,
# read by bench.py), the C4 bench line with its CPU baseline and regimes, C3 / C2 / C5 lines and a
# kernel-trace summary of the C4 bench.  gpurun_out/find/.
export TMPDIR=/tmp
O=gpurun_out/find; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step pmc_c4 300 bash tools/collect_pmc.sh C4 r3
step bench_c4 420 python bench.py
step bench_c3 300 python bench.py --config C3
step bench_c2 200 python bench.py --config C2
step bench_c5 300 python bench.py --config C5
step prof_c4 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python bench.py --no-cpu --no-regimes --steps 12
echo done
