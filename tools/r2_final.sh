#!/bin/bash
# Round-2 validation + measurement on one MI355X: GPU tests, smoke, PMC HBM
# traffic (profiles/r2_pmc_C4.json, read by bench.py), bench lines C4 (default
# flags: CPU baseline and regimes) / C3 / C2 / C5, rocprofv3 kernel stats of
# the C4 bench, clock and wave-state counters.  Logs under gpurun_out/final/.
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step pmc_c4 600 bash tools/collect_pmc.sh C4 r2
step bench_c4 600 python bench.py
step bench_c3 300 python bench.py --config C3 --no-cpu --no-regimes --steps 20
step bench_c2 300 python bench.py --config C2 --no-cpu --no-regimes --steps 50
step bench_c5 400 python bench.py --config C5 --steps 50
step prof_c4 400 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python bench.py --no-cpu --no-regimes --steps 10
TAILN=8 step clock_c4 400 bash tools/pmc_clock.sh c4 --config C4 --ticks 2
echo done
