#!/bin/bash
# Round-2 profiles: fit kernel stats, bench kernel stats (C4 default), PMC
# traffic of the sweep (writes profiles/r2_pmc_C4.json), clock + matrix pipe.
export TMPDIR=/tmp
O=gpurun_out/r2prof; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step fit 300 rocprofv3 --kernel-trace --stats -d $O/fit -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2
step bench 300 rocprofv3 --kernel-trace --stats -d $O/bench -o run --output-format csv -- python bench.py --no-cpu --no-regimes --steps 10
step pmc 600 bash tools/collect_pmc.sh C4 r2
step clock 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $O/clock -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 2
python tools/pmc_clock.py $O/clock > $O/clock.txt
echo done
