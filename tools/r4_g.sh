#!/bin/bash
# Round 4: PMC traffic of the fast sweep (C4, C5) on the final kernels, and
# kernel traces of the warm C4 and C2 fits.
export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pmc_c4 900 bash tools/collect_pmc.sh C4 r4
step fitc4 300 rocprofv3 --kernel-trace --stats -d $O/fitc4 -o run --output-format csv -- python3 tools/fit_timing.py --n 16384 --reps 3
step fitc2 300 rocprofv3 --kernel-trace --stats -d $O/fitc2 -o run --output-format csv -- python3 tools/fit_timing.py --n 2048 --reps 5
echo done
