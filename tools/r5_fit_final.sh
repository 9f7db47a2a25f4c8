#!/bin/bash
# Round 5: fit timing at the library defaults (C2 / C3 size / C4 / box) and
# the C4 fit's kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r5fitfinal; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step timing 300 python -u tools/fit_timing.py --n 2048 8192 16384 --reps 4
step timing_box 300 python -u tools/fit_timing.py --n 16384 --reps 3 --box
step trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/fit_timing.py --n 16384 --reps 2
python3 tools/trace_list.py $O/tr 100 > $O/trace.txt
