#!/bin/bash
# Round 5: the C2 (N = 2048) fit's kernel timeline, with and without the
# precision probe.
export TMPDIR=/tmp
O=gpurun_out/r5c2tr; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/fit_timing.py --n 2048 --reps 3
python3 tools/trace_list.py $O/tr 120 > $O/trace.txt
step trace0 300 rocprofv3 --kernel-trace -d $O/tr0 -o run --output-format csv -- python3 tools/fit_timing.py --n 2048 --reps 3 --prec 0
python3 tools/trace_list.py $O/tr0 120 > $O/trace0.txt
