#!/bin/bash
# Round 5: the C4 fit's kernel timeline on the current build (warm refits:
# the inverse at the adapted digits).
export TMPDIR=/tmp
O=gpurun_out/r5c4tr; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/fit_timing.py --n 16384 --reps 3
python3 tools/trace_list.py $O/tr 110 > $O/trace.txt
