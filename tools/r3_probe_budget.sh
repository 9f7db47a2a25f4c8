#!/bin/bash
# Round 3: the probe's reference at 2^-24 of the fast sweep's largest variance (was 2^-30) --
# the probe values and decisions on every workload, the precision tests, the warm fit's trace.
export TMPDIR=/tmp
O=gpurun_out/pb; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step probe 400 python tools/r3_probe_values.py
step tests 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "precise or lpsc or probe or precision"
step fit_trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python tools/fit_timing.py --n 8192 16384 --reps 3
echo done
