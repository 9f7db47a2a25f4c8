#!/bin/bash
# Round 4: C2 / C4 fit timings by option (what the small-N fit's time is made of)
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -12 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step c2 300 python -u tools/fit_timing.py --n 2048 --reps 5 --chol 1 0 --outer 512 128 --prec -1 0
step c2inv 300 python -u tools/fit_timing.py --n 2048 --reps 5 --inv 1 0 --leaves 1 0 --inv-base 1024 2048
echo done
