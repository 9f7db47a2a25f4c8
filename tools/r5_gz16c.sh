#!/bin/bash
# Round 5: the guard launched after the tile norms (beside the probe): guard
# tests, fit timing, the bench line.
export TMPDIR=/tmp
O=gpurun_out/r5gz16c; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step guard 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_invcheck.py
step timing 300 python -u tools/fit_timing.py --n 2048 8192 16384 --reps 4 --oz 6
step timing_box 300 python -u tools/fit_timing.py --n 16384 --reps 3 --oz 6 --box
step bench 300 python -u bench.py --no-cpu --no-regimes --steps 50 --warmup 3
