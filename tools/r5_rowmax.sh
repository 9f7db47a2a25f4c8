#!/bin/bash
# Round 5: the coalesced row maxima in the inverse's packs: tests, timing.
export TMPDIR=/tmp
O=gpurun_out/r5rowmax; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sliced_inverse or recursive_inverse or inverse_overlap or cholesky or small_append"
step guard 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_invcheck.py
step timing 300 python -u tools/fit_timing.py --n 2048 8192 16384 --reps 4
step timing_box 300 python -u tools/fit_timing.py --n 16384 --reps 3 --box
