#!/bin/bash
# Round 3: the threaded k-d order -- GPU tests (the fit paths and orders) and warm C3/C4 fits.
export TMPDIR=/tmp
O=gpurun_out/kd; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/fit_timing.py --n 8192 16384 --reps 3 > $O/fit.log 2>&1 || exit 12
cat $O/fit.log
