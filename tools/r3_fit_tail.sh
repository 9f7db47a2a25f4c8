#!/bin/bash
# Round 3 fit-tail changes (inverse enqueue order, alpha on aux_stream, widen inside the
# Cholesky, probe reference budget, batched base cases): inverse/fit GPU tests, warm C3/C4 fits
# with the base cases batched or not, a kernel trace of C4 fits.
export TMPDIR=/tmp
O=gpurun_out/ft2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "inverse or cholesky or precise or probe" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/fit_timing.py --n 8192 16384 --reps 3 --leaves 0 1 > $O/fit.log 2>&1 || exit 12
cat $O/fit.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2 > $O/tr.log 2>&1 || exit 13
