#!/bin/bash
# round 3: the inverse's first half beside the Cholesky (SBO_OPT_INV_OVERLAP) -- parity, then fit timing per CU reserve
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "inverse_overlap or recursive_inverse or blocked_cholesky" > gpurun_out/r3_overlap_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 --overlap 0 16 32 64 128 192 > gpurun_out/r3_fit_overlap.log 2>&1 || exit 12
