#!/bin/bash
# round 3: two-level blocked Cholesky (SBO_OPT_CHOL_OUTER) -- parity, then fit timing per outer panel width
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "blocked_cholesky or inverse_overlap or recursive_inverse or jitter or incremental" > gpurun_out/r3_outer_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 --outer 128 256 512 1024 > gpurun_out/r3_fit_outer.log 2>&1 || exit 12
