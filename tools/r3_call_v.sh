#!/bin/bash
# round 3: the recursive inverse's top-level halves side by side -- parity tests, fit timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "recursive_inverse or inverse_overlap or incremental or append or precise" > gpurun_out/r3_invpar_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 > gpurun_out/r3_fit_invpar.log 2>&1 || exit 12
