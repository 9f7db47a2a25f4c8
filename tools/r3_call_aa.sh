#!/bin/bash
# round 3: inverse panels of >= 1024 columns at the 4096 level (rocBLAS dgemm shape), inverse tests, fit timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "recursive_inverse or inverse_overlap or incremental" > gpurun_out/r3_panel_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 --inv-panels 8 16 > gpurun_out/r3_fit_panel.log 2>&1 || exit 12
