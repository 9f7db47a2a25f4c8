#!/bin/bash
# round 3: chain-kernel micro-benchmark, Cholesky tests, fit timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/chol_micro.bin > gpurun_out/r3_chol_micro.log 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "cholesky or not_spd or jitter or recursive_inverse or append" > gpurun_out/r3_chol_tests.log 2>&1 || exit 12
timeout -k 10 300 python -u tools/fit_timing.py --n 8192 16384 --chol 2 1 --reps 3 > gpurun_out/r3_fit_timing.log 2>&1 || exit 13
