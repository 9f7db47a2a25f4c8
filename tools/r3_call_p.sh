#!/bin/bash
# round 3: MFMA diagonal-block Cholesky kernel and MFMA trailing updates -- micro-benchmark, parity tests, fit timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/chol_micro.bin > gpurun_out/r3_chol_micro4.log 2>&1 || exit 10
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "blocked_cholesky or chol_diag or not_spd or jitter or incremental or recursive_inverse" > gpurun_out/r3_trsm_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 --outer 512 > gpurun_out/r3_fit_trsm.log 2>&1 || exit 12
