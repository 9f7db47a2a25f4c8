#!/bin/bash
# round 3: the bf16x3 split trailing update -- probe against rocBLAS, Cholesky parity (SBO_OPT_CHOL_GEMM 3 included), fit timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/r3_update_probe.bin > gpurun_out/r3_update_probe_x3.log 2>&1 || exit 10
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "blocked_cholesky" > gpurun_out/r3_x3_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 --gemm 0 3 > gpurun_out/r3_fit_x3.log 2>&1 || exit 12
