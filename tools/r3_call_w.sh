#!/bin/bash
# round 3: the whole parity file (precise test against the f64-alpha oracle) on the fit changes (two-level Cholesky, MFMA chain kernels, tile_norm, inverse halves side by side), then fit timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r3_parity_fitchanges.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 > gpurun_out/r3_fit_invpar.log 2>&1 || exit 12
