#!/bin/bash
# round 3: fit with the MFMA diagonal kernel and two-level Cholesky -- inverse overlap re-measured, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 --overlap 0 32 64 128 > gpurun_out/r3_fit_overlap2.log 2>&1 || exit 11
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_fitdiag -o run --output-format csv -- \
  python tools/fit_timing.py --n 16384 --reps 2 > gpurun_out/r3_fitdiag.log 2>&1 || exit 12
