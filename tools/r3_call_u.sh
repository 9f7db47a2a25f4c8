#!/bin/bash
# round 3: the recursive inverse's panels at a 256-column floor, then a kernel trace of the C4 fit
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 2 --inv-panels 16 32 64 > gpurun_out/r3_fit_invtune2.log 2>&1 || exit 12
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_fitnew -o run --output-format csv -- \
  python tools/fit_timing.py --n 16384 --reps 2 > gpurun_out/r3_fitnew.log 2>&1 || exit 13
