#!/bin/bash
# round 3: fit timing -- own panel solve vs strsm, CU-reserved trailing updates
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/fit_timing.py --n 16384 --chol 1 2 --reserve 0 8 16 32 --reps 3 > gpurun_out/r3_fit_reserve.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_fitprof16 -o run --output-format csv -- python tools/fit_timing.py --n 16384 --chol 1 --reserve 16 --reps 2 > gpurun_out/r3_fitprof16.log 2>&1 || exit 13
