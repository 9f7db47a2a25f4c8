#!/bin/bash
# round 3: kernel trace of the C4 fit, two-level Cholesky (outer 512) vs one level
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for ou in 128 512; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_fitou$ou -o run --output-format csv -- \
  python tools/fit_timing.py --n 16384 --reps 2 --outer $ou > gpurun_out/r3_fitou$ou.log 2>&1 || exit 11
done
