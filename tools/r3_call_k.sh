#!/bin/bash
# round 3: kernel trace of the C4 fit with the inverse's first half overlapped (SBO_OPT_INV_OVERLAP 64) and without
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for ov in 0 64; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_fitov$ov -o run --output-format csv -- \
  python tools/fit_timing.py --n 16384 --reps 2 --overlap $ov > gpurun_out/r3_fitov$ov.log 2>&1 || exit 11
done
