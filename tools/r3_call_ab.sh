#!/bin/bash
# round 3: kernel trace of the C4 fit (inverse panels rule), for the inverse's per-kernel breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_fitinv -o run --output-format csv -- \
  python tools/fit_timing.py --n 16384 --reps 2 > gpurun_out/r3_fitinv.log 2>&1 || exit 13
