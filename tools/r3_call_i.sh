#!/bin/bash
# round 3: accuracy printouts of the new tests, C4 bitwise across sweep-group counts, C5 re-sort share sweep
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_headline.py \
  -k "lpsc or c2_exact or bitwise" > gpurun_out/r3_headline_printouts.log 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "precise or precision or resort or padding_band" > gpurun_out/r3_parity_printouts.log 2>&1 || exit 12
for r in 10 40; do
  timeout -k 10 300 python -X faulthandler -u bench.py --config C5 --steps 50 --warmup 1 --resort $r --no-cpu > gpurun_out/r3_c5_resort$r.log 2>&1 || exit 13
done
