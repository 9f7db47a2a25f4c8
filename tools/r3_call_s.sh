#!/bin/bash
# round 3: tile_norm at two workgroups per CU -- bound tests, fit timing, C5 bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "tile_gain or budget or precision_levels or incremental or c3_prop" > gpurun_out/r3_tilenorm_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/fit_timing.py --n 16384 8192 --reps 3 > gpurun_out/r3_fit_tilenorm.log 2>&1 || exit 12
timeout -k 10 300 python -u bench.py --config C5 --steps 50 --warmup 1 --no-cpu > gpurun_out/r3_c5_tilenorm.log 2>&1 || exit 13
