#!/bin/bash
# round 3, first GPU call: stress-box accuracy, RCCL world-1 tests, new parity tests, bench --force-pg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/r3_stress_accuracy.py 16384 > gpurun_out/r3_stress_acc.log 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py \
  tests/test_gpu_frontier.py -k "rccl or topology" > gpurun_out/r3_rccl_frontier_tests.log 2>&1 || exit 12
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "padding_band or state_export" > gpurun_out/r3_parity_new.log 2>&1 || exit 13
timeout -k 10 300 python -u bench.py --force-pg --steps 30 --no-regimes --cpu-seconds 6 > gpurun_out/r3_c4_bench_nccl_world1.log 2>&1 || exit 14
