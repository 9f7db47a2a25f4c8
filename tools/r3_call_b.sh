#!/bin/bash
# round 3, second GPU call: precise sweep tests, probe values, bench --force-pg (faulthandler)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py \
  -k "precise or precision or state_export" > gpurun_out/r3_precise_tests.log 2>&1 || exit 11
timeout -k 10 400 python -u tools/r3_probe_values.py > gpurun_out/r3_probe_values.log 2>&1 || exit 12
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_headline.py \
  -k "lpsc" > gpurun_out/r3_lpsc_tests.log 2>&1 || exit 13
timeout -k 10 300 python -X faulthandler -u bench.py --force-pg --steps 30 --no-regimes --no-cpu > gpurun_out/r3_c4_bench_nccl_world1.log 2>&1 || exit 14
