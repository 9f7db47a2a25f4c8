#!/bin/bash
# round 3 validation after the fit work: full GPU suite, bench lines C2/C3/C4 (default, with regimes + CPU) and C5, rocprof kernel stats of C4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r3b_gpu_tests.log 2>&1 || exit 11
timeout -k 10 600 python -X faulthandler -u bench.py > gpurun_out/r3b_c4_bench.log 2>&1 || exit 12
timeout -k 10 300 python -X faulthandler -u bench.py --config C3 --steps 20 --no-regimes > gpurun_out/r3b_c3_bench.log 2>&1 || exit 13
timeout -k 10 300 python -X faulthandler -u bench.py --config C2 --steps 50 --no-regimes > gpurun_out/r3b_c2_bench.log 2>&1 || exit 14
timeout -k 10 300 python -X faulthandler -u bench.py --config C5 --steps 50 --warmup 1 > gpurun_out/r3b_c5_bench.log 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_c4prof -o run --output-format csv -- python bench.py --steps 12 --no-cpu --no-regimes > gpurun_out/r3b_c4prof.log 2>&1 || exit 16
