#!/bin/bash
# round 3: default C4 bench, C5 bench (re-sort on / off), C5 PMC traffic
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -X faulthandler -u bench.py > gpurun_out/r3_c4_bench.log 2>&1 || exit 12
timeout -k 10 300 python -X faulthandler -u bench.py --config C5 --steps 50 --warmup 1 > gpurun_out/r3_c5_bench.log 2>&1 || exit 13
timeout -k 10 300 python -X faulthandler -u bench.py --config C5 --steps 50 --warmup 1 --resort 0 --no-cpu > gpurun_out/r3_c5_bench_noresort.log 2>&1 || exit 14
bash tools/collect_pmc.sh C5 r3 > gpurun_out/r3_pmc_c5.log 2>&1 || exit 15
