#!/bin/bash
mkdir -p gpurun_out/x3
O=gpurun_out/x3
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "precision_levels or query_cost or tile_skip"
step bench_c4 300 python bench.py --no-cpu
