#!/bin/bash
mkdir -p gpurun_out/x3
O=gpurun_out/x3
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 22 3 --rounds 2
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/x3/prof -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 2
