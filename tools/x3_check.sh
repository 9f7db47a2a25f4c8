#!/bin/bash
mkdir -p gpurun_out/x3
O=gpurun_out/x3
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -10 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 3 9 2 0 --rounds 2
