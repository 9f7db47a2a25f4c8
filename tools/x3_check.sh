#!/bin/bash
mkdir -p gpurun_out/x3
O=gpurun_out/x3
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step acc 300 python tools/variant_accuracy.py --n 8192 16384 --variants 3 0
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 3 0 --rounds 2
step ab_c3 300 python tools/ab_variants.py --config C3 --variants 3 --rounds 2
