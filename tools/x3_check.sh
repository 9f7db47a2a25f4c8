#!/bin/bash
mkdir -p gpurun_out/x3
O=gpurun_out/x3
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -12 $O/$name.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "precision_levels or split_operand or tile_skip or query_cost or partition"
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 22 3 40 --rounds 2
step ab_c3 300 python tools/ab_variants.py --config C3 --variants 22 3 40 --rounds 2
step stamps_c4 300 python tools/x3_stamps.py --config C4
