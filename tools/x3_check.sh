#!/bin/bash
mkdir -p gpurun_out/x3
O=gpurun_out/x3
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 22 3 32 33 --rounds 2
step ab_c3 300 python tools/ab_variants.py --config C3 --variants 22 3 32 33 --rounds 2
for v in 22 3; do step c5_$v 300 python bench.py --config C5 --variant $v; done
