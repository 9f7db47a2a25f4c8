#!/bin/bash
mkdir -p gpurun_out/x3
O=gpurun_out/x3
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 3 40 41 --rounds 3
step ab_c3 300 python tools/ab_variants.py --config C3 --variants 3 40 41 --rounds 3
