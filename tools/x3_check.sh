#!/bin/bash
mkdir -p gpurun_out/x3
O=gpurun_out/x3
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -8 $O/$name.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
step ab_c4 300 python tools/ab_variants.py --config C4 --variants 22 3 --rounds 2
step ab_c3 300 python tools/ab_variants.py --config C3 --variants 22 3 --rounds 2
step shards 300 python tools/shard_emulate.py --config C4
