#!/bin/bash
# Round 3: paired one-product steps (variant 62) against the default (3), same process, C4 / C3 / C2
# and the stress box on the fast sweep; max |d| of mu / sd vs variant 3 (expected 0: same arithmetic).
export TMPDIR=/tmp
O=gpurun_out/pair; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; cat $O/$name.log | grep variant; [ $rc -eq 0 ] || exit $rc; }
step c2 120 python tools/ab_variants.py --config C2 --variants 3 62 --rounds 5
step c4 240 python tools/ab_variants.py --config C4 --variants 3 62 --rounds 5
step c3 240 python tools/ab_variants.py --config C3 --variants 3 62 --rounds 5
step box 400 python tools/ab_variants.py --config C4 --box --variants 3 62 --rounds 2 --opt SBO_OPT_PRECISION=0
echo done
