#!/bin/bash
# Round-2 sweep probe on the GPU box: phase stamps (default plan and dense),
# forced-level per-tile times (diagnostic build).  Logs under gpurun_out/probe/.
export TMPDIR=/tmp
O=gpurun_out/probe; mkdir -p $O
D=$PWD/safe_bayesian_optimization_amd/lib/libsbo_diag.so
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -12 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
run stamps_c4 300 env SBO_LIB=$D python tools/x3_stamps.py --config C4
run stamps_c4_dense 300 env SBO_LIB=$D python tools/x3_stamps.py --config C4 --opt SBO_OPT_TILE_SKIP=0
for l in 0 1 2; do
  run force_l$l 300 env SBO_LIB=$D SBO_LVL_FORCE=$l python tools/ab_variants.py --config C4 --variants 3 --rounds 2
done
run ab_default 300 env SBO_LIB=$D python tools/ab_variants.py --config C4 --variants 3 22 --rounds 2
echo done
