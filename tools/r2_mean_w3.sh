#!/bin/bash
# Per-XCD balance with the level-aware mean-row-block weights (default) and a
# per-row-block slope (SBO_RB_SLOPE), C4 / C3 / dense; then sweep times.
export TMPDIR=/tmp
O=gpurun_out/meanw3; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
for sl in 0 5 10; do
  step c4_s$sl 200 env SBO_LIB=$D SBO_RB_SLOPE=$sl python tools/x3_stamps.py --config C4
  step c3_s$sl 200 env SBO_LIB=$D SBO_RB_SLOPE=$sl python tools/x3_stamps.py --config C3
  step f0_s$sl 200 env SBO_LIB=$D SBO_RB_SLOPE=$sl SBO_LVL_FORCE=0 python tools/x3_stamps.py --config C4
done
step dense_s0 300 env SBO_LIB=$D python tools/x3_stamps.py --config C4 --opt SBO_OPT_TILE_SKIP=0
step base_c4 200 env SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_base.so python tools/ab_variants.py --config C4 --variants 3 22 --rounds 3
step new_c4 200 python tools/ab_variants.py --config C4 --variants 3 22 --rounds 3
step base_c3 200 env SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_base.so python tools/ab_variants.py --config C3 --variants 3 --rounds 3
step new_c3 200 python tools/ab_variants.py --config C3 --variants 3 --rounds 3
step base_dense 300 env SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_base.so python tools/ab_variants.py --config C4 --variants 3 --rounds 1 --opt SBO_OPT_TILE_SKIP=0
step new_dense 300 python tools/ab_variants.py --config C4 --variants 3 --rounds 1 --opt SBO_OPT_TILE_SKIP=0
echo done
