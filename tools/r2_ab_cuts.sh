#!/bin/bash
# A/B: per-row-block XCD chunk cuts + item weight (this tree) vs the previous
# build (lib/libsbo_base.so): bitwise outputs, sweep times (default, dense,
# C3), per-workgroup spread (stamp build), GPU tests.
export TMPDIR=/tmp
O=gpurun_out/abc; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
TAILN=2 step cmp 400 python tools/compare_libs.py $L/libsbo_base.so $L/libsbo.so --configs C4 C2 box
for r in 1 2; do
  SBO_LIB=$L/libsbo_base.so step base_c4_$r 200 python tools/ab_variants.py --config C4 --variants 3 22 --rounds 3
  step new_c4_$r 200 python tools/ab_variants.py --config C4 --variants 3 22 --rounds 3
done
SBO_LIB=$L/libsbo_base.so step base_c3 200 python tools/ab_variants.py --config C3 --variants 3 --rounds 3
step new_c3 200 python tools/ab_variants.py --config C3 --variants 3 --rounds 3
SBO_LIB=$L/libsbo_base.so step base_dense 300 python tools/ab_variants.py --config C4 --variants 3 --rounds 1 --opt SBO_OPT_TILE_SKIP=0
step new_dense 300 python tools/ab_variants.py --config C4 --variants 3 --rounds 1 --opt SBO_OPT_TILE_SKIP=0
TAILN=4 step stamps 200 env SBO_LIB=$L/libsbo_diag.so python tools/x3_stamps.py --config C4
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo done
