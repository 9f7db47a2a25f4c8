#!/bin/bash
# Phase shares, per-level body cycles and per-workgroup loop-cycle spread of
# the split sweep (stamp build, variant 39), default plan and forced levels.
export TMPDIR=/tmp
O=gpurun_out/stamps; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-4} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
TAILN=20 step c4 200 env SBO_LIB=$D python tools/x3_stamps.py --config C4
for l in 0 1 2; do
  TAILN=3 step c4_force$l 200 env SBO_LIB=$D SBO_LVL_FORCE=$l python tools/x3_stamps.py --config C4
  step ab_force$l 200 env SBO_LIB=$D SBO_LVL_FORCE=$l python tools/ab_variants.py --config C4 --variants 3 --rounds 2
done
TAILN=20 step c5 200 env SBO_LIB=$D python tools/x3_stamps.py --config C3
echo done
