#!/bin/bash
# Calibrate the mean row block's sweep-time weight per precision level: stamp
# build, every tile forced to one level, mean-row-block weight 100/125/150 %.
export TMPDIR=/tmp
O=gpurun_out/meanw2; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
for l in 1 2; do
  for w in 100 125 150; do
    step f${l}_w$w 200 env SBO_LIB=$D SBO_MEAN_W=$w SBO_LVL_FORCE=$l python tools/x3_stamps.py --config C4
  done
done
for w in 100 115 130; do
  step c3_w$w 200 env SBO_LIB=$D SBO_MEAN_W=$w python tools/x3_stamps.py --config C3
done
echo done
