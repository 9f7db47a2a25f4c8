#!/bin/bash
# Does the mean row block explain the slow first XCD chunk? Stamp build with
# its tiles weighted 100 / 150 / 200 % in the plan's cuts (SBO_MEAN_W).
export TMPDIR=/tmp
O=gpurun_out/meanw; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
for w in 150 200 300; do
  step c4_w$w 200 env SBO_LIB=$D SBO_MEAN_W=$w python tools/x3_stamps.py --config C4
  step c4f0_w$w 200 env SBO_LIB=$D SBO_MEAN_W=$w SBO_LVL_FORCE=0 python tools/x3_stamps.py --config C4
done
echo done
