#!/bin/bash
# Is the slow XCD the hardware or the chunk it sweeps? Stamp build with the
# chunk -> XCD mapping rotated by 0 and 4 (SBO_XCD_ROT, diagnostic build).
export TMPDIR=/tmp
O=gpurun_out/rot; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
for rot in 0 4 2; do
  step c4_rot$rot 200 env SBO_LIB=$D SBO_XCD_ROT=$rot python tools/x3_stamps.py --config C4
  step c4f0_rot$rot 200 env SBO_LIB=$D SBO_XCD_ROT=$rot SBO_LVL_FORCE=0 python tools/x3_stamps.py --config C4
done
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo done
