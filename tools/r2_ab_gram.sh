#!/bin/bash
# A/B: spectral tile bounds from G^16 (this build) vs G^8 (lib/libsbo_base.so): tiles kept and sweep times; bound test.
export TMPDIR=/tmp
O=gpurun_out/abg; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -E "variant|passed|failed" $O/$name.log | tail -3; [ $rc -eq 0 ] || exit $rc; }
for r in 1 2; do
  SBO_LIB=$L/libsbo_base.so step base_c4_$r 200 python tools/ab_variants.py --config C4 --variants 3 --rounds 3
  step new_c4_$r 200 python tools/ab_variants.py --config C4 --variants 3 --rounds 3
done
SBO_LIB=$L/libsbo_base.so step base_c3 200 python tools/ab_variants.py --config C3 --variants 3 --rounds 3
step new_c3 200 python tools/ab_variants.py --config C3 --variants 3 --rounds 3
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bound or budget or headline or c4 or c5 or level or skip"
echo done
