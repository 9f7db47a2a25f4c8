#!/bin/bash
# Round 5: the pair sweep with its table piece prefetched two stages ahead:
# its tests, then kernels 3 / 4 / 10 on one lpsc-box fit (diagnostic build).
export TMPDIR=/tmp
O=gpurun_out/r5pair2; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -k "precise_sweep_matches_oracle or pair_sweep" -x -v -s --timeout 300 --timeout-method thread
SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_diag.so OZ_KERNELS="3 4 10" step ab 600 python -u tools/r4_oz_ab.py 16384 256
