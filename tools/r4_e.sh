#!/bin/bash
# Round 4: product split sweep (csrc/predict_x3.hip) bitwise against the
# diagnostic build's variant 3; int8 sweep tests; int8 vs f64 precise sweep A/B
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step cmp 300 python -u tools/compare_libs.py safe_bayesian_optimization_amd/lib/libsbo.so safe_bayesian_optimization_amd/lib/libsbo_diag.so
step small 300 python -u -m pytest tests/test_gpu_parity.py -k "int8 or precise_sweep or split_operand or rejects or precision_levels" -x -q --timeout 200 --timeout-method thread
step ab 600 python -u tools/r4_oz_ab.py 16384 256
echo done
