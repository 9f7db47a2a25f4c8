#!/bin/bash
# Round 5: the split-bf16 Cholesky updates (SBO_OPT_CHOL_GEMM 3): tests,
# factor / posterior against rocBLAS at C4 and on the box, fit timing.
export TMPDIR=/tmp
O=gpurun_out/r5cx3; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-500; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "cholesky"
step check 300 python -u tools/r5_cholx3_check.py 16384
step timing 300 python -u tools/fit_timing.py --n 2048 8192 16384 --reps 4 --oz 6 --gemm 0 3
