#!/bin/bash
# Round 5: the left-looking panel solve (SBO_OPT_CHOL_DIAG 1) against the
# right-looking one (2) and the VALU kernels (0): bitwise test, the Cholesky
# tests, fit timing at C2 / C3 / C4 sizes and the C2 fit's kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r5trsm; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step tests 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "chol"
step timing 300 python -u tools/fit_timing.py --n 2048 8192 16384 --reps 5 --diag 2 1
step trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/fit_timing.py --n 2048 --reps 3
python3 tools/trace_list.py $O/tr 120 > $O/trace.txt
