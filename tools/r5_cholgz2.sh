#!/bin/bash
# Round 5: the int8-sliced Cholesky updates with CUs reserved for the chain
# (SBO_OPT_CHOL_RESERVE), and a kernel trace of one such fit.
export TMPDIR=/tmp
O=gpurun_out/r5cholgz2; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -8 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step timing 400 python -u tools/fit_timing.py --n 16384 --reps 3 --oz 6 --gemm 0 4 --reserve 0 16 64
step trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/fit_timing.py --n 16384 --reps 2 --oz 6 --gemm 4
python3 tools/trace_list.py $O/tr 100 > $O/trace.txt
