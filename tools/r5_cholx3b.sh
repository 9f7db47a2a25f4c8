#!/bin/bash
# Round 5: the split-bf16 Cholesky updates against the exact posterior, and a
# kernel trace of the C4 fit with them.
export TMPDIR=/tmp
O=gpurun_out/r5cx3b; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-500; [ $rc -eq 0 ] || exit $rc; }
step exact 600 python -u tools/r5_cholx3_exact.py 8192 1024
step trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/fit_timing.py --n 16384 --reps 3 --oz 6 --gemm 3
python3 tools/trace_list.py $O/tr 100 > $O/trace.txt
