#!/bin/bash
# Round 5: the Cholesky's sliced updates on 128 x 128 tiles: tests, timing.
export TMPDIR=/tmp
O=gpurun_out/r5cholgz4; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "cholesky or sliced_inverse or c4_headline"
step timing 300 python -u tools/fit_timing.py --n 8192 16384 --reps 4 --oz 6 --gemm 0 4 5
step timing_box 300 python -u tools/fit_timing.py --n 16384 --reps 3 --oz 6 --box
step trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/fit_timing.py --n 16384 --reps 2 --oz 6
python3 tools/trace_list.py $O/tr 100 > $O/trace.txt
