#!/bin/bash
# Round 4: the int8 sliced precise sweep -- correctness (both kernels against
# the oracle) first, then the lpsc-box A/B.
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step small 300 python -u -m pytest tests/test_gpu_parity.py -k "int8_mfma_k_layout" -x -v -s --timeout 200 --timeout-method thread
step precise 600 python -u -m pytest tests/test_gpu_parity.py -k "precise or precision" -x -v -s --timeout 300 --timeout-method thread
step ab 600 python -u tools/r4_oz_ab.py 16384 1024
step probegrid 600 python -u tools/r4_probe_vs_grid.py
step fitc2 300 rocprofv3 --kernel-trace --stats -d $O/fitc2 -o run --output-format csv -- python3 tools/fit_timing.py --n 2048 --reps 5
echo done
