#!/bin/bash
# Round 4: int8 sweep in balanced base-256 digits -- correctness first, then
# the lpsc-box A/B against the f64 sweep.
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step small 300 python -u -m pytest tests/test_gpu_parity.py -k "int8 or precise_sweep" -x -v --timeout 200 --timeout-method thread
step ab 600 python -u tools/r4_oz_ab.py 16384 1024
step prec 900 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_parity.py -k "precision or probe or stress or lpsc" -x -v --timeout 300 --timeout-method thread
echo done
