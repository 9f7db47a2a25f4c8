#!/bin/bash
# Round 4: the precise-sweep tests with the automatic K* table budget, and the lpsc A/B.
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_headline.py -k "int8 or precise or kstar or precision or probe or lpsc or stress" -x -v --timeout 300 --timeout-method thread
OZ_KERNELS="3" step ab 300 python -u tools/r4_oz_ab.py 16384 256
echo done
