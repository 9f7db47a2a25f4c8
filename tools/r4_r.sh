#!/bin/bash
# Round 4: batch appends from the kept inverse -- append tests, then the C5 streaming bench line.
export TMPDIR=/tmp
O=gpurun_out/r4r; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_headline.py -k "append or c5 or streaming or inverse" -x -v -s --timeout 300 --timeout-method thread
step c5 400 python -u bench.py --config C5
echo done
