#!/bin/bash
# Round 4, first GPU check: the new precision / trigger tests, the overlap test
# (ADVICE r3), and a C4 bench line with the append1 regime.
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step precision 900 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_parity.py -k "precision or overlap or probe or append" -x -v -s --timeout 600 --timeout-method thread
step bench_c4 600 python -u bench.py --steps 100 --cpu-seconds 5
echo done
