#!/bin/bash
# Round 5: the sliced Cholesky updates at other outer panel widths.
export TMPDIR=/tmp
O=gpurun_out/r5cholouter; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "cholesky" > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; exit $rc
