#!/bin/bash
# Round 5 validation: the whole -m gpu suite.
export TMPDIR=/tmp
O=gpurun_out/r5full; mkdir -p $O
timeout -k 10 1120 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 $O/gpu_tests.log | cut -c1-300; exit $rc
