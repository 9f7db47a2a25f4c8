#!/bin/bash
# Round 5: SBO_OPT_INV_OZ_MIN 4096 / 2048 with the sixteen-wave sliced GEMM.
export TMPDIR=/tmp
O=gpurun_out/r5ozmin2; mkdir -p $O
INV_OZ_MIN="4096 2048" timeout -k 10 600 python -u tools/r4_inv_oz_ab.py 16384 6 > $O/ab.log 2>&1; rc=$?
grep -E "^C4|^lpsc" $O/ab.log; exit $rc
