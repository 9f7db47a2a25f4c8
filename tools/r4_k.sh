#!/bin/bash
# Round 4: the bound on the int8 sweep's K* work -- the diagnostic build's
# variant 9 (no K* digits, wrong results) against the product kernel.
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_diag.so OZ_KERNELS="1 9" timeout -k 10 600 python -u tools/r4_oz_ab.py 16384 256 > $O/ab.log 2>&1; rc=$?; tail -4 $O/ab.log | cut -c1-300; exit $rc
