#!/bin/bash
# Round 4: the K* table (SBO_OPT_PRECISE_KERNEL 3) -- parity first, then the
# lpsc-box A/B against the in-sweep K* (1), then the diagnostic bound (9: no K*).
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step small 400 python -u -m pytest tests/test_gpu_parity.py -k "int8 or precise_sweep or kstar_table" -x -v --timeout 300 --timeout-method thread
OZ_KERNELS="3 1" step ab 600 python -u tools/r4_oz_ab.py 16384 512
SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_diag.so OZ_KERNELS="9" step bound 300 python -u tools/r4_oz_ab.py 16384 64
echo done
