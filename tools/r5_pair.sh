#!/bin/bash
# Round 5: the k-tile pair int8 sweep (SBO_OPT_PRECISE_KERNEL 4): its tests,
# then the lpsc-box A/B against the table sweep (kernel 3).
export TMPDIR=/tmp
O=gpurun_out/r5pair; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -k "precise_sweep_matches_oracle or kstar_table_chunks or pair_sweep or int8_mfma" -x -v -s --timeout 300 --timeout-method thread
OZ_KERNELS="3 4" step ab 600 python -u tools/r4_oz_ab.py 16384 1024
