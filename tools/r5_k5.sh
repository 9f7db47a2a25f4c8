#!/bin/bash
# Round 5: kernel 5 without spills (SGPR-base LDS-DMA): tests, bitwise and
# timing against kernel 3 at N = 16384 on the lpsc box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5k5; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
step k5_tests 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "precise_sweep_matches_oracle or kstar_table_chunks or int8_mfma_k_layout"
REF_ACROSS=1 OZ_KERNELS="3 5" BLOCKS="0" step k5_ab 300 python -u tools/r5_plan_block_ab.py 16384
