#!/bin/bash
# Round 5: the 32-query inverse guard (tests + bench fit cost), kernel 5 (A a
# tile ahead: tests, bitwise vs kernel 3 at N = 16384, timing), the precise
# sweep's timing bounds (diagnostic build: kernel 3, without any stage DMA
# (11), without the table's DMA (12)), then the probe query-set diagnostic.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5g32; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
step k5_tests 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "precise_sweep_matches_oracle or kstar_table_chunks or int8_mfma_k_layout"
REF_ACROSS=1 OZ_KERNELS="3 5" BLOCKS="0" step k5_ab 300 python -u tools/r5_plan_block_ab.py 16384
step guard_tests 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_invcheck.py
step bench 300 python -u bench.py --no-cpu --no-regimes --steps 5 --warmup 2
SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_diag.so OZ_KERNELS="3 11 12" step bounds 600 python -u tools/r4_oz_ab.py 16384 256
INV_OZ_MIN="4096 2048" step inv_oz_min 600 python -u tools/r4_inv_oz_ab.py 16384 6
step probe_design 600 python -u tools/r5_probe_design.py 8192 500
