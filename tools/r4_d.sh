#!/bin/bash
# Round 4: int8 sliced sweep A/B (1: no A prefetch, SGPR DMA bases; 2: A digits prefetched)
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step small 300 python -u -m pytest tests/test_gpu_parity.py -k "int8 or precise_sweep" -x -q --timeout 200 --timeout-method thread
OZ_KERNELS="1 2" step ab 600 python -u tools/r4_oz_ab.py 16384 256
echo done
