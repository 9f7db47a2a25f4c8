#!/bin/bash
# Round 3: the separable K* of grid ticks (predict_x3.hip kSep, default variant 3) -- its GPU
# tests, then an interleaved A/B against the direct K* (variant 63) at C2 / C4 / C3 in one process.
export TMPDIR=/tmp
O=gpurun_out/sep; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "separable or grid_query_blocks or padding_band or product_rejects"
step c2 120 python tools/ab_variants.py --config C2 --variants 63 3 --rounds 5
step c4 240 python tools/ab_variants.py --config C4 --variants 63 3 --rounds 5
step c3 240 python tools/ab_variants.py --config C3 --variants 63 3 --rounds 5
echo done
