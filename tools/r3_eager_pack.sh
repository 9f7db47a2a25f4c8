#!/bin/bash
# Round 3: the fit's operand packs (split bf16 planes, f64 operand) on aux_stream beside the tile
# norms -- GPU tests, warm fit timing and its kernel trace, the C4 bench line.  gpurun_out/epack/.
export TMPDIR=/tmp
O=gpurun_out/epack; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step fit_trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python tools/fit_timing.py --n 8192 16384 --reps 3
step bench_c4 300 python bench.py --no-cpu --no-regimes
echo done
