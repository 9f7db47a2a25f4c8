#!/bin/bash
# Round 3: tile_norm_kernel with the squarings' rescale on the MFMA operand and the maxima from
# registers -- bitwise A/B against the previous build (lib/ab/libsbo_a.so: tile bounds and every
# tick output at C4, C2, the stress box), the warm fit's kernel trace.  gpurun_out/tn/.
export TMPDIR=/tmp
O=gpurun_out/tn; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step cmp 400 python tools/compare_libs.py safe_bayesian_optimization_amd/lib/ab/libsbo_a.so safe_bayesian_optimization_amd/lib/libsbo.so --configs C4 C2 box
step fit_trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python tools/fit_timing.py --n 8192 16384 --reps 3
echo done
