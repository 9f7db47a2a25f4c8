#!/bin/bash
# Plan kernel times of the C4 tick: this build vs lib/libsbo_base.so (rocprofv3 kernel stats), outputs compared.
export TMPDIR=/tmp
O=gpurun_out/planp; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
timeout -k 10 300 env SBO_LIB=$L/libsbo_base.so rocprofv3 --kernel-trace --stats -d $O/base -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 4 > $O/base.log 2>&1 && echo base ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/new -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 4 > $O/new.log 2>&1 && echo new ok &&
timeout -k 10 400 python tools/compare_libs.py $L/libsbo_base.so $L/libsbo.so --configs C4 C2 box > $O/cmp.log 2>&1; tail -1 $O/cmp.log
