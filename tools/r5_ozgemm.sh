#!/bin/bash
# Round 5: the sliced GEMM with eight waves (two per SIMD) against the
# four-wave kernel, on the inverse's own top-level products (N = 16384 box).
export TMPDIR=/tmp
O=gpurun_out/r5ozg; mkdir -p $O
for b in ozgemm_bench_4w ozgemm_bench ozgemm_bench_16w; do
  timeout -k 10 300 safe_bayesian_optimization_amd/lib/$b 16384 1.0 2.5 0.4 6 5 1 > $O/$b.log 2>&1 || exit $?
  echo "== $b"; cat $O/$b.log
done
