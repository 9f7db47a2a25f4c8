#!/bin/bash
# round 3: A/B of the sweep's mean-branch removal (58, 59) and the one-wave-per-SIMD shape with variant 3's options (60, 61)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export SBO_LIB=$PWD/safe_bayesian_optimization_amd/lib/libsbo_diag.so
timeout -k 10 300 python -u tools/ab_variants.py --config C4 --variants 3 58 59 60 61 --rounds 3 > gpurun_out/r3_ab_mean_nc2_c4.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/ab_variants.py --config C3 --variants 3 58 59 60 61 --rounds 3 > gpurun_out/r3_ab_mean_nc2_c3.log 2>&1 || exit 12
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r3_pmc_avail.txt 2>&1 || true
