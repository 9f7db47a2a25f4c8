#!/bin/bash
# Round 4: the K* table tests and A/B (tools/r4_l.sh), then the level rank-key
# re-calibration A/B at C4 (diagnostic build).
export TMPDIR=/tmp
bash tools/r4_l.sh || exit $?
O=gpurun_out/r4m; mkdir -p $O
SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_diag.so timeout -k 10 600 python -u tools/r4_lvlkey.py > $O/lvlkey.log 2>&1; rc=$?; tail -8 $O/lvlkey.log | cut -c1-300; exit $rc
