#!/bin/bash
# True per-workgroup spans of the default sweep (variant 46: only s_memtime at
# start/end), default and level-aware mean weights (SBO_MEAN_W=64,42,33 = old).
export TMPDIR=/tmp
O=gpurun_out/span; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step c4_old 200 env SBO_LIB=$D SBO_MEAN_W=64,42,33 python tools/x3_stamps.py --config C4 --variant 46
step c4_new 200 env SBO_LIB=$D python tools/x3_stamps.py --config C4 --variant 46
step c4_s5 200 env SBO_LIB=$D SBO_RB_SLOPE=5 python tools/x3_stamps.py --config C4 --variant 46
step c3_old 200 env SBO_LIB=$D SBO_MEAN_W=64,42,33 python tools/x3_stamps.py --config C3 --variant 46
step f0_old 200 env SBO_LIB=$D SBO_MEAN_W=64,42,33 SBO_LVL_FORCE=0 python tools/x3_stamps.py --config C4 --variant 46
step dense_old 300 env SBO_LIB=$D SBO_MEAN_W=64,42,33 python tools/x3_stamps.py --config C4 --variant 46 --opt SBO_OPT_TILE_SKIP=0
echo done
