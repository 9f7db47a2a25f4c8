#!/bin/bash
# Round 5: the precise sweep's blocked item order (SBO_OPT_PLAN_BLOCK) A/B,
# then the probe-size calibration (tools/r5_calibrate.py).
export TMPDIR=/tmp
O=gpurun_out/r5blk; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -12 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step ab 900 python -u tools/r5_plan_block_ab.py 16384
step calib 900 python -u tools/r5_calibrate.py 8192 500
