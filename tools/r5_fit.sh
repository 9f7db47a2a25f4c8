#!/bin/bash
# Round 5: fit latency with the inverse guard (C2, C4, the lpsc box), a C4 fit
# kernel trace, the C4 shard emulation on the round-5 build, and the
# probe / guard calibration over hyper-parameters.
export TMPDIR=/tmp
O=gpurun_out/r5fit; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step fit 300 python -u tools/fit_timing.py --n 2048 8192 16384 --reps 5 --oz 6
step fitbox 300 python -u tools/fit_timing.py --n 16384 --reps 3 --oz 6 --box
step fittrace 300 rocprofv3 --kernel-trace -d $O/fittrace -o run --output-format csv -- python3 tools/fit_timing.py --n 16384 --reps 2 --oz 6
step shards 300 python -u tools/shard_emulate.py --config C4 --world 1 2 4 8 --reps 5 --balance 0
step calib 900 python -u tools/r5_calibrate.py 8192 500
