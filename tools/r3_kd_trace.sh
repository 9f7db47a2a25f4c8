#!/bin/bash
# Round 3: kernel traces of warm C3 and C4 fits after the threaded k-d order (the host gap
# between one fit's last kernel and the next fit's fill is the staging), plus the order tests.
export TMPDIR=/tmp
O=gpurun_out/kdt; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "order or kd or append or fit" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 11; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python tools/fit_timing.py --n 8192 16384 --reps 3 > $O/tr.log 2>&1 || exit 12
grep N= $O/tr.log
