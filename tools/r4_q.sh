#!/bin/bash
# Round 4: the small-append path (factor rows / inverse / alpha from the kept f64 inverse).
export TMPDIR=/tmp
O=gpurun_out/r4q; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_headline.py -k "append or c5 or streaming or inverse" -x -v -s --timeout 300 --timeout-method thread
step trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/r4_append_trace.py
grep append $O/trace.log
echo done
