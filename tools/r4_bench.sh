#!/bin/bash
# Round 4: the default bench line under a kernel trace, then the K* table chunk-size A/B.
export TMPDIR=/tmp
O=gpurun_out/r4final; mkdir -p $O
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $O/benchprof -o run --output-format csv -- python3 bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' $O/bench.log | tail -1 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/r4_n.sh
