#!/bin/bash
# Round 4: the one-point append at C4 under a kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/r4_append_trace.py > $O/run.log 2>&1; rc=$?
grep append $O/run.log; exit $rc
