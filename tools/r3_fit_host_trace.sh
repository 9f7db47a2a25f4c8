#!/bin/bash
# Round 3: where the warm C4 fit's host time goes -- kernel + HIP runtime trace of tools/fit_timing.py.
export TMPDIR=/tmp
O=gpurun_out/fht; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d $O/tr -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2 > $O/fit.log 2>&1 || exit 21
ls $O/tr/*/ 2>/dev/null | head; ls $O/tr | head
