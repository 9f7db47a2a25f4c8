#!/bin/bash
# Round 3: the inverse's first half beside the two-level Cholesky (SBO_OPT_INV_OVERLAP = R CUs left
# to the factorization): kernel traces of warm C4 fits at R = 0 and 32 for tools/fit_timeline.py.
export TMPDIR=/tmp
O=gpurun_out/ov3; mkdir -p $O
for r in 0 32; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr$r -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2 --overlap $r > $O/tr$r.log 2>&1 || exit 12
done
cat $O/tr*.log
