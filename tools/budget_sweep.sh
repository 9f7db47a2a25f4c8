#!/bin/bash
# Skip-budget trade-off at C4: sweep time (same build, one process per budget)
# and variance error vs a host f64 sweep of the device operand.  Logs under gpurun_out/budget/.
export TMPDIR=/tmp
O=gpurun_out/budget; mkdir -p $O
for B in 22 20 18; do
  timeout -k 10 300 python tools/ab_variants.py --config C4 --variants 3 --rounds 3 --opt SBO_OPT_SKIP_BUDGET=$B > $O/ab_$B.log 2>&1 || exit $?
  echo "B=$B"; tail -2 $O/ab_$B.log
done
timeout -k 10 600 python tools/variant_accuracy.py --n 16384 --variants 3 --budget 22 20 18 > $O/acc.log 2>&1 || exit $?
cat $O/acc.log | tail -4
