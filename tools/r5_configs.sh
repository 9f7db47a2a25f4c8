#!/bin/bash
# Round 5: the C2 / C3 / C5 bench lines (no CPU comparator, no regimes).
export TMPDIR=/tmp
O=gpurun_out/r5cfg; mkdir -p $O
for C in C2 C3 C5; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu --no-regimes > $O/$C.log 2>&1 || exit $?
  echo "$C: $(grep '^{' $O/$C.log | cut -c1-200)"
done
