#!/bin/bash
# Round 5: the K* table kept small enough to stay in the Infinity Cache
# (SBO_OPT_TABLE_MB: chunks of fewer query blocks) -- kernel 3 on the lpsc
# box at N = 16384, sweep time (events over the chunk launches) and tick.
export TMPDIR=/tmp
O=gpurun_out/r5tmb; mkdir -p $O
for MB in 2048 512 256 128; do
  TABLE_MB=$MB OZ_KERNELS="3" timeout -k 10 300 python -u tools/r4_oz_ab.py 16384 64 > $O/mb$MB.log 2>&1 || exit $?
  echo "TABLE_MB=$MB: $(grep '^kernel 3' $O/mb$MB.log)"
done
