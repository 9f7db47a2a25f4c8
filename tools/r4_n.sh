#!/bin/bash
# Round 4: the K* table's chunk size (SBO_OPT_TABLE_MB) on the lpsc box.
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
for mb in 8192 24576; do
  OZ_KERNELS="3" TABLE_MB=$mb timeout -k 10 300 python -u tools/r4_oz_ab.py 16384 64 > $O/tab_$mb.log 2>&1 || exit $?
  echo "TABLE_MB=$mb: $(grep '^kernel' $O/tab_$mb.log)"
done
