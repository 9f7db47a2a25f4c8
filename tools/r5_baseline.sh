#!/bin/bash
# Round 5 start: the GPU suite at HEAD, then PMC passes of the default precise
# kernel (SBO_OPT_PRECISE_KERNEL 3, K* table) on the lpsc box.
export TMPDIR=/tmp
O=gpurun_out/r5base; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step suite 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA
O=$O/pmcoz bash tools/r4_pmc_oz.sh > $O/pmcoz.log 2>&1; echo "pmcoz rc=$?"; cat $O/pmcoz/summary.txt
