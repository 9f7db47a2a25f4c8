#!/bin/bash
# Round 4: int8 sliced sweep -- PMC passes on the lpsc box (tools/r4_pmc_oz.sh).
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c
O=gpurun_out/r4c/pmc timeout -k 10 900 bash tools/r4_pmc_oz.sh > gpurun_out/r4c/pmc.log 2>&1; rc=$?; tail -12 gpurun_out/r4c/pmc.log; exit $rc
