#!/bin/bash
# Stall breakdown of the predictive kernel: clock/matrix pipe, then wave-state
# and instruction-class counters, one rocprofv3 pass per group.
#   bash tools/pmc_stalls.sh TAG [run_predict args...]
set -e
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/stall_$TAG
rm -rf $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/a -o run --output-format csv -- python tools/run_predict.py "$@"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/b -o run --output-format csv -- python tools/run_predict.py "$@"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA -d $OUT/c -o run --output-format csv -- python tools/run_predict.py "$@"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/d -o run --output-format csv -- python tools/run_predict.py "$@"
echo "== $TAG"
for p in a b c d; do python tools/pmc_clock.py $OUT/$p; done
