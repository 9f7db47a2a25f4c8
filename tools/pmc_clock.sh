#!/bin/bash
# Clock / matrix-pipe / wave-state counters of the predictive kernel, one
# rocprofv3 pass per counter group.   bash tools/pmc_clock.sh TAG [run_predict args...]
set -e
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/clk_$TAG
rm -rf $OUT
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/a -o run --output-format csv -- python tools/run_predict.py "$@"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/b -o run --output-format csv -- python tools/run_predict.py "$@"
echo "== $TAG"
python tools/pmc_clock.py $OUT/a
python tools/pmc_clock.py $OUT/b
