#!/bin/bash
# Round 5: clock and matrix-pipe occupancy of the int8 precise sweep against
# its diagnostic bounds (diagnostic build): kernel 3, kernel 11 (no stage DMA
# at all), 12 (no table DMA), 5 (A a tile ahead) -- the lpsc box, 400 x 400
# grid, one tick; counter passes a (clock, MFMA busy), b (issue / waits).
export TMPDIR=/tmp
export SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_diag.so
O=gpurun_out/r5ozpmc2; mkdir -p $O
: > $O/summary.txt
for K in 3 11 12 5; do
  for g in a b; do
    case $g in
      a) C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES";;
      b) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS";;
    esac
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/k$K$g -o run --output-format csv -- python3 tools/run_predict.py --config C4 --box --grid 400 --ticks 1 --opt SBO_OPT_PRECISE_KERNEL=$K > $O/k$K$g.log 2>&1 || exit 21
    echo "kernel $K pass $g" >> $O/summary.txt
    python3 tools/pmc_clock.py $O/k$K$g predict_oz >> $O/summary.txt
  done
done
cat $O/summary.txt
