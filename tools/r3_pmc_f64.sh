#!/bin/bash
# Round 3: what bounds the precise sweep (predict_f64_kernel, 0.75 of the f64 MFMA peak on the
# lpsc box): four counter passes on the stress box at a 400 x 400 grid, one tick each,
# summaries by tools/pmc_clock.py into gpurun_out/pmcf/summary.txt.
export TMPDIR=/tmp
O=gpurun_out/pmcf; mkdir -p $O
: > $O/summary.txt
for g in a b c d; do
  case $g in
    a) C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES";;
    b) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC";;
    c) C="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE";;
    d) C="SQ_WAVE_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_TRANS_F SQ_INST_CYCLES_SALU SQ_LDS_DATA_FIFO_FULL SQ_INSTS_BRANCH";;
  esac
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$g -o run --output-format csv -- python tools/run_predict.py --config C4 --box --grid 400 --ticks 1 > $O/$g.log 2>&1 || exit 21
  python tools/pmc_clock.py $O/$g predict_f64_kernel >> $O/summary.txt
done
cat $O/summary.txt
