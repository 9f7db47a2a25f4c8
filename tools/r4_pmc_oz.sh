#!/bin/bash
# Round 4: what bounds the int8 sliced precise sweep (predict_oz_kernel) on the
# lpsc box (N = 16384, 400 x 400 grid, one tick): four counter passes,
# summaries by tools/pmc_clock.py into $O/summary.txt (the last dispatch is
# the tick; the earlier ones the fit's probe).
export TMPDIR=/tmp
O=${O:-gpurun_out/pmcoz}; mkdir -p $O
: > $O/summary.txt
for g in a b c d; do
  case $g in
    a) C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES";;
    b) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC";;
    c) C="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE";;
    d) C="SQ_WAVE_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_TRANS_F SQ_INST_CYCLES_SALU SQ_LDS_DATA_FIFO_FULL SQ_INSTS_BRANCH";;
  esac
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$g -o run --output-format csv -- python3 tools/run_predict.py --config C4 --box --grid 400 --ticks 1 > $O/$g.log 2>&1 || exit 21
  python3 tools/pmc_clock.py $O/$g predict_oz_kernel >> $O/summary.txt
done
cat $O/summary.txt
