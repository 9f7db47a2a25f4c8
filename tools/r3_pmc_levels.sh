#!/bin/bash
# Round-3 PMC breakdown of the split sweep at C4 by precision level: the
# default plan and every kept tile forced to six / one product(s) (diagnostic build,
# SBO_LVL_FORCE; the fast sweep forced, SBO_OPT_PRECISION 0, since the forced levels fail the probe).  One rocprofv3 pass per counter group (<= 8 SQ counters each), each under
# its own time limit; summaries by tools/pmc_clock.py into gpurun_out/pmcl3/summary.txt.
export TMPDIR=/tmp
O=gpurun_out/pmcl3; mkdir -p $O
D=$PWD/safe_bayesian_optimization_amd/lib/libsbo_diag.so
: > $O/summary.txt
for lv in def 0 2; do
  for g in a b c d; do
    case $g in
      a) C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES";;
      b) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC";;
      c) C="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE";;
      d) C="SQ_WAVE_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_TRANS_F SQ_INST_CYCLES_SALU SQ_LDS_DATA_FIFO_FULL SQ_INSTS_BRANCH";;
    esac
    if [ $lv = def ]; then
      SBO_LIB=$D timeout -s KILL 90 rocprofv3 --pmc $C -d $O/$lv$g -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 2 --opt SBO_OPT_PRECISION=0 > $O/$lv$g.log 2>&1 || exit 11
    else
      SBO_LIB=$D SBO_LVL_FORCE=$lv timeout -s KILL 90 rocprofv3 --pmc $C -d $O/$lv$g -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 2 --opt SBO_OPT_PRECISION=0 > $O/$lv$g.log 2>&1 || exit 12
    fi
  done
  echo "== level $lv (def: the plan's levels; 0: six products; 2: one product)" >> $O/summary.txt
  for g in a b c d; do python tools/pmc_clock.py $O/$lv$g >> $O/summary.txt; done
done
