#!/bin/bash
# PMC breakdown of the split sweep at C4 by precision level (diagnostic build:
# default plan, and every kept tile forced to six / one product(s)).
# One rocprofv3 pass per counter group.  Logs under gpurun_out/pmcl/.
export TMPDIR=/tmp
O=gpurun_out/pmcl; mkdir -p $O
D=$PWD/safe_bayesian_optimization_amd/lib/libsbo_diag.so
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
for lv in def 0 2; do
  if [ $lv = def ]; then E="SBO_LIB=$D"; else E="SBO_LIB=$D SBO_LVL_FORCE=$lv"; fi
  for g in a b c; do
    case $g in
      a) C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES";;
      b) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC";;
      c) C="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA";;
    esac
    env $E timeout -s KILL 90 rocprofv3 --pmc $C -d $O/$lv$g -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 2 > $O/$lv$g.log 2>&1
    echo "$lv$g rc=$?"
  done
  echo "== level $lv"; for g in a b c; do python tools/pmc_clock.py $O/$lv$g; done
done
