#!/bin/bash
# Round 5: what bounds the int8 precise sweep -- the table sweep (kernel 3)
# against the k-tile pair sweep (4), its no-table diagnostic (10) and the
# no-K* diagnostic (9) on one lpsc-box fit (diagnostic build), then counter
# passes of kernels 3 and 4 (the lpsc box, 400 x 400 grid, one tick).
export TMPDIR=/tmp
O=gpurun_out/r5ozpmc; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc; }
SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_diag.so OZ_KERNELS="3 4 10 9" step ab 600 python -u tools/r4_oz_ab.py 16384 256
: > $O/summary.txt
for K in 3 4; do
  for g in a b c; do
    case $g in
      a) C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES";;
      b) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS";;
      c) C="TCC_HIT_sum TCC_MISS_sum";;
    esac
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/k$K$g -o run --output-format csv -- python3 tools/run_predict.py --config C4 --box --grid 400 --ticks 1 --opt SBO_OPT_PRECISE_KERNEL=$K > $O/k$K$g.log 2>&1 || exit 21
    echo "kernel $K pass $g" >> $O/summary.txt
    python3 tools/pmc_clock.py $O/k$K$g predict_oz >> $O/summary.txt
  done
done
cat $O/summary.txt
