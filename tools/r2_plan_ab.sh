#!/bin/bash
# Plan kernel times of the C4 tick: base (HEAD) vs this build vs libsbo_c.so
# (rocprofv3 kernel stats), then outputs compared bitwise.
export TMPDIR=/tmp
O=gpurun_out/planab; mkdir -p $O
L=safe_bayesian_optimization_amd/lib
for v in ${VARS:-base c new}; do
  lib=$L/libsbo_$v.so; [ $v = new ] && lib=$L/libsbo.so
  timeout -k 10 300 env SBO_LIB=$lib rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 6 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  echo "$v ok"
  python - $O/$v/run_kernel_stats.csv <<'P'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'plan' in r['Name'] or 'predict_x3' in r['Name']:
        nm = r['Name'].split('(')[0]
        nm = r['Name'].split('::')[2].split('(')[0] if 'anonymous' in nm else nm
        print('  %-40s %4s avg %9.1f us' % (nm[-40:], r['Calls'], float(r['AverageNs']) / 1e3))
P
done
[ -n "$NOCMP" ] || timeout -k 10 400 python tools/compare_libs.py $L/libsbo_base.so $L/libsbo.so --configs C4 C2 box > $O/cmp.log 2>&1; tail -12 $O/cmp.log
