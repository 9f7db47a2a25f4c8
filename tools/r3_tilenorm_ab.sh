#!/bin/bash
# Round 3: tile_norm A/B in one call -- bitwise comparison against lib/ab/libsbo_a.so, then the
# warm C4 fit's kernel trace under each library (tile_norm durations side by side).  gpurun_out/tnab/.
export TMPDIR=/tmp
O=gpurun_out/tnab; mkdir -p $O
A=safe_bayesian_optimization_amd/lib/ab/libsbo_a.so; B=safe_bayesian_optimization_amd/lib/libsbo.so
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step cmp 400 python tools/compare_libs.py $A $B --configs C4 C2 box
for v in A B A B; do
  L=$A; [ $v = B ] && L=$B
  SBO_LIB=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$v -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 3 > $O/fit_$v.log 2>&1 || exit 22
  python - $O/tr_$v $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)
rows = [r for r in csv.DictReader(open(f[-1])) if 'tile_norm' in r['Kernel_Name']]
print(sys.argv[2], 'tile_norm ms', [round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, 3) for r in rows])
PY
  grep "N=" $O/fit_$v.log | cut -c100-
  rm -rf $O/tr_$v
done
echo done
