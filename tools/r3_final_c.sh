#!/bin/bash
# Round-3 final validation of the last build (threaded k-d order, sbo_kd_order): GPU tests,
# smoke, the C4 bench line, a kernel trace of warm C3/C4 fits (the staging gap), and the
# precise sweep's counter passes (tools/r3_pmc_f64.sh).  gpurun_out/finc/.
export TMPDIR=/tmp
O=gpurun_out/finc; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_c4 400 python bench.py
step fit_trace 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python tools/fit_timing.py --n 8192 16384 --reps 3
step pmc_f64 600 bash tools/r3_pmc_f64.sh
echo done
