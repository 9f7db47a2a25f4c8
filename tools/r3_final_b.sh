#!/bin/bash
# Round-3 final validation, part 2: bench lines for C3, C2, C5 and a rocprofv3 kernel-trace
# summary of the C4 bench (profiles/r3_c4_kernel_stats.csv).  Logs under gpurun_out/fin/.
export TMPDIR=/tmp
O=gpurun_out/fin; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step bench_c3 300 python bench.py --config C3
step bench_c2 200 python bench.py --config C2
step bench_c5 300 python bench.py --config C5
step prof_c4 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python bench.py --no-cpu --no-regimes --steps 12
echo done
