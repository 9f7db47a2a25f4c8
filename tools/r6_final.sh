#!/bin/bash
# Round-6 measurement pass (GPU box, repo root): part A -- smoke, PMC traffic of the C4 sweep (profiles/r6_pmc_C4.json,
# read by bench.py), the default C4 bench line, and a rocprofv3 kernel-trace --stats of the same bench;
# part B -- the C2 / C3 / C5 bench lines and the 1/2/4/8-strip shard emulation; part T -- the -m gpu suite and
# the C4 bench line.   bash tools/r6_final.sh A|B|T [OUTDIR]
export TMPDIR=/tmp
O=${2:-gpurun_out/r6final}; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
if [ "$1" = A ]; then
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pmc_c4 600 bash tools/collect_pmc.sh C4 r6
cp profiles/r6_pmc_C4.json $O/r6_pmc_C4.json
step bench_c4 500 python bench.py
step prof_c4 500 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python bench.py --no-cpu --no-regimes --steps 20
elif [ "$1" = T ]; then
step gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_c4 500 python bench.py --no-cpu
else
step bench_c2 300 python bench.py --config C2
step bench_c3 400 python bench.py --config C3
step bench_c5 400 python bench.py --config C5
step shards 300 python tools/shard_emulate.py --config C4 --balance 0
fi
echo done
