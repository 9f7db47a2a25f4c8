#!/bin/bash
# Full GPU validation + measurement pass (run on the GPU box from the repo root):
#   parity tests, smoke, bench lines for C2-C5, rocprofv3 kernel-trace stats of
#   the default bench, PMC HBM traffic for C3/C4.  Logs under gpurun_out/val/.
#   bash tools/round_validate.sh TAG
TAG=${1:-r1}
export TMPDIR=/tmp
mkdir -p gpurun_out/val
O=gpurun_out/val
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
# PMC traffic first: bench.py reads the summaries for roofline.traffic
step pmc_c4 900 bash tools/collect_pmc.sh C4 $TAG
step pmc_c3 900 bash tools/collect_pmc.sh C3 $TAG
step bench_c4 600 python bench.py
step bench_c3 600 python bench.py --config C3
step bench_c2 300 python bench.py --config C2
step bench_c5 600 python bench.py --config C5
step prof_c4 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python bench.py --no-cpu --steps 3
step clock_c4 900 bash tools/pmc_clock.sh c4 --config C4 --ticks 2
[ -x tools/mfma_probe.bin ] || hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o tools/mfma_probe.bin
step shards 300 python tools/shard_emulate.py --config C4 --balance 0
step mfma_probe 300 ./tools/mfma_probe.bin
echo done
