#!/bin/bash
# HBM traffic of the predictive kernel from PMC counters, one pass per counter
# group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), then a
# summary JSON under profiles/ that bench.py reads for roofline.traffic.
#   bash tools/collect_pmc.sh C4 r1 [run_predict args, e.g. --opt SBO_OPT_KERNEL_VARIANT=3]
set -e
CFG=${1:-C4}; TAG=${2:-r1}; shift 2 || true
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$CFG
rm -rf $OUT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python tools/run_predict.py --config $CFG --ticks 2 "$@"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python tools/run_predict.py --config $CFG --ticks 2 "$@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python tools/run_predict.py --config $CFG --ticks 2 "$@"
python tools/pmc_summary.py $OUT $CFG profiles/${TAG}_pmc_${CFG}.json
cp profiles/${TAG}_pmc_${CFG}.json $OUT/summary.json
