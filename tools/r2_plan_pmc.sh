#!/bin/bash
# Wave-state / instruction-mix counters of plan_count_kernel and plan_write_kernel (C4 ticks).
export TMPDIR=/tmp
O=gpurun_out/planpmc; rm -rf $O; mkdir -p $O
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/a -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 2 > $O/a.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- python tools/run_predict.py --config C4 --ticks 2 > $O/b.log 2>&1 &&
python tools/pmc_clock.py $O/a plan_count && python tools/pmc_clock.py $O/a plan_write && python - <<'PY'
import csv, glob
for d in ("gpurun_out/planpmc/a", "gpurun_out/planpmc/b"):
    agg = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1][:24]
            if "plan_count" not in k and "plan_write" not in k: continue
            agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(d[-1], k, {c: f"{sum(x)/len(x)*len(x)/2:.3g}" for c, x in v.items()})
PY
