#!/bin/bash
# Round 3: LDS bank conflicts and LDS activity of the fit's own kernels (one warm C4 refit),
# summed per kernel name into gpurun_out/fitpmc/summary.txt.
export TMPDIR=/tmp
O=gpurun_out/fitpmc; mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 1 > $O/a.log 2>&1 || exit 21
python - <<'PY' > $O/summary.txt
import csv, glob, collections
f = glob.glob('gpurun_out/fitpmc/a/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
seen = set()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0][-60:]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    d = (k, r['Dispatch_Id'])
    if d not in seen:
        seen.add(d); n[k] += 1
for k, v in sorted(acc.items(), key=lambda x: -x[1].get('SQ_LDS_BANK_CONFLICT', 0)):
    act = v.get('SQ_LDS_IDX_ACTIVE', 0)
    print(f"{k:62s} n={n[k]:4d} bank_conflict={v.get('SQ_LDS_BANK_CONFLICT',0):.3e} lds_idx_active={act:.3e} "
          f"ratio={v.get('SQ_LDS_BANK_CONFLICT',0)/max(act,1):.2f} wave_cycles={v.get('SQ_WAVE_CYCLES',0):.3e}")
PY
head -25 $O/summary.txt
