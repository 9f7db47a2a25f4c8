"""Summarise rocprofv3 PMC passes of the predictive kernel into one JSON.

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters).  On gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read
(MI355X_MICROARCH.md, HBM section), so it is doubled; WRITE_SIZE is exact for
16-B streaming stores.  Both count memory-side (fabric) traffic, i.e. what
leaves L2 (Infinity-Cache hits included)."""
import csv
import glob
import json
import sys


TICKS = 2   # tools/collect_pmc.sh runs tools/run_predict.py --ticks 2


def per_kernel(path, counter):
    """Per kernel: the counter summed per dispatch, averaged over the last
    TICKS dispatches (the ticks' sweeps; earlier ones are the fit's precision
    probe, a 1536-point sweep with another traffic profile)."""
    vals = {}
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            kn = r["Kernel_Name"]
            k = "predict_kernel" if ("predict_kernel" in kn or "predict_x3_kernel" in kn) else (
                "rbf_fill_kernel" if "rbf_fill" in kn else None)
            if k:
                vals.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
                vals[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    last = {k: [v[d] for d in sorted(v, key=int)[-TICKS:]] for k, v in vals.items()}
    return {k: sum(v) / len(v) for k, v in last.items()}, {k: len(v) for k, v in last.items()}


def main(out, cfg, dst):
    fetch, nf = per_kernel(out + "/fetch", "FETCH_SIZE")
    write, nw = per_kernel(out + "/write", "WRITE_SIZE")
    dur = {}
    for f in glob.glob(out + "/trace/**/*kernel_trace.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(f))
                if "predict_kernel" in r["Kernel_Name"] or "predict_x3_kernel" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        last = rows[-TICKS:]
        if last:
            dur["predict_kernel"] = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last) / len(last) * 1e-6
    res = {"config": cfg, "units": "bytes per launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE)"}
    for k in fetch:
        fb = 2.0 * fetch[k] * 1024.0
        wb = write.get(k, 0.0) * 1024.0
        res[k] = {"fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb, "launches_profiled": nf[k],
                  "avg_ms_kernel_trace": dur.get(k)}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
