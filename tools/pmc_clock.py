"""Effective clock and matrix-pipe occupancy of the predictive kernel from a
rocprofv3 counter pass (GRBM_GUI_ACTIVE is summed over the 8 XCDs;
SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles with the matrix pipe busy).

  rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d DIR -o run --output-format csv -- python tools/run_predict.py ...
  python tools/pmc_clock.py DIR"""
import csv
import glob
import sys


def main(d, cus=256, kernel=None):
    per = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel:
                if kernel not in r["Kernel_Name"]:
                    continue
            elif "predict_kernel" not in r["Kernel_Name"] and "predict_x3_kernel" not in r["Kernel_Name"]:
                continue
            e = per.setdefault(r["Dispatch_Id"], {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, e in sorted(per.items()):
        ns = e["ns"]
        line = f"dispatch {k}: {ns / 1e6:.2f} ms"
        if "GRBM_GUI_ACTIVE" in e:
            ghz = e["GRBM_GUI_ACTIVE"] / 8 / ns
            line += f"  clock {ghz:.3f} GHz"
            if "SQ_VALU_MFMA_BUSY_CYCLES" in e:
                busy = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (e["GRBM_GUI_ACTIVE"] / 8 * cus * 4)
                line += f"  matrix pipe busy {busy * 100:.1f}%"
        for c in sorted(e):
            if c.startswith("SQ_") and c not in ("SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES") and "SQ_WAVE_CYCLES" in e:
                line += f"  {c} {e[c] / e['SQ_WAVE_CYCLES'] * 100:.1f}%"
            elif c.startswith("TCC_") or c.startswith("TCP_") or c.startswith("TA_"):
                line += f"  {c} {e[c]:.4g}"
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
            line += f"  L2 hit rate {e['TCC_HIT_sum'] / max(e['TCC_HIT_sum'] + e['TCC_MISS_sum'], 1) * 100:.1f}%"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1], kernel=sys.argv[2] if len(sys.argv) > 2 else None)
