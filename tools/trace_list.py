"""Kernel timeline of the last warm fit in a rocprofv3 kernel trace of
tools/fit_timing.py (from its last rbf_fill to the end of the trace): start,
end (us from the fill), the gap after the previous kernel's end, the name.
    python tools/trace_list.py <rocprof output dir> [max name chars]"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 110
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    i = max(k for k, r in enumerate(rows) if "rbf_fill" in r["Kernel_Name"])
    t0 = int(rows[i]["Start_Timestamp"])
    prev = t0
    for r in rows[i:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f}  gap {(s - prev) / 1e3:7.1f}  {r['Kernel_Name'][:w]}")
        prev = max(prev, e)


if __name__ == "__main__":
    main()
