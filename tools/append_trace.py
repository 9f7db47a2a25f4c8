"""One-point sbo_append at C4 under a kernel trace (what the node's per-change
cost is made of): fit N = 16384, then 6 one-point appends (synchronous), wall
time per append printed; run under rocprofv3 --kernel-trace and list the last
append's kernels with tools/trace_list.py-style output (--list DIR).
    rocprofv3 --kernel-trace -d D -o run --output-format csv -- python3 tools/append_trace.py
    python tools/append_trace.py --list D"""
import csv
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def listing(d):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # the appends are separated by host gaps > 300 us; the last group is the last append
    groups, cur, prev = [], [], None
    for r in rows:
        s = int(r["Start_Timestamp"])
        if prev is not None and s - prev > 300_000:
            groups.append(cur)
            cur = []
        cur.append(r)
        prev = max(prev or 0, int(r["End_Timestamp"]))
    groups.append(cur)
    g = groups[-1]
    t0 = int(g[0]["Start_Timestamp"])
    tot = {}
    for r in g:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:100]}")
        k = r["Kernel_Name"][:60]
        tot[k] = tot.get(k, 0) + (e - s) / 1e3
    print(f"span {(int(g[-1]['End_Timestamp']) - t0) / 1e3:.1f} us, kernels {len(g)}")
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:12]:
        print(f"  {v:8.1f} us  {k}")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--list":
        return listing(sys.argv[2])
    import numpy as np
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd.terrain import more_points
    wl = synthetic(16384, 1000, 1000, seed=0)
    dev = torch.device("cuda:0")
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    ax, ay, ao = more_points(wl, 7, seed=2024)
    for i in range(7):
        torch.cuda.synchronize()
        time.sleep(0.002)
        t0 = time.perf_counter()
        gm.append(t(ax[i:i + 1]), t(ay[i:i + 1]), t(ao[i:i + 1]))
        torch.cuda.synchronize()
        print(f"append {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
