"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace
(--kernel-trace --output-format csv): where the GPU waits for the host.

    python scripts/gap_analysis.py TRACE_DIR [--top 30]
"""
import argparse
import csv
import glob
import os
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--skip", type=int, default=3, help="frames to skip (setup, warmup)")
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    rows.sort()
    # steady state: from the (skip+1)-th frame upload on (frame_kernel marks a frame start)
    starts = [i for i, r in enumerate(rows) if "frame_kernel" in r[2]]
    if len(starts) > a.skip:
        rows = rows[starts[a.skip]:]
        print(f"frames in window: {len(starts) - a.skip}")
    gaps = []
    busy = 0
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        gaps.append((s1 - e0, n0, n1))
    for s, e, n in rows:
        busy += e - s
    span = rows[-1][1] - rows[0][0]
    tot_gap = sum(g for g, _, _ in gaps if g > 0)
    print(f"kernels {len(rows)} span {span/1e6:.2f} ms busy {busy/1e6:.2f} ms gaps {tot_gap/1e6:.2f} ms")
    hist = collections.Counter()
    for g, _, _ in gaps:
        b = "<5us" if g < 5000 else "<20us" if g < 20000 else "<100us" if g < 100000 else "<1ms" if g < 1e6 else ">1ms"
        hist[b] += g
    print({k: round(v / 1e6, 2) for k, v in hist.items()})
    by_pair = collections.defaultdict(float)
    for g, n0, n1 in gaps:
        if g > 20000:
            by_pair[(n0, n1)] += g
    for (n0, n1), g in sorted(by_pair.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{g/1e6:7.2f} ms  {n0}  ->  {n1}")


if __name__ == "__main__":
    main()
