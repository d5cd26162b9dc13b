"""Summarise rocprofv3 runs of bench.py into profiles/<round>_pmc.json.

    python scripts/pmc_summary.py --trace DIR --fetch DIR --write DIR --out profiles/r01_pmc.json

--trace: a `rocprofv3 --kernel-trace --stats --output-format csv` run;
--fetch / --write: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs of
the same command (the two counters do not fit one pass on gfx950).
Kernels are keyed as bench.py keys them: the instantiation name as rocprof
prints it, without namespaces and argument list, plus '@' and the grid size
in work-items (dcvc_last_kernel()).  HBM bytes per launch = 2 x FETCH_SIZE +
WRITE_SIZE (KiB -> bytes): on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads (MI355X_MICROARCH.md, HBM section).
"""
import argparse
import collections
import csv
import glob
import json
import os


def norm(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].strip()


def rows(d, pattern):
    out = []
    for path in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(path) as f:
            out += list(csv.DictReader(f))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--command", default="")
    a = ap.parse_args()

    trace = collections.defaultdict(list)
    for r in rows(a.trace, "*kernel_trace.csv"):
        gs = int(r.get("Grid_Size_X", r.get("Grid_Size", 0))) * int(r.get("Grid_Size_Y", 1)) * \
            int(r.get("Grid_Size_Z", 1))
        trace[f"{norm(r['Kernel_Name'])}@{gs}"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, cname in ((a.fetch, "FETCH_SIZE"), (a.write, "WRITE_SIZE")):
        for r in rows(d, "*counter_collection.csv"):
            if r["Counter_Name"] != cname:
                continue
            ctr[f"{norm(r['Kernel_Name'])}@{int(r['Grid_Size'])}"][cname].append(float(r["Counter_Value"]))
    kernels = []
    for k, durs in trace.items():
        e = {"kernel": k, "launches": len(durs), "avg_us": round(sum(durs) / len(durs) / 1e3, 2),
             "total_ms": round(sum(durs) / 1e6, 3)}
        c = ctr.get(k)
        if c and c.get("FETCH_SIZE") and c.get("WRITE_SIZE"):
            f = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) * 1024
            w = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) * 1024
            e.update({"fetch_bytes_raw": int(f), "write_bytes": int(w), "hbm_bytes_per_launch": int(2 * f + w)})
        kernels.append(e)
    kernels.sort(key=lambda e: -e["total_ms"])
    with open(a.out, "w") as f:
        json.dump({"command": a.command, "note": "hbm_bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE (gfx950)",
                   "kernels": kernels}, f, indent=1)
    print(f"wrote {a.out}: {len(kernels)} kernels")


if __name__ == "__main__":
    main()
