"""Summarise scripts/pmc_blocks.sh: per shape, the dominant kernel's counters
averaged over its dispatches (HBM bytes with the gfx950 calibration of
scripts/pmc_summary.py: 2 x FETCH_SIZE + WRITE_SIZE, KiB units), its time per
launch from the microbench's own JSON line, and the L2 hit rate
TCC_HIT / (TCC_HIT + TCC_MISS), written to gpurun_out/pmcb_<name>/<name>_pmc_blocks.json."""
import csv
import glob
import json
import os
import sys

GROUPS = ("L2", "FETCH", "WRITE", "SQ", "TA")


def read(d):
    """{kernel: {counter: [values per dispatch]}}"""
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                out.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return out


def main(out, name, shapes):
    recs = []
    for sh in shapes:
        per = {g: read(os.path.join(out, f"{sh}.{g}")) for g in GROUPS}
        # the shape's kernel: the one with the most dispatches in the L2 pass
        # (the microbench launches it 3 + reps times)
        src = next((per[g] for g in GROUPS if per[g]), {})
        if not src:
            continue
        kern = max(src, key=lambda k: max(len(v) for v in src[k].values()))
        ctr = {}
        for g in GROUPS:
            for c, v in per[g].get(kern, {}).items():
                ctr[c] = sum(v) / len(v)
        rec = {"shape": sh, "kernel": kern, "counters_per_dispatch": ctr}
        if "FETCH_SIZE" in ctr and "WRITE_SIZE" in ctr:
            rec["hbm_bytes_per_launch"] = int((2 * ctr["FETCH_SIZE"] + ctr["WRITE_SIZE"]) * 1024)
        h, m = ctr.get("TCC_HIT_sum"), ctr.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            rec["l2_hit_rate"] = h / (h + m)
            rec["l2_requests"] = h + m
        if ctr.get("SQ_INSTS_MFMA"):
            rec["valu_per_mfma"] = ctr.get("SQ_INSTS_VALU", 0) / ctr["SQ_INSTS_MFMA"]
            rec["salu_per_mfma"] = ctr.get("SQ_INSTS_SALU", 0) / ctr["SQ_INSTS_MFMA"]
        if ctr.get("SQ_WAVE_CYCLES"):
            rec["wait_frac"] = ctr.get("SQ_WAIT_ANY", 0) / ctr["SQ_WAVE_CYCLES"]
            rec["issue_stall_frac"] = ctr.get("SQ_WAIT_INST_ANY", 0) / ctr["SQ_WAVE_CYCLES"]
        logs = glob.glob(os.path.join(out, f"{sh}.L2.log")) + glob.glob(os.path.join(out, f"{sh}.FETCH.log"))
        for lp in logs:
            with open(lp) as f:
                lines = [json.loads(x) for x in f if x.startswith("{")]
            if lines:
                rec["us_profiled"] = lines[-1]["us"]
                rec["microbench_kernel"] = lines[-1]["kernel"]
                break
        recs.append(rec)
    path = os.path.join(out, f"{name}_pmc_blocks.json")
    with open(path, "w") as f:
        json.dump({"tool": "scripts/pmc_blocks.sh", "shapes": recs}, f, indent=1)
    print(json.dumps(recs)[:4000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
