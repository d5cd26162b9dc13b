"""Average every PMC counter per kernel over the rocprofv3 passes under DIR
(scripts/pmc_shape.sh) and print one JSON line per kernel with a few derived
ratios (MFMA busy fraction of the XCD-corrected active cycles, LDS bank-conflict
share, wait share)."""
import collections
import csv
import glob
import json
import os
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in acc.items():
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        out = {"kernel": name, "launches": max(len(v) for v in cs.values())}
        out.update({k: round(v, 1) for k, v in sorted(m.items())})
        g = m.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs (MI355X_MICROARCH.md,
            # DVFS note): the kernel's cycles are g / 8; MFMA busy counts cycles
            # summed over all 1024 SIMDs
            out["gui_cycles"] = round(g / 8, 1)
            out["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 256 * 4), 3)
        if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_ANY" in m:
            out["wait_any_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        if "SQ_LDS_IDX_ACTIVE" in m and "SQ_LDS_BANK_CONFLICT" in m and m["SQ_LDS_IDX_ACTIVE"]:
            out["lds_conflict_frac"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 3)
        if "FETCH_SIZE" in m:
            out["hbm_bytes"] = int((2 * m["FETCH_SIZE"] + m.get("WRITE_SIZE", 0)) * 1024)
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
