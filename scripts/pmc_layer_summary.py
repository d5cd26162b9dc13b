"""Summarise scripts/pmc_layer.sh: per layer shape, the split conv kernel's
HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 calibration of
scripts/pmc_summary.py) and its algorithmic bytes as dcvc_amd/hip.py counts
them, written to gpurun_out/pmcl_<name>/<name>_pmc_layers.json."""
import csv
import glob
import json
import os
import re
import sys


def counter(d, name):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                if k.startswith(("void sconv", "void sgemm", "void xconv")):
                    vals.setdefault(k, []).append(float(r["Counter_Value"]))
    return vals


def main(out, name, shapes):
    recs = []
    for sh in shapes:
        m = re.fullmatch(r"(\d+)x(\d+)@(\d+)x(\d+)(?:k(\d))?(?:s(\d))?(r?)", sh)
        cin, cout, H, W = (int(m.group(i)) for i in range(1, 5))
        k, s, res = int(m.group(5) or 3), int(m.group(6) or 1), m.group(7) == "r"
        fe = counter(os.path.join(out, f"{sh}.FETCH_SIZE"), "FETCH_SIZE")
        wr = counter(os.path.join(out, f"{sh}.WRITE_SIZE"), "WRITE_SIZE")
        kern = max(fe, key=lambda n: len(fe[n]))
        fetch = sum(fe[kern]) / len(fe[kern]) * 1024
        write = sum(wr[kern]) / len(wr[kern]) * 1024
        # the microbench's last launch name (instantiation@grid) from its JSON line
        with open(os.path.join(out, f"{sh}.FETCH_SIZE.log")) as f:
            line = [json.loads(x) for x in f if x.startswith("{")][-1]
        Ho, Wo = (H + 2 * ((k - 1) // 2) - k) // s + 1, (W + 2 * ((k - 1) // 2) - k) // s + 1
        nb_w = cout * k * k * ((cin + 31) // 32 * 32) * 4   # packed split weights (hi + lo halves, padded)
        recs.append({"shape": sh, "kernel": line["kernel"], "layer": f"k{k}s{s} {cin}->{cout} {H}x{W} f16x3 in0out0",
                     "residual": res, "hbm_bytes_per_launch": int(2 * fetch + write),
                     "algorithmic_bytes_no_weights": 4 * (H * W * cin + Ho * Wo * cout * (2 if res else 1)),
                     "weight_bytes_approx": nb_w, "avg_us": line["us"]})
    path = os.path.join(out, f"{name}_pmc_layers.json")
    with open(path, "w") as f:
        json.dump({"tool": "scripts/pmc_layer.sh", "layers": recs}, f, indent=1)
    print(json.dumps(recs))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
