"""Golden MS-SSIM vectors from the reference's own calc_msssim
(DCVC-DC/src/utils/metrics.py:15-62, numpy/scipy only), imported from
/root/reference by path.  Inputs are regenerated from the seeds stored in the
fixture; the fixture holds only seeds, shapes and the reference's outputs.

    python tests/golden/make_golden_msssim.py
"""
import importlib.util
import json
import os

import numpy as np

REF = "/root/reference/DCVC-DC/src/utils/metrics.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "msssim_golden.json")

# (seed, h, w): plane sizes of the YUV path (Y and 4:2:0 chroma), both level
# counts (5 levels from 176 px, 4 below), odd intermediate sizes
CASES = [(1, 96, 128), (2, 176, 176), (3, 200, 310), (4, 270, 480), (5, 135, 241), (6, 540, 960)]


def planes(seed, h, w):
    """A source plane (uint8 / 255, as float32 -> float64) and a distorted
    recon plane (float32 in [0, 1]) of the same size."""
    g = np.random.Generator(np.random.PCG64(seed))
    src = (g.integers(0, 256, size=(h, w)).astype(np.float32) / np.float32(255))
    noise = g.normal(0, 0.05, size=(h, w)).astype(np.float32)
    rec = np.clip(src + noise, 0, 1).astype(np.float32)
    return src, rec


def main():
    spec = importlib.util.spec_from_file_location("ref_metrics", REF)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    rows = []
    for seed, h, w in CASES:
        src, rec = planes(seed, h, w)
        rows.append({"seed": seed, "h": h, "w": w, "msssim": float(m.calc_msssim(src, rec, data_range=1)),
                     "psnr": float(m.calc_psnr(src, rec, data_range=1))})
    with open(OUT, "w") as f:
        json.dump({"source": "DCVC-DC/src/utils/metrics.py calc_msssim / calc_psnr (data_range=1)",
                   "cases": rows}, f, indent=1)
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
