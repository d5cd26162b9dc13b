"""Host rANS coder microbenchmark on the symbol load of one DCVC-DC 1080p
P-frame (C3): mv_z 64x17x30, z 128x17x30 (factorized tables), then 4
quadtree steps of mv_y (16 ch each) and 4 of y (32 ch each) at 68x120 with
the 256-row Laplace scale table.  Symbols are drawn from each row's own
distribution so the bypass rate matches real streams.

    python scripts/coder_bench.py [--parts 4] [--iters 5]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcvc_amd.entropy import ScaleTable  # noqa: E402
from dcvc_amd.rans import RansEncoder, RansDecoder, CdfTable  # noqa: E402


def draw(tab, idx, g):
    """symbols of row idx: inverse-CDF sample of the quantised CDF, plus 0.2%
    far outliers (bypass path)."""
    cdf, sizes, offs = tab.cdf, tab.sizes, tab.offsets
    u = g.integers(0, 1 << 16, size=idx.size)
    out = np.empty(idx.size, np.int16)
    for r in np.unique(idx):
        m = idx == r
        row = cdf[r, :sizes[r]]
        v = np.searchsorted(row, u[m], side="right") - 1
        out[m] = np.clip(v, 0, sizes[r] - 2) + offs[r]
    far = g.random(idx.size) < 0.002
    out[far] = g.integers(-300, 300, size=int(far.sum()))
    return out


def workload(seed=0):
    g = np.random.Generator(np.random.PCG64(seed))
    st = ScaleTable("laplace")
    yh, yw, zh, zw = 68, 120, 17, 30
    calls = []
    # factorized z tables stand in with table rows of moderate scale
    for ch in (64, 128):
        n = ch * zh * zw
        idx = np.repeat(np.arange(ch) % 64 + 96, zh * zw).astype(np.int16)
        calls.append((draw(st, idx, g), idx))
    for ch in [16] * 4 + [32] * 4:
        n = ch * yh * yw
        idx = np.clip(g.normal(60, 40, size=n), 0, 255).astype(np.int16)
        calls.append((draw(st, idx, g), idx))
    return st, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    st, calls = workload()
    n = sum(c[0].size for c in calls)
    enc = RansEncoder(True, a.parts)
    dec = RansDecoder(a.parts)
    te, tf, td = [], [], []
    for _ in range(a.iters):
        enc.reset()
        t0 = time.perf_counter()
        for s, i in calls:
            enc.encode_table(s, i, st.table)
        t1 = time.perf_counter()
        enc.flush()
        stream = enc.get_encoded_stream()
        t2 = time.perf_counter()
        dec.set_stream(stream)
        for s, i in calls:
            out = dec.decode_table(i, st.table)
            assert np.array_equal(out, s)
        t3 = time.perf_counter()
        te.append(t1 - t0)
        tf.append(t2 - t1)
        td.append(t3 - t2)
    ms = lambda v: round(1e3 * float(np.median(v)), 3)  # noqa: E731
    print({"symbols": n, "parts": a.parts, "bytes": int(stream.size), "encode_calls_ms": ms(te),
           "flush_ms": ms(tf), "decode_ms": ms(td), "total_ms": round(ms(te) + ms(tf) + ms(td), 3)})


if __name__ == "__main__":
    main()
