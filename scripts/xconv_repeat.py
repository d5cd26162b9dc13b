"""Repeat the codec's split 3x3 / 7x7 conv shapes on fixed inputs and count
launches whose output bits differ from sconv.hip's (the reference path of the
same arithmetic): an intermittent race in a kernel's LDS ring or image
buffers shows up as a mismatch in some of the repeats.

    python scripts/xconv_repeat.py [--reps 50] [--shapes 48x48@1088x1920r,...]

Shape syntax: CINxCOUT@HxW[k7][r|rr][u] (residuals, pixel shuffle).  One JSON
line per shape: {"shape", "kernel", "reps", "mismatches"}.
"""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ("48x48@1088x1920,48x48@1088x1920r,48x48@1088x1920rr,64x64@544x960r,64x64@544x960rr,64x64@544x960,"
           "96x48@1088x1920,128x64@544x960,128x192@544x960u,96x96@272x480,64x128@544x960r,80x48@1088x1920,"
           "32x64@1088x1920k7,8x32@1088x1920k7,192x96@272x480")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--shapes", default=DEFAULT)
    a = ap.parse_args()
    import torch
    from dcvc_amd import hip as K
    dev = torch.device("cuda", 0)
    for sh in a.shapes.split(","):
        m = re.fullmatch(r"(\d+)x(\d+)@(\d+)x(\d+)(k7)?(r*)(u?)", sh)
        cin, cout, H, W = (int(m.group(i)) for i in range(1, 5))
        k = 7 if m.group(5) else 3
        nres, shuf = len(m.group(6)), bool(m.group(7))
        g = torch.Generator().manual_seed(cin + cout + H)
        x = K.from_nchw(torch.randn(1, cin, H, W, generator=g).to(dev), K.F32)
        cw = K.ConvW(torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5,
                     torch.randn(cout, generator=g) * 0.1, 1, K.F16X3, dev)
        co = cout // 4 if shuf else cout
        f = 2 if shuf else 1
        rs = [K.from_nchw(torch.randn(1, co, H, W, generator=g).to(dev), K.F32) for _ in range(nres)]
        kw = dict(act=K.ACT_LRELU, slope=0.1, shuffle=shuf, res=rs[0] if nres > 0 else None,
                  res2=rs[1] if nres > 1 else None)
        K.set_option("xconv", 0)
        try:
            ref = K.conv(cw, x, out_dtype=K.F32, **kw)
            torch.cuda.synchronize()
        finally:
            K.set_option("xconv", 1)
        y = K.empty(H * f, W * f, co, K.F32, dev)
        bad = 0
        kern = ""
        for _ in range(a.reps):
            y.buf.fill_(float("nan"))
            K.conv(cw, x, y, **kw)
            torch.cuda.synchronize()
            kern = K.lib().dcvc_last_kernel().decode()
            bad += int(not torch.equal(y.buf, ref.buf))
        print(json.dumps({"shape": sh, "kernel": kern, "reps": a.reps, "mismatches": bad}), flush=True)


if __name__ == "__main__":
    main()
