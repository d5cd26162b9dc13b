"""Time split-fp16 convolutions (sconv.hip) on the DC 1080p P-frame shapes.

    python scripts/sconv_bench.py [--reps 20] [--shapes 48x48@1088x1920k3r,...] [--opt NAME=VALUE]

A shape is CINxCOUT@HxW then kK (kernel size, default 3), sS (stride,
default 1), "r" for an fp32 residual input, "u" for a pixel-shuffled output and "g" for a
ConvFFN2-gated input (2 CIN channels, x1 * lrelu(x2)).  One JSON line per shape:
kernel, us/launch, algorithmic GB/s (fp32 input, split weights, output,
residual once each) and fp32-equivalent TFLOP/s (against 2500/3 = 833 peak).
"""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ("48x48@1088x1920k3r,64x64@544x960k3r,96x48@1088x1920k3,128x192@544x960k3,32x64@1088x1920k7,"
           "64x32@1088x1920k7,48x192@1088x1920k1,192x48@1088x1920k1r,384x384@68x120k1,1024x384@68x120k1,"
           "56x64@1088x1920k3s2")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default=DEFAULT)
    ap.add_argument("--opt", action="append", default=[], help="NAME=VALUE for dcvc_set_option (repeatable)")
    a = ap.parse_args()
    import torch
    from dcvc_amd import hip as K
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for o in a.opt:
        name, val = o.split("=")
        if name != "arm":   # (a label only: which library of an A/B run)
            K.set_option(name, int(val))
    for sh in a.shapes.split(","):
        m = re.fullmatch(r"(\d+)x(\d+)@(\d+)x(\d+)(?:k(\d))?(?:s(\d))?(r{0,2})(u?)(g?)", sh)
        cin, cout, H, W = (int(m.group(i)) for i in range(1, 5))
        k = int(m.group(5) or 3)
        s = int(m.group(6) or 1)
        res = len(m.group(7)) >= 1
        res2 = len(m.group(7)) == 2
        shuf = m.group(8) == "u"
        gate = m.group(9) == "g"
        gk = dict(in_op=K.IN_GATE, in_slope=0.1) if gate else {}
        cw = K.ConvW(torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5, torch.randn(cout) * 0.1, s, K.F16X3, dev)
        x = K.from_nchw(torch.randn(1, 2 * cin if gate else cin, H, W, device=dev), K.F32)
        Ho, Wo = cw.out_hw(H, W)
        r = K.from_nchw(torch.randn(1, cout, Ho, Wo, device=dev), K.F32) if res else None
        if res2:
            gk["res2"] = K.from_nchw(torch.randn(1, cout, Ho, Wo, device=dev), K.F32)
        y = K.empty(Ho * 2, Wo * 2, cout // 4, K.F32, dev) if shuf else K.empty(Ho, Wo, cout, K.F32, dev)
        for _ in range(3):
            K.conv(cw, x, y, act=K.ACT_LRELU, slope=0.1, res=r, shuffle=shuf, **gk)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            K.conv(cw, x, y, act=K.ACT_LRELU, slope=0.1, res=r, shuffle=shuf, **gk)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        nb = 4 * (H * W * cin * (2 if gate else 1) + Ho * Wo * cout * (1 + res + res2)) + cw.w.numel() * 2
        fl = 2.0 * Ho * Wo * cin * cout * k * k
        print(json.dumps({"shape": sh, "opt": a.opt, "kernel": K.lib().dcvc_last_kernel().decode(), "us": round(us, 2),
                          "gbs": round(nb / us / 1e3, 1), "tflops": round(fl / us / 1e6, 1),
                          "frac_mfma": round(fl / us / 1e6 / 833.3, 3)}), flush=True)


if __name__ == "__main__":
    main()
