"""Time the bf16 3x3 stride-1 convolutions of the DC 1080p P-frame.

    python scripts/conv3_bench.py [--reps 30] [--shapes 48x48@1088x1920r,...]

A shape is CINxCOUT@HxW, with a trailing "r" for a bf16 residual input (the
ResBlock form out = x + conv(...)) and / or "k7" for a 7x7 kernel (SpyNet).  Prints one JSON line per shape: the
kernel, us/launch, algorithmic GB/s (input, weights, output and residual read
or written once) and TFLOP/s.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--shapes", default="48x48@1088x1920r,64x64@544x960r,96x96@272x480r")
    ap.add_argument("--opt", action="append", default=[], help="NAME=VALUE for dcvc_set_option (repeatable)")
    a = ap.parse_args()
    import torch
    from dcvc_amd import hip as K
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for o in a.opt:
        name, val = o.split("=")
        K.set_option(name, int(val))
    for sh in a.shapes.split(","):
        k = 7 if "k7" in sh else 3
        base = sh.replace("k7", "")
        res = base.endswith("r")
        ch, hw = base.rstrip("r").split("@")
        cin, cout = (int(v) for v in ch.split("x"))
        H, W = (int(v) for v in hw.split("x"))
        cw = K.ConvW(torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5, torch.randn(cout) * 0.1, 1, K.BF16, dev)
        x = K.from_nchw(torch.randn(1, cin, H, W, device=dev), K.BF16)
        r = K.from_nchw(torch.randn(1, cout, H, W, device=dev), K.BF16) if res else None
        y = K.empty(H, W, cout, K.BF16, dev)
        for _ in range(3):
            K.conv(cw, x, y, act=K.ACT_LRELU, slope=0.1, res=r)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            K.conv(cw, x, y, act=K.ACT_LRELU, slope=0.1, res=r)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        nb = H * W * 2 * (cin + cout * (2 if res else 1)) + cout * cin * k * k * 2
        print(json.dumps({"shape": sh, "opt": a.opt, "kernel": K.lib().dcvc_last_kernel().decode(), "us": round(us, 2),
                          "gbs": round(nb / us / 1e3, 1), "tflops": round(2.0 * H * W * cin * cout * k * k / us / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
