"""Time the fused DepthConvBlock kernels on the DC 1080p P-frame's shapes.

    python scripts/dcb_bench.py [--reps 30] [--shapes 128x128@272x480,...] [--kernels stream,tile]

Kernels: "stream" = dcbs.hip (persistent, streamed weights), "persistent" =
dcbp.hip (resident weights, where it applies), "tile" = dcb.hip.  Prints one
JSON line per (shape, kernel): us/launch, TFLOP/s, and whether the output is
bit-identical to the first kernel's.
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
    ap.add_argument("--shapes", default="128x128@272x480,128x64@544x960,64x128@272x480,64x48@1088x1920")
    ap.add_argument("--kernels", default="stream,tile")
    ap.add_argument("--opt", action="append", default=[], help="NAME=VALUE for dcvc_set_option (repeatable)")
    a = ap.parse_args()
    import torch
    from dcvc_amd import hip as K
    from dcvc_amd import layers as L
    from dcvc_amd.weights import synthetic_state_dict
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for o in a.opt:
        name, val = o.split("=")
        K.set_option(name, int(val))
    opts = {"stream": (1, 0), "persistent": (0, 1), "tile": (0, 0)}
    for sh in a.shapes.split(","):
        ch, hw = sh.split("@")
        cin, cout = (int(v) for v in ch.split("x"))
        H, W = (int(v) for v in hw.split("x"))
        gated = False
        p = "b.block"
        hid = max(min(4 * cout, 1024), 2 * cout)
        spec = [(f"{p}.0.conv1.0.weight", (cin, cin, 1, 1)), (f"{p}.0.conv1.0.bias", (cin,)),
                (f"{p}.0.depth_conv.weight", (cin, 1, 3, 3)), (f"{p}.0.depth_conv.bias", (cin,)),
                (f"{p}.0.conv2.weight", (cout, cin, 1, 1)), (f"{p}.0.conv2.bias", (cout,)),
                (f"{p}.1.conv.0.weight", (hid, cout, 1, 1)), (f"{p}.1.conv.0.bias", (hid,)),
                (f"{p}.1.conv.2.weight", (cout, hid, 1, 1)), (f"{p}.1.conv.2.bias", (cout,))]
        if cin != cout:
            spec += [(f"{p}.0.adaptor.weight", (cout, cin, 1, 1)), (f"{p}.0.adaptor.bias", (cout,))]
        sd = synthetic_state_dict(spec, seed=1, gain=1.5)
        blk = L.DepthConvBlock(L.Ctx(sd, dev, L.Precision.fast()), "b", gated=gated)
        x = K.from_nchw(torch.randn(1, cin, H, W, device=dev), K.BF16)
        y = K.empty(H, W, cout, K.BF16, dev)
        ref = None
        mac = cin * cin + cin * 9 + cout * cin * (2 if cin != cout else 1) + 2 * hid * cout
        for kn in a.kernels.split(","):
            st, pe = opts[kn]
            K.set_option("dcb_stream", st)
            K.set_option("dcb_persistent", pe)
            for _ in range(3):
                blk(x, y=y)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                blk(x, y=y)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            out = y.t().clone()
            same = True if ref is None else bool(torch.equal(out, ref))
            ref = out if ref is None else ref
            print(json.dumps({"shape": sh, "kernel": K.lib().dcvc_last_kernel().decode(), "us": round(us, 2),
                              "tflops": round(2.0 * mac * H * W / us / 1e6, 1), "bit_identical": same}), flush=True)
    K.set_option("dcb_stream", 1)
    K.set_option("dcb_persistent", 1)


if __name__ == "__main__":
    main()
