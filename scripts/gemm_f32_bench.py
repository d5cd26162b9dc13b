"""A/B the fp32 1x1 GEMM tile configurations (gemm1x1f.hip) on the latent
shapes of the DC 1080p P-frame (68x120 pixels).

    python scripts/gemm_f32_bench.py [--reps 50] [--cfgs 0,1,2,...]

Prints us/launch and TFLOP/s per (shape, config); config 0 is the automatic
choice, -1 the generic conv.hip f32 path.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [(384, 384), (1024, 384), (384, 1024), (192, 192), (768, 192), (192, 768), (1024, 256), (256, 1024),
          (384, 256), (512, 128)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cfgs", default="-1,0,1,2,3,4,5,6,7,8,9,10,11")
    ap.add_argument("--H", type=int, default=68)
    ap.add_argument("--W", type=int, default=120)
    ap.add_argument("--k3", action="store_true", help="time HEM's fp32 3x3 latent convs (conv.hip f32 path) instead")
    ap.add_argument("--shapes", default="", help="cin x cout list, e.g. 384x384,1024x384")
    ap.add_argument("--opt", action="append", default=[], help="NAME=VALUE for dcvc_set_option (repeatable)")
    a = ap.parse_args()
    import torch
    from dcvc_amd import hip as K
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for o in a.opt:
        name, val = o.split("=")
        K.set_option(name, int(val))
    rows = []
    k = 3 if a.k3 else 1
    shapes = [(384, 288), (480, 384), (192, 192), (288, 288), (128, 128), (64, 64)] if a.k3 else SHAPES
    if a.shapes:
        shapes = [tuple(int(v) for v in sh.split("x")) for sh in a.shapes.split(",")]
    cfgs = [-1] if a.k3 else [int(c) for c in a.cfgs.split(",")]
    for cin, cout in shapes:
        cw = K.ConvW(torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5, torch.randn(cout) * 0.1, 1, K.F32, dev)
        x = K.from_nchw(torch.randn(1, cin, a.H, a.W, device=dev), K.F32)
        y = K.conv(cw, x)
        ref = None
        for cfg in cfgs:
            K.set_option("gemm1x1_f32", 0 if cfg < 0 else 1)
            K.set_option("gemm1x1_f32_cfg", max(cfg, 0))
            for _ in range(3):
                K.conv(cw, x, y)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                K.conv(cw, x, y)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            out = y.t().clone()
            same = True if ref is None else bool(torch.equal(out, ref))
            ref = out if ref is None else ref
            fl = 2.0 * a.H * a.W * cin * cout * k * k
            rows.append({"shape": f"{cin}->{cout}", "cfg": cfg, "kernel": K.lib().dcvc_last_kernel().decode(),
                         "us": round(us, 2), "tflops": round(fl / us / 1e6, 1), "bit_identical": same})
            print(json.dumps(rows[-1]), flush=True)
    K.set_option("gemm1x1_f32", 1)
    K.set_option("gemm1x1_f32_cfg", 0)


if __name__ == "__main__":
    main()
