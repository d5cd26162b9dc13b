"""Time the fused split-fp16 blocks and gather kernels on the DC P-frame shapes.

    python scripts/block_bench.py [--reps 20] [--shapes ffn128@272x480,dc64x48a@1088x1920,od@1088x1920]

Shapes: ffnC@HxW (ConvFFN C -> 4C -> C, sffn / slffn), dcCINxCOUT[a]@HxW (DepthConv,
"a" with the adaptor, sdc), od@HxW (OffsetDiversity of a 48-channel map).  One JSON
line per shape: kernel, us per launch, algorithmic GB/s and fp32-equivalent TFLOP/s
(the f16x3 peak is 2500 / 3 = 833).
"""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ("ffn128@272x480,ffn64@544x960,ffn48@1088x1920,ffn32@1088x1920,ffn384@68x120,"
           "dc64x48a@1088x1920,dc48x32a@1088x1920,dc64x64@544x960,od@1088x1920")


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
        if name == "arm":          # A/B label (scripts/gpu_lease.sh ab)
            continue
        if name == "od_planar":
            K.OD_PLANAR = bool(int(val))
        else:
            K.set_option(name, int(val))
    for sh in a.shapes.split(","):
        m = re.fullmatch(r"([a-z]+?)(\d*)(?:x(\d+))?(a?)@(\d+)x(\d+)", sh)
        kind, H, W = m.group(1), int(m.group(5)), int(m.group(6))
        if kind == "ffn":
            c = int(m.group(2))
            hid = 4 * c if c <= 128 else {384: 1024, 192: 768}[c]
            fw = K.FfnW(torch.randn(hid, c, 1, 1) / c ** 0.5, torch.randn(hid) * 0.1,
                        torch.randn(c, hid, 1, 1) / hid ** 0.5, torch.randn(c) * 0.1, dev)
            x = K.from_nchw(torch.randn(1, c, H, W, device=dev), K.F32)
            y = K.empty(H, W, c, K.F32, dev)
            run = lambda: K.conv_ffn(fw, x, y, slope=0.1)  # noqa: E731
            fl = 4.0 * H * W * c * hid
            nb = 4 * 2 * H * W * c + fw.w.numel() * 2
        elif kind == "dc":
            cin, cout, ad = int(m.group(2)), int(m.group(3)), m.group(4) == "a"
            r = lambda *s: torch.randn(*s) * 0.2  # noqa: E731
            dw = K.DcW(r(cin, cin, 1, 1), r(cin), r(9, cin).to(dev), r(cin), r(cout, cin, 1, 1), r(cout),
                       r(cout, cin, 1, 1) if ad else None, r(cout) if ad else None, dev)
            x = K.from_nchw(torch.randn(1, cin, H, W, device=dev), K.F32)
            y = K.empty(H, W, cout, K.F32, dev)
            run = lambda: K.depth_conv_split(dw, x, y)  # noqa: E731
            fl = 2.0 * H * W * (cin * cin + 9 * cin + cin * cout * (2 if ad else 1))
            nb = 4 * H * W * (cin + cout) + dw.w.numel() * 2
        elif kind in ("dwc", "dwu"):
            # the DepthConv tail (depthwise + conv2 + identity): fused (sldc.hip,
            # dcvc_dw_conv2_split) or unfused (dwconv3x3, then the 1x1 with the residual)
            c = int(m.group(2))
            r = lambda *s: torch.randn(*s) * 0.2  # noqa: E731
            w9, bd, w2, b2 = r(9, c).contiguous().to(dev), r(c).to(dev), r(c, c, 1, 1), r(c)
            dwc = K.DwcW(w9, bd, w2, b2, dev)
            cw2 = K.ConvW(w2, b2, 1, K.F16X3, dev)
            t = K.from_nchw(torch.randn(1, c, H, W, device=dev), K.F32)
            x = K.from_nchw(torch.randn(1, c, H, W, device=dev), K.F32)
            y = K.empty(H, W, c, K.F32, dev)
            if kind == "dwc":
                run = lambda: K.dw_conv2_split(dwc, t, x, y)  # noqa: E731
            else:
                run = lambda: K.conv(cw2, K.dwconv3x3(t, w9, bd), y, res=x)  # noqa: E731
            fl = 2.0 * H * W * c * (9 + c)
            nb = 4 * H * W * 3 * c
        elif kind in ("od", "odr"):
            # odr: offsets spread like the bench codec's random-weight ones
            # (40 tanh(o) scattered over tens of pixels); od: small, smooth
            feat = K.from_nchw(torch.randn(1, 48, H, W, device=dev), K.F32)
            offs = K.from_nchw(torch.randn(1, 96, H // 2, W // 2, device=dev) * (0.05 if kind == "od" else 1.0), K.F32)
            flow = K.from_nchw(torch.randn(1, 2, H, W, device=dev) * 3, K.F32)
            fw = (torch.randn(48, 6) * 0.3).contiguous().to(dev)
            fb = (torch.randn(48) * 0.1).to(dev)
            grid = (torch.linspace(-1.0, 1.0, W, dtype=torch.float32, device=dev),
                    torch.linspace(-1.0, 1.0, H, dtype=torch.float32, device=dev))
            cat = K.empty(H, W, 96, K.F32, dev)
            y = cat.ch(48, 48)
            run = lambda: K.offset_diversity(feat, offs, flow, fw, fb, grid, y=y)  # noqa: E731
            fl = 0.0
            nb = 4 * H * W * (48 + 48 + 2) + 4 * (H // 2) * (W // 2) * 96
        else:
            raise ValueError(sh)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(json.dumps({"shape": sh, "opt": a.opt, "kernel": K.lib().dcvc_last_kernel().decode(), "us": round(us, 2),
                          "GBps": round(nb / us / 1e3, 1), "TFLOPs": round(fl / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
