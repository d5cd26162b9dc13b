"""Where do xconv's pixel-shuffle outputs land, against sconv's? (diagnostic)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dcvc_amd import hip as h

torch.manual_seed(0)
cin, cout, H, W = 32, 64, 4, 16
x = torch.randn(1, cin, H, W)
w = torch.randn(cout, cin, 3, 3) / 17
b = torch.zeros(cout)
cw = h.ConvW(w, b, 1, h.F16X3)
xa = h.from_nchw(x, h.F32)
outs = []
for o in (1, 0):
    h.set_option("xconv", o)
    y = h.conv(cw, xa, shuffle=True)
    torch.cuda.synchronize()
    print(h.lib().dcvc_last_kernel().decode())
    outs.append(y.nchw().cpu()[0])
h.set_option("xconv", 1)
a, r = outs
print("max abs xconv", a.abs().max().item(), "sconv", r.abs().max().item())
# for a few xconv outputs, find the matching sconv position
flat = r.reshape(-1)
C, HH, WW = r.shape
for (c, yy, xx) in [(0, 0, 0), (0, 0, 1), (0, 1, 0), (1, 0, 0), (2, 0, 0), (5, 1, 3), (0, 2, 0), (4, 0, 0)]:
    v = a[c, yy, xx].item()
    i = (flat - v).abs().argmin().item()
    print((c, yy, xx), v, "->", (i // (HH * WW), (i // WW) % HH, i % WW), flat[i].item())
