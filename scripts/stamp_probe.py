"""Diagnostic: per-segment cycle shares of the resident 3x3 conv loop, from a
stamped build (libdcvc_hip_STAMP.so, built outside the product tree)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["DCVC_HIP_LIB"] = "libdcvc_hip_STAMP.so"
import torch  # noqa: E402
from dcvc_amd import hip as K  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "dcvc_amd", "lib", "libdcvc_hip_STAMP.so"))
buf = (ctypes.c_ulonglong * 8)()
names = ["issue", "compute", "bar1", "put4", "wait+bar2", "store"]
for k, cin, cout, H, W in [(3, 48, 48, 1088, 1920), (3, 64, 64, 544, 960), (3, 96, 96, 272, 480)]:
    dev = torch.device("cuda", 0)
    cw = K.ConvW(torch.randn(cout, cin, k, k) / (cin * 9) ** 0.5, torch.zeros(cout), 1, K.BF16, dev)
    x = K.from_nchw(torch.randn(1, cin, H, W, device=dev), K.BF16)
    y = K.conv(cw, x)
    torch.cuda.synchronize()
    lib.dcvc_debug_stamps(buf, 1)
    for _ in range(5):
        K.conv(cw, x, y)
    torch.cuda.synchronize()
    lib.dcvc_debug_stamps(buf, 1)
    tot = sum(buf[i] for i in range(6))
    print(f"{cin}->{cout} {H}x{W}: waves {buf[6]}, cycles/wave {tot / max(buf[6], 1):.0f}: " +
          ", ".join(f"{n} {100.0 * buf[i] / tot:.1f}%" for i, n in enumerate(names)), flush=True)
