"""Per-stage clock stamps of one xconv launch (diagnostic; needs a library
built with `make XCONV_DBG=1`): for workgroup 0's second tile, per wave, the
cycles from the previous barrier to the point its MFMAs are issued ("work")
and from there past its end-of-stage wait and barrier ("sync").

    python scripts/xconv_stamps.py 48x48@1088x1920k3r
"""
import ctypes
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dcvc_amd import hip as K


def main(sh):
    m = re.fullmatch(r"(\d+)x(\d+)@(\d+)x(\d+)(?:k(\d))?(r?)", sh)
    cin, cout, H, W = (int(m.group(i)) for i in range(1, 5))
    k = int(m.group(5) or 3)
    res = m.group(6) == "r"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cw = K.ConvW(torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5, torch.randn(cout) * 0.1, 1, K.F16X3, dev)
    x = K.from_nchw(torch.randn(1, cin, H, W, device=dev), K.F32)
    r = K.from_nchw(torch.randn(1, cout, H, W, device=dev), K.F32) if res else None
    for _ in range(3):
        y = K.conv(cw, x, act=K.ACT_LRELU, slope=0.1, res=r)
    torch.cuda.synchronize()
    print(K.lib().dcvc_last_kernel().decode())
    buf = (ctypes.c_uint * 512)()
    f = K.lib().dcvc_internal_xconv_stamps
    f.argtypes = [ctypes.c_void_p]
    assert f(ctypes.cast(buf, ctypes.c_void_p)) == 0, "library built without XCONV_DBG"
    st = np.array(buf[:], dtype=np.int64).reshape(8, 64)
    nst = int(np.count_nonzero(st[0])) // 2
    for w in range(8):
        t = st[w, :2 * nst]
        work = [(t[2 * s] - t[2 * s - 1]) % (1 << 32) for s in range(1, nst)]
        sync = [(t[2 * s + 1] - t[2 * s]) % (1 << 32) for s in range(nst)]
        print(f"wave {w} work", " ".join(f"{v:5d}" for v in work))
        print(f"wave {w} sync", " ".join(f"{v:5d}" for v in sync))
    tot = (st[0, 2 * nst - 1] - st[0, 1]) % (1 << 32)
    print("stages", nst, "cycles stage 1..last (wave 0):", tot)


if __name__ == "__main__":
    for a in sys.argv[1:]:
        main(a)
