"""Host side of the split-fp16 convs (no GPU): dcvc_conv_pack_weights with
compute DCVC_F16X3 writes, per 32-channel input chunk, a hi and a lo block
[rows][cout][32] of fp16 halves with w = hi + 2^-11 lo to ~2^-22, and packs
2 / 4 taps per row for a last chunk of <= 16 / <= 8 channels
(dcvc_amd/csrc/hip/sconv.hip, conv.hip:pack_f16x3)."""
import ctypes

import numpy as np
import pytest
import torch


def pack(w):
    from dcvc_amd import hip as h
    wn = np.ascontiguousarray(w.numpy().astype(np.float32))
    cout, cin, kh, kw = wn.shape
    n = h.lib().dcvc_conv_pack_weights(wn.ctypes.data_as(ctypes.c_void_p), cout, cin, kh, kw, h.F16X3, None)
    assert n > 0
    out = np.zeros(n, dtype=np.uint16)
    assert h.lib().dcvc_conv_pack_weights(wn.ctypes.data_as(ctypes.c_void_p), cout, cin, kh, kw, h.F16X3,
                                          out.ctypes.data_as(ctypes.c_void_p)) == n
    return out


def unpack(buf, cout, cin, k):
    """Rebuild [cout][cin][k][k] from the packed layout (independent decoder)."""
    kt = k * k
    nch = (cin + 31) // 32
    full = 2 * kt * cout * 32
    w = np.zeros((cout, cin, k, k))
    for c in range(nch):
        vc = cin - 32 * c if c == nch - 1 else 32
        tpk = (4 if vc <= 8 else 2 if vc <= 16 else 1) if c == nch - 1 else 1
        spt = 4 // tpk
        rows = (kt + tpk - 1) // tpk
        blk = buf[c * full: c * full + 2 * rows * cout * 32]
        hi = blk[:rows * cout * 32].view(np.float16).astype(np.float64).reshape(rows, cout, 32)
        lo = blk[rows * cout * 32:].view(np.float16).astype(np.float64).reshape(rows, cout, 32)
        v = hi + lo / 2048.0
        for r in range(rows):
            for kk in range(32):
                s, e = kk // 8, kk % 8
                tap = tpk * r + s // spt
                ch = c * 32 + (s % spt) * 8 + e
                if tap < kt and ch < cin:
                    w[:, ch, tap // k, tap % k] = v[r, :, kk]
                else:
                    assert np.all(v[r, :, kk] == 0)
    return w


@pytest.mark.parametrize("cout,cin,k", [(48, 48, 3), (64, 80, 3), (32, 8, 7), (2, 16, 7), (64, 2, 3),
                                        (384, 1024, 1), (16, 3, 3), (40, 33, 1)])
def test_pack_f16x3_roundtrip(cout, cin, k):
    g = torch.Generator().manual_seed(cout + cin + k)
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    w[0, 0, 0, 0] = 3e-7       # fp16 subnormal range
    w[-1, -1, -1, -1] = -1.5e3
    got = unpack(pack(w), cout, cin, k)
    ref = w.double().numpy()
    err = np.abs(got - ref)
    assert np.all(err <= np.abs(ref) * 2.0 ** -21 + 2.0 ** -35), err.max()


def test_pack_f16x3_hi_is_round_to_nearest():
    w = torch.tensor([1.0 + 2 ** -11, 1.0 + 3 * 2 ** -11, -0.1, 65000.0]).view(4, 1, 1, 1)
    buf = pack(w)
    hi = buf[:4 * 32].view(np.float16).reshape(4, 32)[:, 0].astype(np.float64)
    assert hi.tolist() == [1.0, 1.0 + 4 * 2 ** -11, float(np.float16(-0.1)), 64992.0]
