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
    w = torch.tensor([1.0 + 2 ** -11, 1.0 + 3 * 2 ** -11, -0.1, 32760.0]).view(4, 1, 1, 1)
    buf = pack(w)
    hi = buf[:4 * 32].view(np.float16).reshape(4, 32)[:, 0].astype(np.float64)
    assert hi.tolist() == [1.0, 1.0 + 4 * 2 ** -11, float(np.float16(-0.1)), 32768.0]


@pytest.mark.parametrize("bad", [32768.0, -65000.0, float("inf"), float("nan")])
def test_pack_f16x3_rejects_out_of_range(bad):
    """A weight outside the split's range (|w| >= 2^15: the fp16 hi / lo pair no
    longer carries it to ~2^-21) is rejected, as the kernels' range guard
    rejects such activations (tests/test_gpu_split_range.py)."""
    from dcvc_amd import hip as h
    wn = np.array([0.5, bad, 1.0, 2.0], np.float32).reshape(4, 1, 1, 1)
    n = h.lib().dcvc_conv_pack_weights(wn.ctypes.data_as(ctypes.c_void_p), 4, 1, 1, 1, h.F16X3, None)
    out = np.zeros(n, dtype=np.uint16)
    assert h.lib().dcvc_conv_pack_weights(wn.ctypes.data_as(ctypes.c_void_p), 4, 1, 1, 1, h.F16X3,
                                          out.ctypes.data_as(ctypes.c_void_p)) == -1


@pytest.mark.parametrize("c,hid", [(48, 192), (128, 512), (32, 128)])
def test_ffn_pack_roundtrip(c, hid):
    """dcvc_ffn_pack_weights: per slice of 32 hidden channels the swizzled LDS
    images of ffn1 ([kc][h][32]) and ffn2 ([n][32], its K order permuted to the
    order ffn1's accumulators leave the hidden values in), hi then lo; decoded
    back they give the weights to ~2^-22."""
    from dcvc_amd import hip as h
    g = torch.Generator().manual_seed(c)
    w1 = (torch.randn(hid, c, generator=g) / c ** 0.5).numpy().astype(np.float32)
    w2 = (torch.randn(c, hid, generator=g) / hid ** 0.5).numpy().astype(np.float32)
    vp = ctypes.c_void_p
    n = h.lib().dcvc_ffn_pack_weights(w1.ctypes.data_as(vp), w2.ctypes.data_as(vp), c, hid, None)
    buf = np.zeros(n, dtype=np.uint16)
    assert h.lib().dcvc_ffn_pack_weights(w1.ctypes.data_as(vp), w2.ctypes.data_as(vp), c, hid,
                                         buf.ctypes.data_as(vp)) == n
    HS = 32
    kc1, c16 = (c + 31) // 32, (c + 15) // 16 * 16
    w1n, w2n = kc1 * HS * 32, c16 * 32
    sl = 2 * w1n + 2 * w2n
    assert n == sl * (hid // HS)

    def at(row, k):
        x = (0x1320 >> (((row >> 2) & 3) << 2)) & 3
        return row * 32 + ((((k >> 3) ^ x) & 3) << 3) + (k & 7)

    def perm(k):   # ffn2's K position 8 q + m holds hidden channel 4 q + m / 16 + 4 q + m - 4
        q, m = k >> 3, k & 7
        return 4 * q + m if m < 4 else 16 + 4 * q + m - 4
    assert sorted(perm(k) for k in range(32)) == list(range(32))
    f = buf.view(np.float16).astype(np.float64)
    g1 = np.zeros((hid, c))
    g2 = np.zeros((c, hid))
    for s in range(hid // HS):
        b = s * sl
        for kc in range(kc1):
            for hh in range(HS):
                for k in range(32):
                    ch = kc * 32 + k
                    q = at(kc * HS + hh, k)
                    v = f[b + q] + f[b + w1n + q] / 2048
                    if ch < c:
                        g1[s * HS + hh, ch] = v
                    else:
                        assert v == 0
        for nn in range(c):
            for k in range(32):
                q = at(nn, k)
                g2[nn, s * HS + perm(k)] = f[b + 2 * w1n + q] + f[b + 2 * w1n + w2n + q] / 2048
    for got, ref in ((g1, w1), (g2, w2)):
        assert np.all(np.abs(got - ref) <= np.abs(ref) * 2.0 ** -21 + 2.0 ** -35)
