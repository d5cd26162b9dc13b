"""The wave-specialised split-fp16 3x3 kernel (wconv.hip) against xconv.hip and fp64.

wconv3_kernel computes xconv3_kernel's products in xconv's K order with its
epilogue, so with dcvc_set_option("wconv", 1) its output must be
bit-identical to xconv's (option 0) and within the split precision's fp64
bound (4e-6 of the output magnitude, as test_gpu_xconv.py).  The shapes are
the 3x3 stride-1 layers wconv takes (48 / 64 / 128 / 192 input channels, at
most one residual, no pixel shuffle) of the DC and HEM feature-rate stacks
(DCVC-DC/src/models/video_net.py:58-76, 129-170, video_model.py:89-118,
173-232), at sizes where every workgroup walks many tiles (producer /
consumer pipeline across tiles) and at ragged sizes, into channel views, and
launched again and again on fixed inputs (a race between the producer waves'
weight ring / image buffers and the consumer waves' reads shows up as an
occasional mismatch there, as in xconv's round-5 ring race).
"""
import re

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 4e-6


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def K():
    from dcvc_amd import hip
    return hip


def rel_err(got, ref):
    scale = ref.abs().max().item() + 1e-12
    return (got.double() - ref).abs().max().item() / scale


def run(h, cw, x, out, wconv, **kw):
    h.set_option("wconv", wconv)
    try:
        h.conv(cw, x, out, **kw)
        torch.cuda.synchronize()
        return h.lib().dcvc_last_kernel().decode()
    finally:
        h.set_option("wconv", 0)


# cin, cout, H, W, residual, in_op leaky ReLU, act
CASES = [
    (48, 48, 272, 480, True, True, True),      # ResBlock conv2 shape: BN 48, one operand set
    (48, 48, 37, 53, False, True, True),       # ragged tiles
    (48, 48, 136, 240, False, False, False),
    (64, 64, 136, 240, True, True, True),      # BN 32, two n-blocks
    (64, 64, 21, 35, True, False, True),
    (128, 64, 68, 120, False, False, True),
    (128, 32, 19, 23, False, False, False),
    (64, 96, 17, 31, False, False, True),      # 96 = 2 x 48
    (64, 128, 34, 60, False, False, True),     # BN 32, four n-blocks
    (192, 192, 34, 60, True, False, True),     # 6 chunks, BN 48 with a residual
    (192, 48, 40, 66, False, True, False),
    (48, 96, 50, 20, True, False, True),
]


@pytest.mark.parametrize("case", CASES)
def test_wconv_matches_xconv_and_fp64(case):
    h = K()
    cin, cout, H, W, res, lrelu, act = case
    g = torch.Generator().manual_seed(cin * 11 + cout + H)
    big = torch.randn(1, cin + 8, H, W, generator=g)
    big[:, :, ::3] *= 1e-3          # small values: the lo parts go subnormal in fp16
    x = big[:, 4:4 + cin]
    w = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    r = torch.randn(1, cout, H, W, generator=g) if res else None
    sc = torch.rand(cout, generator=g) + 0.5
    xd = F.leaky_relu(x.double(), 0.01) if lrelu else x.double()
    ref = F.conv2d(xd, w.double(), b.double(), padding=1)
    if act:
        ref = F.leaky_relu(ref, 0.1)
    if res:
        ref = r.double() + ref
    ref = ref * sc.double().view(1, -1, 1, 1)
    cw = h.ConvW(w, b, 1, h.F16X3)
    xa = h.from_nchw(big, h.F32).ch(4, cin)
    kw = dict(act=h.ACT_LRELU if act else h.ACT_NONE, slope=0.1, scale=sc.cuda(),
              in_op=h.IN_LRELU if lrelu else h.IN_NONE, in_slope=0.01,
              res=h.from_nchw(r, h.F32) if res else None)
    outs = []
    for wv in (1, 0):
        out = h.empty(H, W, cout + 12, h.F32)
        out.buf.fill_(7.0)
        kern = run(h, cw, xa, out.ch(4, cout), wv, **kw)
        assert kern.startswith("wconv3_kernel" if wv else ("xconv3_kernel", "sconv_kernel")), kern
        # nothing written outside the view
        assert bool((out.buf[:, :, :4] == 7.0).all()) and bool((out.buf[:, :, 4 + cout:] == 7.0).all())
        outs.append(out.ch(4, cout).nchw().cpu())
    assert rel_err(outs[0], ref) < TOL
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("shape", ["48x48@1088x1920", "48x48@1088x1920r", "64x64@544x960r", "128x64@544x960",
                                   "192x192@68x120r"])
def test_wconv_repeated_launches_identical(shape):
    """The codec's shapes launched 50 times on fixed inputs, interleaved with
    another shape's launches on the same stream: every launch bit-identical to
    xconv.hip's result."""
    h = K()
    m = re.fullmatch(r"(\d+)x(\d+)@(\d+)x(\d+)(r?)", shape)
    cin, cout, H, W = (int(m.group(i)) for i in range(1, 5))
    g = torch.Generator().manual_seed(cin + cout + H)
    x = h.from_nchw(torch.randn(1, cin, H, W, generator=g), h.F32)
    cw = h.ConvW(torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5,
                 torch.randn(cout, generator=g) * 0.1, 1, h.F16X3)
    cw2 = h.ConvW(torch.randn(32, cin, 3, 3, generator=g) / 20, torch.zeros(32), 1, h.F16X3)
    kw = dict(act=h.ACT_LRELU, slope=0.1,
              res=h.from_nchw(torch.randn(1, cout, H, W, generator=g), h.F32) if m.group(5) else None)
    ref = h.empty(H, W, cout, h.F32)
    assert run(h, cw, x, ref, 0, **kw).startswith("xconv3_kernel")
    y = h.empty(H, W, cout, h.F32)
    y2 = h.empty(H, W, 32, h.F32)
    bad = 0
    for i in range(50):
        y.buf.fill_(float("nan"))
        if i % 5 == 4:
            assert run(h, cw2, x, y2, 1).startswith("wconv3_kernel")
        assert run(h, cw, x, y, 1, **kw).startswith("wconv3_kernel")
        bad += int(not torch.equal(y.buf, ref.buf))
    assert bad == 0, f"{bad} of 50 launches differ"
