"""Repeated launches of the round-5 split kernels on fixed inputs at codec
sizes: every launch must give the first launch's bits.  A race in an LDS ring,
a DMA / barrier schedule or a wave-private strip shows up as an occasional
mismatch that single-launch parity tests can miss (tests/test_gpu_xconv.py
has the same check for xconv against sconv).  50 launches each: a race seen at
about one launch in five then shows with certainty."""
import pytest
import torch

pytestmark = pytest.mark.gpu

REPS = 50


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def K():
    from dcvc_amd import hip
    return hip


def repeat(fn, out):
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    first = out.buf.clone()
    bad = 0
    for _ in range(REPS):
        out.buf.fill_(float("nan"))
        fn()
        torch.cuda.synchronize()
        bad += int(not torch.equal(out.buf, first))
    return bad


# (128 at 68 x 120: the 4-wave streamed-weight build for maps under 65536
# pixels, whose vmcnt(NDW + PFN) waits assume the next tile's prefetch stays
# behind the weight DMA)
@pytest.mark.parametrize("c,H,W", [(128, 272, 480), (128, 68, 120), (64, 544, 960), (48, 1088, 1920)])
def test_sffn_repeatable(c, H, W):
    h = K()
    g = torch.Generator().manual_seed(c)
    hid = 4 * c
    fw = h.FfnW(torch.randn(hid, c, 1, 1, generator=g) / c ** 0.5, torch.randn(hid, generator=g) * 0.1,
                torch.randn(c, hid, 1, 1, generator=g) / hid ** 0.5, torch.randn(c, generator=g) * 0.1)
    x = h.from_nchw(torch.randn(1, c, H, W, generator=g), h.F32)
    y = h.empty(H, W, c, h.F32)
    assert repeat(lambda: h.conv_ffn(fw, x, y, slope=0.1), y) == 0


@pytest.mark.parametrize("cin,cout,adapt,H,W", [(64, 48, True, 1088, 1920), (48, 32, True, 1088, 1920),
                                                (64, 64, False, 544, 960)])
def test_sdc_repeatable(cin, cout, adapt, H, W):
    h = K()
    g = torch.Generator().manual_seed(cin + cout)
    r = lambda *s: torch.randn(*s, generator=g) * 0.2  # noqa: E731
    dw = h.DcW(r(cin, cin, 1, 1), r(cin), r(9, cin).cuda(), r(cin), r(cout, cin, 1, 1), r(cout),
               r(cout, cin, 1, 1) if adapt else None, r(cout) if adapt else None)
    x = h.from_nchw(torch.randn(1, cin, H, W, generator=g), h.F32)
    y = h.empty(H, W, cout, h.F32)
    assert repeat(lambda: h.depth_conv_split(dw, x, y), y) == 0


# cin, cout, k, stride, H, W, pixel shuffle, gated input
CONVS = [(56, 64, 3, 2, 1088, 1920, False, False),    # dconv stride 2
         (128, 128, 1, 1, 272, 480, False, False),    # dconv 1x1, 128-channel blocks
         (64, 128, 1, 1, 544, 960, True, False),      # dconv 1x1 + 64-byte shuffle stores
         (64, 64, 1, 1, 544, 960, False, True),       # dconv gated 1x1
         (768, 768, 1, 1, 68, 120, False, True),      # sgemm gated 1x1 (latent rate, LDS-DMA ring)
         (384, 384, 1, 1, 68, 120, False, False),     # sgemm 1x1 (latent rate)
         (16, 2, 7, 1, 1088, 1920, False, False),     # nconv
         (2, 64, 3, 2, 1088, 1920, False, False)]     # tconv


@pytest.mark.parametrize("case", CONVS)
def test_conv_repeatable(case):
    h = K()
    cin, cout, k, s, H, W, shuf, gate = case
    g = torch.Generator().manual_seed(cin * 3 + cout + k)
    x = h.from_nchw(torch.randn(1, 2 * cin if gate else cin, H, W, generator=g), h.F32)
    cw = h.ConvW(torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5,
                 torch.randn(cout, generator=g) * 0.1, s, h.F16X3)
    Ho, Wo = cw.out_hw(H, W)
    f = 2 if shuf else 1
    y = h.empty(Ho * f, Wo * f, cout // 4 if shuf else cout, h.F32)
    kw = dict(shuffle=shuf, in_op=h.IN_GATE if gate else h.IN_NONE, in_slope=0.1)
    assert repeat(lambda: h.conv(cw, x, y, **kw), y) == 0


@pytest.mark.parametrize("c", [384, 192])
def test_latent_blocks_repeatable(c):
    """The latent DepthConvBlock stages at 68 x 120 (slffn / sldc, 64-pixel
    workgroups at C = 384)."""
    h = K()
    g = torch.Generator().manual_seed(c)
    hid = {384: 1024, 192: 768}[c]
    fw = h.FfnW(torch.randn(hid, c, 1, 1, generator=g) / c ** 0.5, torch.randn(hid, generator=g) * 0.1,
                torch.randn(c, hid, 1, 1, generator=g) / hid ** 0.5, torch.randn(c, generator=g) * 0.1)
    x = h.from_nchw(torch.randn(1, c, 68, 120, generator=g), h.F32)
    y = h.empty(68, 120, c, h.F32)
    assert repeat(lambda: h.conv_ffn(fw, x, y, slope=0.1), y) == 0
    r = lambda *s: torch.randn(*s, generator=g) * 0.2  # noqa: E731
    dwc = h.DwcW(r(9, c).contiguous().cuda(), r(c).cuda(), r(c, c, 1, 1), r(c))
    t = h.from_nchw(torch.randn(1, c, 68, 120, generator=g), h.F32)
    y2 = h.empty(68, 120, c, h.F32)
    assert repeat(lambda: h.dw_conv2_split(dwc, t, x, y2), y2) == 0
