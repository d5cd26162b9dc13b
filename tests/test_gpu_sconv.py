"""The split-fp16 conv kernels (sconv.hip, compute DCVC_F16X3) against fp64
convolutions of the same fp32 operands on the CPU.

The split keeps ~21 bits of every operand (x = hi + 2^-11 lo, the lo * lo
product dropped), so the kernel must land within a few fp32 roundings of the
exact result: the bound is 4e-6 of the output's magnitude, while dropping
one product of a K = 432 sum moves it by ~1e-2 and bf16 operands by ~4e-3.
Shapes cover every kernel size / stride / tap packing the codec uses: 32-
channel chunks, 16- and 8-channel last chunks (2 and 4 taps per MFMA K step),
channel counts below 8 (scalar staging), channel views, every epilogue op.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 4e-6


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)
    # these tests pin sconv.hip / sgemm.hip themselves: the static-shape 3x3
    # kernel (xconv.hip) and the direct kernel (dconv.hip) that take their
    # shapes first are compared with them bit for bit in test_gpu_xconv.py /
    # test_gpu_dconv.py
    from dcvc_amd import hip
    hip.set_option("xconv", 0)
    hip.set_option("dconv", 0)
    hip.set_option("tconv", 0)
    hip.set_option("nconv", 0)
    yield
    hip.set_option("xconv", 1)
    hip.set_option("dconv", 1)
    hip.set_option("tconv", 1)
    hip.set_option("nconv", 1)


def K():
    from dcvc_amd import hip
    return hip


def rel_err(got, ref):
    scale = ref.abs().max().item() + 1e-12
    return (got.double() - ref).abs().max().item() / scale


CASES = [
    # cin, cout, k, stride, H, W
    (48, 48, 3, 1, 37, 53),
    (64, 64, 3, 1, 70, 90),
    (32, 64, 3, 1, 19, 40),
    (96, 48, 3, 1, 21, 35),
    (80, 48, 3, 1, 17, 33),
    (128, 192, 3, 1, 11, 23),
    (3, 48, 3, 1, 20, 33),
    (6, 64, 3, 1, 16, 20),
    (2, 64, 3, 2, 34, 40),
    (51, 64, 3, 2, 34, 40),
    (56, 64, 3, 2, 36, 46),
    (64, 96, 3, 2, 18, 30),
    (8, 32, 7, 1, 23, 29),
    (16, 2, 7, 1, 16, 16),
    (32, 64, 7, 1, 24, 37),
    (64, 32, 7, 1, 20, 21),
    (32, 16, 7, 1, 18, 33),
    (384, 384, 1, 1, 9, 13),
    (1024, 384, 1, 1, 5, 6),
    (48, 192, 1, 1, 33, 47),
    (192, 48, 1, 1, 33, 47),
    (128, 64, 1, 2, 12, 10),
    (2, 64, 1, 2, 30, 34),
    (16, 16, 1, 1, 64, 80),
]


@pytest.mark.parametrize("case", CASES)
def test_sconv_matches_fp64(case):
    h = K()
    cin, cout, k, s, H, W = case
    g = torch.Generator().manual_seed(cin * 1000 + cout + k)
    x = torch.randn(1, cin, H, W, generator=g)
    x[:, :, ::3] *= 1e-3          # small values: the lo parts go subnormal in fp16
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=s, padding=(k - 1) // 2)
    cw = h.ConvW(w, b, s, h.F16X3)
    y = h.conv(cw, h.from_nchw(x, h.F32), out_dtype=h.F32)
    torch.cuda.synchronize()
    kern = h.lib().dcvc_last_kernel().decode()
    want = "sgemm_kernel" if k == 1 and s == 1 and cin % 8 == 0 else "sconv_kernel"
    assert kern.startswith(want), kern
    err = rel_err(y.nchw().cpu(), ref)
    assert err < TOL, (case, err)


# the 1x1 pixel-GEMM kernel (sgemm.hip) in each forced (BN, pixel groups)
# configuration: latent sizes, ragged pixel counts, output channels that pad
# the n-block, in_op lrelu and the whole epilogue on channel views
SGEMM_CFGS = {1: (128, 2), 2: (64, 2), 3: (32, 2), 4: (128, 1), 5: (64, 1), 6: (32, 1)}


@pytest.mark.parametrize("cfg", sorted(SGEMM_CFGS))
@pytest.mark.parametrize("cin,cout,H,W", [(1024, 384, 68, 120), (384, 1024, 17, 23), (192, 48, 9, 7),
                                          (40, 36, 5, 31), (8, 4, 3, 3)])
def test_sgemm_matches_fp64(cfg, cin, cout, H, W):
    h = K()
    g = torch.Generator().manual_seed(cin + cout + cfg)
    x = torch.randn(1, cin, H, W, generator=g)
    x[:, ::5] *= 1e-3
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), b.double())
    cw = h.ConvW(w, b, 1, h.F16X3)
    h.set_option("sgemm", cfg)
    try:
        y = h.conv(cw, h.from_nchw(x, h.F32), out_dtype=h.F32)
        torch.cuda.synchronize()
        bn, pxw = SGEMM_CFGS[cfg]
        assert h.lib().dcvc_last_kernel().decode() == f"sgemm_kernel<{bn}, {pxw}, 2>"
    finally:
        h.set_option("sgemm", 0)
    err = rel_err(y.nchw().cpu(), ref)
    assert err < TOL, err


@pytest.mark.parametrize("cfg", [0, 1, 5])
@pytest.mark.parametrize("cin,cout,H,W", [(64, 256, 13, 21), (128, 256, 9, 40), (64, 128, 17, 16)])
def test_sgemm_pixel_shuffle(cfg, cin, cout, H, W):
    """sgemm.hip's pixel-shuffle epilogue (subpel_conv1x1, DCVC-DC/src/models/
    layers.py:26-31 as the hyperprior decoders and upsamplers use it): bias and
    activation per conv channel, then residuals and the scale in the output
    map, on channel views; against fp64 and the sconv.hip 1x1 path."""
    h = K()
    g = torch.Generator().manual_seed(cin + cout + H + cfg)
    x = torch.randn(1, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    co = cout // 4
    r = torch.randn(1, co, 2 * H, 2 * W, generator=g)
    sc = torch.rand(co, generator=g) + 0.5
    ref = (r.double() + F.pixel_shuffle(F.leaky_relu(F.conv2d(x.double(), w.double(), b.double()), 0.1), 2)) \
        * sc.double().view(1, -1, 1, 1)
    cw = h.ConvW(w, b, 1, h.F16X3)
    xa = h.from_nchw(x, h.F32)
    ra = h.from_nchw(r, h.F32)
    outs = []
    for opt in (cfg, -1):
        out = h.empty(2 * H, 2 * W, co + 8, h.F32)
        out.buf.fill_(7.0)
        h.set_option("sgemm", opt)
        try:
            h.conv(cw, xa, out.ch(4, co), shuffle=True, act=h.ACT_LRELU, slope=0.1, res=ra, scale=sc.cuda())
            torch.cuda.synchronize()
            kern = h.lib().dcvc_last_kernel().decode()
        finally:
            h.set_option("sgemm", 0)
        assert kern.startswith("sgemm_kernel" if opt >= 0 else "sconv_kernel"), kern
        assert bool((out.buf[:, :, :4] == 7.0).all()) and bool((out.buf[:, :, 4 + co:] == 7.0).all())
        outs.append(out.ch(4, co).nchw().cpu())
    assert rel_err(outs[0], ref) < TOL
    assert rel_err(outs[1], ref) < TOL


@pytest.mark.parametrize("pd", [1, 2, 3, 5])
def test_sgemm_stage_depths(pd):
    """sgemm.hip with 1, 2, 3 and 5 stages in flight: same products and K order,
    so bit-identical to each other, and within the fp64 bound."""
    h = K()
    g = torch.Generator().manual_seed(pd)
    cin, cout, H, W = 384, 192, 17, 30
    x = torch.randn(1, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), b.double())
    cw = h.ConvW(w, b, 1, h.F16X3)
    xa = h.from_nchw(x, h.F32)
    h.set_option("sgemm_pd", pd)
    try:
        y = h.conv(cw, xa, out_dtype=h.F32)
        torch.cuda.synchronize()
        assert h.lib().dcvc_last_kernel().decode().endswith(f", {pd}>")
    finally:
        h.set_option("sgemm_pd", 0)
    y0 = h.conv(cw, xa, out_dtype=h.F32)
    torch.cuda.synchronize()
    assert rel_err(y.nchw().cpu(), ref) < TOL
    assert torch.equal(y.nchw().cpu(), y0.nchw().cpu())


@pytest.mark.parametrize("cfg", [0, 2, 6])
def test_sgemm_epilogue_and_views(cfg):
    h = K()
    cin, cout, H, W = 96, 40, 13, 29
    g = torch.Generator().manual_seed(11)
    big = torch.randn(1, cin + 8, H, W, generator=g)
    x = big[:, 4:4 + cin]
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    r = torch.randn(1, cout, H, W, generator=g)
    r2 = torch.randn(1, cout, H, W, generator=g)
    sc = torch.rand(cout, generator=g) + 0.5
    xd = F.leaky_relu(x.double(), 0.2)
    ref = (r2.double() + (r.double() + F.leaky_relu(F.conv2d(xd, w.double(), b.double()), 0.1))) \
        * sc.double().view(1, -1, 1, 1)
    cw = h.ConvW(w, b, 1, h.F16X3)
    xa = h.from_nchw(big, h.F32).ch(4, cin)
    out = h.empty(H, W, cout + 12, h.F32)
    out.buf.fill_(7.0)
    ra = h.empty(H, W, cout + 4, h.F32)
    h.copy(h.from_nchw(r, h.F32), ra.ch(4, cout))
    r2a = h.from_nchw(r2, h.F32)
    h.set_option("sgemm", cfg)
    try:
        h.conv(cw, xa, out.ch(8, cout), in_op=h.IN_LRELU, in_slope=0.2, act=h.ACT_LRELU, slope=0.1,
               res=ra.ch(4, cout), res2=r2a, scale=sc.cuda())
        torch.cuda.synchronize()
        assert h.lib().dcvc_last_kernel().decode().startswith("sgemm_kernel")
    finally:
        h.set_option("sgemm", 0)
    assert rel_err(out.ch(8, cout).nchw().cpu(), ref) < TOL
    # the channels around the view are untouched
    assert bool((out.buf[:, :, :8] == 7.0).all()) and bool((out.buf[:, :, 8 + cout:] == 7.0).all())


def test_sconv_fused_epilogue_and_views():
    """in_op lrelu, bias, act, residual, res2, scale on channel views; pixel
    shuffle; the ConvFFN2 gate input op."""
    h = K()
    cin, cout, H, W = 64, 48, 29, 37
    g = torch.Generator().manual_seed(7)
    big = torch.randn(1, cin + 16, H, W, generator=g)
    x = big[:, 8:8 + cin]
    w = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    r = torch.randn(1, cout, H, W, generator=g)
    r2 = torch.randn(1, cout, H, W, generator=g)
    sc = torch.rand(cout, generator=g) + 0.5
    xd = F.leaky_relu(x.double(), 0.2)
    ref = (r2.double() + (r.double() + F.leaky_relu(F.conv2d(xd, w.double(), b.double(), padding=1), 0.1))) \
        * sc.double().view(1, -1, 1, 1)
    cw = h.ConvW(w, b, 1, h.F16X3)
    xa = h.from_nchw(big, h.F32).ch(8, cin)
    out = h.empty(H, W, cout + 8, h.F32)
    ra = h.empty(H, W, cout + 4, h.F32)
    h.copy(h.from_nchw(r, h.F32), ra.ch(4, cout))
    r2a = h.from_nchw(r2, h.F32)
    h.conv(cw, xa, out.ch(8, cout), in_op=h.IN_LRELU, in_slope=0.2, act=h.ACT_LRELU, slope=0.1,
           res=ra.ch(4, cout), res2=r2a, scale=sc.cuda())
    torch.cuda.synchronize()
    assert rel_err(out.ch(8, cout).nchw().cpu(), ref) < TOL

    # pixel shuffle (subpel_conv3x3: 96 -> 4 x 32)
    cin, cout = 96, 128
    x = torch.randn(1, cin, 15, 22, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    ref = F.pixel_shuffle(F.conv2d(x.double(), w.double(), b.double(), padding=1), 2)
    y = h.conv(h.ConvW(w, b, 1, h.F16X3), h.from_nchw(x, h.F32), shuffle=True)
    torch.cuda.synchronize()
    assert rel_err(y.nchw().cpu(), ref) < TOL

    # ConvFFN2 gate: conv_out(x1 * lrelu(x2, 0.1)) + residual
    c = 64
    x = torch.randn(1, 2 * c, 20, 36, generator=g)
    w = torch.randn(c, c, 1, 1, generator=g) / c ** 0.5
    b = torch.randn(c, generator=g) * 0.1
    x1, x2 = x.double().chunk(2, 1)
    ref = F.conv2d(x1 * F.leaky_relu(x2, 0.1), w.double(), b.double())
    y = h.conv(h.ConvW(w, b, 1, h.F16X3), h.from_nchw(x, h.F32), in_op=h.IN_GATE, in_slope=0.1)
    torch.cuda.synchronize()
    assert rel_err(y.nchw().cpu(), ref) < TOL


def test_sconv_fp16_subnormal_operands():
    """Inputs around 1e-6 .. 1e-4 (fp16 subnormal hi parts): the kernel still
    follows fp64 to the bound, relative to the output's magnitude."""
    h = K()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 32, 16, 16, generator=g) * 1e-5
    w = torch.randn(32, 32, 3, 3, generator=g) * 0.05
    ref = F.conv2d(x.double(), w.double(), None, padding=1)
    y = h.conv(h.ConvW(w, torch.zeros(32), 1, h.F16X3), h.from_nchw(x, h.F32), out_dtype=h.F32)
    torch.cuda.synchronize()
    assert rel_err(y.nchw().cpu(), ref) < 1e-4


@pytest.mark.parametrize("c,H,W", [(48, 37, 53), (32, 20, 70), (64, 33, 31), (128, 17, 30), (128, 200, 331)])
def test_fused_ffn_matches_fp64(c, H, W):
    """sffn.hip: out = scale * (x + lrelu(ffn2(lrelu(ffn1(x) + b1)) + b2))
    (ConvFFN, DCVC-DC/src/models/layers.py:166-179) in one kernel, on channel
    views, against fp64."""
    h = K()
    g = torch.Generator().manual_seed(c + H)
    hid = 4 * c
    big = torch.randn(1, c + 8, H, W, generator=g)
    x = big[:, 4:4 + c]
    w1 = torch.randn(hid, c, 1, 1, generator=g) / c ** 0.5
    b1 = torch.randn(hid, generator=g) * 0.1
    w2 = torch.randn(c, hid, 1, 1, generator=g) / hid ** 0.5
    b2 = torch.randn(c, generator=g) * 0.1
    sc = torch.rand(c, generator=g) + 0.5
    xd = x.double()
    hh = F.leaky_relu(F.conv2d(xd, w1.double(), b1.double()), 0.1)
    ref = (xd + F.leaky_relu(F.conv2d(hh, w2.double(), b2.double()), 0.1)) * sc.double().view(1, -1, 1, 1)
    fw = h.FfnW(w1, b1, w2, b2)
    xa = h.from_nchw(big, h.F32).ch(4, c)
    out = h.empty(H, W, c + 8, h.F32)
    y = h.conv_ffn(fw, xa, out.ch(4, c), scale=sc.cuda(), slope=0.1)
    torch.cuda.synchronize()
    assert y is not None and h.lib().dcvc_last_kernel().decode().startswith("sffn_kernel")
    got = out.ch(4, c).nchw().cpu()
    assert rel_err(got, ref) < TOL
    if c == 128 and H * W >= 512 * 128:
        # feature maps: 8 waves of one pixel tile (the default) and 4 waves of
        # two (dcvc_set_option("sffn128", 0)): the same products in the same
        # order, the same bits
        assert h.lib().dcvc_last_kernel().decode().startswith("sffn_kernel<128, 8, 1, 4>")
        h.set_option("sffn128", 0)
        try:
            h.conv_ffn(fw, xa, out.ch(4, c), scale=sc.cuda(), slope=0.1)
            torch.cuda.synchronize()
            assert h.lib().dcvc_last_kernel().decode().startswith("sffn_kernel<128, 4, 2, 4>")
        finally:
            h.set_option("sffn128", 1)
        assert torch.equal(out.ch(4, c).nchw().cpu(), got)


@pytest.mark.parametrize("c,H,W", [(384, 68, 120), (192, 68, 120), (384, 17, 30), (192, 5, 7), (384, 3, 11)])
def test_latent_ffn_matches_fp64_and_unfused(c, H, W):
    """slffn.hip: the latent ConvFFN (C = 384 / 192, hidden = max(min(4C,
    1024), 2C), DCVC-DC/src/models/layers.py:166-179) in one kernel on a
    channel view, against fp64, and bit-identical to the two unfused
    split-fp16 GEMM launches (same products, same K order); 68 x 120 is the
    1080p latent, the others ragged 32-pixel tiles."""
    h = K()
    g = torch.Generator().manual_seed(c + H * W)
    hid = max(min(4 * c, 1024), 2 * c)
    big = torch.randn(1, c + 8, H, W, generator=g)
    x = big[:, 4:4 + c]
    w1 = torch.randn(hid, c, 1, 1, generator=g) / c ** 0.5
    b1 = torch.randn(hid, generator=g) * 0.1
    w2 = torch.randn(c, hid, 1, 1, generator=g) / hid ** 0.5
    b2 = torch.randn(c, generator=g) * 0.1
    sc = torch.rand(c, generator=g) + 0.5
    xd = x.double()
    hh = F.leaky_relu(F.conv2d(xd, w1.double(), b1.double()), 0.1)
    ref = (xd + F.leaky_relu(F.conv2d(hh, w2.double(), b2.double()), 0.1)) * sc.double().view(1, -1, 1, 1)
    fw = h.FfnW(w1, b1, w2, b2)
    xa = h.from_nchw(big, h.F32).ch(4, c)
    out = h.empty(H, W, c + 8, h.F32)
    out.buf.fill_(7.0)
    y = h.conv_ffn(fw, xa, out.ch(4, c), scale=sc.cuda(), slope=0.1)
    torch.cuda.synchronize()
    assert y is not None and h.lib().dcvc_last_kernel().decode().startswith("slffn_kernel")
    got = out.ch(4, c).nchw().cpu()
    assert rel_err(got, ref) < TOL
    assert bool((out.buf[:, :, :4] == 7.0).all()) and bool((out.buf[:, :, 4 + c:] == 7.0).all())
    c1, c2 = h.ConvW(w1, b1, 1, h.F16X3), h.ConvW(w2, b2, 1, h.F16X3)
    t = h.conv(c1, xa, act=h.ACT_LRELU, slope=0.1)
    y2 = h.conv(c2, t, act=h.ACT_LRELU, slope=0.1, res=xa, scale=sc.cuda())
    torch.cuda.synchronize()
    assert torch.equal(y2.nchw().cpu(), got)


@pytest.mark.parametrize("c,H,W", [(384, 68, 120), (192, 68, 120), (384, 17, 30), (192, 5, 7), (384, 1, 40),
                                   (128, 272, 480), (128, 37, 53)])
def test_latent_dw_conv2_matches_fp64_and_unfused(c, H, W):
    """sldc_kernel (slffn.hip): the tail of a latent DepthConv, conv2(dw3x3(t)
    + bdw) + b2 + x (DCVC-DC/src/models/layers.py:135-163), against fp64 and
    bit-identical to the unfused depthwise + split-fp16 GEMM launches; image
    edges, ragged 32-pixel tiles spanning rows, channel views."""
    h = K()
    g = torch.Generator().manual_seed(c * 3 + H * W)
    tb = torch.randn(1, c + 8, H, W, generator=g)
    xb = torch.randn(1, c + 16, H, W, generator=g)
    wd = torch.randn(c, 1, 3, 3, generator=g) / 3
    bd = torch.randn(c, generator=g) * 0.1
    w2 = torch.randn(c, c, 1, 1, generator=g) / c ** 0.5
    b2 = torch.randn(c, generator=g) * 0.1
    t, x = tb[:, 8:], xb[:, 4:4 + c]
    ref = F.conv2d(F.conv2d(t.double(), wd.double(), bd.double(), padding=1, groups=c), w2.double(), b2.double()) \
        + x.double()
    w9c = wd.reshape(c, 9).t().contiguous()
    dwc = h.DwcW(w9c, bd, w2, b2)
    ta = h.from_nchw(tb, h.F32).ch(8, c)
    xa = h.from_nchw(xb, h.F32).ch(4, c)
    out = h.empty(H, W, c + 4, h.F32)
    y = h.dw_conv2_split(dwc, ta, xa, out.ch(4, c))
    torch.cuda.synchronize()
    assert y is not None and h.lib().dcvc_last_kernel().decode().startswith("sldc_kernel")
    got = out.ch(4, c).nchw().cpu()
    assert rel_err(got, ref) < TOL
    d = h.dwconv3x3(ta, w9c.cuda(), bd.cuda())
    y2 = h.conv(h.ConvW(w2, b2, 1, h.F16X3), d, res=xa)
    torch.cuda.synchronize()
    assert torch.equal(y2.nchw().cpu(), got)


@pytest.mark.parametrize("cin,cout,adapt,H,W", [(64, 48, True, 37, 53), (48, 32, True, 20, 33), (32, 64, True, 17, 16),
                                                (64, 64, False, 9, 70), (48, 48, False, 8, 16), (32, 32, False, 25, 31)])
def test_fused_depthconv_matches_fp64(cin, cout, adapt, H, W):
    """sdc.hip: DepthConv (DCVC-DC/src/models/layers.py:135-163) = conv2(dw3x3(
    lrelu(conv1(x) + b1, 0.01)) + bdw) + b2 + (adaptor(x) | x) in one kernel,
    on channel views and image edges, against fp64."""
    h = K()
    g = torch.Generator().manual_seed(cin * 7 + cout + H)
    big = torch.randn(1, cin + 8, H, W, generator=g)
    x = big[:, 4:4 + cin]
    w1 = torch.randn(cin, cin, 1, 1, generator=g) / cin ** 0.5
    b1 = torch.randn(cin, generator=g) * 0.1
    wd = torch.randn(cin, 1, 3, 3, generator=g) / 3
    bd = torch.randn(cin, generator=g) * 0.1
    w2 = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b2 = torch.randn(cout, generator=g) * 0.1
    wa = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5 if adapt else None
    ba = torch.randn(cout, generator=g) * 0.1 if adapt else None
    xd = x.double()
    t = F.leaky_relu(F.conv2d(xd, w1.double(), b1.double()), 0.01)
    t = F.conv2d(t, wd.double(), bd.double(), padding=1, groups=cin)
    idn = F.conv2d(xd, wa.double(), ba.double()) if adapt else xd
    ref = F.conv2d(t, w2.double(), b2.double()) + idn
    w9c = wd.reshape(cin, 9).t().contiguous()
    dw = h.DcW(w1, b1, w9c, bd, w2, b2, wa, ba)
    xa = h.from_nchw(big, h.F32).ch(4, cin)
    out = h.empty(H, W, cout + 8, h.F32)
    y = h.depth_conv_split(dw, xa, out.ch(8, cout), slope=0.01)
    torch.cuda.synchronize()
    assert y is not None and h.lib().dcvc_last_kernel().decode().startswith("sdc_kernel")
    got = out.ch(8, cout).nchw().cpu()
    assert rel_err(got, ref) < TOL
    # the unfused launches (split 1x1 with the LeakyReLU epilogue, the fp32
    # depthwise kernel, split 1x1 + identity / adaptor): the same bits
    t1 = h.conv(h.ConvW(w1, b1, 1, h.F16X3), xa, act=h.ACT_LRELU, slope=0.01)
    d = h.dwconv3x3(t1, w9c.cuda(), bd.cuda())
    idn = h.conv(h.ConvW(wa, ba, 1, h.F16X3), xa) if adapt else xa
    y2 = h.conv(h.ConvW(w2, b2, 1, h.F16X3), d, res=idn)
    torch.cuda.synchronize()
    assert torch.equal(y2.nchw().cpu(), got)
