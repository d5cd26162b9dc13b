"""The direct split-fp16 convolution (dconv.hip) against sconv.hip and fp64.

dconv_kernel takes the stride-2 3x3 / 1x1 layers of the strided encoders
(DCVC-DC/src/models/video_model.py:66-86, 173-195; ResidualBlockWithStride)
and the feature-rate 1x1 layers (DepthConv, subpel_conv1x1 incl. the
narrow 64 -> 8 one, DCVC-DC/src/models/layers.py:23-34, 135-163).  It
computes the same products
in the same K order (dcvc_conv_pack_weights' chunks, taps packed in a narrow
last chunk) with the same epilogue as sconv_kernel / sgemm_kernel, so its
output must be bit-identical to theirs (dcvc_set_option("dconv", 0) routes
the call to sconv.hip / sgemm.hip) and within the split precision's fp64
bound.  Shapes: the codec's
layers at sizes where every wave walks many tiles and at ragged sizes (odd
rows / columns, segments past the right edge), on channel views, with the
in_op / act / scale epilogue.
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


def K():
    from dcvc_amd import hip
    return hip


def rel_err(got, ref):
    scale = ref.abs().max().item() + 1e-12
    return (got.double() - ref).abs().max().item() / scale


# cin, cout, k, stride, H, W, in_op leaky ReLU, act leaky ReLU[, residuals, pixel shuffle]
CASES = [
    (56, 64, 3, 2, 272, 480, False, True),     # conv_offset.0 / contextual encoder conv1 shape
    (56, 64, 3, 2, 37, 53, False, False),      # ragged
    (48, 64, 3, 2, 96, 130, False, False),     # feature extractor conv2 (16-channel last chunk)
    (64, 96, 3, 2, 68, 120, False, False),     # 96 = 2 x 48-channel blocks
    (64, 64, 3, 2, 34, 62, True, True),
    (64, 64, 1, 2, 68, 122, False, False),     # ResidualBlockWithStride skip
    # stride-1 1x1 layers on feature-rate maps (>= 64 Ki pixels: DepthConv
    # conv1 / conv2 / adaptor, subpel_conv1x1 upsamplers): KS = 1
    (128, 128, 1, 1, 272, 241, False, False, 1, False),
    (48, 48, 1, 1, 256, 330, False, False, 2, False),
    (192, 48, 1, 1, 256, 257, True, False, 1, False),
    (128, 64, 1, 1, 272, 250, False, True, 0, False),
    (64, 256, 1, 1, 256, 260, False, False, 0, True),   # subpel_conv1x1: pixel shuffle on store
    (64, 128, 1, 1, 272, 243, False, True, 0, True),
    # a narrow upsampler (64 -> 8 1x1 + pixel shuffle to 2 channels: element stores)
    (64, 8, 1, 1, 256, 260, False, False, 0, True),
    (64, 8, 1, 1, 256, 263, True, True, 0, True),
]
# shapes dconv leaves to sconv / sgemm / xconv (more than two output-channel
# blocks of a 3x3 stride-2 layer; latent-rate 1x1; SpyNet's 8 -> 32 7x7)
FALLBACK = [(128, 96, 3, 2, 34, 60), (8, 32, 7, 1, 40, 50), (192, 96, 3, 2, 17, 31), (384, 384, 1, 1, 68, 120), (1024, 256, 1, 1, 17, 30)]


@pytest.mark.parametrize("case", FALLBACK)
def test_dconv_leaves_shapes_it_loses_on(case):
    h = K()
    cin, cout, k, s, H, W = case
    cw = h.ConvW(torch.randn(cout, cin, k, k) * 0.01, torch.zeros(cout), s, h.F16X3)
    h.conv(cw, h.from_nchw(torch.randn(1, cin, H, W), h.F32), out_dtype=h.F32)
    torch.cuda.synchronize()
    kern = h.lib().dcvc_last_kernel().decode()
    assert kern.startswith(("sconv_kernel", "sgemm_kernel", "xconv3_kernel")), kern


@pytest.mark.parametrize("case", CASES)
def test_dconv_matches_sconv_and_fp64(case):
    h = K()
    cin, cout, k, s, H, W, lrelu, act = case[:8]
    nres, shuf = (case[8], case[9]) if len(case) > 8 else (0, False)
    g = torch.Generator().manual_seed(cin * 7 + cout + H + k)
    big = torch.randn(1, cin + 8, H, W, generator=g)
    big[:, :, ::3] *= 1e-3          # small values: the lo parts go subnormal in fp16
    x = big[:, 4:4 + cin]
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    co = cout // 4 if shuf else cout
    sc = torch.rand(co, generator=g) + 0.5
    xd = F.leaky_relu(x.double(), 0.01) if lrelu else x.double()
    ref = F.conv2d(xd, w.double(), b.double(), stride=s, padding=k // 2)
    if act:
        ref = F.leaky_relu(ref, 0.1)
    if shuf:
        ref = F.pixel_shuffle(ref, 2)
    Ho, Wo = ref.shape[2], ref.shape[3]
    rs = [torch.randn(1, co, Ho, Wo, generator=g) for _ in range(nres)]
    for r in rs:
        ref = r.double() + ref
    ref = ref * sc.double().view(1, -1, 1, 1)
    cw = h.ConvW(w, b, s, h.F16X3)
    xa = h.from_nchw(big, h.F32).ch(4, cin)
    ra = [h.from_nchw(r, h.F32) for r in rs]
    kw = dict(act=h.ACT_LRELU if act else h.ACT_NONE, slope=0.1, scale=sc.cuda(), shuffle=shuf,
              in_op=h.IN_LRELU if lrelu else h.IN_NONE, in_slope=0.01,
              res=ra[0] if nres > 0 else None, res2=ra[1] if nres > 1 else None)
    outs = []
    # a 4-aligned channel view (16-byte stores) and, for the narrow output,
    # the standalone tensor the codec writes (element stores)
    off, extra = (4, 12) if co % 4 == 0 else (0, 0)
    for on in (1, 0):
        h.set_option("dconv", on)
        try:
            out = h.empty(Ho, Wo, co + extra, h.F32)
            out.buf.fill_(7.0)
            h.conv(cw, xa, out.ch(off, co), **kw)
            torch.cuda.synchronize()
            kern = h.lib().dcvc_last_kernel().decode()
        finally:
            h.set_option("dconv", 1)
        want = "dconv_kernel" if on else ("sgemm_kernel", "sconv_kernel")
        assert kern.startswith(want), kern
        if extra:
            assert bool((out.buf[:, :, :off] == 7.0).all()) and bool((out.buf[:, :, off + co:] == 7.0).all())
        outs.append(out.ch(off, co).nchw().cpu())
    assert rel_err(outs[0], ref) < TOL
    assert torch.equal(outs[0], outs[1])


def test_dconv_repeatable_and_interleaved():
    """The same launch twice, interleaved with another shape's launches on the
    same stream: identical bits."""
    h = K()
    g = torch.Generator().manual_seed(9)
    x = h.from_nchw(torch.randn(1, 56, 544, 960, generator=g), h.F32)
    cw = h.ConvW(torch.randn(64, 56, 3, 3, generator=g) / 20, torch.randn(64, generator=g) * 0.1, 2, h.F16X3)
    cw2 = h.ConvW(torch.randn(96, 56, 3, 3, generator=g) / 20, torch.zeros(96), 2, h.F16X3)
    y0 = h.conv(cw, x, out_dtype=h.F32)
    torch.cuda.synchronize()
    assert h.lib().dcvc_last_kernel().decode().startswith("dconv_kernel")
    ref = y0.buf.clone()
    for _ in range(3):
        h.conv(cw2, x, out_dtype=h.F32)
        h.conv(cw, x, y0)
    torch.cuda.synchronize()
    assert torch.equal(y0.buf, ref)


@pytest.mark.parametrize("case", [(128, 128, 272, 241, False), (64, 256, 256, 260, True), (128, 256, 40, 70, True)])
def test_dconv_bn128_matches_sgemm(case):
    """1x1 layers with 128-channel n-blocks of 16-pixel groups (the default)
    and with 64-channel blocks of 32 pixels (dcvc_set_option("dconv_bn128",
    0)): the same bits as sgemm.hip, with and without the pixel shuffle's
    coalesced store."""
    h = K()
    cin, cout, H, W, shuf = case
    g = torch.Generator().manual_seed(cin + cout + H)
    x = h.from_nchw(torch.randn(1, cin, H, W, generator=g), h.F32)
    cw = h.ConvW(torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5, torch.randn(cout, generator=g) * 0.1, 1,
                 h.F16X3)
    sc = (torch.rand(cout // 4 if shuf else cout, generator=g) + 0.5).cuda()
    outs = []
    for opts in ({"dconv_bn128": 1}, {"dconv_bn128": 0}, {"dconv": 0}):
        for k, v in opts.items():
            h.set_option(k, v)
        try:
            y = h.conv(cw, x, out_dtype=h.F32, scale=sc, shuffle=shuf, act=h.ACT_LRELU, slope=0.1)
            torch.cuda.synchronize()
            kern = h.lib().dcvc_last_kernel().decode()
        finally:
            h.set_option("dconv_bn128", 1)
            h.set_option("dconv", 1)
        outs.append((kern, y.buf.cpu()))
    big = H * W >= 65536
    assert outs[0][0].startswith("dconv_kernel<1, 128, 1," if big else ("sgemm_kernel", "sconv_kernel")), outs[0][0]
    assert outs[1][0].startswith("dconv_kernel<1, 64, 2," if big else ("sgemm_kernel", "sconv_kernel")), outs[1][0]
    assert outs[2][0].startswith(("sgemm_kernel", "sconv_kernel")), outs[2][0]
    assert torch.equal(outs[0][1], outs[2][1]) and torch.equal(outs[1][1], outs[2][1])


@pytest.mark.parametrize("cin,cout,H,W", [(64, 64, 256, 260), (96, 48, 272, 250), (128, 32, 256, 257), (64, 16, 260, 256)])
def test_dconv_gated_1x1_matches_sconv(cin, cout, H, W):
    """ConvFFN2's gated second 1x1 (DCVC-DC/src/models/layers.py:182-197:
    conv_out(x1 * lrelu(x2)) + x, in_op DCVC_IN_GATE on a 2 cin-channel
    input): dconv against sconv.hip's gated path, bit for bit, and fp64."""
    h = K()
    g = torch.Generator().manual_seed(cin + cout + H)
    x = torch.randn(1, 2 * cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    r = torch.randn(1, cout, H, W, generator=g)
    xd = x.double()
    gated = xd[:, :cin] * F.leaky_relu(xd[:, cin:], 0.1)
    ref = r.double() + F.conv2d(gated, w.double(), b.double())
    cw = h.ConvW(w, b, 1, h.F16X3)
    xa, ra = h.from_nchw(x, h.F32), h.from_nchw(r, h.F32)
    outs = []
    for on in (1, 0):
        h.set_option("dconv", on)
        h.set_option("sgemm_gate", on)
        try:
            y = h.conv(cw, xa, out_dtype=h.F32, in_op=h.IN_GATE, in_slope=0.1, res=ra)
            torch.cuda.synchronize()
            kern = h.lib().dcvc_last_kernel().decode()
        finally:
            h.set_option("dconv", 1)
            h.set_option("sgemm_gate", 1)
        assert (kern.startswith("dconv_kernel<1") and ", true>" in kern) if on else kern.startswith("sconv_kernel"), kern
        outs.append(y.nchw().cpu())
    assert rel_err(outs[0], ref) < TOL
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("cin,cout,H,W", [(512, 256, 68, 120), (1536, 768, 68, 120), (1024, 512, 68, 120),
                                          (512, 256, 136, 240), (256, 128, 34, 60), (96, 40, 17, 23)])
def test_sgemm_gated_1x1_matches_sconv(cin, cout, H, W):
    """The intra codec's latent-rate ConvFFN2 gated 1x1s (DCVC-DC
    image_model.py:62-91 DepthConvBlock2 at 1/16 and 1/8 scale, layers.py:182-
    197), below dconv.hip's pixel count: the pixel-GEMM kernel with the gate
    applied to its DMA-staged operand, against sconv.hip's gated path bit for
    bit (same K order and gate order) and fp64; a ragged last pixel block."""
    h = K()
    g = torch.Generator().manual_seed(cin + cout + H)
    x = torch.randn(1, 2 * cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    r = torch.randn(1, cout, H, W, generator=g)
    xd = x.double()
    gated = xd[:, :cin] * F.leaky_relu(xd[:, cin:], 0.1)
    ref = r.double() + F.conv2d(gated, w.double(), b.double())
    cw = h.ConvW(w, b, 1, h.F16X3)
    xa, ra = h.from_nchw(x, h.F32), h.from_nchw(r, h.F32)
    outs = []
    for on in (1, 0):
        h.set_option("sgemm_gate", on)
        try:
            y = h.conv(cw, xa, out_dtype=h.F32, in_op=h.IN_GATE, in_slope=0.1, res=ra)
            torch.cuda.synchronize()
            kern = h.lib().dcvc_last_kernel().decode()
        finally:
            h.set_option("sgemm_gate", 1)
        assert (kern.startswith("sgemm_kernel") and ", true>" in kern) if on else kern.startswith("sconv_kernel"), kern
        outs.append(y.nchw().cpu())
    assert rel_err(outs[0], ref) < TOL
    assert torch.equal(outs[0], outs[1])
