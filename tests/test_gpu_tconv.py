"""The thin fp32-VALU convolutions (tconv.hip) against fp64 and sconv.hip.

tconv takes the split-precision layers whose input has 2 channels: the
motion encoder's first ResidualBlockWithStride on the flow (3x3 and 1x1
stride 2, 2 -> 64, DCVC-DC/src/models/video_model.py:121-140).
The weights are the split-packed ones rebuilt as hi + 2^-11 lo (22 bits)
and every product is an fp32 FMA, so the kernels are held to
the same fp64 bound as the split kernels (4e-6 of the output's magnitude) and
to sconv.hip (dcvc_set_option("tconv", 0)) within twice that, not bit for
bit.  Shapes: the codec's at sizes with many workgroups, ragged edges, input
and output channel views, the in_op / act / residual / scale epilogue.
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


# cin, cout, k, stride, H, W, in_op leaky ReLU, act leaky ReLU, residual, scale, input channel view
CASES = [
    (2, 64, 3, 2, 272, 480, False, True, False, False, False),   # MvEnc conv1 on the flow
    (2, 64, 1, 2, 272, 480, False, False, False, False, False),  # and its stride-2 skip
    (2, 64, 3, 2, 37, 51, True, True, True, True, True),
    (2, 128, 3, 1, 17, 30, False, False, True, False, True),
    (2, 64, 1, 1, 9, 13, False, True, False, True, False),
]


@pytest.mark.parametrize("case", CASES)
def test_tconv_matches_fp64_and_sconv(case):
    h = K()
    cin, cout, k, s, H, W, lrelu, act, res, scaled, view = case
    g = torch.Generator().manual_seed(cin * 13 + cout + H + k)
    big = torch.randn(1, cin + 8, H, W, generator=g)
    big[:, :, ::3] *= 1e-3
    x = big[:, 4:4 + cin]
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    sc = torch.rand(cout, generator=g) + 0.5
    xd = F.leaky_relu(x.double(), 0.01) if lrelu else x.double()
    ref = F.conv2d(xd, w.double(), b.double(), stride=s, padding=k // 2)
    if act:
        ref = F.leaky_relu(ref, 0.1)
    Ho, Wo = ref.shape[2], ref.shape[3]
    r = torch.randn(1, cout, Ho, Wo, generator=g)
    if res:
        ref = r.double() + ref
    if scaled:
        ref = ref * sc.double().view(1, -1, 1, 1)
    cw = h.ConvW(w, b, s, h.F16X3)
    xa = h.from_nchw(big, h.F32).ch(4, cin) if view else h.from_nchw(x.contiguous(), h.F32)
    kw = dict(act=h.ACT_LRELU if act else h.ACT_NONE, slope=0.1, scale=sc.cuda() if scaled else None,
              in_op=h.IN_LRELU if lrelu else h.IN_NONE, in_slope=0.01, res=h.from_nchw(r, h.F32) if res else None)
    outs = []
    for on in (1, 0):
        h.set_option("tconv", on)
        try:
            # a 4-aligned channel view of a wider map
            extra = 8
            out = h.empty(Ho, Wo, cout + extra, h.F32)
            out.buf.fill_(7.0)
            yv = out.ch(4, cout)
            h.conv(cw, xa, yv, **kw)
            torch.cuda.synchronize()
            kern = h.lib().dcvc_last_kernel().decode()
        finally:
            h.set_option("tconv", 1)
        assert kern.startswith("tconv_" if on else ("sconv_kernel", "xconv3_kernel", "dconv_kernel")), kern
        assert bool((out.buf[:, :, :4] == 7.0).all()) and bool((out.buf[:, :, 4 + cout:] == 7.0).all())
        outs.append(yv.nchw().cpu())
    assert rel_err(outs[0], ref) < TOL
    assert rel_err(outs[0], outs[1].double()) < 2 * TOL


def test_tconv_leaves_other_shapes():
    """Everything but 2-channel inputs stays on the split kernels, and so do
    pixel shuffles."""
    h = K()
    for cin, cout, k, s, shuf in [(8, 32, 7, 1, False), (6, 64, 3, 1, False), (16, 8, 3, 1, False),
                                  (16, 4, 3, 2, False), (2, 64, 3, 1, True), (16, 2, 7, 1, False),
                                  (48, 3, 3, 1, False)]:
        cw = h.ConvW(torch.randn(cout, cin, k, k) * 0.1, torch.zeros(cout), s, h.F16X3)
        h.conv(cw, h.from_nchw(torch.randn(1, cin, 20, 24), h.F32), out_dtype=h.F32, shuffle=shuf)
        torch.cuda.synchronize()
        assert not h.lib().dcvc_last_kernel().decode().startswith("tconv_"), (cin, cout, k, s, shuf)
