"""The few-output-channel split convolution (nconv.hip) against fp64 and sconv.hip.

nconv_kernel takes the stride-1 7x7 layers with COUT x KS <= 16: SpyNet's
last 7x7 of every basic module (16 -> 2, DCVC-DC/src/models/video_net.py:
79-100); the 3x3 heads (48 -> 3) stay on sconv.hip.  Pixels sit on the MFMA's M rows
and (output channel, tap column) pairs on its N columns; an output is the sum
of the tap columns' partials.  The products are sconv.hip's split, the K order
and the final dx sum are not, so the kernel is held to the split kernels'
fp64 bound (4e-6 of the output's magnitude) and to sconv.hip
(dcvc_set_option("nconv", 0)) within twice that.  Shapes: the codec's at
sizes with many waves per launch, ragged rows (column tiles past the right
edge), channel-view inputs, narrow standalone outputs and an output view,
the in_op / act / residual / scale epilogue.
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


# cin, cout, k, H, W, in_op leaky ReLU, act leaky ReLU, residual, scale, input channel view, output view
CASES = [
    (16, 2, 7, 272, 480, False, False, False, False, True, False),   # SpyNet's last layer
    (16, 2, 7, 37, 53, False, False, False, False, False, False),
    (16, 2, 7, 5, 3, True, False, False, False, False, True),
    (32, 2, 7, 40, 81, False, True, True, False, True, False),
    (16, 1, 7, 23, 17, False, False, False, True, False, False),
    (32, 2, 7, 18, 161, True, False, True, True, True, True),
]


@pytest.mark.parametrize("case", CASES)
def test_nconv_matches_fp64_and_sconv(case):
    h = K()
    cin, cout, k, H, W, lrelu, act, res, scaled, view, oview = case
    g = torch.Generator().manual_seed(cin * 31 + cout + H + k)
    big = torch.randn(1, cin + 8, H, W, generator=g)
    big[:, :, ::3] *= 1e-3          # small values: the lo parts go subnormal in fp16
    x = big[:, 4:4 + cin]
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    sc = torch.rand(cout, generator=g) + 0.5
    xd = F.leaky_relu(x.double(), 0.01) if lrelu else x.double()
    ref = F.conv2d(xd, w.double(), b.double(), padding=k // 2)
    if act:
        ref = F.leaky_relu(ref, 0.1)
    r = torch.randn(1, cout, H, W, generator=g)
    if res:
        ref = r.double() + ref
    if scaled:
        ref = ref * sc.double().view(1, -1, 1, 1)
    cw = h.ConvW(w, b, 1, h.F16X3)
    xa = h.from_nchw(big, h.F32).ch(4, cin) if view else h.from_nchw(x.contiguous(), h.F32)
    kw = dict(act=h.ACT_LRELU if act else h.ACT_NONE, slope=0.1, scale=sc.cuda() if scaled else None,
              in_op=h.IN_LRELU if lrelu else h.IN_NONE, in_slope=0.01, res=h.from_nchw(r, h.F32) if res else None)
    outs = []
    for on in (1, 0):
        h.set_option("nconv", on)
        try:
            extra = 5 if oview else 0
            out = h.empty(H, W, cout + extra, h.F32)
            out.buf.fill_(7.0)
            yv = out.ch(2, cout) if oview else out
            h.conv(cw, xa, yv, **kw)
            torch.cuda.synchronize()
            kern = h.lib().dcvc_last_kernel().decode()
        finally:
            h.set_option("nconv", 1)
        assert kern.startswith("nconv_kernel" if on else "sconv_kernel"), kern
        if oview:
            assert bool((out.buf[:, :, :2] == 7.0).all()) and bool((out.buf[:, :, 2 + cout:] == 7.0).all())
        outs.append(yv.nchw().cpu())
    assert rel_err(outs[0], ref) < TOL
    assert rel_err(outs[0], outs[1].double()) < 2 * TOL


def test_nconv_range_guard():
    """The fp16 range guard of the split kernels covers nconv's split too."""
    h = K()
    cw = h.ConvW(torch.randn(2, 16, 7, 7) * 0.01, torch.zeros(2), 1, h.F16X3)
    for big, want in ((3e4, False), (1e5, True)):
        x = torch.randn(1, 16, 20, 30)
        x[0, 3, 5, 7] = big
        h.split_guard_arm(torch.device("cuda", 0))
        try:
            h.conv(cw, h.from_nchw(x, h.F32), out_dtype=h.F32)
            torch.cuda.synchronize()
            assert h.lib().dcvc_last_kernel().decode().startswith("nconv_kernel")
            assert h.split_guard_tripped() == want
        finally:
            h.split_guard_disarm()


def test_nconv_leaves_3x3_heads():
    h = K()
    cw = h.ConvW(torch.randn(3, 48, 3, 3) * 0.1, torch.zeros(3), 1, h.F16X3)
    h.conv(cw, h.from_nchw(torch.randn(1, 48, 20, 24), h.F32), out_dtype=h.F32)
    torch.cuda.synchronize()
    assert h.lib().dcvc_last_kernel().decode().startswith("sconv_kernel")
