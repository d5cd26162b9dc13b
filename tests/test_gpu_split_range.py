"""The fp16 range guard of the split-fp16 kernels (dcvc_split_range_flag).

A split operand carries an fp32 value as hi + 2^-11 lo of two fp16 numbers:
~2^-21 of the value while |v| < 2^15, silently saturated above (the HEM
random-weight latents of SURVEY section 7 grow without bound).  Every split
kernel raises the calling thread's flag when a value it splits reaches 2^15;
the codecs check it once per frame (layers.split_guarded) and raise
SplitRangeError.  Here: inputs just under the limit still match fp64 at the
split bound; inputs around 1e5 raise, through every split kernel family (3x3
static kernel, generic sconv, 1x1 sgemm, fused ConvFFN / DepthConv).
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
    return (got.double() - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)


# (cin, cout, k, stride, kernel family expected)
CONVS = [(48, 48, 3, 1, "xconv3_kernel"), (6, 64, 3, 1, "sconv_kernel"), (56, 64, 3, 2, "sconv_kernel"),
         (32, 64, 7, 1, "xconv3_kernel"), (8, 32, 7, 1, "sconv_kernel"), (96, 48, 1, 1, "sgemm_kernel")]


@pytest.mark.parametrize("case", CONVS)
@pytest.mark.parametrize("peak", [3.0e4, 1.0e5])
def test_split_conv_range(case, peak):
    h = K()
    cin, cout, k, s, fam = case
    g = torch.Generator().manual_seed(cin + cout + k)
    x = torch.randn(1, cin, 24, 40, generator=g)
    x = x / x.abs().max() * peak
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g)
    cw = h.ConvW(w, b, s, h.F16X3)
    dev = torch.device("cuda", 0)
    h.split_guard_arm(dev)
    h.split_guard_check()   # clear
    y = h.conv(cw, h.from_nchw(x, h.F32), out_dtype=h.F32)
    torch.cuda.synchronize()
    assert h.lib().dcvc_last_kernel().decode().startswith(fam)
    if peak < 32768:
        h.split_guard_check()   # must not raise
        ref = F.conv2d(x.double(), w.double(), b.double(), stride=s, padding=(k - 1) // 2)
        assert rel_err(y.nchw().cpu(), ref) < TOL
    else:
        with pytest.raises(h.SplitRangeError):
            h.split_guard_check()
        h.split_guard_check()   # the flag was cleared


def test_split_fused_blocks_range():
    """A ConvFFN (sffn.hip) whose hidden layer, a fused intermediate that never
    reaches HBM, leaves the range raises too; the same block in range does not."""
    h = K()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    C, HID = 64, 256
    w1 = torch.randn(HID, C, 1, 1, generator=g) / C ** 0.5
    w2 = torch.randn(C, HID, 1, 1, generator=g) * 1e-3
    x0 = torch.randn(1, C, 40, 48, generator=g)
    h.split_guard_arm(dev)
    h.split_guard_check()
    # hidden ~ N(0, (xs * gain)^2): 1 in range; 1e5 out of it, with the input
    # (|x| < 5e3) and the weights (|w| < 1e2) themselves in range
    for xs, gain, raises in ((1.0, 1.0, False), (1.0e3, 1.0e2, True)):
        fw = h.FfnW(w1 * gain, torch.zeros(HID), w2, torch.zeros(C), dev)
        assert h.conv_ffn(fw, h.from_nchw(x0 * xs, h.F32)) is not None
        torch.cuda.synchronize()
        if raises:
            with pytest.raises(h.SplitRangeError):
                h.split_guard_check()
        else:
            h.split_guard_check()


def test_codec_frame_in_range_does_not_raise(dc_golden):
    """A whole split-precision frame of the golden sequence: in range, no raise
    (encode_decode checks the flag itself)."""
    import tempfile
    import os
    from dcvc_amd.dc import IntraNoAR
    from dcvc_amd.layers import Precision
    net = IntraNoAR(precision=Precision.split()).load_state_dict(dc_golden.i_state_dict())
    net.update(force=True)
    x, xp = dc_golden.frame_tensor("B", 0)
    with tempfile.TemporaryDirectory() as td:
        r = net.encode_decode(xp.cuda(), False, 40, os.path.join(td, "i.bin"), pic_width=x.shape[3],
                              pic_height=x.shape[2])
    assert r["bit"] > 0
