"""The fp16 range guard of the split-fp16 kernels (dcvc_split_range_flag).

A split operand carries an fp32 value as hi + 2^-11 lo of two fp16 numbers:
~2^-21 of the value while |v| < 2^15, silently saturated above (the HEM
random-weight latents of SURVEY section 7 grow without bound).  Every split
kernel raises the calling thread's flag when a value it splits reaches 2^15;
the codecs check it once per frame (layers.split_guarded) and raise
SplitRangeError.  Here: inputs just under the limit still match fp64 at the
split bound; inputs around 1e5 raise, through every split kernel family (3x3
static kernel, generic sconv, direct dconv (stride 2, 1x1, narrow 7x7), fused
ConvFFN / DepthConv).
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
CONVS = [(48, 48, 3, 1, "xconv3_kernel"), (6, 64, 3, 1, "sconv_kernel"), (56, 64, 3, 2, "dconv_kernel"),
         (32, 64, 7, 1, "xconv3_kernel"), (8, 32, 7, 1, "xconv3_kernel"), (96, 48, 1, 1, "sgemm_kernel"),
         (64, 48, 3, 2, "dconv_kernel"), (8, 48, 7, 1, "sconv_kernel")]


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


# (parameter pair, stage that trips): conv A's weights and bias times 2^16,
# conv B's weights times 2^-16, a positively homogeneous map between them
# (ResBlock conv1 -> lrelu -> conv2, DCVC-DC/src/models/video_net.py:58-76;
# ResidualBlockWithStride's conv1 -> lrelu -> conv2, layers.py:42-73;
# ResidualBlockUpsample's subpel conv -> pixel shuffle -> lrelu -> conv,
# layers.py:76-101; ConvFFN's conv.0 -> lrelu -> conv.2, layers.py:166-180).
# In fp32 arithmetic scaling by a power of two is exact and a leaky ReLU (and
# a pixel shuffle) commutes with it, so the network's output is bit for bit
# that of the unscaled weights while A's output (B's input) leaves the split's
# range (|v| >= 2^15) -- provided A's outputs reach 2^-1 on the golden
# sequence: the pairs come from the oracle's activation maxima on frame A
# (DC P-frame: mv_encoder.enc_2.conv1 1.30, the recon UNet's FFN 0.67; the
# SpyNet and contextual-decoder pairs tried first stay below 0.56 and did not
# trip).  "compress" pairs trip in the encoder, "decompress" pairs only in
# the decoder.
HOT_PAIRS = {
    ("hem", "P", "compress"): ("y_prior_fusion.0", "y_prior_fusion.2"),
    ("hem", "P", "decompress"): ("contextual_decoder.res1.conv1", "contextual_decoder.res1.conv2"),
    ("hem", "I", "compress"): ("enc.0.conv1", "enc.0.conv2"),
    ("hem", "I", "decompress"): ("dec.1.subpel_conv.0", "dec.1.conv"),
    ("dc", "P", "compress"): ("mv_encoder.enc_2.conv1", "mv_encoder.enc_2.conv2"),
    ("dc", "P", "decompress"): ("recon_generation_net.unet_2.context_refine.1.block.1.conv.0",
                                "recon_generation_net.unet_2.context_refine.1.block.1.conv.2"),
    ("dc", "I", "compress"): ("enc.enc_1.0.conv1", "enc.enc_1.0.conv2"),
    ("dc", "I", "decompress"): ("dec.dec_1.1.subpel_conv.0", "dec.dec_1.1.conv"),
}


def _hot(sd, pair):
    a, b = pair
    out = dict(sd)
    out[a + ".weight"] = sd[a + ".weight"] * 65536.0
    out[a + ".bias"] = sd[a + ".bias"] * 65536.0
    out[b + ".weight"] = sd[b + ".weight"] / 65536.0
    return out


@pytest.mark.parametrize("case", sorted(HOT_PAIRS))
def test_frame_out_of_range_falls_back(case, dc_golden):
    """A whole frame (golden sequence A; DCVC-HEM or DCVC-DC, I- or P-frame)
    whose activations pass 2^15 in the encoder or in the decoder
    (DCVC-HEM/src/models/common_model.py:32-37: the reference codes any fp32
    range): the split codec does not abort or leave a stream of a failed
    attempt behind; the frame is coded again by its fp32 twin, the output file
    holds that stream, its decode is lossless, the twin's calls, bits and
    reconstruction are those of an fp32 codec on the unscaled weights, and the
    frame meets the strict teacher-forced bar against the oracle run on the
    unscaled weights (the same function, comment above)."""
    import os
    import tempfile
    import numpy as np
    from tests.test_gpu_parity_strict import HemPair, Pair, psnr
    from tests.parity import compare_frame, check_frame
    from dcvc_amd.layers import Precision
    model, kind, stage = case
    if model == "hem":
        from tests.hem_fixtures import HEMGolden
        from dcvc_amd.hem import DMC, IntraNoAR
        g = HEMGolden()
        meta = g.meta["A"]
        isd, psd = g.i_state_dict(), g.p_state_dict()
        pair = HemPair(isd, psd, g.q("A"), "split")
        q = None
    else:
        from dcvc_amd.dc import DMC, IntraNoAR
        g = dc_golden
        meta = g.meta["A"]
        isd, psd = g.i_state_dict(), g.p_state_dict()
        pair = Pair(isd, psd, "split")
        q = meta["q_index"]
    h, w = meta["h"], meta["w"]
    cls, sd = (IntraNoAR, isd) if kind == "I" else (DMC, psd)
    hot = cls(precision=Precision.split()).load_state_dict(_hot(sd, HOT_PAIRS[case]))
    hot.update(force=True)
    ref = cls(precision=Precision.parity()).load_state_dict(sd)   # the twin's arithmetic, unscaled weights
    ref.update(force=True)
    frames = [g.frame_tensor("A", t) for t in range(2)]
    t = 0 if kind == "I" else 1
    dpb_o = None
    if t:
        _, _, _, dpb_o = pair.oracle(0, frames[0][1], None, q, 0)
    x, xp = frames[t]
    calls, tap, bits_o, dpb_next = pair.oracle(t, xp, dpb_o, q, t)
    with tempfile.TemporaryDirectory() as td:
        res = {}
        for name, net in (("hot", hot), ("ref", ref)):
            if t:
                pair.pp = net
            else:
                pair.pi = net
            path = os.path.join(td, f"{name}.bin")
            enc, bits, rec = pair.product(t, xp, dpb_o, q, t, path, h, w)   # asserts decoder == encoder
            res[name] = (enc, bits, rec, os.path.getsize(path) * 8, getattr(net, "fallbacks", 0))
    enc, bits, rec, fbits, nfb = res["hot"]
    assert nfb == 1, "the split codec did not fall back"
    assert fbits == bits, "the output file is not the stream the frame reports"
    enc_r, bits_r, rec_r, _, _ = res["ref"]
    # the fallback IS the fp32 path: same calls, bits and reconstruction
    assert bits == bits_r
    for (s1, i1), (s2, i2) in zip(enc, enc_r):
        np.testing.assert_array_equal(s1.reshape(-1), s2.reshape(-1))
        np.testing.assert_array_equal(i1.reshape(-1), i2.reshape(-1))
    assert torch.equal(rec.cpu(), rec_r.cpu())
    st = compare_frame(enc, calls, tap)
    check_frame(st, bits, bits_o, psnr(rec[:, :, :h, :w], x), psnr(dpb_next["ref_frame"][:, :, :h, :w], x),
                f"{model}_A {kind} fallback ({stage})")


def test_guard_cleared_between_calls(dc_golden):
    """an unguarded split call that leaves the range (a direct
    kernel call here) must not be charged to the next guarded frame: arming
    clears the flag, and a guarded call disarms it on the way out."""
    import tempfile
    import os
    from dcvc_amd.dc import IntraNoAR
    from dcvc_amd.layers import Precision
    h = K()
    dev = torch.device("cuda", 0)
    h.split_guard_arm(dev)
    h.split_guard_disarm()
    # out of range with the guard off: nothing may be recorded
    x = torch.full((1, 48, 16, 16), 1.0e5)
    cw = h.ConvW(torch.randn(48, 48, 3, 3) * 0.01, torch.zeros(48), 1, h.F16X3)
    h.conv(cw, h.from_nchw(x, h.F32), out_dtype=h.F32)
    torch.cuda.synchronize()
    assert not h.split_guard_tripped()
    # out of range with a stale armed flag, then a guarded in-range frame
    h.split_guard_arm(dev)
    h.conv(cw, h.from_nchw(x, h.F32), out_dtype=h.F32)
    torch.cuda.synchronize()
    assert h.split_guard_tripped()
    net = IntraNoAR(precision=Precision.split()).load_state_dict(dc_golden.i_state_dict())
    net.update(force=True)
    xf, xp = dc_golden.frame_tensor("B", 0)
    with tempfile.TemporaryDirectory() as td:
        r = net.encode_decode(xp.cuda(), False, 40, os.path.join(td, "i.bin"), pic_width=xf.shape[3],
                              pic_height=xf.shape[2])
    assert "precision_fallback" not in r and getattr(net, "fallbacks", 0) == 0
    # the guarded call disarmed the flag on its way out
    h.conv(cw, h.from_nchw(x, h.F32), out_dtype=h.F32)
    torch.cuda.synchronize()
    assert not h.split_guard_tripped()
