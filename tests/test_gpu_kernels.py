"""Kernel-level parity of libdcvc_hip against plain PyTorch fp32 on the CPU.

f32-compute convs are an exact fp32 fma chain in a different summation order
than the CPU, so they are held to a relative tolerance of 2e-5 of the
output's magnitude.  bf16-compute convs (bf16 operands, fp32 accumulation)
are compared with fp64 convolutions of the SAME bf16-rounded operands, so
what remains is the fp32 accumulation order: 1e-4 of the output's magnitude
for fp32 outputs, and for bf16 outputs one bf16 rounding of each element
(bf16_err) -- a kernel that dropped one tap-channel product of a K = 432 sum
(~1 % of the magnitude) fails both.  Gather/resample kernels in f32 follow
the CPU kernels' operation order and must match to 1e-6.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)


def K():
    from dcvc_amd import hip
    return hip


def to_act(x, dtype):
    return K().from_nchw(x, dtype)


def back(a):
    return a.nchw().cpu()


def rel_err(got, ref):
    scale = ref.abs().max().item() + 1e-6
    return (got.double() - ref.double()).abs().max().item() / scale


def bf16r(t):
    """t rounded to bf16 (round to nearest even, as the kernels stage operands)."""
    return t.bfloat16().double()


def bf16_err(got, ref, rel=2.0 ** -8):
    """Error of a bf16 output beyond one bf16 rounding of the exact value:
    max(|got - ref| - rel |ref|, 0) relative to the output's magnitude.
    Between two bf16 outputs (two kernels, each rounding once) the bound is
    one whole bf16 ulp: rel = 2^-7."""
    ref = ref.double()
    excess = ((got.double() - ref).abs() - ref.abs() * rel).clamp(min=0.0)
    return excess.max().item() / (ref.abs().max().item() + 1e-6)


TOL_BF16 = 1e-4   # fp32 accumulation order, fp32 outputs (and bf16_err's floor)


CONV_CASES = [
    # cin, cout, k, stride, H, W
    (48, 48, 3, 1, 37, 53),
    (3, 48, 3, 1, 20, 33),
    (51, 64, 3, 2, 34, 40),
    (8, 32, 7, 1, 23, 29),
    (16, 2, 7, 1, 16, 16),
    (64, 96, 3, 2, 18, 30),
    (384, 384, 1, 1, 9, 13),
    (128, 64, 1, 2, 12, 10),
    (64, 128, 2, 2, 8, 8),
    (96, 256, 3, 1, 7, 11),
    (1024, 384, 1, 1, 5, 6),
    (64, 64, 3, 1, 70, 90),
    (32, 128, 1, 1, 40, 64),
    (128, 512, 1, 1, 33, 47),
    (256, 768, 1, 1, 17, 30),
]


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_conv_vector_paths_with_channel_views(mode):
    """16-byte staging and 4-channel stores on views with aligned offsets."""
    h = K()
    comp = h.F32 if mode == "f32" else h.BF16
    dt = h.F32 if mode == "f32" else h.BF16
    cin, cout, H, W = 64, 48, 29, 37
    big = torch.randn(1, cin + 16, H, W)
    x = big[:, 8:8 + cin]
    w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout) * 0.1
    r = torch.randn(1, cout, H, W)
    if mode == "f32":
        ref = F.leaky_relu(F.conv2d(x, w, b, padding=1), 0.1) + r
    else:   # bf16 input map and weights, bf16 residual copy, one bf16 rounding of the output
        ref = F.leaky_relu(F.conv2d(bf16r(x), bf16r(w), b.double(), padding=1), 0.1) + bf16r(r)
    cw = h.ConvW(w, b, 1, comp)
    xa = to_act(big, dt).ch(8, cin)
    out = h.empty(H, W, cout + 8, dt)
    ra = h.empty(H, W, cout + 4, dt)
    h.copy(to_act(r, h.F32), ra.ch(4, cout))
    h.conv(cw, xa, out.ch(8, cout), act=h.ACT_LRELU, slope=0.1, res=ra.ch(4, cout))
    torch.cuda.synchronize()
    if mode == "f32":
        assert rel_err(back(out.ch(8, cout)), ref) < 2e-5
    else:
        assert bf16_err(back(out.ch(8, cout)), ref) < TOL_BF16


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_conv_matches_torch(case, mode):
    h = K()
    cin, cout, k, s, H, W = case
    x = torch.randn(1, cin, H, W)
    w = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pad = (k - 1) // 2
    if mode == "f32":
        ref = F.conv2d(x, w, b, stride=s, padding=pad)
    else:
        ref = F.conv2d(bf16r(x), bf16r(w), b.double(), stride=s, padding=pad)
    comp = h.F32 if mode == "f32" else h.BF16
    dt = h.F32 if mode == "f32" else h.BF16
    cw = h.ConvW(w, b, s, comp)
    xa = to_act(x, dt if mode == "bf16" else h.F32)
    y = h.conv(cw, xa, out_dtype=h.F32)
    torch.cuda.synchronize()
    err = rel_err(back(y), ref)
    assert err < (2e-5 if mode == "f32" else TOL_BF16), err


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_conv_fused_epilogue(mode):
    """in_op lrelu, act, residual, res2, scale, pixel shuffle, channel views."""
    h = K()
    comp = h.F32 if mode == "f32" else h.BF16
    tol = 2e-5 if mode == "f32" else TOL_BF16
    cin, cout, H, W = 40, 64, 19, 21
    big = torch.randn(1, cin + 8, H, W)
    x = big[:, 5:5 + cin]
    w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout) * 0.1
    r1 = torch.randn(1, cout // 4, 2 * H, 2 * W)
    r2 = torch.randn(1, cout // 4, 2 * H, 2 * W)
    sc = torch.rand(cout // 4) + 0.5
    t = F.leaky_relu(x.double(), 0.1)
    wr = w.double()
    if mode == "bf16":   # the input op runs in fp32, then the operands are staged as bf16
        t, wr = bf16r(t), bf16r(w)
    t = F.pixel_shuffle(F.leaky_relu(F.conv2d(t, wr, b.double(), padding=1), 0.01), 2)
    ref = (r2.double() + (r1.double() + t)) * sc.double().view(1, -1, 1, 1)
    cw = h.ConvW(w, b, 1, comp)
    xa = to_act(big, h.F32).ch(5, cin)
    out = h.empty(2 * H, 2 * W, cout // 4 + 3, h.F32)
    y = out.ch(3, cout // 4)
    h.conv(cw, xa, y, in_op=h.IN_LRELU, in_slope=0.1, act=h.ACT_LRELU, slope=0.01, shuffle=True,
           scale=sc.cuda(), res=to_act(r1, h.F32), res2=to_act(r2, h.F32))
    torch.cuda.synchronize()
    assert rel_err(back(y), ref) < tol


def test_conv_gate_input():
    """ConvFFN2 gate: x1 * lrelu(x2, 0.1) fed to a 1x1 conv."""
    h = K()
    c = 24
    x = torch.randn(1, 2 * c, 9, 14)
    w = torch.randn(c, c, 1, 1) / c ** 0.5
    b = torch.randn(c)
    x1, x2 = x.chunk(2, 1)
    ref = F.conv2d(x1 * F.leaky_relu(x2, 0.1), w, b)
    cw = h.ConvW(w, b, 1, h.F32)
    y = h.conv(cw, to_act(x, h.F32), in_op=h.IN_GATE, in_slope=0.1)
    torch.cuda.synchronize()
    assert rel_err(back(y), ref) < 2e-5


@pytest.mark.parametrize("C,H,W", [(48, 17, 23), (64, 9, 200), (128, 5, 61)])
def test_dwconv3x3(C, H, W):
    # (64, 9, 200): several workgroups per image row (the kernel's 2D grid)
    h = K()
    x = torch.randn(1, C, H, W)
    w = torch.randn(C, 1, 3, 3)
    b = torch.randn(C)
    ref = F.conv2d(x, w, b, padding=1, groups=C)
    w9c = w.reshape(C, 9).t().contiguous().cuda()
    y = h.dwconv3x3(to_act(x, h.F32), w9c, b.cuda())
    torch.cuda.synchronize()
    assert rel_err(back(y), ref) < 1e-5


def _grid(H, W):
    return (torch.linspace(-1.0, 1.0, W, dtype=torch.float32).cuda(),
            torch.linspace(-1.0, 1.0, H, dtype=torch.float32).cuda())


def test_flow_warp_matches_reference_formula():
    from oracle.dc_oracle import flow_warp
    h = K()
    x = torch.randn(1, 48, 30, 44)
    flow = torch.randn(1, 2, 30, 44) * 6
    ref = flow_warp(x, flow)
    y = h.flow_warp(to_act(x, h.F32), to_act(flow, h.F32), _grid(30, 44))
    torch.cuda.synchronize()
    assert (back(y) - ref).abs().max().item() < 1e-5


def test_flow_warp_bf16_vector_path():
    """bf16 maps with 8-channel-aligned views take the 16-byte-per-corner
    kernel: per-channel arithmetic in fp32 from the bf16 inputs, one bf16
    rounding, i.e. the reference formula on the bf16-rounded input."""
    from oracle.dc_oracle import flow_warp
    h = K()
    H, W = 33, 47
    x = torch.randn(1, 64, H, W)
    flow = torch.randn(1, 2, H, W) * 6
    xa = to_act(x, h.BF16)
    y = h.empty(H, W, 56, h.BF16)
    h.flow_warp(xa.ch(8, 48), to_act(flow, h.F32), _grid(H, W), y=y.ch(8, 48))
    torch.cuda.synchronize()
    ref = flow_warp(x[:, 8:56].bfloat16().float(), flow).bfloat16().float()
    got = back(y)[:, 8:56]
    assert (got - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    assert (got == ref).float().mean().item() > 0.99


def test_flow_warp_f32_vector_path_bit_identical():
    """fp32 maps with 4-channel-aligned views take the 16-byte-per-corner
    kernel (warp4_kernel); a view at an odd channel offset takes the scalar
    kernel: the same per-channel arithmetic, so identical bits, and the
    reference formula within fp32 rounding."""
    from oracle.dc_oracle import flow_warp
    h = K()
    H, W = 37, 61
    x = torch.randn(1, 56, H, W)
    flow = torch.randn(1, 2, H, W) * 6
    xa = to_act(x, h.F32)
    fa = to_act(flow, h.F32)
    y4 = h.empty(H, W, 56, h.F32)
    y1 = h.empty(H, W, 56, h.F32)
    y4.buf.fill_(3.0)
    h.flow_warp(xa.ch(4, 48), fa, _grid(H, W), y=y4.ch(4, 48))
    h.flow_warp(xa.ch(4, 48), fa, _grid(H, W), y=y1.ch(5, 48))   # odd output offset: scalar kernel
    torch.cuda.synchronize()
    got4 = back(y4)[:, 4:52]
    assert torch.equal(got4, back(y1)[:, 5:53])
    assert bool((back(y4)[:, :4] == 3.0).all()) and bool((back(y4)[:, 52:] == 3.0).all())
    ref = flow_warp(x[:, 4:52], flow)
    assert (got4 - ref).abs().max().item() < 1e-5


def test_dwconv3x3_f32_row_blocked_bit_identical():
    """fp32 4-channel-aligned views take the row-blocked kernel (dw4r_kernel,
    4 output rows per thread); a view at an even, not 4-aligned channel offset
    takes the scalar kernel: same taps in the same order, identical bits."""
    h = K()
    C, H, W = 128, 19, 37
    g = torch.Generator().manual_seed(11)
    big = torch.randn(1, C + 8, H, W, generator=g)
    w = torch.randn(C, 1, 3, 3, generator=g)
    b = torch.randn(C, generator=g)
    w9c = w.reshape(C, 9).t().contiguous().cuda()
    xa = h.from_nchw(big, h.F32)
    y4 = h.empty(H, W, C + 8, h.F32)
    y2 = h.empty(H, W, C + 8, h.F32)
    h.dwconv3x3(xa.ch(4, C), w9c, b.cuda(), y=y4.ch(4, C))
    h.dwconv3x3(xa.ch(2, C), w9c, b.cuda(), y=y2.ch(2, C))
    torch.cuda.synchronize()
    a4 = back(y4)[:, 4:4 + C]
    ref = F.conv2d(big[:, 4:4 + C], w, b, padding=1, groups=C)
    assert rel_err(a4, ref) < 1e-5
    ref2 = F.conv2d(big[:, 2:2 + C], w, b, padding=1, groups=C)
    a2 = back(y2)[:, 2:2 + C]
    assert rel_err(a2, ref2) < 1e-5
    # same input channels through both kernels: shift the scalar path's view
    y3 = h.empty(H, W, C + 8, h.F32)
    big2 = torch.cat([big[:, 2:], big[:, :2]], dim=1)   # channel 4 + k of big at 2 + k
    h.dwconv3x3(h.from_nchw(big2, h.F32).ch(2, C), w9c, b.cuda(), y=y3.ch(2, C))
    torch.cuda.synchronize()
    assert torch.equal(a4, back(y3)[:, 2:2 + C])


def test_resize_and_pool():
    from oracle.dc_oracle import up2, down2
    h = K()
    x = torch.randn(1, 5, 14, 22)
    xa = to_act(x, h.F32)
    up = h.resize2x(xa, True, 2.0)
    dn = h.resize2x(xa, False, 0.5)
    ap = h.pool2x2(xa, False)
    mp = h.pool2x2(xa, True)
    torch.cuda.synchronize()
    assert (back(up) - up2(x) * 2.0).abs().max().item() < 1e-6
    assert (back(dn) - down2(x) / 2).abs().max().item() < 1e-6
    assert (back(ap) - F.avg_pool2d(x, 2, 2)).abs().max().item() < 1e-6
    assert torch.equal(back(mp), F.max_pool2d(x, 2, 2))


@pytest.mark.parametrize("zero_pad", [False, True])
def test_frame_to_nhwc_padding(zero_pad):
    """uint8 CHW frame -> float NHWC /255, padded to the harness's multiple:
    replicate for DC (test_video.py:130), zeros for HEM (test_video.py:113-119)."""
    h = K()
    u8 = torch.randint(0, 256, (3, 37, 50), dtype=torch.uint8)
    ref = u8.float().unsqueeze(0) / 255.0
    ref = F.pad(ref, (0, 14, 0, 27), mode="constant", value=0) if zero_pad else F.pad(ref, (0, 14, 0, 27),
                                                                                    mode="replicate")
    y = h.empty(64, 64, 3, h.F32, torch.device("cuda"))
    h.frame_to_nhwc(u8.cuda(), 37, 50, y, zero_pad=zero_pad)
    torch.cuda.synchronize()
    assert torch.equal(back(y), ref)


@pytest.mark.parametrize("H,W", [(24, 32), (6, 2), (10, 18)])
def test_offset_diversity_matches_oracle(H, W):
    # (6, 2): a one-column offset map; pixel pairs {2q-1, 2q} share its corners
    from oracle import dc_oracle as O
    h = K()
    feat = torch.randn(1, 48, H, W)
    flow = torch.randn(1, 2, H, W) * 3
    offs = torch.randn(1, 96, H // 2, W // 2) * 0.05
    fw = torch.randn(48, 6, 1, 1) * 0.3
    fb = torch.randn(48) * 0.1
    # oracle path from the up-sampled offset map onwards (video_model.py:46-61)
    out = O.up2(offs)
    o1, o2, mask = torch.chunk(out, 3, dim=1)
    mask = torch.sigmoid(mask)
    offset = 40 * torch.tanh(torch.cat((o1, o2), dim=1)) + flow.repeat(1, 32, 1, 1)
    xx = feat.view(16, 3, H, W).repeat(2, 1, 1, 1)
    xx = O.flow_warp(xx, offset.view(32, 2, H, W)) * mask.view(32, 1, H, W)
    ref = F.conv2d(xx.view(1, 96, H, W), fw, fb, groups=16)
    y = h.offset_diversity(to_act(feat, h.F32), to_act(offs, h.F32), to_act(flow, h.F32),
                           fw.reshape(48, 6).contiguous().cuda(), fb.cuda(), _grid(H, W))
    torch.cuda.synchronize()
    assert (back(y) - ref).abs().max().item() < 1e-4


def test_quadtree_encode_decode_steps_match_oracle():
    from oracle import dc_oracle as O
    h = K()
    C, H, W = 16, 6, 10
    y = torch.randn(1, C, H, W) * 4
    params = torch.cat([torch.rand(1, C, H, W) + 0.3, torch.rand(1, C, H, W) * 3,
                        torch.randn(1, C, H, W)], dim=1)
    sms = [torch.cat([torch.rand(1, C, H, W) * 2, torch.randn(1, C, H, W)], 1) for _ in range(3)]
    it = iter(sms)
    # oracle with the adaptor + spatial prior replaced by the fixed step tensors
    orig_conv = O.conv
    O.conv = lambda P, name, x, stride=1, groups=1: x
    try:
        sym_w, sc_w, _, y_hat, _ = O.four_part_prior(None, y, params, ["a", "b", "c"], lambda x: next(it))
    finally:
        O.conv = orig_conv
    buf = h.zeros(H, W, 4 * C, h.F32)
    h.copy(to_act(params, h.F32), buf.ch(C, 3 * C))
    yh = h.empty(H, W, C, h.F32)
    n = C // 4 * H * W
    log_min = math.log(0.01)
    log_step = (math.log(64.0) - log_min) / 255
    for k in range(4):
        sm = None if k == 0 else to_act(sms[k - 1], h.F32)
        sym = torch.empty(n, dtype=torch.int16, device="cuda")
        idx = torch.empty(n, dtype=torch.int16, device="cuda")
        h.qt_encode_step(to_act(y, h.F32), buf.ch(C, 3 * C), sm, k, buf.ch(0, C), yh, sym, idx, log_min, log_step)
        torch.cuda.synchronize()
        assert torch.equal(sym.cpu(), sym_w[k].clamp(-30000, 30000).to(torch.int16).reshape(-1))
        ref_idx = O.build_indexes(sc_w[k], log_min, log_step).to(torch.int16).reshape(-1)
        assert (idx.cpu() != ref_idx).sum().item() <= 1
    assert torch.equal(back(yh), y_hat)


@pytest.mark.parametrize("case", [(48, 192, 37, 61), (384, 384, 9, 13), (96, 48, 20, 33), (40, 64, 17, 19),
                                  (1024, 384, 5, 6), (64, 256, 30, 40)])
@pytest.mark.parametrize("xdt", ["f32", "bf16"])
def test_gemm1x1_equals_generic_conv(case, xdt):
    """The double-buffered 1x1 GEMM kernel and the generic conv kernel
    accumulate the same 32-channel MFMA blocks in the same order: outputs are
    bit-identical, including lrelu input op, residual, scale and shuffle."""
    h = K()
    cin, cout, H, W = case
    dt = h.F32 if xdt == "f32" else h.BF16
    x = torch.randn(1, cin, H, W)
    w = torch.randn(cout, cin, 1, 1) / cin ** 0.5
    b = torch.randn(cout) * 0.1
    cw = h.ConvW(w, b, 1, h.BF16)
    xa = to_act(x, dt)
    outs = []
    rt = torch.randn(1, cout, H, W)
    for use in (1, 0):
        h.set_option("gemm1x1", use)
        r = h.empty(H, W, cout, h.BF16)
        h.copy(to_act(rt, h.F32), r)
        y = h.conv(cw, xa, out_dtype=h.BF16, in_op=h.IN_LRELU, in_slope=0.1, act=h.ACT_LRELU, slope=0.01, res=r)
        y2 = h.conv(cw, xa, shuffle=cout % 4 == 0, out_dtype=h.F32) if cout % 4 == 0 else y
        torch.cuda.synchronize()
        outs.append((back(y), back(y2)))
    h.set_option("gemm1x1", 1)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    ref = F.leaky_relu(F.conv2d(F.leaky_relu(x, 0.1), w, b), 0.01) + rt
    assert rel_err(back(y), ref) < 2e-2


@pytest.mark.parametrize("case", [(384, 384, 68, 120), (1024, 384, 17, 30), (384, 1024, 9, 13), (192, 192, 68, 120),
                                  (768, 192, 20, 33), (40, 64, 17, 19), (128, 512, 33, 47), (96, 288, 34, 60),
                                  (64, 2, 8, 9), (104, 16, 5, 7)])
@pytest.mark.parametrize("cfg,upfront,direct", [(0, 1, 1), (0, 1, 0), (0, 0, 0), (8, 1, 1), (12, 1, 1), (13, 1, 1),
                                                (13, 0, 1), (14, 1, 1), (15, 1, 1)])
def test_gemm1x1_f32_equals_generic_conv(case, cfg, upfront, direct):
    """The fp32 1x1 GEMM (gemm1x1f.hip; cfg 0 = automatic tile choice, 12-15
    force the v_mfma_f32_32x32x2_f32 variants; upfront 1 / 0 = a step's LDS
    operands read up front / per MFMA group; direct 1 / 0 = epilogue from the
    accumulators / through the LDS tile) and conv.hip's f32 path run
    the same exact-f32 MFMA chain (k ascending): bit-identical outputs with
    the lrelu input op, activation, residual and shuffle; and within f32
    tolerance of torch."""
    h = K()
    cin, cout, H, W = case
    h.set_option("gemm1x1_f32_cfg", cfg)
    h.set_option("gemm1x1_f32_upfront", upfront)
    h.set_option("gemm1x1_f32_direct", direct)
    x = torch.randn(1, cin, H, W)
    w = torch.randn(cout, cin, 1, 1) / cin ** 0.5
    b = torch.randn(cout) * 0.1
    cw = h.ConvW(w, b, 1, h.F32)
    xa = to_act(x, h.F32)
    rt = torch.randn(1, cout, H, W)
    rt2 = torch.randn(1, cout, H, W)
    sc = (torch.rand(cout) + 0.5).cuda()
    outs = []
    for use in (1, 0):
        h.set_option("gemm1x1_f32", use)
        r = to_act(rt, h.F32)
        r2 = to_act(rt2, h.F32)
        y = h.conv(cw, xa, out_dtype=h.F32, in_op=h.IN_LRELU, in_slope=0.1, act=h.ACT_LRELU, slope=0.01, res=r)
        y1 = h.conv(cw, xa, out_dtype=h.F32)
        y2 = h.conv(cw, xa, shuffle=True, out_dtype=h.F32) if cout % 4 == 0 else y1
        y3 = h.conv(cw, xa, out_dtype=h.F32, act=h.ACT_LRELU, slope=0.1, res=r, res2=r2, scale=sc)
        torch.cuda.synchronize()
        outs.append((back(y), back(y1), back(y2), back(y3)))
    h.set_option("gemm1x1_f32", 1)
    h.set_option("gemm1x1_f32_cfg", 0)
    h.set_option("gemm1x1_f32_upfront", 1)
    h.set_option("gemm1x1_f32_direct", 1)
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    ref = F.leaky_relu(F.conv2d(F.leaky_relu(x, 0.1), w, b), 0.01) + rt
    assert rel_err(outs[0][0], ref) < 2e-5
    assert rel_err(outs[0][1], F.conv2d(x, w, b)) < 2e-5


@pytest.mark.parametrize("case", [(384, 288, 68, 120), (480, 384, 34, 60), (192, 192, 17, 30), (40, 64, 17, 19),
                                  (128, 128, 9, 13), (64, 16, 5, 70)])
def test_gemm3x3_f32_equals_generic_conv(case):
    """fp32 3x3 stride-1 convs as nine shifted GEMMs (gemm1x1f.hip, K3) run
    conv.hip's f32 MFMA chain in its order (32-channel chunk-major, taps
    inside): bit-identical outputs with the lrelu input op, activation and
    residual; within f32 tolerance of torch."""
    h = K()
    cin, cout, H, W = case
    x = torch.randn(1, cin, H, W)
    w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout) * 0.1
    cw = h.ConvW(w, b, 1, h.F32)
    xa = to_act(x, h.F32)
    rt = torch.randn(1, cout, H, W)
    outs, names = [], []
    for use in (1, 0):
        h.set_option("gemm3x3_f32", use)
        try:
            r = to_act(rt, h.F32)
            y = h.conv(cw, xa, out_dtype=h.F32, in_op=h.IN_LRELU, in_slope=0.1, act=h.ACT_LRELU, slope=0.01, res=r)
            names.append(h.lib().dcvc_last_kernel().decode())
            y1 = h.conv(cw, xa, out_dtype=h.F32)
            torch.cuda.synchronize()
            outs.append((back(y), back(y1)))
        finally:
            h.set_option("gemm3x3_f32", 1)
    assert names[0].startswith("gemm1x1f_kernel") and names[1].startswith("conv_kernel"), names
    for a_, c_ in zip(outs[0], outs[1]):
        assert torch.equal(a_, c_)
    ref = F.leaky_relu(F.conv2d(F.leaky_relu(x, 0.1), w, b, padding=1), 0.01) + rt
    assert rel_err(outs[0][0], ref) < 2e-5
    assert rel_err(outs[0][1], F.conv2d(x, w, b, padding=1)) < 2e-5


C3_CASES = [
    # cin, cout, H, W, coff (input channel view offset in a wider buffer)
    (64, 64, 37, 61, 0), (96, 192, 20, 33, 0), (128, 128, 9, 13, 0), (192, 96, 11, 70, 0),
    (128, 192, 40, 36, 0), (96, 96, 25, 70, 0), (64, 128, 300, 20, 0),
    (64, 3, 33, 47, 0), (32, 256, 18, 17, 32),
    (48, 48, 40, 50, 0), (80, 48, 17, 19, 0), (16, 32, 30, 30, 0), (48, 64, 21, 35, 16),
]


@pytest.mark.parametrize("case", C3_CASES)
def test_conv3x3_fixed_geometry_kernel(case):
    """The fixed-geometry 3x3 kernel vs the generic conv kernel: bit-identical
    when Cin % 32 == 0 (same K order), fp32-rounding-close with a 16-channel
    tail chunk (two taps per MFMA); both vs torch fp32 with bf16 tolerance.
    Exercises lrelu input op, bias + act, residual, scale, shuffle, f32 out,
    a channel-offset input view and ragged tile edges."""
    h = K()
    cin, cout, H, W, coff = case
    x = torch.randn(1, cin + coff + 8, H, W)
    w = torch.randn(cout, cin, 3, 3) / (9 * cin) ** 0.5
    b = torch.randn(cout) * 0.1
    cw = h.ConvW(w, b, 1, h.BF16)
    xbuf = to_act(x, h.BF16)
    xa = xbuf.ch(coff, cin)
    rt = torch.randn(1, cout, H, W)
    sc = torch.rand(cout if cout % 4 else cout // 4) + 0.5
    outs = []
    for use, res in ((1, 2), (0, 1), (1, 0)):
        h.set_option("conv3x3", use)
        h.set_option("conv3x3_resident", res)
        r = h.empty(H, W, cout, h.BF16)
        h.copy(to_act(rt, h.F32), r)
        y = h.conv(cw, xa, out_dtype=h.BF16, in_op=h.IN_LRELU, in_slope=0.1, act=h.ACT_LRELU, slope=0.01,
                   res=r)
        y2 = h.conv(cw, xa, out_dtype=h.F32, shuffle=cout % 4 == 0,
                    scale=sc.cuda() if cout % 4 == 0 else None)
        torch.cuda.synchronize()
        outs.append((back(y), back(y2)))
    h.set_option("conv3x3", 1)
    h.set_option("conv3x3_resident", 1)
    xs = bf16r(x[:, coff:coff + cin])
    wb, bd = bf16r(w), b.double()
    # lrelu of a bf16 value is re-rounded to bf16 on staging
    ref = F.leaky_relu(F.conv2d(bf16r(F.leaky_relu(xs, 0.1)), wb, bd, padding=1), 0.01) + bf16r(rt)
    assert bf16_err(outs[0][0], ref) < TOL_BF16
    ref2 = F.conv2d(xs, wb, bd, padding=1)
    if cout % 4 == 0:
        ref2 = F.pixel_shuffle(ref2, 2) * sc.double().view(1, -1, 1, 1)
    assert rel_err(outs[0][1], ref2) < TOL_BF16
    # resident-weight and per-workgroup variants run the same K order
    assert torch.equal(outs[0][0], outs[2][0])
    assert torch.equal(outs[0][1], outs[2][1])
    if cin % 32 == 0:
        assert torch.equal(outs[0][0], outs[1][0])
        assert torch.equal(outs[0][1], outs[1][1])
    else:
        assert rel_err(outs[0][1], outs[1][1]) < 1e-5


P3_CASES = [
    # cin, cout, H, W, coff: grids of >= 2 tiles per CU so the persistent kernel takes them
    (48, 48, 261, 533, 0), (96, 48, 130, 1030, 0), (64, 64, 270, 500, 8), (80, 48, 260, 520, 0),
    (128, 64, 250, 530, 0), (96, 96, 200, 700, 0), (64, 128, 260, 520, 0), (32, 32, 300, 470, 16),
]


@pytest.mark.parametrize("emode,rows4", [(3, 0), (2, 0), (1, 0), (0, 0), (0, 1)])
@pytest.mark.parametrize("case", P3_CASES)
def test_conv3x3_persistent_kernel(case, emode, rows4):
    """The persistent resident-weight 3x3 kernel (conv3x3p.hip) is
    bit-identical to the per-workgroup kernel (same K order, same fp32
    epilogue order) with every epilogue option on: lrelu input, bias +
    lrelu, two residuals, per-channel scale, ragged image edges, a channel
    view of a wider input; in each epilogue mode (2: straight from the
    accumulators with two input images, 1: one image, 0: the fp32 LDS
    tile, 3: mode 2 also for 8-row tiles); rows4: 32-row tiles where they
    fit (calls without a second residual)."""
    h = K()
    h.set_option("conv3x3_epilogue", emode)
    h.set_option("conv3x3_rows4", rows4)
    cin, cout, H, W, coff = case
    x = torch.randn(1, cin + coff + 8, H, W)
    w = torch.randn(cout, cin, 3, 3) / (9 * cin) ** 0.5
    b = torch.randn(cout) * 0.1
    cw = h.ConvW(w, b, 1, h.BF16)
    xa = to_act(x, h.BF16).ch(coff, cin)
    r1, r2 = to_act(torch.randn(1, cout, H, W), h.BF16), to_act(torch.randn(1, cout, H, W), h.BF16)
    sc = (torch.rand(cout) + 0.5).cuda()
    rf = to_act(torch.randn(1, cout, H, W), h.F32)
    shuf = cout % 32 == 0
    r3 = to_act(torch.randn(1, cout // 4, 2 * H, 2 * W), h.BF16) if shuf else None
    sc4 = (torch.rand(cout // 4) + 0.5).cuda() if shuf else None
    outs, names = [], []
    for pers in (1, 0):
        h.set_option("conv3x3_persistent", pers)
        h.set_option("conv3x3_resident", 0)
        y = h.conv(cw, xa, out_dtype=h.BF16, in_op=h.IN_LRELU, in_slope=0.1, act=h.ACT_LRELU, slope=0.01,
                   res=r1, res2=r2, scale=sc)
        names.append(h.lib().dcvc_last_kernel().decode())
        y2 = h.conv(cw, xa, out_dtype=h.BF16)
        y3 = h.conv(cw, xa, out_dtype=h.F32, act=h.ACT_LRELU, slope=0.1, res=rf)
        names.append(h.lib().dcvc_last_kernel().decode())
        y5 = h.conv(cw, xa, out_dtype=h.BF16, in_op=h.IN_LRELU, in_slope=0.1, act=h.ACT_LRELU, slope=0.01,
                    res=r1, scale=sc)
        names.append(h.lib().dcvc_last_kernel().decode())
        got = [back(y), back(y2), back(y3), back(y5)]
        if shuf:
            y4 = h.conv(cw, xa, out_dtype=h.BF16, shuffle=True, res=r3, scale=sc4)
            names.append(h.lib().dcvc_last_kernel().decode())
            got.append(back(y4))
        torch.cuda.synchronize()
        outs.append(got)
    h.set_option("conv3x3_persistent", 1)
    h.set_option("conv3x3_resident", 1)
    h.set_option("conv3x3_epilogue", 0)
    h.set_option("conv3x3_rows4", 1)
    k = len(names) // 2
    assert all(n.startswith("conv3p_kernel") for n in names[:k]), names
    if emode == 0:
        assert all(n.split(">")[0].endswith(", 0") for n in names[:k]), names
    assert not any(n.startswith("conv3p_kernel") for n in names[k:]), names
    for a, b_ in zip(outs[0], outs[1]):
        assert torch.equal(a, b_)
    xs = bf16r(x[:, coff:coff + cin])
    ref = F.conv2d(xs, bf16r(w), b.double(), padding=1)
    assert bf16_err(outs[0][1], ref) < TOL_BF16
    # the fp32-output call: lrelu(conv + b, 0.1) + fp32 residual
    ref3 = F.leaky_relu(ref, 0.1) + back(rf).double()
    assert rel_err(outs[0][2], ref3) < TOL_BF16
    if shuf:
        ref4 = (F.pixel_shuffle(ref, 2) + back(r3).double()) * sc4.cpu().double().view(1, -1, 1, 1)
        assert bf16_err(outs[0][4], ref4) < TOL_BF16


DCB_SHAPES = [(48, 32, False), (32, 64, False), (64, 128, False), (128, 128, False), (128, 64, False),
              (64, 48, False), (64, 64, False), (16, 32, True), (32, 64, True), (64, 128, True),
              (128, 128, True), (128, 64, True), (64, 16, True)]


def _dcb_state(cin, cout, gated, seed):
    from dcvc_amd.weights import synthetic_state_dict
    p = "b.block"
    spec = [(f"{p}.0.conv1.0.weight", (cin, cin, 1, 1)), (f"{p}.0.conv1.0.bias", (cin,)),
            (f"{p}.0.depth_conv.weight", (cin, 1, 3, 3)), (f"{p}.0.depth_conv.bias", (cin,)),
            (f"{p}.0.conv2.weight", (cout, cin, 1, 1)), (f"{p}.0.conv2.bias", (cout,))]
    if cin != cout:
        spec += [(f"{p}.0.adaptor.weight", (cout, cin, 1, 1)), (f"{p}.0.adaptor.bias", (cout,))]
    if gated:
        spec += [(f"{p}.1.conv.weight", (4 * cout, cout, 1, 1)), (f"{p}.1.conv.bias", (4 * cout,)),
                 (f"{p}.1.conv_out.weight", (cout, 2 * cout, 1, 1)), (f"{p}.1.conv_out.bias", (cout,))]
    else:
        hid = max(min(4 * cout, 1024), 2 * cout)
        spec += [(f"{p}.1.conv.0.weight", (hid, cout, 1, 1)), (f"{p}.1.conv.0.bias", (hid,)),
                 (f"{p}.1.conv.2.weight", (cout, hid, 1, 1)), (f"{p}.1.conv.2.bias", (cout,))]
    return synthetic_state_dict(spec, seed=seed, gain=1.5)


@pytest.mark.parametrize("shape", DCB_SHAPES)
def test_fused_depthconv_block_matches_unfused(shape):
    """The fused DepthConvBlock kernel reproduces the unfused bf16 kernel
    sequence (same roundings, same accumulation order) and the fp32 oracle."""
    from dcvc_amd import layers as L
    from oracle import dc_oracle as O
    h = K()
    cin, cout, gated = shape
    sd = _dcb_state(cin, cout, gated, seed=cin * 7 + cout)
    ctx = L.Ctx(sd, torch.device("cuda"), L.Precision.fast())
    blk = L.DepthConvBlock(ctx, "b", gated=gated)
    H, W = 37, 45
    x = torch.randn(1, cin, H, W)
    xa = to_act(x, h.BF16)
    sc = torch.rand(cout) + 0.5
    outs = []
    for fuse in (True, False):
        L.FUSE_DCB = fuse
        outs.append(back(blk(xa, scale=sc.cuda())))
    L.FUSE_DCB = True
    torch.cuda.synchronize()
    diff = (outs[0] - outs[1]).abs().max().item()
    assert diff <= 1e-2 * outs[1].abs().max().item(), diff
    fn = O.depth_conv_block2 if gated else O.depth_conv_block
    ref = fn(O.Params(sd), "b", x.to(torch.bfloat16).float()) * sc.view(1, -1, 1, 1)
    assert rel_err(outs[0], ref) < 3e-2


@pytest.mark.parametrize("shape", [(64, 48), (48, 32), (32, 64), (64, 64)])
def test_persistent_depthconv_block_equals_per_tile_kernel(shape):
    """dcbp.hip (persistent, resident weights) vs dcb.hip on a map of >= 2
    tiles per CU: same K order and rounding points, so bit-identical."""
    from dcvc_amd import layers as L
    h = K()
    cin, cout = shape
    sd = _dcb_state(cin, cout, False, seed=cin * 3 + cout)
    ctx = L.Ctx(sd, torch.device("cuda"), L.Precision.fast())
    blk = L.DepthConvBlock(ctx, "b")
    H, W = 133, 541
    xa = to_act(torch.randn(1, cin, H, W), h.BF16)
    sc = (torch.rand(cout) + 0.5).cuda()
    outs, names = [], []
    h.set_option("dcb_stream", 0)
    try:
        for pers in (1, 0):
            h.set_option("dcb_persistent", pers)
            outs.append(back(blk(xa, scale=sc)))
            names.append(h.lib().dcvc_last_kernel().decode())
    finally:
        h.set_option("dcb_persistent", 1)
        h.set_option("dcb_stream", 1)
    torch.cuda.synchronize()
    assert names[0].startswith("dcbp_kernel") and names[1].startswith("dcb_kernel"), names
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("shape", [(128, 128, False), (128, 64, False), (64, 128, False)])
@pytest.mark.parametrize("hw", [(133, 541), (21, 35), (272, 480)])
def test_streamed_depthconv_block_equals_per_tile_kernel(shape, hw):
    """dcbs.hip (persistent, 8 waves, weights streamed through two LDS
    buffers two chunks ahead, tiles chained across the stream) vs dcb.hip:
    same K order and rounding points, so bit-identical; 133x541 gives every
    workgroup 2-3 tiles, 21x35 fewer tiles than CUs, 272x480 the 1080p
    quarter-resolution map."""
    from dcvc_amd import layers as L
    h = K()
    cin, cout, gated = shape
    sd = _dcb_state(cin, cout, gated, seed=cin * 5 + cout)
    ctx = L.Ctx(sd, torch.device("cuda"), L.Precision.fast())
    blk = L.DepthConvBlock(ctx, "b", gated=gated)
    H, W = hw
    xa = to_act(torch.randn(1, cin, H, W), h.BF16)
    sc = (torch.rand(cout) + 0.5).cuda()
    outs, names = [], []
    h.set_option("dcb_persistent", 0)
    try:
        for on in (1, 0):
            h.set_option("dcb_stream", on)
            outs.append(back(blk(xa, scale=sc)))
            names.append(h.lib().dcvc_last_kernel().decode())
    finally:
        h.set_option("dcb_stream", 1)
        h.set_option("dcb_persistent", 1)
    torch.cuda.synchronize()
    assert names[0].startswith("dcbs_kernel") and names[1].startswith("dcb_kernel"), names
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("cin,cout,H,W,res,out32", [(8, 32, 544, 960, False, False), (16, 2, 544, 960, True, True),
                                                    (8, 32, 37, 45, False, False), (16, 2, 21, 19, True, True),
                                                    (8, 16, 40, 70, True, False)])
def test_conv7_small_cin_matches_torch(cin, cout, H, W, res, out32):
    """conv7s.hip (SpyNet's 8- and 16-channel 7x7 layers, taps packed into
    the MFMA K dimension) vs torch fp32 on the bf16-rounded operands and vs
    the generic conv.hip path; 544x960 gives each persistent workgroup
    several tiles, the small maps partial tiles."""
    h = K()
    x = torch.randn(1, cin, H, W)
    w = torch.randn(cout, cin, 7, 7) / (cin * 49) ** 0.5
    b = torch.randn(cout) * 0.1
    r = torch.randn(1, cout, H, W) if res else None
    ref = F.conv2d(bf16r(x), bf16r(w), b.double(), padding=3)
    if not res:
        ref = F.relu(ref)
    else:
        ref = ref + (r.double() if out32 else bf16r(r))
    cw = h.ConvW(w, b, 1, h.BF16)
    xa = to_act(x, h.BF16)
    odt = h.F32 if out32 else h.BF16
    ra = to_act(r, odt) if res else None
    outs, names = [], []
    for on in (1, 0):
        h.set_option("conv7_small_cin", on)
        try:
            y = h.conv(cw, xa, out_dtype=odt, act=h.ACT_NONE if res else h.ACT_LRELU, slope=0.0, res=ra)
        finally:
            h.set_option("conv7_small_cin", 1)
        outs.append(back(y))
        names.append(h.lib().dcvc_last_kernel().decode())
    torch.cuda.synchronize()
    assert names[0].startswith("conv7s_kernel") and names[1].startswith("conv_kernel"), names
    # fp32 sums of exact bf16 products (+ one bf16 output rounding)
    err = rel_err(outs[0], ref) if out32 else bf16_err(outs[0], ref)
    assert err < (2e-5 if out32 else TOL_BF16), err
    assert (rel_err(outs[0], outs[1]) if out32 else bf16_err(outs[0], outs[1].double(), 2.0 ** -7)) < TOL_BF16


@pytest.mark.parametrize("cin,cout,H,W", [(32, 64, 272, 480), (64, 32, 272, 480), (32, 16, 272, 480),
                                         (32, 64, 37, 45), (64, 32, 21, 19), (32, 16, 9, 70)])
def test_conv7_wide_cin_matches_torch(cin, cout, H, W):
    """conv7w.hip (SpyNet's 32- and 64-channel 7x7 layers: persistent,
    resident weights, slot-rotated halo image) vs torch fp32 on the
    bf16-rounded operands and vs the generic conv.hip path (ReLU, bf16 out)."""
    h = K()
    x = torch.randn(1, cin, H, W)
    w = torch.randn(cout, cin, 7, 7) / (cin * 49) ** 0.5
    b = torch.randn(cout) * 0.1
    ref = F.relu(F.conv2d(bf16r(x), bf16r(w), b.double(), padding=3))
    cw = h.ConvW(w, b, 1, h.BF16)
    xa = to_act(x, h.BF16)
    outs, names = [], []
    for on in (1, 0):
        h.set_option("conv7_wide_cin", on)
        try:
            y = h.conv(cw, xa, out_dtype=h.BF16, act=h.ACT_LRELU, slope=0.0)
        finally:
            h.set_option("conv7_wide_cin", 1)
        outs.append(back(y))
        names.append(h.lib().dcvc_last_kernel().decode())
    torch.cuda.synchronize()
    assert names[0].startswith("conv7w_kernel") and names[1].startswith("conv_kernel"), names
    assert bf16_err(outs[0], ref) < TOL_BF16
    assert bf16_err(outs[0], outs[1].double(), 2.0 ** -7) < TOL_BF16


@pytest.mark.parametrize("cin,cout,H,W,res,coff", [(56, 64, 544, 960, False, 0), (48, 64, 545, 961, True, 8),
                                                   (64, 96, 544, 962, False, 0), (64, 64, 547, 959, True, 0)])
def test_conv3x3_stride2_persistent_matches_torch(cin, cout, H, W, res, coff):
    """conv3s2.hip (persistent stride-2 3x3, resident weights, column-
    de-interleaved input image) vs torch fp32 on the bf16-rounded operands and
    vs the generic conv.hip path: odd map sizes, an input channel view, the
    residual epilogue, two n-blocks (96 outputs); maps of >= 2 output tiles
    per CU (smaller ones take the per-tile kernel)."""
    h = K()
    big = torch.randn(1, cin + coff, H, W)
    x = big[:, coff:coff + cin]
    w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout) * 0.1
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    r = torch.randn(1, cout, Ho, Wo) if res else None
    ref = F.leaky_relu(F.conv2d(bf16r(x), bf16r(w), b.double(), stride=2, padding=1), 0.1)
    if res:
        ref = ref + bf16r(r)
    cw = h.ConvW(w, b, 2, h.BF16)
    xa = to_act(big, h.BF16).ch(coff, cin)
    ra = to_act(r, h.BF16) if res else None
    outs, names = [], []
    for on in (1, 0):
        h.set_option("conv3x3_s2", on)
        try:
            y = h.conv(cw, xa, out_dtype=h.BF16, act=h.ACT_LRELU, slope=0.1, res=ra)
        finally:
            h.set_option("conv3x3_s2", 1)
        outs.append(back(y))
        names.append(h.lib().dcvc_last_kernel().decode())
    torch.cuda.synchronize()
    assert names[0].startswith("conv3s2_kernel") and names[1].startswith("conv_kernel"), names
    assert bf16_err(outs[0], ref) < TOL_BF16
    assert bf16_err(outs[0], outs[1].double(), 2.0 ** -7) < TOL_BF16


@pytest.mark.parametrize("dt,C,view", [("f32", 64, False), ("bf16", 64, False), ("bf16", 256, False),
                                       ("bf16", 48, True), ("f32", 36, False)])
def test_se_layer_matches_torch(dt, C, view):
    """SELayer (DCVC-HEM/src/models/video_net.py:157-170) + the residual
    apply of ConvBlockResidual (:173-188): vector and scalar-view paths."""
    h = K()
    dtype = h.F32 if dt == "f32" else h.BF16
    R = max(1, C // 16)
    x = torch.randn(1, C, 45, 77)
    a = torch.randn(1, C, 45, 77)
    w1 = torch.randn(R, C) * 0.3
    w2 = torch.randn(C, R) * 0.3
    if view:   # channel view at offset 3 of a wider buffer: scalar path
        big = torch.randn(1, C + 16, 45, 77)
        big[:, 3:3 + C] = x
        xa = to_act(big, dtype).ch(3, C)
    else:
        xa = to_act(x, dtype)
    x = back(xa)
    aa = to_act(a, dtype)
    a = back(aa)
    work = torch.empty(256 * C, dtype=torch.float32, device="cuda")
    s = torch.empty(C, dtype=torch.float32, device="cuda")
    h.se_scale(xa, w1.cuda(), w2.cuda(), work, s)
    y = h.se_apply(aa, xa, s)
    torch.cuda.synchronize()
    ref_s = torch.sigmoid(w2 @ torch.relu(w1 @ x.mean((-1, -2))[0]))
    assert (s.cpu() - ref_s).abs().max().item() < 1e-5
    ref_y = a + x * ref_s[None, :, None, None]
    tol = 1e-5 if dt == "f32" else 1e-2
    assert rel_err(back(y), ref_y) < tol


@pytest.mark.parametrize("src_dt,dst_dt", [(0, 0), (1, 1), (1, 0), (0, 1)])
@pytest.mark.parametrize("coff,C,pad", [(8, 48, 0), (3, 48, 0), (64, 64, 0), (0, 16, 5)])
def test_copy_and_pad_views(src_dt, dst_dt, coff, C, pad):
    """dcvc_copy / dcvc_pad_replicate into a channel window of a wider buffer,
    on the 8-channel vector path (aligned windows) and the scalar path: an
    exact copy (with dtype conversion), replicate padding, other channels
    untouched."""
    k = K()
    H, W = 37, 53
    x = torch.randn(1, C, H, W)
    xa = to_act(x, src_dt)
    dst = k.zeros(H + pad, W + pad, coff + C + 8, dst_dt)
    if pad:
        k.pad_replicate(xa, dst.ch(coff, C))
    else:
        k.copy(xa, dst.ch(coff, C))
    ref = F.pad(back(xa), (0, pad, 0, pad), mode="replicate")
    if dst_dt == 1:
        ref = ref.to(torch.bfloat16).float()
    got = dst.t().float().cpu()
    assert torch.equal(got[:, :, coff:coff + C].permute(2, 0, 1).unsqueeze(0), ref)
    assert not got[:, :, :coff].any() and not got[:, :, coff + C:].any()


@pytest.mark.parametrize("H,W", [(40, 56), (6, 2), (10, 18)])
def test_offset_diversity_paired_bf16_loads_bit_identical(H, W):
    """bf16 features: the paired-load path (even channel stride / offset) is
    bit-identical to the per-channel path (odd offset view of a wider buffer),
    including a one-column offset map (6x2) and a map whose width is not a
    multiple of the kernel's pixel tiles (10x18)."""
    h = K()
    feat = torch.randn(1, 48, H, W)
    flow = torch.randn(1, 2, H, W) * 3
    offs = torch.randn(1, 96, H // 2, W // 2) * 0.05
    fw = (torch.randn(48, 6) * 0.3).contiguous().cuda()
    fb = (torch.randn(48) * 0.1).cuda()
    fa = to_act(feat, h.BF16)                       # standalone 48-ch buffer: paired path
    wide = h.zeros(H, W, 50, h.BF16)
    h.copy(fa, wide.ch(1, 48))                      # coff 1: per-channel path
    oa, fl = to_act(offs, h.F32), to_act(flow, h.F32)
    y1 = h.offset_diversity(fa, oa, fl, fw, fb, _grid(H, W))
    y2 = h.offset_diversity(wide.ch(1, 48), oa, fl, fw, fb, _grid(H, W))
    torch.cuda.synchronize()
    assert torch.equal(y1.t().cpu(), y2.t().cpu())


@pytest.mark.parametrize("H,W,oscale", [(6, 2, 0.05), (10, 18, 0.05), (24, 130, 2.0), (68, 256, 0.5),
                                        (1088, 1920, 0.05)])
def test_offset_diversity_planar_bit_identical(H, W, oscale):
    """fp32 OffsetDiversity: the group-planar kernel pair (feature copied to
    [16][H][W][3], one group per wave, offsets and outputs staged in LDS;
    dcvc_offset_diversity_ws) gives the pixel-major kernel's bits, on the
    codec's views (input a wider buffer's channel window, output written into
    the 96-channel concat buffer at channel 48), with widths that are not a
    multiple of its 64-pixel runs and offsets large enough to clamp at the
    borders (oscale 2: 40 tanh(o) near +-40 pixels)."""
    h = K()
    g = torch.Generator().manual_seed(H * 7 + W)
    feat = torch.randn(1, 48, H, W, generator=g)
    flow = torch.randn(1, 2, H, W, generator=g) * 3
    offs = torch.randn(1, 96, H // 2, W // 2, generator=g) * oscale
    fw = (torch.randn(48, 6, generator=g) * 0.3).contiguous().cuda()
    fb = (torch.randn(48, generator=g) * 0.1).cuda()
    wide = h.zeros(H, W, 56, h.F32)
    h.copy(to_act(feat, h.F32), wide.ch(4, 48))
    fa = wide.ch(4, 48)
    oa, fl = to_act(offs, h.F32), to_act(flow, h.F32)
    gx, gy = _grid(H, W)
    y_ref = h.zeros(H, W, 96, h.F32)
    h.check(h.lib().dcvc_offset_diversity(fa.c(), oa.c(), fl.c(), y_ref.ch(48, 48).c(), fw.data_ptr(), fb.data_ptr(),
                                          gx.data_ptr(), gy.data_ptr(), 40.0, h.stream()), "od")
    y = h.zeros(H, W, 96, h.F32)
    old, h.OD_PLANAR = h.OD_PLANAR, True
    try:
        h.offset_diversity(fa, oa, fl, fw, fb, (gx, gy), y=y.ch(48, 48))
    finally:
        h.OD_PLANAR = old
    torch.cuda.synchronize()
    assert torch.equal(y.t().cpu(), y_ref.t().cpu())
