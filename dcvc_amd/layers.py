"""Network blocks of the DCVC-DC hot path on libdcvc_hip.

Each block is built from a reference-format state_dict prefix (same key names
as DCVC-DC/src/models/*.py, so reference checkpoints load) and runs entirely
on our kernels: convs with fused epilogues, depthwise conv, pooling, resize.
Concatenations are never materialised by copying: producers write into
channel windows of one NHWC buffer (``Act.ch``).

Precision policy (``Precision``): feature-domain activations (full to 1/8
resolution) are stored in ``feat`` and convolved with ``feat_compute``;
latent-domain tensors (1/16 and 1/64: y, z, priors, entropy parameters) are
stored fp32 and convolved with ``latent_compute``.
  * ``Precision.split()`` (the bench default): fp32 storage everywhere, every
    dense conv on split-fp16 operands (x = hi + 2^-11 lo, three f16 MFMAs per
    product, fp32 accumulation; sconv.hip): held to the strict parity bar.
  * ``Precision.parity()``: fp32 everywhere on f32 MFMA (exact fp32 fma chains).
  * ``Precision.fast()``: bf16 feature maps and bf16 MFMA, fp32 latents; not
    held to the strict bar (labelled lines only).
"""
import torch

from . import hip as K
from .hip import Act, F32, BF16, F16X3, ACT_LRELU, ACT_NONE, IN_LRELU, IN_GATE


FUSE_DCB = True   # fused DepthConvBlock kernel where instantiated (A/B switch)
FUSE_FFN = True   # split precision: fused ConvFFN kernel (sffn.hip) where instantiated (A/B switch)
FUSE_DC = True    # split precision: fused DepthConv kernel (sdc.hip) where instantiated (A/B switch)
DW128 = True      # split precision: the 128-channel feature-rate DepthConv tail (depthwise + conv2 + identity) in one kernel (A/B)
# (cin, cout, adaptor) of the fused DepthConv instantiations (sdc.hip supported())
SDC_SHAPES = {(64, 48, True), (48, 32, True), (32, 64, True), (64, 64, False), (48, 48, False), (32, 32, False)}


class Precision:
    def __init__(self, feat, feat_compute, latent_compute):
        self.feat = feat
        self.feat_compute = feat_compute
        self.latent = F32
        self.latent_compute = latent_compute

    @staticmethod
    def parity():
        return Precision(F32, F32, F32)

    @staticmethod
    def fast(latent_compute=F32):
        return Precision(BF16, BF16, latent_compute)

    @staticmethod
    def split():
        return Precision(F32, F16X3, F16X3)

    @property
    def name(self):
        if self.feat_compute == F16X3:
            return "split"
        if self.feat == F32:
            return "parity"
        return "fast" if self.latent_compute == F32 else "fast-bf16-tail"


def split_checkpoint(codec, stage):
    """Inside a guarded encode_decode (split_guarded): raise
    hip.SplitRangeError now if a split kernel of this frame has seen a value
    outside the split's range.  The codecs call it right after ``compress``
    (before the stream file is written) and after ``decompress``."""
    if codec.prec.feat_compute == F16X3 and getattr(codec, "_guard_on", False):
        K.split_guard_check(f"{type(codec).__name__}.{stage}")


def parity_twin(codec):
    """The fp32 (Precision.parity) twin of a split codec, built once, lazily,
    from the same state_dict and constructor arguments; it shares the codec's
    entropy coder (same stream_part / ec_thread, same tables)."""
    t = getattr(codec, "_parity_twin", None)
    if t is None:
        kw = dict(codec._init_kw, precision=Precision.parity(), device=codec.dev)
        t = type(codec)(**kw).load_state_dict(codec.sd)
        if codec.entropy_coder is not None:
            t.update(force=True)
        codec._parity_twin = t
    if codec.entropy_coder is not None:
        t.entropy_coder = codec.entropy_coder
    return t


def split_guarded(fn):
    """encode_decode of a codec in Precision.split(): the fp16 range guard of
    the split kernels (dcvc_split_range_flag) is armed (and cleared) for the
    calling thread for the frame, checked by the codec after ``compress``
    (before the file is written) and after ``decompress``
    (``split_checkpoint``), and disarmed on the way out whatever happens.

    A frame that trips it is coded again, whole, by the codec's fp32 twin
    (``parity_twin``: the same state_dict on the fp32 HIP kernels, the
    reference's own arithmetic), so a drop-in run of an input the split cannot
    carry (DCVC-HEM's random init grows its latents, common_model.py:32-37)
    still gets a valid stream: write mode rewrites the same output file, and
    the result dict says ``precision_fallback: "parity"``.  The encoder and
    the decoder of a frame always run in one precision."""
    import functools

    @functools.wraps(fn)
    def run(self, *args, **kw):
        if self.prec.feat_compute != F16X3:
            return fn(self, *args, **kw)
        ec = self.entropy_coder
        trace = getattr(ec, "trace", None) if ec is not None else None
        n0 = len(trace) if trace is not None else 0
        K.split_guard_arm(self.dev)
        self._guard_on = True
        try:
            out = fn(self, *args, **kw)
            K.split_guard_check(f"{type(self).__name__}.encode_decode")
            return out
        except K.SplitRangeError as e:
            reason = str(e)
        finally:
            self._guard_on = False
            K.split_guard_disarm()
        # the fp32 twin codes the frame again (its encoder and decoder);
        # the coder trace keeps only the twin's calls
        if trace is not None:
            del trace[n0:]
        self.fallbacks = getattr(self, "fallbacks", 0) + 1
        out = parity_twin(self).encode_decode(*args, **kw)
        out["precision_fallback"] = "parity"
        out["precision_fallback_reason"] = reason
        return out
    return run


class Ctx:
    """Builds layers from a state_dict on one device under one precision."""

    def __init__(self, state_dict, device, prec):
        self.sd = state_dict
        self.dev = device
        self.prec = prec
        self.used = set()

    def has(self, name):
        return name + ".weight" in self.sd

    def take(self, key):
        if key not in self.sd:
            raise KeyError(f"missing key in state_dict: {key}")
        self.used.add(key)
        return self.sd[key]

    def check_strict(self, extra_used=()):
        """load_state_dict(strict=True): every key must be consumed."""
        unused = set(self.sd) - self.used - set(extra_used)
        if unused:
            raise RuntimeError(f"unexpected key(s) in state_dict: {sorted(unused)[:8]}")

    def conv(self, name, stride=1, latent=False, compute=None, cin_pad=None, out_perm=None, in_perm=None):
        """cin_pad: zero-pad the input channels to this count, for inputs whose
        concat buffer carries zero channels up to an 8-channel multiple (the
        kernels' 16-byte staging path); the products of the pad are exact
        zeros, so the result is unchanged.  out_perm: output channel order
        (a permutation of the reference's), so a producer can write a
        consumer's concat layout directly; per-channel results are unchanged.
        in_perm: input channel j of the buffer is the reference's input
        channel in_perm[j] (a concat laid out with its 16-byte-aligned part
        first); the sum over input channels is the same set of products."""
        if compute is None:
            compute = self.prec.latent_compute if latent else self.prec.feat_compute
        b = self.take(name + ".bias") if name + ".bias" in self.sd else None
        w = self.take(name + ".weight")
        if in_perm is not None:
            w = w.detach().float()[:, torch.as_tensor(in_perm, dtype=torch.long)]
        if cin_pad is not None and cin_pad > w.shape[1]:
            w = torch.nn.functional.pad(w.detach().float(), (0, 0, 0, 0, 0, cin_pad - w.shape[1]))
        if out_perm is not None:
            perm = torch.as_tensor(out_perm, dtype=torch.long)
            w = w.detach().float()[perm]
            if b is not None:
                b = b.detach().float()[perm]
        return K.ConvW(w, b, stride, compute, self.dev)

    def dw(self, name):
        w = self.take(name + ".weight").detach().float().cpu()  # [C,1,3,3]
        C = w.shape[0]
        w9c = w.reshape(C, 9).t().contiguous().to(self.dev)  # [9][C]
        b = self.take(name + ".bias").detach().float().contiguous().to(self.dev)
        return w9c, b

    def dtype(self, latent):
        return self.prec.latent if latent else self.prec.feat

    def fit(self, x, compute):
        """f32 / f16x3 compute needs f32 inputs; cast a view when a layer crosses domains."""
        if compute != BF16 and x.dtype != F32:
            return cast(x, F32)
        return x


def cast(x, dtype):
    if x.dtype == dtype:
        return x
    y = K.empty(x.H, x.W, x.C, dtype, x.buf.device)
    return K.copy(x, y)


# ------------------------------------------------------------------ layers.py
class DepthConvBlock:
    """DepthConv + ConvFFN (DepthConvBlock) or + ConvFFN2 (DepthConvBlock2),
    DCVC-DC/src/models/layers.py:135-222."""

    def __init__(self, ctx, p, gated=False, latent=False, slope_dc=0.01, slope_ffn=0.1):
        self.ctx, self.latent, self.gated = ctx, latent, gated
        self.slope_dc, self.slope_ffn = slope_dc, slope_ffn
        d = p + ".block.0"
        f = p + ".block.1"
        self.conv1 = ctx.conv(d + ".conv1.0", latent=latent)
        self.dw = ctx.dw(d + ".depth_conv")
        self.conv2 = ctx.conv(d + ".conv2", latent=latent)
        self.adaptor = ctx.conv(d + ".adaptor", latent=latent) if ctx.has(d + ".adaptor") else None
        if gated:
            self.ffn1 = ctx.conv(f + ".conv", latent=latent)
            self.ffn2 = ctx.conv(f + ".conv_out", latent=latent)
        else:
            self.ffn1 = ctx.conv(f + ".conv.0", latent=latent)
            self.ffn2 = ctx.conv(f + ".conv.2", latent=latent)
        self.cout = self.ffn2.cout
        # split precision: DepthConv and ConvFFN as fused kernels (sdc.hip,
        # sffn.hip) where one is instantiated for the block's widths; t1, the
        # depthwise output and the 4x-wide hidden layer stay in LDS
        self.dcw = None
        sd = ctx.sd
        if (FUSE_DC and self.conv1.compute == F16X3 and not latent and
                (self.conv1.cin, self.conv2.cout, self.adaptor is not None) in SDC_SHAPES):
            self.dcw = K.DcW(sd[d + ".conv1.0.weight"], sd[d + ".conv1.0.bias"], self.dw[0], self.dw[1],
                             sd[d + ".conv2.weight"], sd[d + ".conv2.bias"],
                             sd[d + ".adaptor.weight"] if self.adaptor is not None else None,
                             sd[d + ".adaptor.bias"] if self.adaptor is not None else None, ctx.dev)
        # split precision, the entropy model's adaptor-free 192 / 384-channel
        # latent blocks: depthwise + conv2 + identity in one kernel (slffn.hip)
        self.dwc = None
        if (FUSE_DC and self.conv1.compute == F16X3 and self.adaptor is None and self.conv1.cin == self.conv2.cout
                and ((latent and self.conv2.cin in (192, 384)) or (DW128 and not latent and self.conv2.cin == 128))):
            self.dwc = K.DwcW(self.dw[0], self.dw[1], sd[d + ".conv2.weight"], sd[d + ".conv2.bias"], ctx.dev)
        self.ffn = None
        # (sffn.hip for the feature-rate widths; slffn.hip for the latent
        # 192 / 384-channel blocks of the entropy model)
        if (FUSE_FFN and not gated and self.ffn2.compute == F16X3 and self.cout in (32, 48, 64, 128, 192, 384)
                and self.ffn1.cout % (64 if self.cout != 128 else 32) == 0):
            sd = ctx.sd
            self.ffn = K.FfnW(sd[f + ".conv.0.weight"], sd[f + ".conv.0.bias"], sd[f + ".conv.2.weight"],
                              sd[f + ".conv.2.bias"], ctx.dev)

    def __call__(self, x, y=None, scale=None):
        ctx = self.ctx
        dt = ctx.dtype(self.latent)
        if (FUSE_DCB and not self.latent and x.dtype == BF16 and dt == BF16
                and self.conv1.compute == BF16 and self.cout <= 128 and x.C <= 128):
            out = y if y is not None else K.empty(x.H, x.W, self.cout, BF16, x.buf.device)
            if K.depthconv_block(self, x, out, scale) is not None:
                return out
        x = ctx.fit(x, self.conv1.compute)
        dc = None
        if self.dcw is not None:
            dc = K.depth_conv_split(self.dcw, x, slope=self.slope_dc)
        if dc is not None:
            pass
        elif self.adaptor is not None:
            idn = K.conv(self.adaptor, x, out_dtype=dt)
        else:
            idn = cast(x, dt)
        if dc is None:
            t = K.conv(self.conv1, x, out_dtype=dt, act=ACT_LRELU, slope=self.slope_dc)
            if self.dwc is not None:
                dc = K.dw_conv2_split(self.dwc, t, idn)
            if dc is None:
                t = K.dwconv3x3(t, *self.dw)
                dc = K.conv(self.conv2, t, res=idn)
        if self.gated:
            h = K.conv(self.ffn1, dc)
            return K.conv(self.ffn2, h, y, in_op=IN_GATE, in_slope=self.slope_ffn, res=dc, scale=scale)
        if self.ffn is not None:
            out = K.conv_ffn(self.ffn, dc, y, scale=scale, slope=self.slope_ffn)
            if out is not None:
                return out
        # the hidden layer feeds only ffn2: with bf16 compute ffn2 rounds it
        # to bf16 on staging anyway, so it is stored as bf16 (same values,
        # half the traffic of the 4x-wide map)
        hid = BF16 if self.ffn2.compute == BF16 else dt
        h = K.conv(self.ffn1, dc, out_dtype=hid, act=ACT_LRELU, slope=self.slope_ffn)
        return K.conv(self.ffn2, h, y, out_dtype=dc.dtype, act=ACT_LRELU, slope=self.slope_ffn, res=dc,
                      scale=scale)


class ResidualBlockWithStride:
    """layers.py:42-73."""

    def __init__(self, ctx, p, latent=False):
        self.ctx, self.latent = ctx, latent
        self.conv1 = ctx.conv(p + ".conv1", 2, latent)
        self.conv2 = ctx.conv(p + ".conv2", 1, latent)
        self.down = ctx.conv(p + ".downsample", 2, latent)

    def __call__(self, x, y=None, scale=None):
        dt = self.ctx.dtype(self.latent)
        x = self.ctx.fit(x, self.conv1.compute)
        t = K.conv(self.conv1, x, out_dtype=dt, act=ACT_LRELU, slope=0.01)
        idn = K.conv(self.down, x, out_dtype=dt)
        return K.conv(self.conv2, t, y, act=ACT_LRELU, slope=0.1, res=idn, scale=scale)


class ResidualBlockUpsample:
    """layers.py:76-101."""

    def __init__(self, ctx, p, latent=False):
        self.ctx, self.latent = ctx, latent
        self.sub = ctx.conv(p + ".subpel_conv.0", 1, latent)
        self.conv = ctx.conv(p + ".conv", 1, latent)
        self.up = ctx.conv(p + ".upsample.0", 1, latent)

    def __call__(self, x, y=None, scale=None):
        dt = self.ctx.dtype(self.latent)
        x = self.ctx.fit(x, self.sub.compute)
        t = K.conv(self.sub, x, out_dtype=dt, shuffle=True, act=ACT_LRELU, slope=0.01)
        idn = K.conv(self.up, x, out_dtype=dt, shuffle=True)
        return K.conv(self.conv, t, y, act=ACT_LRELU, slope=0.1, res=idn, scale=scale)


# ------------------------------------------------------------ video_net.py
class ResBlock:
    """video_net.py:58-76: x + [lrelu?](conv2(lrelu(conv1(lrelu(x)))))."""

    def __init__(self, ctx, p, slope=0.01, end_with_relu=False, latent=False):
        self.ctx, self.latent = ctx, latent
        self.slope, self.end = slope, end_with_relu
        self.conv1 = ctx.conv(p + ".conv1", 1, latent)
        self.conv2 = ctx.conv(p + ".conv2", 1, latent)

    def __call__(self, x, y=None, res2=None, scale=None):
        t = K.conv(self.conv1, x, in_op=IN_LRELU, in_slope=self.slope, act=ACT_LRELU, slope=self.slope)
        return K.conv(self.conv2, t, y, act=ACT_LRELU if self.end else ACT_NONE, slope=self.slope,
                      res=x, res2=res2, scale=scale)


class UNet:
    """UNet / UNet2 (video_net.py:129-214) with cat-free skip buffers."""

    def __init__(self, ctx, p, gated=False):
        self.ctx = ctx
        B = lambda n: DepthConvBlock(ctx, f"{p}.{n}", gated=gated)  # noqa: E731
        self.conv1, self.conv2, self.conv3 = B("conv1"), B("conv2"), B("conv3")
        self.refine = [B(f"context_refine.{i}") for i in range(4)]
        self.up3 = ctx.conv(p + ".up3.0")
        self.up_conv3 = B("up_conv3")
        self.up2 = ctx.conv(p + ".up2.0")
        self.up_conv2 = B("up_conv2")

    def __call__(self, x, y=None):
        dt = self.ctx.prec.feat
        H, W = x.H, x.W
        c1 = self.conv1.cout
        c2 = self.conv2.cout
        cat2 = K.empty(H, W, c1 + self.up2.cout // 4, dt, x.buf.device)
        x1 = self.conv1(x, cat2.ch(0, c1))
        x2p = K.pool2x2(x1, True)
        cat3 = K.empty(H // 2, W // 2, c2 + self.up3.cout // 4, dt, x.buf.device)
        x2 = self.conv2(x2p, cat3.ch(0, c2))
        x3 = self.conv3(K.pool2x2(x2, True))
        for b in self.refine:
            x3 = b(x3)
        K.conv(self.up3, x3, cat3.ch(c2, self.up3.cout // 4), shuffle=True)
        d3 = self.up_conv3(cat3)
        K.conv(self.up2, d3, cat2.ch(c1, self.up2.cout // 4), shuffle=True)
        return self.up_conv2(cat2, y)


class SpyNet:
    """ME_Spynet + MEBasic (video_net.py:79-126).  Flows are fp32."""

    def __init__(self, ctx, p, grids):
        self.ctx, self.grids = ctx, grids
        self.levels = [[ctx.conv(f"{p}.moduleBasic.{lv}.conv{i}") for i in range(1, 6)] for lv in range(4)]

    def __call__(self, im1, im2):
        dev = im1.buf.device
        p1, p2 = [im1], [im2]
        for _ in range(3):
            p1.append(K.pool2x2(p1[-1], False))
            p2.append(K.pool2x2(p2[-1], False))
        flow = K.zeros(p2[3].H // 2, p2[3].W // 2, 2, F32, dev)
        cdt = self.ctx.prec.feat_compute
        in_dt = F32 if cdt == F32 else self.ctx.prec.feat
        for lv in range(4):
            k = 3 - lv
            H, W = p1[k].H, p1[k].W
            cat = K.empty(H, W, 8, F32, dev)  # [im1 | warp(im2, flow_up) | flow_up]
            flow_up = K.resize2x(flow, True, 2.0, y=cat.ch(6, 2))
            K.copy(p1[k], cat.ch(0, 3))
            K.flow_warp(p2[k], flow_up, self.grids(H, W), y=cat.ch(3, 3))
            convs = self.levels[lv]
            t = cast(cat, in_dt)
            for c in convs[:4]:
                t = K.conv(c, t, out_dtype=in_dt, act=ACT_LRELU, slope=0.0)
            flow = K.conv(convs[4], t, out_dtype=F32, res=cast(flow_up, F32) if flow_up.dtype != F32 else flow_up)
        return flow


def hyper_enc(ctx, p, reduce_enc_layer):
    """get_hyper_enc_dec_models encoder (video_net.py:217-237)."""
    if reduce_enc_layer:
        convs = [(ctx.conv(p + ".0", 1, True), True), (ctx.conv(p + ".2", 2, True), True),
                 (ctx.conv(p + ".4", 2, True), False)]
    else:
        convs = [(ctx.conv(p + ".0", 1, True), True), (ctx.conv(p + ".2", 1, True), True),
                 (ctx.conv(p + ".4", 2, True), True), (ctx.conv(p + ".6", 1, True), True),
                 (ctx.conv(p + ".8", 2, True), False)]

    def run(x):
        for c, relu in convs:
            x = K.conv(c, ctx.fit(x, c.compute), out_dtype=F32, act=ACT_LRELU if relu else K.ACT_ROUND,
                       slope=0.01)
        return x  # last conv rounds: z_hat = round(z)
    return run


def hyper_dec(ctx, p):
    """get_hyper_enc_dec_models decoder (video_net.py:239-249)."""
    c0, c4, c8 = (ctx.conv(f"{p}.{i}", 1, True) for i in (0, 4, 8))
    c2, c6 = (ctx.conv(f"{p}.{i}.0", 1, True) for i in (2, 6))  # subpel_conv1x1 = Sequential(conv, shuffle)

    def run(x, y=None):
        x = K.conv(c0, x, act=ACT_LRELU, slope=0.01)
        x = K.conv(c2, x, shuffle=True, act=ACT_LRELU, slope=0.01)
        x = K.conv(c4, x, act=ACT_LRELU, slope=0.01)
        x = K.conv(c6, x, shuffle=True, act=ACT_LRELU, slope=0.01)
        return K.conv(c8, x, y)
    return run


class Grids:
    """The reference's cached fp32 linspace grids (video_net.py:11-19),
    computed once per size on the host with the CPU linspace so the values
    are those of the CPU reference."""

    def __init__(self, device):
        self.dev = device
        self.cache = {}

    def __call__(self, H, W):
        key = (H, W)
        if key not in self.cache:
            gx = torch.linspace(-1.0, 1.0, W, dtype=torch.float32).to(self.dev)
            gy = torch.linspace(-1.0, 1.0, H, dtype=torch.float32).to(self.dev)
            self.cache[key] = (gx, gy)
        return self.cache[key]
