"""DCVC-HEM network blocks on libdcvc_hip (DCVC-HEM/src/models/video_net.py,
src/layers/layers.py).  Blocks shared with DCVC-DC (ResidualBlockWithStride,
ResidualBlockUpsample, SpyNet, hyperprior decoder) come from dcvc_amd.layers;
this module adds HEM's ResBlock variants, ConvBlockResidual with its
squeeze-excitation layer, the HEM UNet and the enc/dec towers."""
import torch

from .. import hip as K
from ..hip import F32, BF16, ACT_LRELU, ACT_NONE, IN_LRELU, IN_NONE
from ..layers import ResidualBlockWithStride, ResidualBlockUpsample


class ResBlock:
    """ResBlock (video_net.py:82-108): x + [act](conv2(act(conv1([act](x)))));
    slope 0 is nn.ReLU (leaky ReLU with slope 0 gives the same values)."""

    def __init__(self, ctx, p, slope=0.01, start_from_relu=True, end_with_relu=False, latent=False):
        self.slope = 0.0 if slope < 0.0001 else slope
        self.start, self.end = start_from_relu, end_with_relu
        self.conv1 = ctx.conv(p + ".conv1", 1, latent)
        self.conv2 = ctx.conv(p + ".conv2", 1, latent)

    def __call__(self, x, y=None, res2=None):
        t = K.conv(self.conv1, x, in_op=IN_LRELU if self.start else IN_NONE, in_slope=self.slope, act=ACT_LRELU,
                   slope=self.slope)
        return K.conv(self.conv2, t, y, act=ACT_LRELU if self.end else ACT_NONE, slope=self.slope, res=x,
                      res2=res2)


class ResidualBlock:
    """ResidualBlock (layers/layers.py:105-128): x + lrelu(conv2(lrelu(conv1(x))))."""

    def __init__(self, ctx, p):
        self.conv1 = ctx.conv(p + ".conv1")
        self.conv2 = ctx.conv(p + ".conv2")

    def __call__(self, x, y=None):
        t = K.conv(self.conv1, x, act=ACT_LRELU, slope=0.01)
        return K.conv(self.conv2, t, y, act=ACT_LRELU, slope=0.01, res=x)


class ConvBlockResidual:
    """ConvBlockResidual + SELayer (video_net.py:157-188):
    up_dim(x) + SE(conv2(lrelu(conv1(x))))."""

    def __init__(self, ctx, p):
        self.c0 = ctx.conv(p + ".conv.0")
        self.c2 = ctx.conv(p + ".conv.2")
        self.up = ctx.conv(p + ".up_dim")
        self.w1 = ctx.take(p + ".conv.3.fc.0.weight").detach().float().contiguous().to(ctx.dev)
        self.w2 = ctx.take(p + ".conv.3.fc.2.weight").detach().float().contiguous().to(ctx.dev)
        self.dev = ctx.dev
        self.dt = ctx.prec.feat

    def __call__(self, x, y=None):
        t = K.conv(self.c0, x, act=ACT_LRELU, slope=0.01)
        u = K.conv(self.c2, t)
        work = torch.empty(256 * u.C, dtype=torch.float32, device=self.dev)
        s = torch.empty(u.C, dtype=torch.float32, device=self.dev)
        K.se_scale(u, self.w1, self.w2, work, s)
        a = K.conv(self.up, x, out_dtype=u.dtype)
        return K.se_apply(a, u, s, y)


class UNet:
    """UNet (video_net.py:191-236) with cat-free skip buffers."""

    def __init__(self, ctx, p):
        self.ctx = ctx
        self.conv1 = ConvBlockResidual(ctx, p + ".conv1")
        self.conv2 = ConvBlockResidual(ctx, p + ".conv2")
        self.conv3 = ConvBlockResidual(ctx, p + ".conv3")
        self.refine = [ResBlock(ctx, f"{p}.context_refine.{i}", slope=0) for i in range(4)]
        self.up3 = ctx.conv(p + ".up3.0")
        self.up_conv3 = ConvBlockResidual(ctx, p + ".up_conv3")
        self.up2 = ctx.conv(p + ".up2.0")
        self.up_conv2 = ConvBlockResidual(ctx, p + ".up_conv2")

    def __call__(self, x, y=None):
        dt, dev = self.ctx.prec.feat, x.buf.device
        H, W = x.H, x.W
        c1 = self.conv1.c2.cout
        c2 = self.conv2.c2.cout
        cat2 = K.empty(H, W, c1 + self.up2.cout // 4, dt, dev)
        x1 = self.conv1(x, cat2.ch(0, c1))
        cat3 = K.empty(H // 2, W // 2, c2 + self.up3.cout // 4, dt, dev)
        x2 = self.conv2(K.pool2x2(x1, True), cat3.ch(0, c2))
        x3 = self.conv3(K.pool2x2(x2, True))
        for b in self.refine:
            x3 = b(x3)
        K.conv(self.up3, x3, cat3.ch(c2, self.up3.cout // 4), shuffle=True)
        d3 = self.up_conv3(cat3)
        K.conv(self.up2, d3, cat2.ch(c1, self.up2.cout // 4), shuffle=True)
        return self.up_conv2(cat2, y)


class EncTower:
    """get_enc_dec_models encoder (video_net.py:239-249)."""

    def __init__(self, ctx, p):
        self.blocks = []
        for i in (0, 2, 4):
            self.blocks += [ResidualBlockWithStride(ctx, f"{p}.{i}"), ResidualBlock(ctx, f"{p}.{i + 1}")]
        self.last = ctx.conv(p + ".6", 2)

    def __call__(self, x):
        for b in self.blocks:
            x = b(x)
        return K.conv(self.last, x, out_dtype=F32)


class DecTower:
    """get_enc_dec_models decoder (video_net.py:251-262)."""

    def __init__(self, ctx, p):
        self.blocks = []
        for i in (0, 2, 4):
            self.blocks += [ResidualBlock(ctx, f"{p}.{i}"), ResidualBlockUpsample(ctx, f"{p}.{i + 1}")]
        self.blocks.append(ResidualBlock(ctx, p + ".6"))
        self.last = ctx.conv(p + ".7.0")

    def __call__(self, x, out_dtype=None):
        for b in self.blocks:
            x = b(x)
        return K.conv(self.last, x, out_dtype=out_dtype, shuffle=True)


class Seq3:
    """The 3-conv prior networks (mv/y prior fusion, spatial priors,
    video_model.py:153-214): conv, lrelu(0.2), conv, lrelu(0.2), conv.  The
    last conv's outputs can be permuted (out_perm) and written into a view."""

    def __init__(self, ctx, p, out_perm=None):
        self.c0 = ctx.conv(p + ".0", latent=True)
        self.c2 = ctx.conv(p + ".2", latent=True)
        self.c4 = ctx.conv(p + ".4", latent=True, out_perm=out_perm)

    def __call__(self, x, y=None):
        # the two intermediate maps feed only the next conv: with bf16 compute
        # that conv rounds its input to bf16 on staging, so storing them as
        # bf16 (the epilogue's identical RNE rounding) changes no value and
        # halves their traffic; parity mode (f32 compute) keeps fp32
        mid0 = BF16 if self.c2.compute == BF16 else F32
        mid1 = BF16 if self.c4.compute == BF16 else F32
        x = K.conv(self.c0, x, out_dtype=mid0, act=ACT_LRELU, slope=0.2)
        x = K.conv(self.c2, x, out_dtype=mid1, act=ACT_LRELU, slope=0.2)
        return K.conv(self.c4, x, y, out_dtype=F32)


def chunk3_to_buffer_order(C):
    """prior fusion output chunk(3) = (q_step, scales, means) -> the dual
    prior buffer order (means, scales, q_step) (common_model.py:124)."""
    return list(range(2 * C, 3 * C)) + list(range(C, 2 * C)) + list(range(0, C))
