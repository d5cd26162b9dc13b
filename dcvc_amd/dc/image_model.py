"""DCVC-DC intra codec (IntraNoAR) on MI355X.

API of DCVC-DC/src/models/image_model.py:61-252: ``IntraNoAR(N, anchor_num,
ec_thread, stream_part, inplace)``, ``load_state_dict``, ``update``,
``get_q_scales_from_ckpt``, ``compress``, ``decompress``, ``forward``
(estimate mode) and ``encode_decode`` (both modes).  ``x_hat`` is an NHWC fp32 ``Act``.
"""
import torch

from .. import hip as K
from ..hip import F32, ACT_LRELU, ACT_CLAMP01
from ..layers import split_guarded, split_checkpoint, Ctx, Precision, DepthConvBlock, ResidualBlockWithStride, ResidualBlockUpsample, UNet
from ..entropy import ScaleTable, FactorizedTable, EntropyCoder
from ..stream_helper import get_downsampled_shape, encode_i, decode_i, filesize, get_state_dict
from .common import SymbolBuffer, QuadtreePrior, BitCounter, bits_result, pad_for_y, crop_to, q_fine, curr_q
from .video_model import as_act


class IntraNoAR:
    def __init__(self, N=256, anchor_num=4, ec_thread=False, stream_part=1, inplace=False, precision=None,
                 device=None):
        self.N = N
        self.ec_thread, self.stream_part = ec_thread, stream_part
        self._init_kw = dict(N=N, anchor_num=anchor_num, ec_thread=ec_thread, stream_part=stream_part,
                             inplace=inplace)
        self.prec = precision if precision is not None else Precision.split()
        self.dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.entropy_coder = None

    def load_state_dict(self, state_dict, strict=True):
        sd = {k: v for k, v in state_dict.items()}
        self.sd = sd
        ctx = Ctx(sd, self.dev, self.prec)
        self.ctx = ctx
        D2 = lambda p, latent=False: DepthConvBlock(ctx, p, gated=True, latent=latent)  # noqa: E731
        # IntraEncoder (image_model.py:16-35)
        self.e1 = ResidualBlockWithStride(ctx, "enc.enc_1.0")
        self.e1b = D2("enc.enc_1.1")
        self.e2 = [ResidualBlockWithStride(ctx, "enc.enc_2.0"), D2("enc.enc_2.1"),
                   ResidualBlockWithStride(ctx, "enc.enc_2.2"), D2("enc.enc_2.3")]
        self.e2c = ctx.conv("enc.enc_2.4", 2)
        # hyper (image_model.py:68-78)
        self.he0 = D2("hyper_enc.0", latent=True)
        self.he1 = ctx.conv("hyper_enc.1", 2, latent=True)
        self.he3 = ctx.conv("hyper_enc.3", 2, latent=True)
        self.hd = [ResidualBlockUpsample(ctx, "hyper_dec.0", latent=True),
                   ResidualBlockUpsample(ctx, "hyper_dec.1", latent=True), D2("hyper_dec.2", latent=True)]
        self.pf = [D2("y_prior_fusion.0", latent=True), D2("y_prior_fusion.1", latent=True)]
        self.prior = QuadtreePrior(ctx, [f"y_spatial_prior_adaptor_{i}" for i in (1, 2, 3)], "y_spatial_prior",
                                   self.N, gated=True)
        # IntraDecoder (image_model.py:38-58) + refine
        self.d1 = [D2("dec.dec_1.0"), ResidualBlockUpsample(ctx, "dec.dec_1.1"), D2("dec.dec_1.2"),
                   ResidualBlockUpsample(ctx, "dec.dec_1.3"), D2("dec.dec_1.4")]
        self.d1u = ResidualBlockUpsample(ctx, "dec.dec_1.5")
        self.d2 = D2("dec.dec_2.0")
        self.d2u = ResidualBlockUpsample(ctx, "dec.dec_2.1")
        self.refine_unet = UNet(ctx, "refine.0", gated=True)
        self.refine_conv = ctx.conv("refine.1")
        self.fine = {k: q_fine(sd[k]) for k in ("q_scale_enc", "q_scale_dec")}
        self._q_cache = {}
        if strict:
            ctx.check_strict([k for k in sd if k.startswith("bit_estimator") or k.startswith("q_")])
        # weights were packed / uploaded on this thread's stream: finish before
        # any other stream (a GOP lane) reads them
        if torch.device(self.dev).type == "cuda":
            torch.cuda.current_stream(self.dev).synchronize()
        return self

    # nn.Module calls test_video.py makes on the model (:301-302, :77)
    def to(self, device):
        return self

    def eval(self):
        return self

    def parameters(self):
        yield torch.empty(0, device=self.dev)

    def update(self, force=False):
        if self.entropy_coder is not None and not force:
            return
        self.entropy_coder = EntropyCoder(self.ec_thread, self.stream_part)
        self.scale_table = ScaleTable("gaussian")
        self.z_table = FactorizedTable(self.sd, "bit_estimator_z", self.N)

    @staticmethod
    def get_q_scales_from_ckpt(ckpt_path):
        ckpt = get_state_dict(ckpt_path)
        return ckpt["q_scale_enc"].reshape(-1), ckpt["q_scale_dec"].reshape(-1)

    def get_q_for_inference(self, q_in_ckpt, q_index):
        key = (bool(q_in_ckpt), int(q_index))
        if key not in self._q_cache:
            out = []
            for tab, basic in (("q_scale_enc", "q_basic_enc"), ("q_scale_dec", "q_basic_dec")):
                table = self.sd[tab].detach().float().cpu()[:, 0, 0, 0] if q_in_ckpt else self.fine[tab]
                out.append(curr_q(table, self.sd[basic], q_index, self.dev))
            self._q_cache[key] = out
        return self._q_cache[key]

    def _params(self, z_hat, yh, yw):
        p = z_hat
        for b in self.hd:
            p = b(p)
        p = self.pf[0](p)
        buf = self.prior.new_buffer(yh, yw)
        full = self.pf[1](p)
        crop_to(full, yh, yw, y=buf.ch(self.N, 3 * self.N))
        return buf

    def _decode_image(self, y_hat, q, clamp=True):
        """dec + refine; write mode clamps (image_model.py:251), estimate
        mode returns refine's output unclamped (image_model.py:129-130)."""
        f = y_hat
        for b in self.d1:
            f = b(f)
        f = self.d1u(f, scale=q)
        f = self.d2u(self.d2(f))
        f = self.refine_unet(f)
        return K.conv(self.refine_conv, f, out_dtype=F32, act=ACT_CLAMP01 if clamp else K.ACT_NONE)

    def _analysis(self, x, q_enc):
        """IntraEncoder + hyper encoder: (y, z_hat)."""
        f = self.e1(x)
        f = self.e1b(f, scale=q_enc)
        for b in self.e2:
            f = b(f)
        y = K.conv(self.e2c, f, out_dtype=F32)
        z = self.he0(pad_for_y(y))
        z = K.conv(self.he1, z, act=ACT_LRELU, slope=0.01)
        return y, K.conv(self.he3, z, act=K.ACT_ROUND)

    def forward(self, x, q_in_ckpt=False, q_index=None):
        """Estimate mode, image_model.py:114-149: Gaussian bits for y,
        factorized bits for z, summed on the GPU."""
        x = as_act(x)
        q_enc, q_dec = self.get_q_for_inference(q_in_ckpt, q_index)
        y, z_hat = self._analysis(x, q_enc)
        bc = BitCounter(self.dev, ("y", "z"))
        bc.factorized("z", z_hat, self.z_table)
        params = self._params(z_hat, y.H, y.W)
        y_hat = self.prior.estimate(y, params, bc.buffer("y", self.N * y.H * y.W), True)
        x_hat = self._decode_image(y_hat, q_dec, clamp=False)
        r = bits_result(bc.totals(), x.H * x.W, ("y", "z"))
        return {"x_hat": x_hat.nchw_view(), "bit": r["bit"], "bpp": r["bpp"], "bpp_y": r["bpp_y"],
                "bpp_z": r["bpp_z"]}

    def compress(self, x, q_in_ckpt, q_index):
        """image_model.py:198-229 (without the unused encoder recon)."""
        x = as_act(x)
        q_enc, _ = self.get_q_for_inference(q_in_ckpt, q_index)
        y, z_hat = self._analysis(x, q_enc)
        yh, yw = y.H, y.W
        params = self._params(z_hat, yh, yw)
        sb = SymbolBuffer(self.dev)
        c_z = sb.plan("z", self.N * z_hat.H * z_hat.W)
        c_y = [sb.plan("y", self.N // 4 * yh * yw) for _ in range(4)]
        sb.alloc()
        K.to_symbols(z_hat, sb.sym_slice(c_z))
        self.prior.encode(y, params, sb, c_y, self.scale_table)
        host = sb.to_host()
        ec = self.entropy_coder
        ec.reset()
        ec.encode(host[c_z][0], self.z_table.indexes(z_hat.H, z_hat.W), self.z_table.table)
        for c in c_y:
            ec.encode(host[c][0], host[c][1], self.scale_table.table)
        ec.flush()
        return {"bit_stream": ec.get_encoded_stream(), "x_hat": None}

    def decompress(self, bit_stream, height, width, q_in_ckpt, q_index):
        """image_model.py:231-252."""
        _, q_dec = self.get_q_for_inference(q_in_ckpt, q_index)
        ec = self.entropy_coder
        ec.set_stream(bit_stream)
        zh, zw = get_downsampled_shape(height, width, 64)
        yh, yw = get_downsampled_shape(height, width, 16)
        z = ec.decode(self.z_table.indexes(zh, zw), self.z_table.table)
        z_hat = K.empty(zh, zw, self.N, F32, self.dev)
        K.from_symbols(torch.from_numpy(z.copy()).to(self.dev), z_hat)
        params = self._params(z_hat, yh, yw)
        y_hat = self.prior.decode(params, lambda idx: ec.decode(idx, self.scale_table.table), self.scale_table)
        return {"x_hat": self._decode_image(y_hat, q_dec)}

    @split_guarded
    def encode_decode(self, x, q_in_ckpt, q_index, output_path=None, pic_width=None, pic_height=None):
        """image_model.py:169-196: write mode, or estimate mode when
        output_path is None."""
        if output_path is None:
            enc = self.forward(x, q_in_ckpt, q_index)
            return {"bit": enc["bit"], "x_hat": enc["x_hat"]}
        assert pic_height is not None and pic_width is not None
        enc = self.compress(x, q_in_ckpt, q_index)
        split_checkpoint(self, "compress")   # before the file is written
        encode_i(pic_height, pic_width, q_in_ckpt, q_index, enc["bit_stream"], output_path)
        bit = filesize(output_path) * 8
        height, width, q_in_ckpt, q_index, bit_stream = decode_i(output_path)
        dec = self.decompress(bit_stream, height, width, q_in_ckpt, q_index)
        split_checkpoint(self, "decompress")
        return {"bit": bit, "x_hat": dec["x_hat"].nchw_view()}
