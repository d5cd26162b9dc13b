"""DCVC-HEM intra codec (IntraNoAR) on MI355X.

API of DCVC-HEM/src/models/image_model.py:15-171: ``IntraNoAR(N,
anchor_num)``, ``load_state_dict``, ``update``, ``get_q_scales_from_ckpt``,
``compress``, ``decompress``, ``forward`` (estimate mode) and
``encode_decode(x, q_scale, output_path, pic_width, pic_height)``.
"""
import torch

from .. import hip as K
from ..hip import F32, ACT_CLAMP01
from ..layers import split_guarded, split_checkpoint, Ctx, Precision, hyper_enc, hyper_dec
from ..entropy import ScaleTable, FactorizedTable
from ..stream_helper import get_downsampled_shape, filesize, get_state_dict
from ..dc.common import SymbolBuffer, BitCounter, bits_result
from ..dc.video_model import as_act
from .common import DualPrior, HemEntropyCoder, lower_bound_q, get_rounded_q
from .layers import EncTower, DecTower, UNet, Seq3, chunk3_to_buffer_order
from .stream_helper import encode_i, decode_i


class IntraNoAR:
    def __init__(self, N=192, anchor_num=4, precision=None, device=None):
        self.N = N
        self.anchor_num = anchor_num
        self._init_kw = dict(N=N, anchor_num=anchor_num)
        self.prec = precision if precision is not None else Precision.split()
        self.dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.entropy_coder = None

    def load_state_dict(self, state_dict, strict=True):
        sd = {k: v for k, v in state_dict.items()}
        self.sd = sd
        ctx = Ctx(sd, self.dev, self.prec)
        self.ctx = ctx
        N = self.N
        self.enc = EncTower(ctx, "enc")
        self.dec = DecTower(ctx, "dec")
        self.refine_unet = UNet(ctx, "refine.0")
        self.refine_conv = ctx.conv("refine.1")
        self.henc = hyper_enc(ctx, "hyper_enc", False)
        self.hdec = hyper_dec(ctx, "hyper_dec")
        self.fusion = Seq3(ctx, "y_prior_fusion", out_perm=chunk3_to_buffer_order(N))
        self.prior = DualPrior(ctx, "y_spatial_prior", N)
        self._q_cache = {}
        if strict:
            ctx.check_strict([k for k in sd if k.startswith("bit_estimator") or k.startswith("q_")])
        # weights were packed / uploaded on this thread's stream: finish before
        # any other stream (a GOP lane) reads them
        if torch.device(self.dev).type == "cuda":
            torch.cuda.current_stream(self.dev).synchronize()
        return self

    def to(self, device):
        return self

    def eval(self):
        return self

    def parameters(self):
        yield torch.empty(0, device=self.dev)

    def update(self, force=False):
        if self.entropy_coder is not None and not force:
            return
        self.entropy_coder = HemEntropyCoder()
        self.scale_table = ScaleTable("gaussian")
        self.z_table = FactorizedTable(self.sd, "bit_estimator_z", self.N)

    @staticmethod
    def get_q_scales_from_ckpt(ckpt_path):
        return get_state_dict(ckpt_path)["q_scale"].reshape(-1)

    def _q(self, q_scale):
        key = float(q_scale)
        if key not in self._q_cache:
            self._q_cache[key] = lower_bound_q(self.sd["q_basic"], key, self.dev)
        return self._q_cache[key]

    def _params(self, z_hat):
        """hyper_dec + y_prior_fusion into the dual prior buffer (:58-60)."""
        p = self.hdec(z_hat)
        buf = self.prior.new_buffer(p.H, p.W)
        self.fusion(p, y=self.prior.params_view(buf))
        return buf

    def _analysis(self, x, q):
        y = self.enc(x)
        y = K.channel_div(y, q, y)
        return y, self.henc(y)

    def _synthesis(self, y_hat, clamp):
        f = self.dec(y_hat)
        f = self.refine_unet(f)
        return K.conv(self.refine_conv, f, out_dtype=F32, act=ACT_CLAMP01 if clamp else K.ACT_NONE)

    def compress(self, x, q_scale):
        """image_model.py:134-157."""
        x = as_act(x)
        q = self._q(q_scale)
        y, z_hat = self._analysis(x, q)
        yh, yw = y.H, y.W
        sb = SymbolBuffer(self.dev, torch.int32)
        c_z = sb.plan("z", self.N * z_hat.H * z_hat.W)
        c_y = [sb.plan("y", self.N // 2 * yh * yw) for _ in range(2)]
        sb.alloc()
        K.to_symbols_i32(z_hat, sb.sym_slice(c_z))
        buf = self._params(z_hat)
        self.prior.encode(y, buf, q, [sb.sym_slice(c) for c in c_y], [sb.idx_slice(c) for c in c_y],
                          self.scale_table)
        host = sb.to_host()
        ec = self.entropy_coder
        ec.reset_encoder()
        ec.encode(host[c_z][0], self.z_table.indexes(z_hat.H, z_hat.W).astype("int32"), self.z_table.table)
        for c in c_y:
            ec.encode(host[c][0], host[c][1].astype("int32"), self.scale_table.table)
        return {"bit_stream": ec.flush_encoder()}

    def decompress(self, bit_stream, height, width, q_scale):
        """image_model.py:159-171."""
        q = self._q(q_scale)
        ec = self.entropy_coder
        ec.set_stream(bit_stream)
        zh, zw = get_downsampled_shape(height, width, 64)
        z = ec.decode(self.z_table.indexes(zh, zw).astype("int32"), self.z_table.table)
        z_hat = K.empty(zh, zw, self.N, F32, self.dev)
        K.from_symbols_i32(torch.from_numpy(z.copy()).to(self.dev), z_hat)
        buf = self._params(z_hat)
        y_hat = self.prior.decode(buf, q, lambda idx: ec.decode(idx.astype("int32"), self.scale_table.table),
                                  self.scale_table)
        return {"x_hat": self._synthesis(y_hat, clamp=True)}

    def forward(self, x, q_scale=None):
        """Estimate mode (image_model.py:53-99); the mse / ssim entries of
        the reference's dict are not produced."""
        x = as_act(x)
        q = self._q(q_scale)
        y, z_hat = self._analysis(x, q)
        bc = BitCounter(self.dev, ("y", "z"))
        bc.factorized("z", z_hat, self.z_table)
        buf = self._params(z_hat)
        y_hat = self.prior.estimate(y, buf, q, bc.buffer("y", self.N * y.H * y.W), True)
        x_hat = self._synthesis(y_hat, clamp=False)
        r = bits_result(bc.totals(), x.H * x.W, ("y", "z"))
        return {"x_hat": x_hat.nchw_view(), "bit": r["bit"], "bpp": r["bpp"], "bpp_y": r["bpp_y"],
                "bpp_z": r["bpp_z"]}

    @split_guarded
    def encode_decode(self, x, q_scale, output_path=None, pic_width=None, pic_height=None):
        """image_model.py:106-131."""
        if output_path is None:
            return self.forward(x, q_scale)
        assert pic_height is not None and pic_width is not None
        q_scale, q_index = get_rounded_q(q_scale)
        enc = self.compress(x, q_scale)
        split_checkpoint(self, "compress")   # before the file is written
        encode_i(pic_height, pic_width, q_index, enc["bit_stream"], output_path)
        bit = filesize(output_path) * 8
        height, width, q_index, bit_stream = decode_i(output_path)
        dec = self.decompress(bit_stream, height, width, q_index / 100)
        split_checkpoint(self, "decompress")
        return {"bit": bit, "x_hat": dec["x_hat"].nchw_view()}
