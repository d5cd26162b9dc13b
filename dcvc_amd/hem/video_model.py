"""DCVC-HEM P-frame codec (DMC) on MI355X.

API of DCVC-HEM/src/models/video_model.py:136-515: ``DMC(anchor_num)``,
``load_state_dict``, ``update``, ``get_q_scales_from_ckpt``, ``compress``,
``decompress``, ``forward_one_frame`` and ``encode_decode(x, dpb,
output_path, pic_width, pic_height, mv_y_q_scale, y_q_scale)`` with the
reference's return dicts.  Frames and DPB entries are NHWC ``Act`` views on
the GPU (``x`` may also be a (1, 3, H, W) tensor).  In write mode the encoder
skips compress()'s reconstruction (:303-305), which the reference computes
and discards (encode_decode returns the decoder's dpb).
"""
import time

import torch

from .. import hip as K
from ..hip import F32, ACT_LRELU, ACT_CLAMP01
from ..layers import split_guarded, split_checkpoint, Ctx, Precision, SpyNet, Grids, ResidualBlockWithStride, hyper_enc, hyper_dec
from ..entropy import ScaleTable, FactorizedTable
from ..stream_helper import get_downsampled_shape, filesize, get_state_dict
from ..dc.common import SymbolBuffer, BitCounter, bits_result
from ..dc.video_model import as_act, dpb_in, Contexts
from .common import DualPrior, HemEntropyCoder, lower_bound_q, get_rounded_q
from .layers import ResBlock, EncTower, DecTower, UNet, Seq3, chunk3_to_buffer_order
from .stream_helper import encode_p, decode_p

CH_MV, CH_N, CH_M = 64, 64, 96  # video_model.py:140-142


class DMC:
    def __init__(self, anchor_num=4, precision=None, device=None):
        self.anchor_num = anchor_num
        self._init_kw = dict(anchor_num=anchor_num)
        self.prec = precision if precision is not None else Precision.split()
        self.dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.entropy_coder = None

    # ------------------------------------------------------------ building
    def load_state_dict(self, state_dict, strict=True):
        sd = {k: v for k, v in state_dict.items()}
        self.sd = sd
        ctx = Ctx(sd, self.dev, self.prec)
        self.ctx = ctx
        self.grids = Grids(self.dev)
        self.optic_flow = SpyNet(ctx, "optic_flow", self.grids)
        self.mv_enc = EncTower(ctx, "mv_encoder")
        self.mv_dec = DecTower(ctx, "mv_decoder")
        self.mv_henc = hyper_enc(ctx, "mv_hyper_prior_encoder", False)
        self.mv_hdec = hyper_dec(ctx, "mv_hyper_prior_decoder")
        self.mv_fusion = Seq3(ctx, "mv_y_prior_fusion", out_perm=chunk3_to_buffer_order(CH_MV))
        self.mv_prior = DualPrior(ctx, "mv_y_spatial_prior", CH_MV)
        self.fa_I = ctx.conv("feature_adaptor_I")
        self.fa_P = ctx.conv("feature_adaptor_P")
        fe = "feature_extractor"
        self.fe_c1, self.fe_r1 = ctx.conv(fe + ".conv1"), ResBlock(ctx, fe + ".res_block1")
        self.fe_c2, self.fe_r2 = ctx.conv(fe + ".conv2", 2), ResBlock(ctx, fe + ".res_block2")
        self.fe_c3, self.fe_r3 = ctx.conv(fe + ".conv3", 2), ResBlock(ctx, fe + ".res_block3")
        cf = "context_fusion_net"
        self.cf_c3up, self.cf_r3up = ctx.conv(cf + ".conv3_up.0"), ResBlock(ctx, cf + ".res_block3_up")
        self.cf_c3out, self.cf_r3out = ctx.conv(cf + ".conv3_out"), ResBlock(ctx, cf + ".res_block3_out")
        self.cf_c2up, self.cf_r2up = ctx.conv(cf + ".conv2_up.0"), ResBlock(ctx, cf + ".res_block2_up")
        self.cf_c2out, self.cf_r2out = ctx.conv(cf + ".conv2_out"), ResBlock(ctx, cf + ".res_block2_out")
        self.cf_c1out, self.cf_r1out = ctx.conv(cf + ".conv1_out"), ResBlock(ctx, cf + ".res_block1_out")
        ce = "contextual_encoder"
        # buffer order cat(context1, x, 0 x5), the reference's cat(x, context1)
        # by input permutation (aligned 64-channel copy)
        self.ce_c1 = ctx.conv(ce + ".conv1", 2, cin_pad=72, in_perm=list(range(3, 3 + CH_N)) + [0, 1, 2])
        self.ce_r1 = ResBlock(ctx, ce + ".res1", 0.1, True, True)
        self.ce_c2 = ctx.conv(ce + ".conv2", 2)
        self.ce_r2 = ResBlock(ctx, ce + ".res2", 0.1, True, True)
        self.ce_c3 = ctx.conv(ce + ".conv3", 2)
        self.ce_c4 = ctx.conv(ce + ".conv4", 2)
        self.y_henc = hyper_enc(ctx, "contextual_hyper_prior_encoder", True)
        self.y_hdec = hyper_dec(ctx, "contextual_hyper_prior_decoder")
        self.tpe0 = ctx.conv("temporal_prior_encoder.0", 2)
        self.tpe2 = ctx.conv("temporal_prior_encoder.2", 2)
        self.y_fusion = Seq3(ctx, "y_prior_fusion", out_perm=chunk3_to_buffer_order(CH_M))
        self.y_prior = DualPrior(ctx, "y_spatial_prior", CH_M)
        cd = "contextual_decoder"
        self.cd_up1, self.cd_up2 = ctx.conv(cd + ".up1.0"), ctx.conv(cd + ".up2.0")
        self.cd_r1 = ResBlock(ctx, cd + ".res1", 0.1, True, True)
        self.cd_up3 = ctx.conv(cd + ".up3.0")
        self.cd_r2 = ResBlock(ctx, cd + ".res2", 0.1, True, True)
        self.cd_up4 = ctx.conv(cd + ".up4.0")
        rg = "recon_generation_net"
        self.rg_first = ctx.conv(rg + ".first_conv")
        self.rg_u1, self.rg_u2 = UNet(ctx, rg + ".unet_1"), UNet(ctx, rg + ".unet_2")
        self.rg_out = ctx.conv(rg + ".recon_conv")
        self._q_cache = {}
        self._zpad = {}
        if strict:
            ctx.check_strict([k for k in sd if k.startswith("bit_estimator") or "_q_" in k])
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
        """CompressionModel.update (common_model.py:72-77)."""
        if self.entropy_coder is not None and not force:
            return
        self.entropy_coder = HemEntropyCoder()
        self.scale_table = ScaleTable("laplace")
        self.z_table = FactorizedTable(self.sd, "bit_estimator_z", CH_N)
        self.mvz_table = FactorizedTable(self.sd, "bit_estimator_z_mv", CH_MV)

    @staticmethod
    def get_q_scales_from_ckpt(ckpt_path):
        ckpt = get_state_dict(ckpt_path)
        return ckpt["y_q_scale"].reshape(-1), ckpt["mv_y_q_scale"].reshape(-1)

    def _q(self, mv_y_q_scale, y_q_scale):
        key = (float(mv_y_q_scale), float(y_q_scale))
        if key not in self._q_cache:
            self._q_cache[key] = (lower_bound_q(self.sd["mv_y_q_basic"], float(mv_y_q_scale), self.dev),
                                  lower_bound_q(self.sd["y_q_basic"], float(y_q_scale), self.dev))
        return self._q_cache[key]

    def _padded(self, key, H, W, C):
        k = (key, H, W)
        if k not in self._zpad:
            self._zpad[k] = K.zeros(H, W, C, self.prec.feat, self.dev)
        return self._zpad[k]

    # ---------------------------------------------------------- sub-graphs
    def _mv_params(self, mv_z_hat, ref_mv_y, yh, yw):
        """mv hyper decoder + mv_y_prior_fusion into the dual prior buffer."""
        cat = K.empty(yh, yw, 3 * CH_MV, F32, self.dev)
        self.mv_hdec(mv_z_hat, y=cat.ch(0, 2 * CH_MV))
        if ref_mv_y is None:
            K.fill(cat.ch(2 * CH_MV, CH_MV), 0.0)  # torch.zeros_like(mv_y) (:274-276)
        else:
            K.copy(ref_mv_y, cat.ch(2 * CH_MV, CH_MV))
        buf = self.mv_prior.new_buffer(yh, yw)
        self.mv_fusion(cat, y=self.mv_prior.params_view(buf))
        return buf

    def _y_params(self, z_hat, c3, ref_y, yh, yw):
        """temporal + hierarchical params + ref_y, y_prior_fusion (:286-297)."""
        cat = K.empty(yh, yw, 5 * CH_M, F32, self.dev)
        t = K.conv(self.tpe0, c3, act=ACT_LRELU, slope=0.1)
        K.conv(self.tpe2, t, cat.ch(0, 2 * CH_M))
        self.y_hdec(z_hat, y=cat.ch(2 * CH_M, 2 * CH_M))
        if ref_y is None:
            K.fill(cat.ch(4 * CH_M, CH_M), 0.0)  # torch.zeros_like(y) (:291-293)
        else:
            K.copy(ref_y, cat.ch(4 * CH_M, CH_M))
        buf = self.y_prior.new_buffer(yh, yw)
        self.y_fusion(cat, y=self.y_prior.params_view(buf))
        return buf

    def _motion_compensation(self, dpb, mv):
        """multi_scale_feature_extractor + motion_compensation +
        MultiScaleContextFusion (:17-68, 225-242)."""
        feat, dev = self.prec.feat, self.dev
        H, W = mv.H, mv.W
        mv2 = K.resize2x(mv, False, 0.5)
        mv3 = K.resize2x(mv2, False, 0.5)
        if dpb["ref_feature"] is None:
            f = K.conv(self.fa_I, dpb["ref_frame"], out_dtype=feat)
        else:
            f = K.conv(self.fa_P, dpb["ref_feature"])
        l1 = self.fe_r1(K.conv(self.fe_c1, f))
        l2 = self.fe_r2(K.conv(self.fe_c2, l1))
        l3 = self.fe_r3(K.conv(self.fe_c3, l2))
        cat1 = K.empty(H, W, 2 * CH_N, feat, dev)                      # cat(context2_up, context1)
        c1 = K.flow_warp(l1, mv, self.grids(H, W), y=cat1.ch(CH_N, CH_N))
        cat2 = K.empty(H // 2, W // 2, 2 * CH_N, feat, dev)            # cat(context3_up, context2)
        c2 = K.flow_warp(l2, mv2, self.grids(H // 2, W // 2), y=cat2.ch(CH_N, CH_N))
        c3 = K.flow_warp(l3, mv3, self.grids(H // 4, W // 4))
        # each context written straight into the concat buffers its consumers
        # read (dc.video_model.Contexts: b1 = cat(up4 (32), c1, x, 0 x5))
        ctx = Contexts(self, H, W, CH_N, CH_N, CH_N)
        self.cf_r3up(K.conv(self.cf_c3up, c3, shuffle=True), y=cat2.ch(0, CH_N))
        self.cf_r3out(K.conv(self.cf_c3out, c3), res2=c3, y=ctx.c3)
        self.cf_r2up(K.conv(self.cf_c2up, cat2, shuffle=True), y=cat1.ch(0, CH_N))
        self.cf_r2out(K.conv(self.cf_c2out, cat2), res2=c2, y=ctx.c2)
        self.cf_r1out(K.conv(self.cf_c1out, cat1), res2=c1, y=ctx.c1)
        return ctx

    def _contextual_encoder(self, x, ctx, yq):
        """ContextualEncoder (:71-95), then y / curr_y_q."""
        K.copy(x, ctx.b1.ch(32 + CH_N, 3))
        K.conv(self.ce_c1, ctx.b1.ch(32, 72), ctx.b2.ch(0, CH_N))     # cat(context1, x, 0 x5)
        f = self.ce_r1(ctx.b2)                                         # cat(., context2)
        K.conv(self.ce_c2, f, ctx.b3.ch(0, CH_N))
        f = self.ce_r2(ctx.b3)                                         # cat(., context3)
        f = K.conv(self.ce_c3, f)
        y = K.conv(self.ce_c4, f, out_dtype=F32)
        return K.channel_div(y, yq, y)

    def _recon(self, y_hat, ctx, clamp=True):
        """ContextualDecoder + ReconGeneration (:98-128)."""
        f = K.conv(self.cd_up1, y_hat, out_dtype=self.prec.feat, shuffle=True)
        K.conv(self.cd_up2, f, ctx.b3.ch(0, CH_N), shuffle=True)
        f = self.cd_r1(ctx.b3)                                         # cat(., context3)
        K.conv(self.cd_up3, f, ctx.b2.ch(0, CH_N), shuffle=True)
        f = self.cd_r2(ctx.b2)                                         # cat(., context2)
        K.conv(self.cd_up4, f, ctx.b1.ch(0, 32), shuffle=True)
        f = K.conv(self.rg_first, ctx.b1.ch(0, 32 + CH_N))            # cat(., context1)
        f = self.rg_u1(f)
        feature = self.rg_u2(f)
        x_hat = K.conv(self.rg_out, feature, out_dtype=F32, act=ACT_CLAMP01 if clamp else K.ACT_NONE)
        return x_hat, feature

    def _analysis(self, x, dpb, mvq, yq, mv_prior_fn, y_prior_fn, bc=None):
        """The encoder graph up to both dual priors; returns what the caller's
        prior functions returned and the contexts."""
        est_mv = self.optic_flow(x, dpb["ref_frame"])
        mv_y = self.mv_enc(est_mv)
        mv_y = K.channel_div(mv_y, mvq, mv_y)
        yh, yw = mv_y.H, mv_y.W
        mv_z_hat = self.mv_henc(mv_y)
        if bc is not None:
            bc.factorized("mv_z", mv_z_hat, self.mvz_table)
        mv_buf = self._mv_params(mv_z_hat, dpb["ref_mv_y"], yh, yw)
        mv_y_hat = mv_prior_fn(mv_y, mv_buf)
        mv_hat = self.mv_dec(mv_y_hat, out_dtype=F32)
        ctx = self._motion_compensation(dpb, mv_hat)
        y = self._contextual_encoder(x, ctx, yq)
        z_hat = self.y_henc(y)
        if bc is not None:
            bc.factorized("z", z_hat, self.z_table)
        buf = self._y_params(z_hat, ctx.c3, dpb["ref_y"], yh, yw)
        y_hat = y_prior_fn(y, buf)
        return mv_z_hat, mv_y_hat, z_hat, y_hat, ctx

    # --------------------------------------------------------------- codec
    def compress(self, x, dpb, mv_y_q_scale, y_q_scale):
        """video_model.py:263-330 without the discarded reconstruction."""
        x = as_act(x)
        dpb = dpb_in(dpb)
        mvq, yq = self._q(mv_y_q_scale, y_q_scale)
        H, W = x.H, x.W
        yh, yw = H // 16, W // 16
        zh, zw = H // 64, W // 64
        sb = SymbolBuffer(self.dev, torch.int32)
        c_mvz = sb.plan("mvz", CH_MV * zh * zw)
        c_mv = [sb.plan("y", CH_MV // 2 * yh * yw) for _ in range(2)]
        c_z = sb.plan("z", CH_N * zh * zw)
        c_y = [sb.plan("y", CH_M // 2 * yh * yw) for _ in range(2)]
        sb.alloc()
        st = self.scale_table

        def mv_prior(mv_y, buf):
            return self.mv_prior.encode(mv_y, buf, mvq, [sb.sym_slice(c) for c in c_mv],
                                        [sb.idx_slice(c) for c in c_mv], st)

        def y_prior(y, buf):
            return self.y_prior.encode(y, buf, yq, [sb.sym_slice(c) for c in c_y], [sb.idx_slice(c) for c in c_y],
                                       st)
        mv_z_hat, _, z_hat, _, _ = self._analysis(x, dpb, mvq, yq, mv_prior, y_prior)
        K.to_symbols_i32(mv_z_hat, sb.sym_slice(c_mvz))
        K.to_symbols_i32(z_hat, sb.sym_slice(c_z))
        host = sb.to_host()
        ec = self.entropy_coder
        ec.reset_encoder()
        ec.encode(host[c_mvz][0], self.mvz_table.indexes(zh, zw).astype("int32"), self.mvz_table.table)
        for c in c_mv:
            ec.encode(host[c][0], host[c][1].astype("int32"), st.table)
        ec.encode(host[c_z][0], self.z_table.indexes(zh, zw).astype("int32"), self.z_table.table)
        for c in c_y:
            ec.encode(host[c][0], host[c][1].astype("int32"), st.table)
        return {"dbp": None, "bit_stream": ec.flush_encoder()}

    def decompress(self, dpb, string, height, width, mv_y_q_scale, y_q_scale):
        """video_model.py:332-375."""
        mvq, yq = self._q(mv_y_q_scale, y_q_scale)
        dpb = dpb_in(dpb)
        ec, dev, st = self.entropy_coder, self.dev, self.scale_table
        ec.set_stream(string)
        zh, zw = get_downsampled_shape(height, width, 64)
        yh, yw = 4 * zh, 4 * zw  # the hyper decoders upsample z by 4 (HEM pads frames to 64)
        mvz = ec.decode(self.mvz_table.indexes(zh, zw).astype("int32"), self.mvz_table.table)
        mv_z_hat = K.empty(zh, zw, CH_MV, F32, dev)
        K.from_symbols_i32(K.upload(mvz, dev, "mv_z"), mv_z_hat)

        def dec(idx):
            return ec.decode(idx.astype("int32"), st.table)
        mv_buf = self._mv_params(mv_z_hat, dpb["ref_mv_y"], yh, yw)
        mv_y_hat = self.mv_prior.decode(mv_buf, mvq, dec, st)
        mv_hat = self.mv_dec(mv_y_hat, out_dtype=F32)
        ctx = self._motion_compensation(dpb, mv_hat)
        z = ec.decode(self.z_table.indexes(zh, zw).astype("int32"), self.z_table.table)
        z_hat = K.empty(zh, zw, CH_N, F32, dev)
        K.from_symbols_i32(K.upload(z, dev, "z"), z_hat)
        buf = self._y_params(z_hat, ctx.c3, dpb["ref_y"], yh, yw)
        y_hat = self.y_prior.decode(buf, yq, dec, st)
        x_hat, feature = self._recon(y_hat, ctx)
        return {"dpb": {"ref_frame": x_hat.nchw_view(), "ref_feature": feature, "ref_y": y_hat,
                        "ref_mv_y": mv_y_hat}}

    def forward_one_frame(self, x, dpb, mv_y_q_scale=None, y_q_scale=None):
        """Estimate mode (video_model.py:417-515), bits summed on the GPU.
        mse / ssim / BDQ entries of the reference's training outputs are not
        produced (MS-SSIM needs pytorch_msssim)."""
        x = as_act(x)
        dpb = dpb_in(dpb)
        mvq, yq = self._q(mv_y_q_scale, y_q_scale)
        H, W = x.H, x.W
        yh, yw = H // 16, W // 16
        bc = BitCounter(self.dev, ("mv_y", "mv_z", "y", "z"))

        def mv_prior(mv_y, buf):
            return self.mv_prior.estimate(mv_y, buf, mvq, bc.buffer("mv_y", CH_MV * yh * yw), False)

        def y_prior(y, buf):
            return self.y_prior.estimate(y, buf, yq, bc.buffer("y", CH_M * yh * yw), False)
        _, mv_y_hat, _, y_hat, ctx = self._analysis(x, dpb, mvq, yq, mv_prior, y_prior, bc)
        x_hat, feature = self._recon(y_hat, ctx, clamp=False)
        out = bits_result(bc.totals(), H * W, ("mv_y", "mv_z", "y", "z"))
        out["dpb"] = {"ref_frame": x_hat.nchw_view(), "ref_feature": feature, "ref_y": y_hat, "ref_mv_y": mv_y_hat}
        return out

    @split_guarded
    def encode_decode(self, x, dpb, output_path=None, pic_width=None, pic_height=None, mv_y_q_scale=None,
                      y_q_scale=None):
        """video_model.py:377-415."""
        if output_path is None:
            enc = self.forward_one_frame(x, dpb, mv_y_q_scale=mv_y_q_scale, y_q_scale=y_q_scale)
            return {"dpb": enc["dpb"], "bit_y": enc["bit_y"], "bit_z": enc["bit_z"], "bit_mv_y": enc["bit_mv_y"],
                    "bit_mv_z": enc["bit_mv_z"], "bit": enc["bit"], "decoding_time": 0}
        mv_y_q_scale, mv_y_q_index = get_rounded_q(mv_y_q_scale)
        y_q_scale, y_q_index = get_rounded_q(y_q_scale)
        enc = self.compress(x, dpb, mv_y_q_scale, y_q_scale)
        split_checkpoint(self, "compress")   # before the file is written
        encode_p(enc["bit_stream"], mv_y_q_index, y_q_index, output_path)
        bits = filesize(output_path) * 8
        mv_y_q_index, y_q_index, string = decode_p(output_path)
        torch.cuda.current_stream(self.dev).synchronize()
        start = time.time()
        dec = self.decompress(dpb, string, pic_height, pic_width, mv_y_q_index / 100, y_q_index / 100)
        split_checkpoint(self, "decompress")
        torch.cuda.current_stream(self.dev).synchronize()
        return {"dpb": dec["dpb"], "bit": bits, "decoding_time": time.time() - start}
