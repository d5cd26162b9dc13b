"""DCVC-DC P-frame codec (DMC) on MI355X.

API of DCVC-DC/src/models/video_model.py:235-628: ``DMC(anchor_num,
ec_thread, stream_part, inplace)``, ``load_state_dict``, ``update``,
``get_q_scales_from_ckpt``, ``compress``, ``decompress``, ``encode_decode``.
Frames and DPB entries are NHWC ``Act`` views on the GPU (``x`` may also be
passed as a (1, 3, H, W) tensor).  Write mode (``output_path`` given) is the
real-bitstream path; ``output_path=None`` runs estimate mode
(``forward_one_frame``) with the bits summed on the GPU.  The encoder skips compress()'s dead reconstruction
(video_model.py:468), whose output the reference discards in write mode.
"""
import time

import torch

from .. import hip as K
from ..hip import F32, ACT_LRELU, ACT_CLAMP01
from ..layers import (split_guarded, split_checkpoint, Ctx, Precision, DepthConvBlock, ResidualBlockWithStride, ResidualBlockUpsample,
                      ResBlock, UNet, SpyNet, Grids, hyper_enc, hyper_dec, cast)
from ..entropy import ScaleTable, FactorizedTable, EntropyCoder
from ..stream_helper import (get_downsampled_shape, encode_p, decode_p, filesize, get_state_dict)
from .common import SymbolBuffer, QuadtreePrior, BitCounter, bits_result, pad_for_y, crop_to, q_fine, curr_q

G1, G2, G4, G8, G16 = 48, 64, 96, 96, 128  # video_model.py:19-23


def as_act(x, dtype=F32):
    """Act view of a frame / DPB entry.  A (1, C, H, W) tensor that is the NCHW
    view of a contiguous NHWC buffer (Act.nchw_view, what encode_decode hands
    back to the harness) is wrapped without a copy; other tensors are copied
    into a fresh NHWC buffer."""
    if isinstance(x, K.Act):
        return x
    if x.dim() == 4 and x.shape[0] == 1 and x.is_cuda and x.dtype == K._TORCH[dtype]:
        hwc = x[0].permute(1, 2, 0)
        if hwc.is_contiguous():
            return K.Act(hwc)
    return K.from_nchw(x, dtype)


def dpb_in(dpb):
    return {k: (as_act(v) if isinstance(v, torch.Tensor) else v) for k, v in dpb.items()}


class Contexts:
    """The three contexts of MultiScaleContextFusion (video_model.py:103-118),
    each written by its producer straight into the concatenation its consumers
    read, so no context is copied into a concat buffer:
      b1 = cat(cd_up4 out (32), c1 (48), x (3), 0 x5) at full size: the
           contextual encoder reads channels 32..87 (its cat(c1, x, 0 x5)),
           the reconstruction channels 0..79 (cat(up4, c1));
      b2 = cat(first conv out, c2) at 1/2, b3 = cat(first conv out, c3) at 1/4:
           the encoder (video_model.py:173-195) and the reconstruction
           (:197-232) each write the first half, one after the other on the
           frame's stream, and read the context in the second.
    b1's pad channels stay zero (a cached buffer, allocated zeroed)."""

    def __init__(self, net, H, W, C1=G1, C2=G2, C3=G4):
        # (DCVC-HEM: 64 channels at every scale, its encoder's cat(c1, x, 0 x5) is 72 wide)
        feat, dev = net.prec.feat, net.dev
        self.b1 = net._padded("ctx1", H, W, 32 + C1 + 8)
        self.b2 = K.empty(H // 2, W // 2, 2 * C2, feat, dev)
        self.b3 = K.empty(H // 4, W // 4, 2 * C3, feat, dev)
        self.c1, self.c2, self.c3 = self.b1.ch(32, C1), self.b2.ch(C2, C2), self.b3.ch(C3, C3)

    def __iter__(self):   # c1, c2, c3 = ctx (diagnostics that checksum the contexts)
        return iter((self.c1, self.c2, self.c3))


class DMC:
    def __init__(self, anchor_num=4, ec_thread=False, stream_part=1, inplace=False, precision=None,
                 device=None):
        self.anchor_num = anchor_num
        self.ec_thread, self.stream_part = ec_thread, stream_part
        self._init_kw = dict(anchor_num=anchor_num, ec_thread=ec_thread, stream_part=stream_part, inplace=inplace)
        self.prec = precision if precision is not None else Precision.split()
        self.dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.entropy_coder = None
        self.sd = None

    # ------------------------------------------------------------ building
    def load_state_dict(self, state_dict, strict=True):
        sd = {k: v for k, v in state_dict.items()}
        self.sd = sd
        ctx = Ctx(sd, self.dev, self.prec)
        self.ctx = ctx
        self.grids = Grids(self.dev)
        self.optic_flow = SpyNet(ctx, "optic_flow", self.grids)
        # OffsetDiversity (video_model.py:26-63)
        self.off_c0 = ctx.conv("align.conv_offset.0", 2, cin_pad=56)
        self.off_c2 = ctx.conv("align.conv_offset.2")
        self.off_c4 = ctx.conv("align.conv_offset.4")
        self.fusion_w = ctx.take("align.fusion.weight").detach().float().reshape(48, 6).contiguous().to(self.dev)
        self.fusion_b = ctx.take("align.fusion.bias").detach().float().contiguous().to(self.dev)
        # MvEnc (video_model.py:121-146)
        self.me1 = ResidualBlockWithStride(ctx, "mv_encoder.enc_1.0")
        self.me1b = DepthConvBlock(ctx, "mv_encoder.enc_1.1")
        self.me2 = ResidualBlockWithStride(ctx, "mv_encoder.enc_2")
        self.me_ad0 = DepthConvBlock(ctx, "mv_encoder.adaptor_0")
        self.me_ad1 = DepthConvBlock(ctx, "mv_encoder.adaptor_1")
        self.me3 = ResidualBlockWithStride(ctx, "mv_encoder.enc_3.0")
        self.me3b = DepthConvBlock(ctx, "mv_encoder.enc_3.1")
        self.me3c = ctx.conv("mv_encoder.enc_3.2", 2)
        self.mv_henc = hyper_enc(ctx, "mv_hyper_prior_encoder", False)
        self.mv_hdec = hyper_dec(ctx, "mv_hyper_prior_decoder")
        self.mv_fa0 = DepthConvBlock(ctx, "mv_y_prior_fusion_adaptor_0", latent=True)
        self.mv_fa1 = DepthConvBlock(ctx, "mv_y_prior_fusion_adaptor_1", latent=True)
        self.mv_f = [DepthConvBlock(ctx, f"mv_y_prior_fusion.{i}", latent=True) for i in range(2)]
        self.mv_prior = QuadtreePrior(ctx, [f"mv_y_spatial_prior_adaptor_{i}" for i in (1, 2, 3)],
                                      "mv_y_spatial_prior", 64, gated=False)
        # MvDec (video_model.py:149-170)
        self.md = [DepthConvBlock(ctx, "mv_decoder.dec_1.0"), ResidualBlockUpsample(ctx, "mv_decoder.dec_1.1"),
                   DepthConvBlock(ctx, "mv_decoder.dec_1.2"), ResidualBlockUpsample(ctx, "mv_decoder.dec_1.3"),
                   DepthConvBlock(ctx, "mv_decoder.dec_1.4")]
        self.md2 = ResidualBlockUpsample(ctx, "mv_decoder.dec_2")
        self.md3 = DepthConvBlock(ctx, "mv_decoder.dec_3.0")
        self.md3c = ctx.conv("mv_decoder.dec_3.1.0")
        # feature extraction + context fusion (video_model.py:66-118, 343-364)
        self.fa_I = ctx.conv("feature_adaptor_I")
        self.fa = [ctx.conv(f"feature_adaptor.{i}") for i in range(3)]
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
        # contextual encoder / decoder / recon (video_model.py:173-232)
        ce = "contextual_encoder"
        # buffer order cat(c1, x, 0 x5): the 48 context channels at offset 0
        # (16-byte aligned copy), the reference's cat(x, c1) by input permutation
        self.ce_c1 = ctx.conv(ce + ".conv1", 2, cin_pad=56, in_perm=list(range(3, 3 + G1)) + [0, 1, 2])
        self.ce_r1 = ResBlock(ctx, ce + ".res1", 0.1, True)
        self.ce_c2 = ctx.conv(ce + ".conv2", 2)
        self.ce_r2 = ResBlock(ctx, ce + ".res2", 0.1, True)
        self.ce_c3 = ctx.conv(ce + ".conv3", 2)
        self.ce_c4 = ctx.conv(ce + ".conv4", 2)
        self.y_henc = hyper_enc(ctx, "contextual_hyper_prior_encoder", True)
        self.y_hdec = hyper_dec(ctx, "contextual_hyper_prior_decoder")
        self.tpe0 = ctx.conv("temporal_prior_encoder.0", 2)
        self.tpe2 = ctx.conv("temporal_prior_encoder.2", 2)
        self.y_fa0 = DepthConvBlock(ctx, "y_prior_fusion_adaptor_0", latent=True)
        self.y_fa1 = DepthConvBlock(ctx, "y_prior_fusion_adaptor_1", latent=True)
        self.y_f = [DepthConvBlock(ctx, f"y_prior_fusion.{i}", latent=True) for i in range(2)]
        self.y_prior = QuadtreePrior(ctx, [f"y_spatial_prior_adaptor_{i}" for i in (1, 2, 3)],
                                     "y_spatial_prior", G16, gated=False)
        cd = "contextual_decoder"
        self.cd_up1, self.cd_up2 = ctx.conv(cd + ".up1.0"), ctx.conv(cd + ".up2.0")
        self.cd_r1 = ResBlock(ctx, cd + ".res1", 0.1, True)
        self.cd_up3 = ctx.conv(cd + ".up3.0")
        self.cd_r2 = ResBlock(ctx, cd + ".res2", 0.1, True)
        self.cd_up4 = ctx.conv(cd + ".up4.0")
        rg = "recon_generation_net"
        self.rg_first = ctx.conv(rg + ".first_conv")
        self.rg_u1, self.rg_u2 = UNet(ctx, rg + ".unet_1"), UNet(ctx, rg + ".unet_2")
        self.rg_out = ctx.conv(rg + ".recon_conv")
        # q tables (video_model.py:325-341)
        self.fine = {k: q_fine(sd[k]) for k in
                     ("mv_y_q_scale_enc", "mv_y_q_scale_dec", "y_q_scale_enc", "y_q_scale_dec")}
        self._q_cache = {}
        self._zpad = {}
        if strict:
            ctx.check_strict([k for k in sd if k.startswith("bit_estimator") or "_q_" in k])
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
        """CompressionModel.update (common_model.py:63-68)."""
        if self.entropy_coder is not None and not force:
            return
        self.entropy_coder = EntropyCoder(self.ec_thread, self.stream_part)
        self.scale_table = ScaleTable("laplace")
        self.z_table = FactorizedTable(self.sd, "bit_estimator_z", G16)
        self.mvz_table = FactorizedTable(self.sd, "bit_estimator_z_mv", 64)

    @staticmethod
    def get_q_scales_from_ckpt(ckpt_path):
        ckpt = get_state_dict(ckpt_path)
        return tuple(ckpt[k].reshape(-1) for k in
                     ("y_q_scale_enc", "y_q_scale_dec", "mv_y_q_scale_enc", "mv_y_q_scale_dec"))

    def get_q_for_inference(self, q_in_ckpt, q_index):
        key = (bool(q_in_ckpt), int(q_index))
        if key not in self._q_cache:
            out = []
            for tab, basic in (("mv_y_q_scale_enc", "mv_y_q_basic_enc"), ("mv_y_q_scale_dec", "mv_y_q_basic_dec"),
                               ("y_q_scale_enc", "y_q_basic_enc"), ("y_q_scale_dec", "y_q_basic_dec")):
                table = self.sd[tab].detach().float().cpu() if q_in_ckpt else self.fine[tab]
                out.append(curr_q(table, self.sd[basic], q_index, self.dev))
            self._q_cache[key] = out
        return self._q_cache[key]

    def _padded(self, key, H, W, C):
        """A cached concat buffer of C channels whose channels beyond the ones
        the producers write stay zero (allocated zeroed once per shape)."""
        k = (key, H, W)
        if k not in self._zpad:
            self._zpad[k] = K.zeros(H, W, C, self.prec.feat, self.dev)
        return self._zpad[k]

    # ---------------------------------------------------------- sub-graphs
    def _mv_encoder(self, est_mv, ref_mv_feature, q):
        out = self.me1(est_mv)
        out = self.me1b(out, scale=q)
        out = self.me2(out)
        if ref_mv_feature is None:
            out = self.me_ad0(out)
        else:
            cat = K.empty(out.H, out.W, out.C + ref_mv_feature.C, self.prec.feat, self.dev)
            K.copy(out, cat.ch(0, out.C))
            K.copy(ref_mv_feature, cat.ch(out.C, ref_mv_feature.C))
            out = self.me_ad1(cat)
        out = self.me3(out)
        out = self.me3b(out)
        return K.conv(self.me3c, out, out_dtype=F32)

    def _mv_prior_params(self, mv_z_hat, dpb, yh, yw):
        p = crop_to(self.mv_hdec(mv_z_hat), yh, yw)
        buf = self.mv_prior.new_buffer(yh, yw)
        if dpb["ref_mv_y"] is None:
            p = self.mv_fa0(p)
        else:
            cat = K.empty(yh, yw, 128, F32, self.dev)
            K.copy(p, cat.ch(0, 64))
            K.copy(dpb["ref_mv_y"], cat.ch(64, 64))
            p = self.mv_fa1(cat)
        p = self.mv_f[0](p)
        self.mv_f[1](p, y=buf.ch(64, 192))
        return buf

    def _res_prior_params(self, z_hat, dpb, c3, yh, yw):
        C = G16
        cat = K.empty(yh, yw, 3 * C if dpb["ref_y"] is not None else 2 * C, F32, self.dev)
        t = K.conv(self.tpe0, c3, act=ACT_LRELU, slope=0.1)
        K.conv(self.tpe2, t, cat.ch(0, C))                                # temporal params
        h = self.y_hdec(z_hat)                                           # hierarchical params
        crop_to(h, yh, yw, y=cat.ch(C, C))
        if dpb["ref_y"] is not None:
            K.copy(dpb["ref_y"], cat.ch(2 * C, C))
            p = self.y_fa1(cat)
        else:
            p = self.y_fa0(cat)
        buf = self.y_prior.new_buffer(yh, yw)
        p = self.y_f[0](p)
        self.y_f[1](p, y=buf.ch(C, 3 * C))
        return buf

    def _mv_decoder(self, mv_y_hat, q):
        f = mv_y_hat
        for b in self.md:
            f = b(f)
        out = self.md2(f, scale=q)
        out = self.md3(out)
        mv = K.conv(self.md3c, out, out_dtype=F32, shuffle=True)
        return mv, f

    def _motion_compensation(self, dpb, mv, frame_idx):
        """motion_compensation + OffsetDiversity + MultiScaleContextFusion."""
        feat, dev = self.prec.feat, self.dev
        H, W = mv.H, mv.W
        ref = dpb["ref_frame"]
        aux = self._padded("aux", H, W, 56)                             # cat(c1_init, warpframe, mv, 0 x3)
        K.flow_warp(ref, mv, self.grids(H, W), y=aux.ch(G1, 3))
        mv2 = K.resize2x(mv, False, 0.5)
        mv3 = K.resize2x(mv2, False, 0.5)
        if dpb["ref_feature"] is None:
            f = K.conv(self.fa_I, ref, out_dtype=feat)
        else:
            f = K.conv(self.fa[[0, 1, 0, 2][frame_idx % 4]], dpb["ref_feature"])
        r1 = self.fe_r1(K.conv(self.fe_c1, f))
        r2 = self.fe_r2(K.conv(self.fe_c2, r1))
        r3 = self.fe_r3(K.conv(self.fe_c3, r2))
        K.flow_warp(r1, mv, self.grids(H, W), y=aux.ch(0, G1))
        K.copy(mv, aux.ch(G1 + 3, 2))
        o = K.conv(self.off_c0, aux, act=ACT_LRELU, slope=0.1)  # 56 = 53 + 3 zero channels
        o = K.conv(self.off_c2, o, act=ACT_LRELU, slope=0.1)
        o = K.conv(self.off_c4, o, out_dtype=F32)
        cat1 = K.empty(H, W, G1 + G1, feat, dev)                       # cat(c2_up, c1)
        c1 = K.offset_diversity(r1, o, mv, self.fusion_w, self.fusion_b, self.grids(H, W), y=cat1.ch(G1, G1))
        cat2 = K.empty(H // 2, W // 2, G2 + G2, feat, dev)             # cat(c3_up, c2)
        c2 = K.flow_warp(r2, mv2, self.grids(H // 2, W // 2), y=cat2.ch(G2, G2))
        c3 = K.flow_warp(r3, mv3, self.grids(H // 4, W // 4))
        # MultiScaleContextFusion (video_model.py:103-118), each context
        # written straight into the concat buffers its consumers read (Contexts)
        ctx = Contexts(self, H, W)
        self.cf_r3up(K.conv(self.cf_c3up, c3, shuffle=True), y=cat2.ch(0, G2))
        self.cf_r3out(K.conv(self.cf_c3out, c3), res2=c3, y=ctx.c3)
        self.cf_r2up(K.conv(self.cf_c2up, cat2, shuffle=True), y=cat1.ch(0, G1))
        self.cf_r2out(K.conv(self.cf_c2out, cat2), res2=c2, y=ctx.c2)
        self.cf_r1out(K.conv(self.cf_c1out, cat1), res2=c1, y=ctx.c1)
        return ctx

    def _contextual_encoder(self, x, ctx, q):
        K.copy(x, ctx.b1.ch(32 + G1, 3))
        K.conv(self.ce_c1, ctx.b1.ch(32, 56), ctx.b2.ch(0, G2))       # cat(c1, x, 0 x5)
        f = self.ce_r1(ctx.b2, scale=q)                                # cat(., c2)
        K.conv(self.ce_c2, f, ctx.b3.ch(0, G4))
        f = self.ce_r2(ctx.b3)                                         # cat(., c3)
        f = K.conv(self.ce_c3, f)
        return K.conv(self.ce_c4, f, out_dtype=F32)

    def _recon(self, y_hat, ctx, q):
        """get_recon_and_feature (video_model.py:401-405)."""
        feat = self.prec.feat
        f = K.conv(self.cd_up1, y_hat, out_dtype=feat, shuffle=True)
        K.conv(self.cd_up2, f, ctx.b3.ch(0, G4), shuffle=True)
        f = self.cd_r1(ctx.b3)                                         # cat(., c3)
        K.conv(self.cd_up3, f, ctx.b2.ch(0, G2), shuffle=True, scale=q)
        f = self.cd_r2(ctx.b2)                                         # cat(., c2)
        K.conv(self.cd_up4, f, ctx.b1.ch(0, 32), shuffle=True)
        f = K.conv(self.rg_first, ctx.b1.ch(0, 32 + G1))              # cat(., c1)
        f = self.rg_u1(f)
        feature = self.rg_u2(f)
        x_hat = K.conv(self.rg_out, feature, out_dtype=F32, act=ACT_CLAMP01)
        return x_hat, feature

    # --------------------------------------------------------------- codec
    def compress(self, x, dpb, q_in_ckpt, q_index, frame_idx):
        """video_model.py:425-481.  Returns {"bit_stream": bytes, "dpb": None}
        (the encoder-side reconstruction is not computed: write mode returns
        the decoder's dpb, which is bit-identical)."""
        x = as_act(x)
        dpb = dpb_in(dpb)
        mv_q_enc, mv_q_dec, y_q_enc, y_q_dec = self.get_q_for_inference(q_in_ckpt, q_index)
        dev = self.dev
        est_mv = self.optic_flow(x, dpb["ref_frame"])
        mv_y = self._mv_encoder(est_mv, dpb["ref_mv_feature"], mv_q_enc)
        yh, yw = mv_y.H, mv_y.W
        mv_z_hat = self.mv_henc(pad_for_y(mv_y))
        mv_params = self._mv_prior_params(mv_z_hat, dpb, yh, yw)

        sb = SymbolBuffer(dev)
        zn = mv_z_hat.H * mv_z_hat.W
        c_mvz = sb.plan("mvz", 64 * zn)
        c_z = sb.plan("z", G16 * zn)
        c_mv = [sb.plan("y", 16 * yh * yw) for _ in range(4)]
        c_y = [sb.plan("y", 32 * yh * yw) for _ in range(4)]
        sb.alloc()
        K.to_symbols(mv_z_hat, sb.sym_slice(c_mvz))
        mv_y_hat = self.mv_prior.encode(mv_y, mv_params, sb, c_mv, self.scale_table)
        mv_hat, _ = self._mv_decoder(mv_y_hat, mv_q_dec)
        ctx = self._motion_compensation(dpb, mv_hat, frame_idx)
        y = self._contextual_encoder(x, ctx, y_q_enc)
        z_hat = self.y_henc(pad_for_y(y))
        K.to_symbols(z_hat, sb.sym_slice(c_z))
        params = self._res_prior_params(z_hat, dpb, ctx.c3, yh, yw)
        self.y_prior.encode(y, params, sb, c_y, self.scale_table)
        host = sb.to_host()

        ec = self.entropy_coder
        ec.reset()
        zh, zw = mv_z_hat.H, mv_z_hat.W
        ec.encode(host[c_mvz][0], self.mvz_table.indexes(zh, zw), self.mvz_table.table)
        ec.encode(host[c_z][0], self.z_table.indexes(zh, zw), self.z_table.table)
        for c in c_mv + c_y:
            ec.encode(host[c][0], host[c][1], self.scale_table.table)
        ec.flush()
        return {"dpb": None, "bit_stream": ec.get_encoded_stream()}

    def decompress(self, dpb, string, height, width, q_in_ckpt, q_index, frame_idx):
        """video_model.py:483-520."""
        _, mv_q_dec, _, y_q_dec = self.get_q_for_inference(q_in_ckpt, q_index)
        dpb = dpb_in(dpb)
        ec, dev = self.entropy_coder, self.dev
        ec.set_stream(string)
        zh, zw = get_downsampled_shape(height, width, 64)
        yh, yw = get_downsampled_shape(height, width, 16)
        mvz = ec.decode(self.mvz_table.indexes(zh, zw), self.mvz_table.table)
        z = ec.decode(self.z_table.indexes(zh, zw), self.z_table.table)
        zs = K.upload(mvz, dev, "mv_z")
        mv_z_hat = K.empty(zh, zw, 64, F32, dev)
        K.from_symbols(zs, mv_z_hat)
        zs2 = K.upload(z, dev, "z")
        z_hat = K.empty(zh, zw, G16, F32, dev)
        K.from_symbols(zs2, z_hat)

        def dec(idx):
            return ec.decode(idx, self.scale_table.table)

        mv_params = self._mv_prior_params(mv_z_hat, dpb, yh, yw)
        mv_y_hat = self.mv_prior.decode(mv_params, dec, self.scale_table)
        mv_hat, mv_feature = self._mv_decoder(mv_y_hat, mv_q_dec)
        ctx = self._motion_compensation(dpb, mv_hat, frame_idx)
        params = self._res_prior_params(z_hat, dpb, ctx.c3, yh, yw)
        y_hat = self.y_prior.decode(params, dec, self.scale_table)
        x_hat, feature = self._recon(y_hat, ctx, y_q_dec)
        return {"dpb": {"ref_frame": x_hat.nchw_view(), "ref_feature": feature, "ref_mv_feature": mv_feature,
                        "ref_y": y_hat, "ref_mv_y": mv_y_hat}}

    def forward_one_frame(self, x, dpb, q_in_ckpt=False, q_index=None, frame_idx=0):
        """Estimate mode, video_model.py:559-628: the encoder graph with the
        four-part prior run in estimate form, the reconstruction, and the
        estimated bits (Laplace bits for y / mv_y, factorized bits for z /
        mv_z) summed on the GPU.  Returns the reference's dict with Python
        floats for the bpp / bit entries."""
        x = as_act(x)
        dpb = dpb_in(dpb)
        mv_q_enc, mv_q_dec, y_q_enc, y_q_dec = self.get_q_for_inference(q_in_ckpt, q_index)
        bc = BitCounter(self.dev, ("mv_y", "mv_z", "y", "z"))
        est_mv = self.optic_flow(x, dpb["ref_frame"])
        mv_y = self._mv_encoder(est_mv, dpb["ref_mv_feature"], mv_q_enc)
        yh, yw = mv_y.H, mv_y.W
        mv_z_hat = self.mv_henc(pad_for_y(mv_y))
        bc.factorized("mv_z", mv_z_hat, self.mvz_table)
        mv_params = self._mv_prior_params(mv_z_hat, dpb, yh, yw)
        mv_y_hat = self.mv_prior.estimate(mv_y, mv_params, bc.buffer("mv_y", 64 * yh * yw), False)
        mv_hat, mv_feature = self._mv_decoder(mv_y_hat, mv_q_dec)
        ctx = self._motion_compensation(dpb, mv_hat, frame_idx)
        y = self._contextual_encoder(x, ctx, y_q_enc)
        z_hat = self.y_henc(pad_for_y(y))
        bc.factorized("z", z_hat, self.z_table)
        params = self._res_prior_params(z_hat, dpb, ctx.c3, yh, yw)
        y_hat = self.y_prior.estimate(y, params, bc.buffer("y", G16 * yh * yw), False)
        x_hat, feature = self._recon(y_hat, ctx, y_q_dec)
        out = bits_result(bc.totals(), x.H * x.W, ("mv_y", "mv_z", "y", "z"))
        out["dpb"] = {"ref_frame": x_hat.nchw_view(), "ref_feature": feature, "ref_mv_feature": mv_feature,
                      "ref_y": y_hat, "ref_mv_y": mv_y_hat}
        return out

    @split_guarded
    def encode_decode(self, x, dpb, q_in_ckpt, q_index, output_path=None, pic_width=None, pic_height=None,
                      frame_idx=0):
        """video_model.py:522-557: write mode (output_path given: real
        bitstream through a file, bit = filesize * 8) or estimate mode."""
        if output_path is None:
            enc = self.forward_one_frame(x, dpb, q_in_ckpt=q_in_ckpt, q_index=q_index, frame_idx=frame_idx)
            return {"dpb": enc["dpb"], "bit": enc["bit"], "encoding_time": 0, "decoding_time": 0}
        torch.cuda.current_stream(self.dev).synchronize()
        t0 = time.time()
        enc = self.compress(x, dpb, q_in_ckpt, q_index, frame_idx)
        split_checkpoint(self, "compress")   # before the file is written
        encode_p(enc["bit_stream"], q_in_ckpt, q_index, frame_idx, output_path)
        bits = filesize(output_path) * 8
        torch.cuda.current_stream(self.dev).synchronize()
        t1 = time.time()
        q_in_ckpt, q_index, frame_idx, string = decode_p(output_path)
        dec = self.decompress(dpb, string, pic_height, pic_width, q_in_ckpt, q_index, frame_idx)
        split_checkpoint(self, "decompress")
        torch.cuda.current_stream(self.dev).synchronize()
        t2 = time.time()
        return {"dpb": dec["dpb"], "bit": bits, "encoding_time": t1 - t0, "decoding_time": t2 - t1}
