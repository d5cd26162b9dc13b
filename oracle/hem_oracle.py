"""DCVC-HEM CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/ (and ``__graft_entry__.smoke()``) may import this module, and only
as the checker.  The product path (``dcvc_amd``) never imports it.

A functional restatement, in plain PyTorch fp32 on the CPU, of the DCVC-HEM
P-frame codec (``DMC``) and intra codec (``IntraNoAR``) in write mode
(compress / decompress around an entropy coder) and estimate mode
(forward_one_frame / forward), driven by a reference-format state_dict.
Every function cites the reference code it follows (paths relative to
/root/reference/DCVC-HEM/src).  The op order is the reference's, so on the
CPU the results are bitwise equal to it; tests/test_oracle_hem.py pins that
against the fixtures tests/golden/make_golden_hem.py recorded from the
reference itself.
"""
import torch
import torch.nn.functional as F

from .dc_oracle import (Params, conv, lrelu, subpel, flow_warp, down2, spynet, EntropyTables, bit_estimator_cdf,
                        build_indexes, index_float, laplace_bits, z_bits, probs_to_bits, get_downsampled_shape)

CH_MV, CH_N, CH_M = 64, 64, 96  # models/video_model.py:140-142


# ----------------------------------------------------------- layers.py
def residual_block_with_stride(P, p, x):
    """ResidualBlockWithStride (layers/layers.py:43-74)."""
    out = lrelu(conv(P, p + ".conv1", x, stride=2))
    out = lrelu(conv(P, p + ".conv2", out), 0.1)
    return out + conv(P, p + ".downsample", x, stride=2)


def residual_block_upsample(P, p, x):
    """ResidualBlockUpsample (layers/layers.py:77-102)."""
    out = lrelu(subpel(P, p + ".subpel_conv", x))
    out = lrelu(conv(P, p + ".conv", out), 0.1)
    return out + subpel(P, p + ".upsample", x)


def residual_block(P, p, x):
    """ResidualBlock (layers/layers.py:105-128)."""
    out = lrelu(conv(P, p + ".conv1", x))
    out = lrelu(conv(P, p + ".conv2", out))
    return out + x


# --------------------------------------------------------- video_net.py
def res_block(P, p, x, slope=0.01, start_from_relu=True, end_with_relu=False):
    """ResBlock (models/video_net.py:82-108); slope 0 is nn.ReLU."""
    act = (lambda t: F.relu(t)) if slope < 0.0001 else (lambda t: lrelu(t, slope))  # noqa: E731
    out = act(x) if start_from_relu else x
    out = act(conv(P, p + ".conv1", out))
    out = conv(P, p + ".conv2", out)
    if end_with_relu:
        out = act(out)
    return x + out


def se_layer(P, p, x):
    """SELayer (models/video_net.py:157-170)."""
    y = torch.mean(x, dim=(-1, -2))
    y = F.relu(F.linear(y, P[p + ".fc.0.weight"]))
    y = torch.sigmoid(F.linear(y, P[p + ".fc.2.weight"]))
    return x * y[:, :, None, None]


def conv_block_residual(P, p, x):
    """ConvBlockResidual (models/video_net.py:173-188)."""
    x1 = lrelu(conv(P, p + ".conv.0", x))
    x1 = se_layer(P, p + ".conv.3", conv(P, p + ".conv.2", x1))
    return conv(P, p + ".up_dim", x) + x1


def unet(P, p, x):
    """UNet (models/video_net.py:191-236)."""
    x1 = conv_block_residual(P, p + ".conv1", x)
    x2 = conv_block_residual(P, p + ".conv2", F.max_pool2d(x1, 2, 2))
    x3 = conv_block_residual(P, p + ".conv3", F.max_pool2d(x2, 2, 2))
    for i in range(4):
        x3 = res_block(P, f"{p}.context_refine.{i}", x3, slope=0)
    d3 = conv_block_residual(P, p + ".up_conv3", torch.cat((x2, subpel(P, p + ".up3", x3)), dim=1))
    return conv_block_residual(P, p + ".up_conv2", torch.cat((x1, subpel(P, p + ".up2", d3)), dim=1))


def enc_model(P, p, x):
    """get_enc_dec_models encoder (models/video_net.py:239-249)."""
    for i in (0, 2, 4):
        x = residual_block_with_stride(P, f"{p}.{i}", x)
        x = residual_block(P, f"{p}.{i + 1}", x)
    return conv(P, p + ".6", x, stride=2)


def dec_model(P, p, x):
    """get_enc_dec_models decoder (models/video_net.py:251-262)."""
    for i in (0, 2, 4):
        x = residual_block(P, f"{p}.{i}", x)
        x = residual_block_upsample(P, f"{p}.{i + 1}", x)
    x = residual_block(P, p + ".6", x)
    return subpel(P, p + ".7", x)


def hyper_enc(P, p, x):
    """get_hyper_enc_dec_models encoder (models/video_net.py:267-278)."""
    x = lrelu(conv(P, p + ".0", x))
    x = lrelu(conv(P, p + ".2", x))
    x = lrelu(conv(P, p + ".4", x, stride=2))
    x = lrelu(conv(P, p + ".6", x))
    return conv(P, p + ".8", x, stride=2)


def hyper_dec(P, p, x):
    """get_hyper_enc_dec_models decoder (models/video_net.py:280-290)."""
    x = lrelu(conv(P, p + ".0", x))
    x = lrelu(subpel(P, p + ".2", x))
    x = lrelu(conv(P, p + ".4", x))
    x = lrelu(subpel(P, p + ".6", x))
    return conv(P, p + ".8", x)


def ctx_hyper_enc(P, y):
    """contextual_hyper_prior_encoder (models/video_model.py:167-173)."""
    p = "contextual_hyper_prior_encoder"
    x = lrelu(conv(P, p + ".0", y))
    x = lrelu(conv(P, p + ".2", x, stride=2))
    return conv(P, p + ".4", x, stride=2)


def seq3(P, p, x, slope=0.2):
    """the 3-conv prior networks (y/mv prior fusion, spatial priors)."""
    x = lrelu(conv(P, p + ".0", x), slope)
    x = lrelu(conv(P, p + ".2", x), slope)
    return conv(P, p + ".4", x)


# --------------------------------------------------- dual (checkerboard) prior
def dual_masks(h, w):
    """CompressionModel.get_mask (models/common_model.py:84-90)."""
    micro = torch.tensor(((1, 0), (0, 1)), dtype=torch.float32)
    m0 = micro.repeat(h // 2, w // 2)[None, None]
    return m0, torch.ones_like(m0) - m0


def _masked(y, scales, means, mask, force=None):
    """process_with_mask (models/common_model.py:92-100); ``force(pre, y_q,
    mask)``: test instrumentation (dc_oracle.Forcer)."""
    scales_hat = scales * mask
    means_hat = means * mask
    y_res = (y - means_hat) * mask
    y_q = torch.round(y_res)
    if force is not None:
        y_q = force(y_res, y_q, mask)
    return y_res, y_q, y_q + means_hat, scales_hat


def dual_prior(P, y, means, scales, quant_step, spatial, write=False, res_out=None, force=None, call_base=0):
    """forward_dual_prior (models/common_model.py:102-156).  ``res_out`` (a
    list) receives the two coder calls' pre-rounding y - means (test
    instrumentation, tests/parity.py); ``force`` (a dc_oracle.Forcer) replays
    coder calls call_base, call_base + 1 at rounding ties."""
    f0 = f1 = None
    if force is not None:
        f0 = lambda pre, q, m: force.apply(call_base, pre, q, m)       # noqa: E731
        f1 = lambda pre, q, m: force.apply(call_base + 1, pre, q, m)   # noqa: E731
    _, _, H, W = y.size()
    m0, m1 = dual_masks(H, W)
    quant_step = torch.max(quant_step, torch.ones_like(quant_step) * 0.5)
    y = y / quant_step
    y_0, y_1 = y.chunk(2, 1)
    s_0, s_1 = scales.chunk(2, 1)
    mu_0, mu_1 = means.chunk(2, 1)
    r00, q00, h00, sh00 = _masked(y_0, s_0, mu_0, m0, f0)
    r11, q11, h11, sh11 = _masked(y_1, s_1, mu_1, m1, f0)
    params = torch.cat((h00, h11, means, scales, quant_step), dim=1)
    s_0, mu_0, s_1, mu_1 = spatial(params).chunk(4, 1)
    r01, q01, h01, sh01 = _masked(y_0, s_0, mu_0, m1, f1)
    r10, q10, h10, sh10 = _masked(y_1, s_1, mu_1, m0, f1)
    y_q = torch.cat((q00 + q01, q11 + q10), dim=1)
    y_hat = torch.cat((h00 + h01, h11 + h10), dim=1)
    scales_hat = torch.cat((sh00 + sh01, sh11 + sh10), dim=1)
    y_hat = y_hat * quant_step
    if res_out is not None:
        res_out += [r00 + r11, r01 + r10]
    if write:
        return q00 + q11, q01 + q10, sh00 + sh11, sh01 + sh10, y_hat
    return y_q, y_hat, scales_hat


def dual_decompress(P, means, scales, quant_step, spatial, decode):
    """decompress_dual_prior (models/common_model.py:161-188); decode(scales)
    returns the decoded symbols (float tensor, scales' shape)."""
    _, _, H, W = means.size()
    m0, m1 = dual_masks(H, W)
    quant_step = torch.clamp_min(quant_step, 0.5)
    s_0, s_1 = scales.chunk(2, 1)
    mu_0, mu_1 = means.chunk(2, 1)
    q0 = decode(s_0 * m0 + s_1 * m1)
    h00 = (q0 + mu_0) * m0
    h11 = (q0 + mu_1) * m1
    params = torch.cat((h00, h11, means, scales, quant_step), dim=1)
    s_0, mu_0, s_1, mu_1 = spatial(params).chunk(4, 1)
    q1 = decode(s_0 * m1 + s_1 * m0)
    h01 = (q1 + mu_0) * m1
    h10 = (q1 + mu_1) * m0
    return torch.cat((h00 + h01, h11 + h10), dim=1) * quant_step


def gaussian_bits(y, sigma):
    """get_y_gaussian_bits (models/common_model.py:58-63): sigma clamped at 0.11."""
    sigma = sigma.clamp(0.11, 1e10)
    d = torch.distributions.normal.Normal(torch.zeros_like(sigma), sigma)
    return probs_to_bits(d.cdf(y + 0.5) - d.cdf(y - 0.5))


def lower_bound_q(P, name, q_scale):
    """get_curr_q / get_curr_*_q: LowerBound(q_basic, 0.5) * q_scale."""
    q = P[name]
    return torch.max(q, torch.ones_like(q) * 0.5) * q_scale


# ------------------------------------------------------------ video_model.py
class DMCOracle:
    """DMC (models/video_model.py:136-330, 377-515)."""

    def __init__(self, state_dict, quantize):
        self.P = Params(state_dict)
        self.tab_y = EntropyTables.gaussian("laplace", quantize)
        self.tab_z = EntropyTables.bit_estimator(self.P, "bit_estimator_z", CH_N, quantize)
        self.tab_mvz = EntropyTables.bit_estimator(self.P, "bit_estimator_z_mv", CH_MV, quantize)

    def motion_compensation(self, dpb, mv):
        """multi_scale_feature_extractor + motion_compensation (:225-242)."""
        P = self.P
        mv2 = down2(mv) / 2
        mv3 = down2(mv2) / 2
        if dpb["ref_feature"] is None:
            f = conv(P, "feature_adaptor_I", dpb["ref_frame"])
        else:
            f = conv(P, "feature_adaptor_P", dpb["ref_feature"])
        fe = "feature_extractor"
        l1 = res_block(P, fe + ".res_block1", conv(P, fe + ".conv1", f))
        l2 = res_block(P, fe + ".res_block2", conv(P, fe + ".conv2", l1, stride=2))
        l3 = res_block(P, fe + ".res_block3", conv(P, fe + ".conv3", l2, stride=2))
        c1, c2, c3 = flow_warp(l1, mv), flow_warp(l2, mv2), flow_warp(l3, mv3)
        cf = "context_fusion_net"
        c3u = res_block(P, cf + ".res_block3_up", subpel(P, cf + ".conv3_up", c3))
        c3o = res_block(P, cf + ".res_block3_out", conv(P, cf + ".conv3_out", c3))
        cat = torch.cat((c3u, c2), dim=1)
        c2u = res_block(P, cf + ".res_block2_up", subpel(P, cf + ".conv2_up", cat))
        c2o = res_block(P, cf + ".res_block2_out", conv(P, cf + ".conv2_out", cat))
        c1o = res_block(P, cf + ".res_block1_out", conv(P, cf + ".conv1_out", torch.cat((c2u, c1), dim=1)))
        return c1 + c1o, c2 + c2o, c3 + c3o

    def contextual_encoder(self, x, c1, c2, c3):
        P, p = self.P, "contextual_encoder"
        f = conv(P, p + ".conv1", torch.cat([x, c1], dim=1), stride=2)
        f = res_block(P, p + ".res1", torch.cat([f, c2], dim=1), 0.1, True, True)
        f = conv(P, p + ".conv2", f, stride=2)
        f = res_block(P, p + ".res2", torch.cat([f, c3], dim=1), 0.1, True, True)
        f = conv(P, p + ".conv3", f, stride=2)
        return conv(P, p + ".conv4", f, stride=2)

    def recon(self, y_hat, c1, c2, c3):
        """contextual_decoder + recon_generation_net (:71-128)."""
        P, p = self.P, "contextual_decoder"
        f = subpel(P, p + ".up1", y_hat)
        f = subpel(P, p + ".up2", f)
        f = res_block(P, p + ".res1", torch.cat([f, c3], dim=1), 0.1, True, True)
        f = subpel(P, p + ".up3", f)
        f = res_block(P, p + ".res2", torch.cat([f, c2], dim=1), 0.1, True, True)
        f = subpel(P, p + ".up4", f)
        g = "recon_generation_net"
        feature = conv(P, g + ".first_conv", torch.cat((f, c1), dim=1))
        feature = unet(P, g + ".unet_1", feature)
        feature = unet(P, g + ".unet_2", feature)
        return feature, conv(P, g + ".recon_conv", feature)

    def mv_params(self, mv_z_hat, ref_mv_y, like):
        P = self.P
        p = hyper_dec(P, "mv_hyper_prior_decoder", mv_z_hat)
        if ref_mv_y is None:
            ref_mv_y = torch.zeros_like(like) if like is not None else torch.zeros(
                (1, p.shape[1] // 2) + tuple(p.shape[2:]))
        return seq3(P, "mv_y_prior_fusion", torch.cat((p, ref_mv_y), dim=1)).chunk(3, 1)

    def y_params(self, z_hat, c3, ref_y, like):
        P = self.P
        hier = hyper_dec(P, "contextual_hyper_prior_decoder", z_hat)
        temp = conv(P, "temporal_prior_encoder.2",
                    lrelu(conv(P, "temporal_prior_encoder.0", c3, stride=2), 0.1), stride=2)
        if ref_y is None:
            ref_y = torch.zeros_like(like) if like is not None else torch.zeros(
                (1, temp.shape[1] // 2) + tuple(temp.shape[2:]))
        return seq3(P, "y_prior_fusion", torch.cat((temp, hier, ref_y), dim=1)).chunk(3, 1)

    def spatial(self, prefix):
        return lambda t: seq3(self.P, prefix, t)

    def compress(self, x, dpb, mv_y_q_scale, y_q_scale, tap=None, recon=False, force=None):
        """compress (:263-330): the coder calls [(table, symbols, scales)].
        Test instrumentation: ``tap`` (a dict) receives per call the
        pre-rounding values ("pre"), the pre-truncation scale indexes
        ("idx_f") and the dependency order; ``recon=True`` also returns the
        decoder-side dpb built from the encoder's y_hat (what decompress()
        reconstructs from the stream)."""
        P = self.P
        mvq = lower_bound_q(P, "mv_y_q_basic", mv_y_q_scale)
        yq = lower_bound_q(P, "y_q_basic", y_q_scale)
        est_mv = spynet(P, "optic_flow", x, dpb["ref_frame"])
        mv_y = enc_model(P, "mv_encoder", est_mv) / mvq
        mv_z = hyper_enc(P, "mv_hyper_prior_encoder", mv_y)
        mv_z_hat = torch.round(mv_z) if force is None else force.apply(0, mv_z, torch.round(mv_z))
        mv_q_step, mv_scales, mv_means = self.mv_params(mv_z_hat, dpb["ref_mv_y"], mv_y)
        res = []
        mq0, mq1, ms0, ms1, mv_y_hat = dual_prior(P, mv_y, mv_means, mv_scales, mv_q_step,
                                                  self.spatial("mv_y_spatial_prior"), write=True, res_out=res,
                                                  force=force, call_base=1)
        mv_y_hat = mv_y_hat * mvq
        mv_hat = dec_model(P, "mv_decoder", mv_y_hat)
        c1, c2, c3 = self.motion_compensation(dpb, mv_hat)
        y = self.contextual_encoder(x, c1, c2, c3) / yq
        z = ctx_hyper_enc(P, y)
        z_hat = torch.round(z) if force is None else force.apply(3, z, torch.round(z))
        q_step, scales, means = self.y_params(z_hat, c3, dpb["ref_y"], y)
        q0, q1, s0, s1, y_hat = dual_prior(P, y, means, scales, q_step, self.spatial("y_spatial_prior"),
                                           write=True, res_out=res, force=force, call_base=4)
        calls = [("p_mvz", mv_z_hat, None), ("p_y", mq0, ms0), ("p_y", mq1, ms1), ("p_z", z_hat, None),
                 ("p_y", q0, s0), ("p_y", q1, s1)]
        if tap is not None:
            lm, st = self.tab_y[3], self.tab_y[4]
            tap["pre"] = [mv_z, res[0], res[1], z, res[2], res[3]]
            tap["idx_f"] = [None if sc is None else index_float(sc, lm, st) for _, _, sc in calls]
            tap["order"] = [0, 1, 2, 3, 4, 5]
        if recon:
            y_hat = y_hat * yq
            feature, rec = self.recon(y_hat, c1, c2, c3)
            return calls, {"ref_frame": rec.clamp(0, 1), "ref_feature": feature, "ref_y": y_hat,
                           "ref_mv_y": mv_y_hat}
        return calls

    def decompress(self, dpb, decoder, height, width, mv_y_q_scale, y_q_scale):
        """decompress (:332-375); decoder(kind, indexes) -> int symbols."""
        P = self.P
        mvq = lower_bound_q(P, "mv_y_q_basic", mv_y_q_scale)
        yq = lower_bound_q(P, "y_q_basic", y_q_scale)
        zh, zw = get_downsampled_shape(height, width, 64)
        mv_z_hat = decoder("p_mvz", channel_indexes(CH_MV, zh, zw)).float().reshape(1, CH_MV, zh, zw)
        mv_q_step, mv_scales, mv_means = self.mv_params(mv_z_hat, dpb["ref_mv_y"], None)
        mv_y_hat = dual_decompress(P, mv_means, mv_scales, mv_q_step, self.spatial("mv_y_spatial_prior"),
                                   self._dec_y(decoder, "p_y"))
        mv_y_hat = mv_y_hat * mvq
        mv_hat = dec_model(P, "mv_decoder", mv_y_hat)
        c1, c2, c3 = self.motion_compensation(dpb, mv_hat)
        z_hat = decoder("p_z", channel_indexes(CH_N, zh, zw)).float().reshape(1, CH_N, zh, zw)
        q_step, scales, means = self.y_params(z_hat, c3, dpb["ref_y"], None)
        y_hat = dual_decompress(P, means, scales, q_step, self.spatial("y_spatial_prior"),
                                self._dec_y(decoder, "p_y"))
        y_hat = y_hat * yq
        feature, recon = self.recon(y_hat, c1, c2, c3)
        return {"ref_frame": recon.clamp(0, 1), "ref_feature": feature, "ref_y": y_hat, "ref_mv_y": mv_y_hat}

    def _dec_y(self, decoder, kind):
        log_min, step = self.tab_y[3], self.tab_y[4]

        def dec(scales):
            idx = build_indexes(scales, log_min, step)
            return decoder(kind, idx.reshape(-1)).float().reshape(scales.shape)
        return dec

    def forward_one_frame(self, x, dpb, mv_y_q_scale, y_q_scale):
        """Estimate mode (:417-515): (bit, dpb)."""
        P = self.P
        mvq = lower_bound_q(P, "mv_y_q_basic", mv_y_q_scale)
        yq = lower_bound_q(P, "y_q_basic", y_q_scale)
        est_mv = spynet(P, "optic_flow", x, dpb["ref_frame"])
        mv_y = enc_model(P, "mv_encoder", est_mv) / mvq
        mv_z_hat = torch.round(hyper_enc(P, "mv_hyper_prior_encoder", mv_y))
        mv_q_step, mv_scales, mv_means = self.mv_params(mv_z_hat, dpb["ref_mv_y"], mv_y)
        mv_y_q, mv_y_hat, mv_scales_hat = dual_prior(P, mv_y, mv_means, mv_scales, mv_q_step,
                                                     self.spatial("mv_y_spatial_prior"))
        mv_y_hat = mv_y_hat * mvq
        mv_hat = dec_model(P, "mv_decoder", mv_y_hat)
        c1, c2, c3 = self.motion_compensation(dpb, mv_hat)
        y = self.contextual_encoder(x, c1, c2, c3) / yq
        z_hat = torch.round(ctx_hyper_enc(P, y))
        q_step, scales, means = self.y_params(z_hat, c3, dpb["ref_y"], y)
        y_q, y_hat, scales_hat = dual_prior(P, y, means, scales, q_step, self.spatial("y_spatial_prior"))
        y_hat = y_hat * yq
        feature, recon = self.recon(y_hat, c1, c2, c3)
        _, _, H, W = x.size()
        n = H * W
        bpp_y = torch.sum(laplace_bits(y_q, scales_hat), dim=(1, 2, 3)) / n
        bpp_z = torch.sum(z_bits(P, "bit_estimator_z", z_hat), dim=(1, 2, 3)) / n
        bpp_mv_y = torch.sum(laplace_bits(mv_y_q, mv_scales_hat), dim=(1, 2, 3)) / n
        bpp_mv_z = torch.sum(z_bits(P, "bit_estimator_z_mv", mv_z_hat), dim=(1, 2, 3)) / n
        bit = torch.sum(bpp_y + bpp_z + bpp_mv_y + bpp_mv_z) * n
        return bit.item(), {"ref_frame": recon, "ref_feature": feature, "ref_y": y_hat, "ref_mv_y": mv_y_hat}


def channel_indexes(C, h, w):
    """BitEstimator.build_indexes (entropy_models/entropy_models.py:176-180), flattened."""
    return torch.arange(C).view(C, 1, 1).expand(C, h, w).reshape(-1).int()


# ------------------------------------------------------------ image_model.py
class IntraOracle:
    """IntraNoAR (models/image_model.py:15-171), N = 192."""

    def __init__(self, state_dict, quantize, N=192):
        self.P = Params(state_dict)
        self.N = N
        self.tab_y = EntropyTables.gaussian("gaussian", quantize)
        self.tab_z = EntropyTables.bit_estimator(self.P, "bit_estimator_z", N, quantize)

    def _prior(self, z_hat):
        P = self.P
        return seq3(P, "y_prior_fusion", hyper_dec(P, "hyper_dec", z_hat)).chunk(3, 1)

    def _refine(self, y_hat):
        P = self.P
        return conv(P, "refine.1", unet(P, "refine.0", dec_model(P, "dec", y_hat)))

    def compress(self, x, q_scale, tap=None, recon=False, force=None):
        """compress (:150-154); ``tap`` / ``recon`` / ``force`` as in DMCOracle.compress."""
        P = self.P
        q = lower_bound_q(P, "q_basic", q_scale)
        y = enc_model(P, "enc", x) / q
        z = hyper_enc(P, "hyper_enc", y)
        z_hat = torch.round(z) if force is None else force.apply(0, z, torch.round(z))
        q_step, scales, means = self._prior(z_hat)
        res = []
        q0, q1, s0, s1, y_hat = dual_prior(P, y, means, scales, q_step, lambda t: seq3(P, "y_spatial_prior", t),
                                           write=True, res_out=res, force=force, call_base=1)
        calls = [("i_z", z_hat, None), ("i_y", q0, s0), ("i_y", q1, s1)]
        if tap is not None:
            lm, st = self.tab_y[3], self.tab_y[4]
            tap["pre"] = [z, res[0], res[1]]
            tap["idx_f"] = [None, index_float(s0, lm, st), index_float(s1, lm, st)]
            tap["order"] = [0, 1, 2]
        if recon:
            return calls, self._refine(y_hat * q).clamp_(0, 1)
        return calls

    def decompress(self, decoder, height, width, q_scale):
        P = self.P
        q = lower_bound_q(P, "q_basic", q_scale)
        zh, zw = get_downsampled_shape(height, width, 64)
        z_hat = decoder("i_z", channel_indexes(self.N, zh, zw)).float().reshape(1, self.N, zh, zw)
        q_step, scales, means = self._prior(z_hat)
        log_min, step = self.tab_y[3], self.tab_y[4]

        def dec(scales_r):
            idx = build_indexes(scales_r, log_min, step)
            return decoder("i_y", idx.reshape(-1)).float().reshape(scales_r.shape)
        y_hat = dual_decompress(P, means, scales, q_step, lambda t: seq3(P, "y_spatial_prior", t), dec) * q
        return self._refine(y_hat).clamp_(0, 1)

    def forward(self, x, q_scale):
        """Estimate mode (:53-99): (bit, x_hat)."""
        P = self.P
        q = lower_bound_q(P, "q_basic", q_scale)
        y = enc_model(P, "enc", x) / q
        z_hat = torch.round(hyper_enc(P, "hyper_enc", y))
        q_step, scales, means = self._prior(z_hat)
        y_q, y_hat, scales_hat = dual_prior(P, y, means, scales, q_step, lambda t: seq3(P, "y_spatial_prior", t))
        x_hat = self._refine(y_hat * q)
        _, _, H, W = x.size()
        n = H * W
        bpp_y = torch.sum(gaussian_bits(y_q, scales_hat), dim=(1, 2, 3)) / n
        bpp_z = torch.sum(z_bits(P, "bit_estimator_z", z_hat), dim=(1, 2, 3)) / n
        return (torch.sum(bpp_y + bpp_z) * n).item(), x_hat
