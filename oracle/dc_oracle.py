"""DCVC-DC CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module, and only as the checker / the timed CPU baseline.  The
product path (``dcvc_amd``) never imports it.

A functional restatement, in plain PyTorch fp32 on the CPU, of the DCVC-DC
P-frame codec (``DMC``) and intra codec (``IntraNoAR``), driven directly by a
reference-format ``state_dict`` (same key names, so reference checkpoints load).
Every function cites the reference code it follows (paths relative to
/root/reference/DCVC-DC/src).  The op sequence — including operand order of
adds, the cached-grid warp and the mask arithmetic of the quadtree prior — is
kept identical to the reference so that on the CPU the results are bitwise
equal to the reference's; the committed fixtures under tests/golden/ pin it.

The entropy coder used in write mode is the C restatement in
``oracle/rans_oracle.c`` (loaded through ``oracle.rans_oracle``).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

G1, G2, G4, G8, G16 = 48, 64, 96, 96, 128  # models/video_model.py:19-23


# ------------------------------------------------------------------ helpers
class Params:
    """state_dict accessor (fp32 CPU tensors)."""

    def __init__(self, sd):
        self.sd = {k: v.detach().float().cpu() for k, v in sd.items()}

    def __getitem__(self, k):
        return self.sd[k]

    def has(self, k):
        return k in self.sd


def conv(P, name, x, stride=1, groups=1):
    """nn.Conv2d with padding (k-1)//2 as every conv of the reference uses."""
    w = P[name + ".weight"]
    k = w.shape[-1]
    return F.conv2d(x, w, P[name + ".bias"], stride=stride, padding=(k - 1) // 2, groups=groups)


def lrelu(x, slope=0.01):
    return F.leaky_relu(x, slope)


def subpel(P, name, x, r=2):
    """subpel_conv3x3 / subpel_conv1x1 (models/layers.py:23-34)."""
    return F.pixel_shuffle(conv(P, name + ".0", x), r)


# -------------------------------------------------------------- layers.py
def residual_block_with_stride(P, p, x, stride=2):
    """ResidualBlockWithStride (models/layers.py:42-73)."""
    out = lrelu(conv(P, p + ".conv1", x, stride=stride))
    out = lrelu(conv(P, p + ".conv2", out), 0.1)
    identity = conv(P, p + ".downsample", x, stride=stride) if stride != 1 else x
    return out + identity


def residual_block_upsample(P, p, x):
    """ResidualBlockUpsample (models/layers.py:76-101)."""
    out = lrelu(subpel(P, p + ".subpel_conv", x))
    out = lrelu(conv(P, p + ".conv", out), 0.1)
    identity = subpel(P, p + ".upsample", x)
    return out + identity


def depth_conv(P, p, x, slope=0.01, stride=1):
    """DepthConv (models/layers.py:135-163)."""
    identity = x
    if P.has(p + ".adaptor.weight"):
        identity = conv(P, p + ".adaptor", identity, stride=stride)
    out = lrelu(conv(P, p + ".conv1.0", x, stride=stride), slope)
    out = conv(P, p + ".depth_conv", out, groups=out.shape[1])
    out = conv(P, p + ".conv2", out)
    return out + identity


def conv_ffn(P, p, x, slope=0.1):
    """ConvFFN (models/layers.py:166-179)."""
    h = lrelu(conv(P, p + ".conv.0", x), slope)
    h = lrelu(conv(P, p + ".conv.2", h), slope)
    return x + h


def conv_ffn2(P, p, x, slope=0.1):
    """ConvFFN2 (models/layers.py:182-196)."""
    x1, x2 = conv(P, p + ".conv", x).chunk(2, 1)
    out = x1 * lrelu(x2, slope)
    return x + conv(P, p + ".conv_out", out)


def depth_conv_block(P, p, x, stride=1):
    """DepthConvBlock (models/layers.py:199-209)."""
    return conv_ffn(P, p + ".block.1", depth_conv(P, p + ".block.0", x, stride=stride))


def depth_conv_block2(P, p, x, stride=1):
    """DepthConvBlock2 (models/layers.py:212-222)."""
    return conv_ffn2(P, p + ".block.1", depth_conv(P, p + ".block.0", x, stride=stride))


# ------------------------------------------------------------ video_net.py
_GRID = {}


def flow_warp(feature, flow):
    """torch_warp / add_grid_cache (models/video_net.py:11-38): cached fp32
    linspace grid + normalised flow, grid_sample(bilinear, border,
    align_corners=True)."""
    key = str(flow.size())
    if key not in _GRID:
        N, _, H, W = flow.size()
        hor = torch.linspace(-1.0, 1.0, W, dtype=torch.float32).view(1, 1, 1, W).expand(N, -1, H, -1)
        ver = torch.linspace(-1.0, 1.0, H, dtype=torch.float32).view(1, 1, H, 1).expand(N, -1, -1, W)
        _GRID[key] = torch.cat([hor, ver], 1)
    flow = torch.cat([flow[:, 0:1, :, :] / ((feature.size(3) - 1.0) / 2.0),
                      flow[:, 1:2, :, :] / ((feature.size(2) - 1.0) / 2.0)], 1)
    grid = _GRID[key] + flow
    return F.grid_sample(feature, grid.permute(0, 2, 3, 1), mode="bilinear",
                         padding_mode="border", align_corners=True)


def up2(x):
    """bilinearupsacling (models/video_net.py:41-47)."""
    return F.interpolate(x, (x.size(2) * 2, x.size(3) * 2), mode="bilinear", align_corners=False)


def down2(x):
    """bilineardownsacling (models/video_net.py:50-55)."""
    return F.interpolate(x, (x.size(2) // 2, x.size(3) // 2), mode="bilinear", align_corners=False)


def res_block(P, p, x, slope=0.01, end_with_relu=False):
    """ResBlock (models/video_net.py:58-76)."""
    out = lrelu(x, slope)
    out = lrelu(conv(P, p + ".conv1", out), slope)
    out = conv(P, p + ".conv2", out)
    if end_with_relu:
        out = lrelu(out, slope)
    return x + out


def me_basic(P, p, x):
    """MEBasic (models/video_net.py:79-95)."""
    for i in range(1, 5):
        x = F.relu(conv(P, f"{p}.conv{i}", x))
    return conv(P, p + ".conv5", x)


def spynet(P, p, im1, im2):
    """ME_Spynet (models/video_net.py:98-126)."""
    l1, l2 = [im1], [im2]
    for lv in range(3):
        l1.append(F.avg_pool2d(l1[lv], kernel_size=2, stride=2))
        l2.append(F.avg_pool2d(l2[lv], kernel_size=2, stride=2))
    h, w = l2[3].shape[2:]
    flow = torch.zeros([im1.size(0), 2, h // 2, w // 2], dtype=im1.dtype)
    for lv in range(4):
        flow_up = up2(flow) * 2.0
        k = 3 - lv
        flow = flow_up + me_basic(P, f"{p}.moduleBasic.{lv}",
                                  torch.cat([l1[k], flow_warp(l2[k], flow_up), flow_up], 1))
    return flow


def unet(P, p, x, block=depth_conv_block):
    """UNet / UNet2 (models/video_net.py:129-214)."""
    x1 = block(P, p + ".conv1", x)
    x2 = F.max_pool2d(x1, 2, 2)
    x2 = block(P, p + ".conv2", x2)
    x3 = F.max_pool2d(x2, 2, 2)
    x3 = block(P, p + ".conv3", x3)
    for i in range(4):
        x3 = block(P, f"{p}.context_refine.{i}", x3)
    d3 = block(P, p + ".up_conv3", torch.cat((x2, subpel(P, p + ".up3", x3)), dim=1))
    d2 = block(P, p + ".up_conv2", torch.cat((x1, subpel(P, p + ".up2", d3)), dim=1))
    return d2


def hyper_enc(P, p, x, reduce_enc_layer):
    """get_hyper_enc_dec_models encoder (models/video_net.py:217-237)."""
    if reduce_enc_layer:
        x = lrelu(conv(P, p + ".0", x))
        x = lrelu(conv(P, p + ".2", x, stride=2))
        return conv(P, p + ".4", x, stride=2)
    x = lrelu(conv(P, p + ".0", x))
    x = lrelu(conv(P, p + ".2", x))
    x = lrelu(conv(P, p + ".4", x, stride=2))
    x = lrelu(conv(P, p + ".6", x))
    return conv(P, p + ".8", x, stride=2)


def hyper_dec(P, p, x):
    """get_hyper_enc_dec_models decoder (models/video_net.py:239-249)."""
    x = lrelu(conv(P, p + ".0", x))
    x = lrelu(subpel(P, p + ".2", x))
    x = lrelu(conv(P, p + ".4", x))
    x = lrelu(subpel(P, p + ".6", x))
    return conv(P, p + ".8", x)


# ------------------------------------------------------- stream_helper.py
def get_padding_size(h, w, p=64):
    """utils/stream_helper.py:22-31."""
    nh = (h + p - 1) // p * p
    nw = (w + p - 1) // p * p
    return 0, nw - w, 0, nh - h


def get_downsampled_shape(h, w, p):
    """utils/stream_helper.py:34-37."""
    nh = (h + p - 1) // p * p
    nw = (w + p - 1) // p * p
    return int(nh / p + 0.5), int(nw / p + 0.5)


# --------------------------------------------------------- entropy models
class EntropyTables:
    """Quantised CDF tables (models/entropy_models.py:228-267 GaussianEncoder.update,
    :124-178 BitEstimator.update).  ``quantize`` maps a float PMF to a CDF."""

    @staticmethod
    def pmf_to_cdf(pmf, tail_mass, pmf_length, max_length, quantize):
        cdf = torch.zeros((len(pmf_length), max_length + 2), dtype=torch.int32)
        for i, p in enumerate(pmf):
            prob = torch.cat((p[: pmf_length[i]], tail_mass[i]), dim=0)
            c = torch.IntTensor(quantize(prob.tolist(), 16))
            cdf[i, : c.size(0)] = c
        return cdf

    @staticmethod
    def gaussian(distribution, quantize):
        if distribution == "laplace":
            dist, smin, smax = torch.distributions.laplace.Laplace, 0.01, 64.0
        else:
            dist, smin, smax = torch.distributions.normal.Normal, 0.11, 64.0
        table = torch.exp(torch.linspace(math.log(smin), math.log(smax), 256))
        center = torch.zeros_like(table) + 50
        scales = torch.zeros_like(center) + table
        d = dist(torch.zeros_like(scales), scales)
        for i in range(50, 1, -1):
            probs = torch.squeeze(d.cdf(torch.zeros_like(center) + i))
            center = torch.where(probs > torch.zeros_like(center) + 0.9999,
                                 torch.zeros_like(center) + i, center)
        center = center.int()
        length = 2 * center + 1
        max_length = torch.max(length).item()
        samples = (torch.arange(max_length) - center[:, None]).float()
        scales = torch.zeros_like(samples) + table[:, None]
        d = dist(torch.zeros_like(scales), scales)
        upper = d.cdf(samples + 0.5)
        lower = d.cdf(samples - 0.5)
        pmf = upper - lower
        tail = 2 * lower[:, :1]
        cdf = EntropyTables.pmf_to_cdf(pmf, tail, length, max_length, quantize)
        log_min = math.log(smin)
        step = (math.log(smax) - log_min) / 255
        return cdf.numpy(), (length + 2).int().numpy(), (-center).int().numpy(), log_min, step

    @staticmethod
    def bit_estimator(P, p, channel, quantize):
        med = torch.zeros(channel)
        minima = med + 50
        for i in range(50, 1, -1):
            probs = torch.squeeze(bit_estimator_cdf(P, p, (torch.zeros_like(med) - i)[None, :, None, None]))
            minima = torch.where(probs < torch.zeros_like(med) + 0.0001, torch.zeros_like(med) + i, minima)
        maxima = med + 50
        for i in range(50, 1, -1):
            probs = torch.squeeze(bit_estimator_cdf(P, p, (torch.zeros_like(med) + i)[None, :, None, None]))
            maxima = torch.where(probs > torch.zeros_like(med) + 0.9999, torch.zeros_like(med) + i, maxima)
        minima = minima.int()
        maxima = maxima.int()
        offset = -minima
        pmf_start = med - minima
        length = maxima + minima + 1
        max_length = length.max()
        samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
        lower = bit_estimator_cdf(P, p, samples - 0.5).squeeze(0)
        upper = bit_estimator_cdf(P, p, samples + 0.5).squeeze(0)
        pmf = (upper - lower)[:, 0, :]
        tail = lower[:, 0, :1] + (1.0 - upper[:, 0, -1:])
        cdf = EntropyTables.pmf_to_cdf(pmf, tail, length, max_length, quantize)
        return cdf.numpy(), (length + 2).int().numpy(), offset.int().numpy()


def bit_estimator_cdf(P, p, x):
    """BitEstimator.get_cdf with 4 Bitparm layers (models/entropy_models.py:58-77, 111-122)."""
    for i in range(1, 5):
        q = f"{p}.f{i}"
        x = x * F.softplus(P[q + ".h"]) + P[q + ".b"]
        if i < 4:
            x = x + torch.tanh(x) * torch.tanh(P[q + ".a"])
    return torch.sigmoid(x)


def build_indexes(scales, log_min, step):
    """GaussianEncoder.build_indexes (models/entropy_models.py:269-273)."""
    return index_float(scales, log_min, step).clamp_(0, 255).int()


def index_float(scales, log_min, step):
    """build_indexes before the clamp and the int() truncation (the value whose
    distance to an integer says how close an index is to flipping)."""
    scales = torch.maximum(scales, torch.zeros_like(scales) + 1e-5)
    return (torch.log(scales) - log_min) / step


def probs_to_bits(probs):
    """common_model.py:39-43."""
    return torch.clamp_min(-1.0 * torch.log(probs + 1e-5) / math.log(2.0), 0)


def laplace_bits(y, sigma):
    """common_model.py:52-57."""
    sigma = sigma.clamp(1e-5, 1e10)
    d = torch.distributions.laplace.Laplace(torch.zeros_like(sigma), sigma)
    return probs_to_bits(d.cdf(y + 0.5) - d.cdf(y - 0.5))


def gaussian_bits(y, sigma):
    """common_model.py:45-50."""
    sigma = sigma.clamp(1e-5, 1e10)
    d = torch.distributions.normal.Normal(torch.zeros_like(sigma), sigma)
    return probs_to_bits(d.cdf(y + 0.5) - d.cdf(y - 0.5))


def z_bits(P, p, z):
    """common_model.py:59-61."""
    return probs_to_bits(bit_estimator_cdf(P, p, z + 0.5) - bit_estimator_cdf(P, p, z - 0.5))


# ------------------------------------------------------ quadtree prior
_MASKS = {}


def four_part_masks(h, w):
    """get_mask_four_parts (common_model.py:102-129)."""
    key = (h, w)
    if key not in _MASKS:
        ms = []
        for micro in (((1, 0), (0, 0)), ((0, 1), (0, 0)), ((0, 0), (1, 0)), ((0, 0), (0, 1))):
            m = torch.tensor(micro, dtype=torch.float32).repeat((h + 1) // 2, (w + 1) // 2)
            ms.append(m[:h, :w][None, None])
        _MASKS[key] = ms
    return _MASKS[key]


class Forcer:
    """Test instrumentation (tests/parity.py, strict bar): replays another
    coder's symbols at the oracle's rounding ties.  ``syms[c]`` holds the
    symbols of coder call c (stream order, flattened NCHW); wherever the
    oracle's pre-rounding value lies within ``eps`` of a half-integer and its
    rounded symbol differs from ``syms[c]``, the oracle takes ``syms[c]``, so
    every later step of the frame runs on the same y_hat as that coder.  A
    difference away from a tie is left in place (the comparison then reports
    it as unexplained)."""

    def __init__(self, syms, eps):
        self.syms = syms
        self.eps = eps
        self.forced = 0

    def apply(self, call, pre, q, mask=None):
        if self.syms is None or self.syms[call] is None:
            return q
        P = torch.as_tensor(np.asarray(self.syms[call]).astype(np.float32)).reshape(q.shape)
        a = pre.double().abs()
        sel = ((a - torch.floor(a) - 0.5).abs() < self.eps) & (P != q)
        if mask is not None:
            sel &= mask.bool()
        self.forced += int(sel.sum())
        return torch.where(sel, P, q)


def _masked(y, scales, means, mask, force=None):
    """process_with_mask (common_model.py:92-100); ``force(pre, y_q, mask)``:
    test instrumentation (Forcer)."""
    s_hat = scales * mask
    m_hat = means * mask
    y_res = (y - m_hat) * mask
    y_q = torch.round(y_res)
    if force is not None:
        y_q = force(y_res, y_q, mask)
    return y_res, y_q, y_q + m_hat, s_hat


# Which mask each channel quarter uses at step k (common_model.py:168-220):
# step 0 -> (0,1,2,3), step 1 -> (3,2,1,0), step 2 -> (2,3,0,1), step 3 -> (1,0,3,2)
STEP_MASK = ((0, 1, 2, 3), (3, 2, 1, 0), (2, 3, 0, 1), (1, 0, 3, 2))


def four_part_prior(P, y, common_params, adaptors, spatial, yres_out=None, force=None, call_base=0):
    """forward_four_part_prior with write=True (common_model.py:142-252).
    Returns (per-step symbols y_q_w_k, per-step scales_w_k, y_q, y_hat, scales_hat).
    ``yres_out`` (a list) receives each step's pre-rounding y - means in the
    layout of y_q_w_k (test instrumentation: distance to a rounding tie);
    ``force`` (a Forcer) replays coder call call_base + step's symbols at ties."""
    quant_step, scales, means = common_params.chunk(3, 1)
    _, _, H, W = y.size()
    masks = four_part_masks(H, W)
    quant_step = torch.clamp_min(quant_step, 0.5)
    y = y / quant_step
    ys = y.chunk(4, 1)
    sc, me = scales.chunk(4, 1), means.chunk(4, 1)
    res = [[None] * 4 for _ in range(4)]  # res[quarter][mask] = (y_res, y_q, y_hat, s_hat)
    y_hat_so_far = None
    for step in range(4):
        if step > 0:
            params = torch.cat((y_hat_so_far, common_params), dim=1)
            out = spatial(conv(P, adaptors[step - 1], params)).chunk(8, 1)
            sc, me = out[:4], out[4:]
        cur = []
        fk = None
        if force is not None:
            fk = (lambda c: (lambda pre, yq, m: force.apply(c, pre, yq, m)))(call_base + step)
        for q in range(4):
            mk = STEP_MASK[step][q]
            res[q][mk] = _masked(ys[q], sc[q], me[q], masks[mk], fk)
            cur.append(res[q][mk][2])
        cur = torch.cat(cur, dim=1)
        y_hat_so_far = cur if step == 0 else y_hat_so_far + cur

    def combine(field):
        return torch.cat([res[q][0][field] + res[q][1][field] + res[q][2][field] + res[q][3][field]
                          for q in range(4)], dim=1)

    y_q, y_hat, scales_hat = combine(1), combine(2), combine(3)
    y_hat = y_hat * quant_step
    sym_w, sc_w = [], []
    for step in range(4):
        mks = STEP_MASK[step]
        sym_w.append(res[0][mks[0]][1] + res[1][mks[1]][1] + res[2][mks[2]][1] + res[3][mks[3]][1])
        sc_w.append(res[0][mks[0]][3] + res[1][mks[1]][3] + res[2][mks[2]][3] + res[3][mks[3]][3])
        if yres_out is not None:
            yres_out.append(res[0][mks[0]][0] + res[1][mks[1]][0] + res[2][mks[2]][0] + res[3][mks[3]][0])
    return sym_w, sc_w, y_q, y_hat, scales_hat


def four_part_decompress(P, common_params, adaptors, spatial, decode):
    """decompress_four_part_prior (common_model.py:261-321); ``decode(scales_r)``
    returns the decoded symbol tensor of that step."""
    quant_step, scales, means = common_params.chunk(3, 1)
    _, _, H, W = means.size()
    masks = four_part_masks(H, W)
    quant_step = torch.clamp_min(quant_step, 0.5)
    sc, me = scales.chunk(4, 1), means.chunk(4, 1)
    y_hat_so_far = None
    for step in range(4):
        if step > 0:
            params = torch.cat((y_hat_so_far, common_params), dim=1)
            out = spatial(conv(P, adaptors[step - 1], params)).chunk(8, 1)
            sc, me = out[:4], out[4:]
        mk = STEP_MASK[step]
        scales_r = sc[0] * masks[mk[0]] + sc[1] * masks[mk[1]] + sc[2] * masks[mk[2]] + sc[3] * masks[mk[3]]
        y_q_r = decode(scales_r)
        cur = torch.cat([(y_q_r + me[q]) * masks[mk[q]] for q in range(4)], dim=1)
        y_hat_so_far = cur if step == 0 else y_hat_so_far + cur
    return y_hat_so_far * quant_step


def pad_for_y(y):
    """common_model.py:70-78."""
    _, _, H, W = y.size()
    l, r, t, b = get_padding_size(H, W, 4)
    return F.pad(y, (l, r, t, b), mode="replicate"), (-l, -r, -t, -b)


def slice_to_y(p, slice_shape):
    return F.pad(p, slice_shape)


def q_fine(q_scale):
    """load_state_dict fine table (video_model.py:325-341, image_model.py:158-167)."""
    return np.exp(np.linspace(np.log(q_scale[0, 0, 0, 0]), np.log(q_scale[3, 0, 0, 0]), 64))


def curr_q(q_scale_table, q_basic, q_index):
    """get_curr_q (common_model.py:35-37)."""
    return q_basic * q_scale_table[q_index]


# ------------------------------------------------------------ DMC (P-frame)
def offset_diversity(P, p, x, aux, flow, group_num=16, offset_num=2, max_mag=40):
    """OffsetDiversity (models/video_model.py:26-63)."""
    B, C, H, W = x.shape
    out = conv(P, p + ".conv_offset.0", aux, stride=2)
    out = lrelu(out, 0.1)
    out = lrelu(conv(P, p + ".conv_offset.2", out), 0.1)
    out = conv(P, p + ".conv_offset.4", out)
    out = up2(out)
    o1, o2, mask = torch.chunk(out, 3, dim=1)
    mask = torch.sigmoid(mask)
    offset = max_mag * torch.tanh(torch.cat((o1, o2), dim=1))
    offset = offset + flow.repeat(1, group_num * offset_num, 1, 1)
    offset = offset.view(B * group_num * offset_num, 2, H, W)
    mask = mask.view(B * group_num * offset_num, 1, H, W)
    x = x.view(B * group_num, C // group_num, H, W).repeat(offset_num, 1, 1, 1)
    x = flow_warp(x, offset) * mask
    x = x.view(B, C * offset_num, H, W)
    return conv(P, p + ".fusion", x, groups=group_num)


def feature_extractor(P, p, f):
    """FeatureExtractor (models/video_model.py:66-86)."""
    l1 = res_block(P, p + ".res_block1", conv(P, p + ".conv1", f))
    l2 = res_block(P, p + ".res_block2", conv(P, p + ".conv2", l1, stride=2))
    l3 = res_block(P, p + ".res_block3", conv(P, p + ".conv3", l2, stride=2))
    return l1, l2, l3


def context_fusion(P, p, c1, c2, c3):
    """MultiScaleContextFusion (models/video_model.py:89-118)."""
    c3_up = res_block(P, p + ".res_block3_up", subpel(P, p + ".conv3_up", c3))
    c3_out = res_block(P, p + ".res_block3_out", conv(P, p + ".conv3_out", c3))
    c2_up = res_block(P, p + ".res_block2_up", subpel(P, p + ".conv2_up", torch.cat((c3_up, c2), dim=1)))
    c2_out = res_block(P, p + ".res_block2_out", conv(P, p + ".conv2_out", torch.cat((c3_up, c2), dim=1)))
    c1_out = res_block(P, p + ".res_block1_out", conv(P, p + ".conv1_out", torch.cat((c2_up, c1), dim=1)))
    return c1 + c1_out, c2 + c2_out, c3 + c3_out


def mv_enc(P, p, x, context, q):
    """MvEnc (models/video_model.py:121-146)."""
    out = residual_block_with_stride(P, p + ".enc_1.0", x)
    out = depth_conv_block(P, p + ".enc_1.1", out)
    out = out * q
    out = residual_block_with_stride(P, p + ".enc_2", out)
    if context is None:
        out = depth_conv_block(P, p + ".adaptor_0", out)
    else:
        out = depth_conv_block(P, p + ".adaptor_1", torch.cat((out, context), dim=1))
    out = residual_block_with_stride(P, p + ".enc_3.0", out)
    out = depth_conv_block(P, p + ".enc_3.1", out)
    return conv(P, p + ".enc_3.2", out, stride=2)


def mv_dec(P, p, x, q):
    """MvDec (models/video_model.py:149-170)."""
    f = depth_conv_block(P, p + ".dec_1.0", x)
    f = residual_block_upsample(P, p + ".dec_1.1", f)
    f = depth_conv_block(P, p + ".dec_1.2", f)
    f = residual_block_upsample(P, p + ".dec_1.3", f)
    f = depth_conv_block(P, p + ".dec_1.4", f)
    out = residual_block_upsample(P, p + ".dec_2", f)
    out = out * q
    out = depth_conv_block(P, p + ".dec_3.0", out)
    return subpel(P, p + ".dec_3.1", out), f


def contextual_encoder(P, p, x, c1, c2, c3, q):
    """ContextualEncoder (models/video_model.py:173-193)."""
    f = conv(P, p + ".conv1", torch.cat([x, c1], dim=1), stride=2)
    f = res_block(P, p + ".res1", torch.cat([f, c2], dim=1), 0.1, True)
    f = f * q
    f = conv(P, p + ".conv2", f, stride=2)
    f = res_block(P, p + ".res2", torch.cat([f, c3], dim=1), 0.1, True)
    f = conv(P, p + ".conv3", f, stride=2)
    return conv(P, p + ".conv4", f, stride=2)


def contextual_decoder(P, p, x, c2, c3, q):
    """ContextualDecoder (models/video_model.py:196-216)."""
    f = subpel(P, p + ".up1", x)
    f = subpel(P, p + ".up2", f)
    f = res_block(P, p + ".res1", torch.cat([f, c3], dim=1), 0.1, True)
    f = subpel(P, p + ".up3", f)
    f = f * q
    f = res_block(P, p + ".res2", torch.cat([f, c2], dim=1), 0.1, True)
    return subpel(P, p + ".up4", f)


def recon_generation(P, p, ctx, res):
    """ReconGeneration (models/video_model.py:219-232)."""
    f = conv(P, p + ".first_conv", torch.cat((ctx, res), dim=1))
    f = unet(P, p + ".unet_1", f)
    f = unet(P, p + ".unet_2", f)
    return f, conv(P, p + ".recon_conv", f)


class DMCOracle:
    """DMC (models/video_model.py:235-628) as functions of a state_dict."""

    def __init__(self, state_dict, quantize):
        self.P = P = Params(state_dict)
        self.fine = {k: q_fine(P[k].numpy()) for k in
                     ("mv_y_q_scale_enc", "mv_y_q_scale_dec", "y_q_scale_enc", "y_q_scale_dec")}
        g = EntropyTables.gaussian("laplace", quantize)
        self.y_cdf, self.y_sizes, self.y_offsets, self.log_min, self.log_step = g
        self.z_tab = EntropyTables.bit_estimator(P, "bit_estimator_z", G16, quantize)
        self.mvz_tab = EntropyTables.bit_estimator(P, "bit_estimator_z_mv", 64, quantize)

    def get_q(self, q_in_ckpt, q_index):
        """get_q_for_inference (video_model.py:413-423)."""
        P = self.P
        out = []
        for tab, basic in (("mv_y_q_scale_enc", "mv_y_q_basic_enc"), ("mv_y_q_scale_dec", "mv_y_q_basic_dec"),
                           ("y_q_scale_enc", "y_q_basic_enc"), ("y_q_scale_dec", "y_q_basic_dec")):
            table = P[tab] if q_in_ckpt else self.fine[tab]
            out.append(curr_q(table, P[basic], q_index))
        return out

    def mv_prior(self, mv_z_hat, dpb, slice_shape):
        """mv_prior_param_decoder (video_model.py:375-385)."""
        P = self.P
        p = slice_to_y(hyper_dec(P, "mv_hyper_prior_decoder", mv_z_hat), slice_shape)
        if dpb["ref_mv_y"] is None:
            p = depth_conv_block(P, "mv_y_prior_fusion_adaptor_0", p)
        else:
            p = depth_conv_block(P, "mv_y_prior_fusion_adaptor_1", torch.cat((p, dpb["ref_mv_y"]), dim=1))
        p = depth_conv_block(P, "mv_y_prior_fusion.0", p)
        return depth_conv_block(P, "mv_y_prior_fusion.1", p)

    def res_prior(self, z_hat, dpb, c3, slice_shape):
        """res_prior_param_decoder (video_model.py:387-399)."""
        P = self.P
        h = slice_to_y(hyper_dec(P, "contextual_hyper_prior_decoder", z_hat), slice_shape)
        t = lrelu(conv(P, "temporal_prior_encoder.0", c3, stride=2), 0.1)
        t = conv(P, "temporal_prior_encoder.2", t, stride=2)
        if dpb["ref_y"] is None:
            p = depth_conv_block(P, "y_prior_fusion_adaptor_0", torch.cat((t, h), dim=1))
        else:
            p = depth_conv_block(P, "y_prior_fusion_adaptor_1", torch.cat((t, h, dpb["ref_y"]), dim=1))
        p = depth_conv_block(P, "y_prior_fusion.0", p)
        return depth_conv_block(P, "y_prior_fusion.1", p)

    def spatial(self, prefix):
        P = self.P
        return lambda x: depth_conv_block(P, prefix + ".2", depth_conv_block(
            P, prefix + ".1", depth_conv_block(P, prefix + ".0", x)))

    def motion_compensation(self, dpb, mv, frame_idx):
        """motion_compensation + multi_scale_feature_extractor (video_model.py:343-364)."""
        P = self.P
        warpframe = flow_warp(dpb["ref_frame"], mv)
        mv2 = down2(mv) / 2
        mv3 = down2(mv2) / 2
        if dpb["ref_feature"] is None:
            f = conv(P, "feature_adaptor_I", dpb["ref_frame"])
        else:
            f = conv(P, f"feature_adaptor.{[0, 1, 0, 2][frame_idx % 4]}", dpb["ref_feature"])
        r1, r2, r3 = feature_extractor(P, "feature_extractor", f)
        c1_init = flow_warp(r1, mv)
        c1 = offset_diversity(P, "align", r1, torch.cat((c1_init, warpframe, mv), dim=1), mv)
        c2 = flow_warp(r2, mv2)
        c3 = flow_warp(r3, mv3)
        return context_fusion(P, "context_fusion_net", c1, c2, c3)

    def recon(self, y_hat, c1, c2, c3, y_q_dec):
        """get_recon_and_feature (video_model.py:401-405)."""
        P = self.P
        r = contextual_decoder(P, "contextual_decoder", y_hat, c2, c3, y_q_dec)
        feature, x_hat = recon_generation(P, "recon_generation_net", r, c1)
        return x_hat.clamp_(0, 1), feature

    _MV_AD = ["mv_y_spatial_prior_adaptor_1", "mv_y_spatial_prior_adaptor_2", "mv_y_spatial_prior_adaptor_3"]
    _Y_AD = ["y_spatial_prior_adaptor_1", "y_spatial_prior_adaptor_2", "y_spatial_prior_adaptor_3"]

    def compress(self, x, dpb, q_in_ckpt, q_index, frame_idx, tap=None, recon=False, force=None):
        """compress (video_model.py:425-481) minus the encoder-side
        reconstruction, whose output is unused in write mode.  Returns the
        ordered list of coder calls [(kind, symbols, indexes)] and the dpb.

        Test instrumentation: ``tap`` (a dict) receives, per coder call, the
        pre-rounding values ("pre": z or y - means) and the pre-truncation
        scale indexes ("idx_f", y calls), plus the calls in dependency order
        ("order": mv_z, mv_y steps, z, y steps).  ``recon=True`` also returns
        the decoder-side dpb, built from the encoder's y_hat (the same values
        decompress() reconstructs from the stream).  ``force`` (a Forcer over
        the calls in stream order) replays another coder's symbols at ties."""
        P = self.P
        fa = force.apply if force is not None else (lambda c, pre, q, m=None: q)
        mv_q_enc, mv_q_dec, y_q_enc, y_q_dec = self.get_q(q_in_ckpt, q_index)
        est_mv = spynet(P, "optic_flow", x, dpb["ref_frame"])
        mv_y = mv_enc(P, "mv_encoder", est_mv, dpb["ref_mv_feature"], mv_q_enc)
        mv_y_pad, ss = pad_for_y(mv_y)
        mv_z = hyper_enc(P, "mv_hyper_prior_encoder", mv_y_pad, False)
        mv_z_hat = fa(0, mv_z, torch.round(mv_z))
        mv_params = self.mv_prior(mv_z_hat, dpb, ss)
        mv_res, y_res = [], []
        mv_sym, mv_sc, _, mv_y_hat, _ = four_part_prior(P, mv_y, mv_params, self._MV_AD,
                                                        self.spatial("mv_y_spatial_prior"), mv_res, force, 2)
        mv_hat, mv_feature = mv_dec(P, "mv_decoder", mv_y_hat, mv_q_dec)
        c1, c2, c3 = self.motion_compensation(dpb, mv_hat, frame_idx)
        y = contextual_encoder(P, "contextual_encoder", x, c1, c2, c3, y_q_enc)
        y_pad, ss = pad_for_y(y)
        z = hyper_enc(P, "contextual_hyper_prior_encoder", y_pad, True)
        z_hat = fa(1, z, torch.round(z))
        params = self.res_prior(z_hat, dpb, c3, ss)
        y_sym, y_sc, _, y_hat, _ = four_part_prior(P, y, params, self._Y_AD, self.spatial("y_spatial_prior"), y_res,
                                                   force, 6)
        calls = [("mvz", mv_z_hat, channel_indexes(mv_z_hat)), ("z", z_hat, channel_indexes(z_hat))]
        for s, sc in zip(mv_sym, mv_sc):
            calls.append(("y", s, build_indexes(sc, self.log_min, self.log_step)))
        for s, sc in zip(y_sym, y_sc):
            calls.append(("y", s, build_indexes(sc, self.log_min, self.log_step)))
        if tap is not None:
            tap["pre"] = [mv_z, z] + mv_res + y_res
            tap["idx_f"] = [None, None] + [index_float(sc, self.log_min, self.log_step) for sc in mv_sc + y_sc]
            tap["order"] = [0, 2, 3, 4, 5, 1, 6, 7, 8, 9]
        if recon:
            x_hat, feature = self.recon(y_hat, c1, c2, c3, y_q_dec)
            return calls, {"ref_frame": x_hat, "ref_feature": feature, "ref_mv_feature": mv_feature,
                           "ref_y": y_hat, "ref_mv_y": mv_y_hat}
        return calls

    def decompress(self, dpb, decoder, height, width, q_in_ckpt, q_index, frame_idx):
        """decompress (video_model.py:483-520); ``decoder(kind, indexes)``
        returns decoded symbols as an int array."""
        P = self.P
        _, mv_q_dec, _, y_q_dec = self.get_q(q_in_ckpt, q_index)
        zh, zw = get_downsampled_shape(height, width, 64)
        yh, yw = get_downsampled_shape(height, width, 16)
        l, r, t, b = get_padding_size(yh, yw, 4)
        ss = (-l, -r, -t, -b)
        mvz_idx = channel_indexes(torch.zeros(1, 64, zh, zw))
        mv_z_hat = torch.tensor(decoder("mvz", mvz_idx), dtype=torch.float32).reshape(1, 64, zh, zw)
        z_idx = channel_indexes(torch.zeros(1, G16, zh, zw))
        z_hat = torch.tensor(decoder("z", z_idx), dtype=torch.float32).reshape(1, G16, zh, zw)

        def dec_y(scales_r):
            idx = build_indexes(scales_r, self.log_min, self.log_step)
            return torch.tensor(decoder("y", idx), dtype=torch.float32).reshape(scales_r.shape)

        mv_params = self.mv_prior(mv_z_hat, dpb, ss)
        mv_y_hat = four_part_decompress(P, mv_params, self._MV_AD, self.spatial("mv_y_spatial_prior"), dec_y)
        mv_hat, mv_feature = mv_dec(P, "mv_decoder", mv_y_hat, mv_q_dec)
        c1, c2, c3 = self.motion_compensation(dpb, mv_hat, frame_idx)
        params = self.res_prior(z_hat, dpb, c3, ss)
        y_hat = four_part_decompress(P, params, self._Y_AD, self.spatial("y_spatial_prior"), dec_y)
        x_hat, feature = self.recon(y_hat, c1, c2, c3, y_q_dec)
        return {"ref_frame": x_hat, "ref_feature": feature, "ref_mv_feature": mv_feature,
                "ref_y": y_hat, "ref_mv_y": mv_y_hat}

    def forward_one_frame(self, x, dpb, q_in_ckpt, q_index, frame_idx):
        """Estimate mode (video_model.py:559-628): returns (bits, dpb)."""
        P = self.P
        mv_q_enc, mv_q_dec, y_q_enc, y_q_dec = self.get_q(q_in_ckpt, q_index)
        est_mv = spynet(P, "optic_flow", x, dpb["ref_frame"])
        mv_y = mv_enc(P, "mv_encoder", est_mv, dpb["ref_mv_feature"], mv_q_enc)
        mv_y_pad, ss = pad_for_y(mv_y)
        mv_z_hat = torch.round(hyper_enc(P, "mv_hyper_prior_encoder", mv_y_pad, False))
        mv_params = self.mv_prior(mv_z_hat, dpb, ss)
        _, _, mv_y_q, mv_y_hat, mv_scales_hat = four_part_prior(
            P, mv_y, mv_params, self._MV_AD, self.spatial("mv_y_spatial_prior"))
        mv_hat, mv_feature = mv_dec(P, "mv_decoder", mv_y_hat, mv_q_dec)
        c1, c2, c3 = self.motion_compensation(dpb, mv_hat, frame_idx)
        y = contextual_encoder(P, "contextual_encoder", x, c1, c2, c3, y_q_enc)
        y_pad, ss = pad_for_y(y)
        z_hat = torch.round(hyper_enc(P, "contextual_hyper_prior_encoder", y_pad, True))
        params = self.res_prior(z_hat, dpb, c3, ss)
        _, _, y_q, y_hat, scales_hat = four_part_prior(P, y, params, self._Y_AD, self.spatial("y_spatial_prior"))
        x_hat, feature = self.recon(y_hat, c1, c2, c3, y_q_dec)
        _, _, H, W = x.size()
        n = H * W
        bpp = (torch.sum(laplace_bits(y_q, scales_hat), dim=(1, 2, 3)) / n
               + torch.sum(z_bits(P, "bit_estimator_z", z_hat), dim=(1, 2, 3)) / n
               + torch.sum(laplace_bits(mv_y_q, mv_scales_hat), dim=(1, 2, 3)) / n
               + torch.sum(z_bits(P, "bit_estimator_z_mv", mv_z_hat), dim=(1, 2, 3)) / n)
        bit = torch.sum(bpp) * n
        dpb = {"ref_frame": x_hat, "ref_feature": feature, "ref_mv_feature": mv_feature,
               "ref_y": y_hat, "ref_mv_y": mv_y_hat}
        return bit.item(), dpb


def channel_indexes(x):
    """BitEstimator.build_indexes (models/entropy_models.py:179-183)."""
    N, C, H, W = x.shape
    return torch.arange(C, dtype=torch.int).view(1, -1, 1, 1).repeat(N, 1, H, W)


# ------------------------------------------------------- IntraNoAR (I-frame)
class IntraOracle:
    """IntraNoAR (models/image_model.py:61-252) as functions of a state_dict."""

    def __init__(self, state_dict, quantize, N=256):
        self.P = P = Params(state_dict)
        self.N = N
        self.fine = {k: q_fine(P[k].numpy()) for k in ("q_scale_enc", "q_scale_dec")}
        g = EntropyTables.gaussian("gaussian", quantize)
        self.y_cdf, self.y_sizes, self.y_offsets, self.log_min, self.log_step = g
        self.z_tab = EntropyTables.bit_estimator(P, "bit_estimator_z", N, quantize)

    def get_q(self, q_in_ckpt, q_index):
        """get_q_for_inference (image_model.py:107-112)."""
        P = self.P
        enc = P["q_scale_enc"][:, 0, 0, 0] if q_in_ckpt else self.fine["q_scale_enc"]
        dec = P["q_scale_dec"][:, 0, 0, 0] if q_in_ckpt else self.fine["q_scale_dec"]
        return curr_q(enc, P["q_basic_enc"], q_index), curr_q(dec, P["q_basic_dec"], q_index)

    def enc(self, x, q):
        """IntraEncoder (image_model.py:16-35)."""
        P = self.P
        out = residual_block_with_stride(P, "enc.enc_1.0", x)
        out = depth_conv_block2(P, "enc.enc_1.1", out)
        out = out * q
        out = residual_block_with_stride(P, "enc.enc_2.0", out)
        out = depth_conv_block2(P, "enc.enc_2.1", out)
        out = residual_block_with_stride(P, "enc.enc_2.2", out)
        out = depth_conv_block2(P, "enc.enc_2.3", out)
        return conv(P, "enc.enc_2.4", out, stride=2)

    def dec(self, x, q):
        """IntraDecoder (image_model.py:38-58)."""
        P = self.P
        out = depth_conv_block2(P, "dec.dec_1.0", x)
        out = residual_block_upsample(P, "dec.dec_1.1", out)
        out = depth_conv_block2(P, "dec.dec_1.2", out)
        out = residual_block_upsample(P, "dec.dec_1.3", out)
        out = depth_conv_block2(P, "dec.dec_1.4", out)
        out = residual_block_upsample(P, "dec.dec_1.5", out)
        out = out * q
        out = depth_conv_block2(P, "dec.dec_2.0", out)
        return residual_block_upsample(P, "dec.dec_2.1", out)

    def refine(self, x):
        """refine = UNet2 + conv3x3 (image_model.py:95-98)."""
        return conv(self.P, "refine.1", unet(self.P, "refine.0", x, block=depth_conv_block2))

    def hyper(self, y):
        P = self.P
        y_pad, ss = pad_for_y(y)
        z = depth_conv_block2(P, "hyper_enc.0", y_pad)
        z = lrelu(conv(P, "hyper_enc.1", z, stride=2))
        z = conv(P, "hyper_enc.3", z, stride=2)
        return torch.round(z), ss

    def prior(self, z_hat, ss):
        P = self.P
        p = residual_block_upsample(P, "hyper_dec.0", z_hat)
        p = residual_block_upsample(P, "hyper_dec.1", p)
        p = depth_conv_block2(P, "hyper_dec.2", p)
        p = depth_conv_block2(P, "y_prior_fusion.0", p)
        p = depth_conv_block2(P, "y_prior_fusion.1", p)
        return slice_to_y(p, ss)

    def spatial(self, x):
        P = self.P
        for i in range(3):
            x = depth_conv_block2(P, f"y_spatial_prior.{i}", x)
        return x

    _AD = ["y_spatial_prior_adaptor_1", "y_spatial_prior_adaptor_2", "y_spatial_prior_adaptor_3"]

    def compress(self, x, q_in_ckpt, q_index, tap=None, recon=False, force=None):
        """compress (image_model.py:198-229) without the unused encoder recon;
        ``tap`` / ``recon`` / ``force`` as in DMCOracle.compress."""
        q_enc, q_dec = self.get_q(q_in_ckpt, q_index)
        y = self.enc(x, q_enc)
        y_pad, ss = pad_for_y(y)
        P = self.P
        z = depth_conv_block2(P, "hyper_enc.0", y_pad)
        z = lrelu(conv(P, "hyper_enc.1", z, stride=2))
        z = conv(P, "hyper_enc.3", z, stride=2)
        z_hat = torch.round(z) if force is None else force.apply(0, z, torch.round(z))
        params = self.prior(z_hat, ss)
        y_res = []
        sym, sc, _, y_hat, _ = four_part_prior(self.P, y, params, self._AD, self.spatial, y_res, force, 1)
        calls = [("z", z_hat, channel_indexes(z_hat))]
        for s, c in zip(sym, sc):
            calls.append(("y", s, build_indexes(c, self.log_min, self.log_step)))
        if tap is not None:
            tap["pre"] = [z] + y_res
            tap["idx_f"] = [None] + [index_float(c, self.log_min, self.log_step) for c in sc]
            tap["order"] = [0, 1, 2, 3, 4]
        if recon:
            return calls, self.refine(self.dec(y_hat, q_dec)).clamp_(0, 1)
        return calls

    def decompress(self, decoder, height, width, q_in_ckpt, q_index):
        """decompress (image_model.py:231-252)."""
        _, q_dec = self.get_q(q_in_ckpt, q_index)
        zh, zw = get_downsampled_shape(height, width, 64)
        yh, yw = get_downsampled_shape(height, width, 16)
        l, r, t, b = get_padding_size(yh, yw, 4)
        z_idx = channel_indexes(torch.zeros(1, self.N, zh, zw))
        z_hat = torch.tensor(decoder("z", z_idx), dtype=torch.float32).reshape(1, self.N, zh, zw)
        params = self.prior(z_hat, (-l, -r, -t, -b))

        def dec_y(scales_r):
            idx = build_indexes(scales_r, self.log_min, self.log_step)
            return torch.tensor(decoder("y", idx), dtype=torch.float32).reshape(scales_r.shape)

        y_hat = four_part_decompress(self.P, params, self._AD, self.spatial, dec_y)
        return self.refine(self.dec(y_hat, q_dec)).clamp_(0, 1)

    def forward(self, x, q_in_ckpt, q_index):
        """Estimate mode (image_model.py:114-149): returns (bits, x_hat)."""
        q_enc, q_dec = self.get_q(q_in_ckpt, q_index)
        y = self.enc(x, q_enc)
        z_hat, ss = self.hyper(y)
        params = self.prior(z_hat, ss)
        _, _, y_q, y_hat, scales_hat = four_part_prior(self.P, y, params, self._AD, self.spatial)
        x_hat = self.refine(self.dec(y_hat, q_dec))
        _, _, H, W = x.size()
        n = H * W
        bpp = (torch.sum(gaussian_bits(y_q, scales_hat), dim=(1, 2, 3)) / n
               + torch.sum(z_bits(self.P, "bit_estimator_z", z_hat), dim=(1, 2, 3)) / n)
        return (torch.sum(bpp) * n).item(), x_hat
