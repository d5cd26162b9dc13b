"""Shared pieces of the DC codecs: the quadtree (four-part) prior driver and
per-frame symbol staging (DCVC-DC/src/models/common_model.py:13-321)."""
import numpy as np
import torch

from .. import hip as K
from ..hip import F32
from ..layers import DepthConvBlock, cast
from ..stream_helper import get_padding_size


class SymbolBuffer:
    """Device int16 staging for one frame's coder calls: every call's
    symbols (and indexes) land in one device buffer that is copied to pinned
    host memory with a single transfer."""

    def __init__(self, device, sym_dtype=torch.int16):
        self.dev = device
        self.sym_dtype = sym_dtype  # int16 (DC coder) or int32 (HEM coder)
        self.sizes = []
        self.kinds = []

    def plan(self, kind, n):
        self.kinds.append(kind)
        self.sizes.append(n)
        return len(self.sizes) - 1

    def alloc(self):
        total = int(sum(self.sizes))
        self.sym = torch.empty(total, dtype=self.sym_dtype, device=self.dev)
        self.idx = torch.empty(total, dtype=torch.int16, device=self.dev)
        self.offs = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
        return self

    def sym_slice(self, i):
        return self.sym[self.offs[i]:self.offs[i + 1]]

    def idx_slice(self, i):
        return self.idx[self.offs[i]:self.offs[i + 1]]

    def to_host(self):
        s = K.pinned("sb_sym", self.sym.numel(), self.sym_dtype)
        x = K.pinned("sb_idx", self.idx.numel(), torch.int16)
        s.copy_(self.sym, non_blocking=K.ASYNC_COPIES)
        x.copy_(self.idx, non_blocking=K.ASYNC_COPIES)
        torch.cuda.current_stream().synchronize()
        s, x = s.numpy(), x.numpy()
        return [(s[self.offs[i]:self.offs[i + 1]], x[self.offs[i]:self.offs[i + 1]]) for i in range(len(self.sizes))]


class QuadtreePrior:
    """forward/compress/decompress_four_part_prior (common_model.py:142-321).

    The spatial-prior input cat(y_hat_so_far, common_params) is one fp32
    NHWC buffer of 4C channels: the prior fusion writes common_params into
    channels [C, 4C) and the quantise kernels write y_hat_so_far into [0, C).
    """

    def __init__(self, ctx, adaptor_names, spatial_prefix, C, gated, nblocks=3):
        self.C = C
        self.adaptors = [ctx.conv(n, latent=True) for n in adaptor_names]
        self.spatial = [DepthConvBlock(ctx, f"{spatial_prefix}.{i}", gated=gated, latent=True)
                        for i in range(nblocks)]
        self.ctx = ctx

    def new_buffer(self, h, w):
        buf = K.empty(h, w, 4 * self.C, F32, self.ctx.dev)
        K.fill(buf.ch(0, self.C), 0.0)  # y_hat_so_far starts at zero
        return buf

    def step_params(self, buf, k):
        x = K.conv(self.adaptors[k - 1], buf)
        for b in self.spatial:
            x = b(x)
        return x  # 2C: scales_0..3 | means_0..3

    def encode(self, y, buf, symbuf, calls, scale_table):
        C = self.C
        yhat = K.empty(y.H, y.W, C, F32, self.ctx.dev)
        params = buf.ch(C, 3 * C)
        for k in range(4):
            sm = None if k == 0 else self.step_params(buf, k)
            K.qt_encode_step(y, params, sm, k, buf.ch(0, C), yhat, symbuf.sym_slice(calls[k]),
                             symbuf.idx_slice(calls[k]), scale_table.log_min, scale_table.log_step)
        return yhat

    def estimate(self, y, buf, bits, gaussian):
        """forward_four_part_prior (write=False) on the GPU: y_hat and, per
        element, its estimated bits (bits: fp32 device tensor of C*h*w)."""
        C = self.C
        yhat = K.empty(y.H, y.W, C, F32, self.ctx.dev)
        params = buf.ch(C, 3 * C)
        n = y.H * y.W * (C // 4)
        for k in range(4):
            sm = None if k == 0 else self.step_params(buf, k)
            K.qt_estimate_step(y, params, sm, k, buf.ch(0, C), yhat, bits[k * n:(k + 1) * n], gaussian)
        return yhat

    def decode(self, buf, decode_fn, scale_table):
        """decode_fn(host int16 indexes) -> host int16 symbols."""
        C = self.C
        h, w = buf.H, buf.W
        n = h * w * (C // 4)
        dev = self.ctx.dev
        yhat = K.empty(h, w, C, F32, dev)
        params = buf.ch(C, 3 * C)
        idx_d = torch.empty(n, dtype=torch.int16, device=dev)
        idx_h = K.pinned("prior_idx", n, torch.int16)
        sym_h = K.pinned("prior_sym", n, torch.int16)
        sym_d = torch.empty(n, dtype=torch.int16, device=dev)
        for k in range(4):
            sm = None if k == 0 else self.step_params(buf, k)
            K.qt_indexes_step(params, sm, k, idx_d, scale_table.log_min, scale_table.log_step)
            idx_h.copy_(idx_d, non_blocking=K.ASYNC_COPIES)
            torch.cuda.current_stream().synchronize()
            sym_h.numpy()[:] = decode_fn(idx_h.numpy())
            sym_d.copy_(sym_h, non_blocking=K.ASYNC_COPIES)
            K.qt_decode_step(params, sm, k, sym_d, buf.ch(0, C), yhat)
        return yhat


class BitCounter:
    """Estimate-mode bit totals on the GPU: per-element bits buffers summed
    in a fixed order (dcvc_sum_f32), one host transfer for all totals."""

    def __init__(self, device, names):
        self.dev = device
        self.names = list(names)
        self.tot = torch.empty(len(self.names), dtype=torch.float32, device=device)
        self.bufs = {}

    def buffer(self, name, n):
        b = torch.empty(n, dtype=torch.float32, device=self.dev)
        self.bufs[name] = b
        return b

    def factorized(self, name, z, table):
        b = self.buffer(name, z.H * z.W * z.C)
        K.factorized_bits(z, table.chain_on(self.dev), b)

    def totals(self):
        for i, n in enumerate(self.names):
            K.sum_f32(self.bufs[n], self.tot[i:i + 1])
        host = self.tot.cpu().numpy()
        return {n: np.float32(host[i]) for i, n in enumerate(self.names)}


def bits_result(tot, pixel_num, names):
    """bpp_k = sum(bits_k) / pixel_num, bit = sum(bpp) * pixel_num, in fp32
    as the reference computes them (video_model.py:602-612)."""
    n = np.float32(pixel_num)
    bpp = {k: np.float32(tot[k]) / n for k in names}
    total = np.float32(0)
    for k in names:
        total = np.float32(total + bpp[k])
    out = {"bpp_" + k: float(bpp[k]) for k in names}
    out["bpp"] = float(total)
    out["bit"] = float(np.float32(total * n))
    for k in names:
        out["bit_" + k] = float(np.float32(bpp[k] * n))
    return out


def pad_for_y(y):
    """common_model.py:70-78: replicate-pad the latent to a multiple of 4."""
    _, r, _, b = get_padding_size(y.H, y.W, 4)
    if r == 0 and b == 0:
        return y
    out = K.empty(y.H + b, y.W + r, y.C, y.dtype, y.buf.device)
    return K.pad_replicate(y, out)


def crop_to(x, h, w, y=None):
    """slice_to_y (common_model.py:85-86): top-left crop."""
    if x.H == h and x.W == w and y is None:
        return x
    if y is None:
        y = K.empty(h, w, x.C, x.dtype, x.buf.device)
    return K.pad_replicate(x, y)


def q_fine(q_scale):
    """load_state_dict fine tables (video_model.py:325-341)."""
    q = q_scale.detach().float().cpu()
    return np.exp(np.linspace(np.log(q[0, 0, 0, 0]), np.log(q[3, 0, 0, 0]), 64))


def curr_q(table, basic, q_index, device):
    """get_curr_q (common_model.py:35-37) on the host CPU, uploaded as a
    per-channel fp32 vector."""
    q = basic.detach().float().cpu() * table[q_index]
    return q.reshape(-1).contiguous().to(device)


__all__ = ["SymbolBuffer", "QuadtreePrior", "BitCounter", "bits_result", "pad_for_y", "crop_to", "q_fine", "curr_q", "cast"]
