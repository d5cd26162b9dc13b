"""Shared pieces of the HEM codecs: the dual (checkerboard) prior driver
(DCVC-HEM/src/models/common_model.py:84-188), the q-step helpers and the
HEM entropy coder session (single headerless int32 stream,
DCVC-HEM/src/entropy_models/entropy_models.py:9-51)."""
import numpy as np
import torch

from .. import hip as K
from ..hip import F32
from ..rans import BufferedRansEncoder, HemRansDecoder
from .layers import Seq3


class DualPrior:
    """forward/compress/decompress_dual_prior on the GPU.  The spatial
    prior's input is one fp32 NHWC buffer of 4C channels,
    [y_hat_0_0 | y_hat_1_1 | means | scales | quant_step]; the prior fusion
    writes channels [C, 4C) (its last conv permuted to that order) and step 0
    writes the y_hat part."""

    def __init__(self, ctx, spatial_prefix, C):
        self.C = C
        self.spatial = Seq3(ctx, spatial_prefix)
        self.ctx = ctx

    def new_buffer(self, h, w):
        return K.empty(h, w, 4 * self.C, F32, self.ctx.dev)

    def params_view(self, buf):
        return buf.ch(self.C, 3 * self.C)

    def encode(self, y, buf, post, sym_slices, idx_slices, scale_table):
        yhat = K.empty(y.H, y.W, self.C, F32, self.ctx.dev)
        for k in range(2):
            sm = None if k == 0 else self.spatial(buf)
            K.dp_encode_step(y, buf, sm, k, yhat, post, sym_slices[k], idx_slices[k], scale_table.log_min,
                             scale_table.log_step)
        return yhat

    def estimate(self, y, buf, post, bits, gaussian):
        yhat = K.empty(y.H, y.W, self.C, F32, self.ctx.dev)
        n = y.H * y.W * (self.C // 2)
        smin = 0.11 if gaussian else 1e-5  # get_y_gaussian_bits / get_y_laplace_bits
        for k in range(2):
            sm = None if k == 0 else self.spatial(buf)
            K.dp_estimate_step(y, buf, sm, k, yhat, post, bits[k * n:(k + 1) * n], gaussian, smin)
        return yhat

    def decode(self, buf, post, decode_fn, scale_table):
        """decode_fn(host int16 indexes) -> host int32 symbols."""
        dev = self.ctx.dev
        n = buf.H * buf.W * (self.C // 2)
        yhat = K.empty(buf.H, buf.W, self.C, F32, dev)
        idx_d = torch.empty(n, dtype=torch.int16, device=dev)
        idx_h = K.pinned("prior_idx", n, torch.int16)
        sym_h = K.pinned("prior_sym", n, torch.int32)
        sym_d = torch.empty(n, dtype=torch.int32, device=dev)
        for k in range(2):
            sm = None if k == 0 else self.spatial(buf)
            K.dp_indexes_step(buf, sm, k, idx_d, scale_table.log_min, scale_table.log_step)
            idx_h.copy_(idx_d, non_blocking=K.ASYNC_COPIES)
            torch.cuda.current_stream().synchronize()
            sym_h.numpy()[:] = decode_fn(idx_h.numpy())
            sym_d.copy_(sym_h, non_blocking=K.ASYNC_COPIES)
            K.dp_decode_step(buf, sm, k, sym_d, yhat, post)
        return yhat


def lower_bound_q(basic, q_scale, device):
    """get_curr_q (LowerBound(q_basic, 0.5) * q_scale, video_model.py:251-261)
    in fp32 on the host CPU, uploaded as a per-channel vector."""
    b = basic.detach().float().cpu()
    q = torch.max(b, torch.ones_like(b) * 0.5) * q_scale
    return q.reshape(-1).contiguous().to(device)


def get_rounded_q(q_scale):
    """stream_helper.get_rounded_q (DCVC-HEM/src/utils/stream_helper.py:40-44)."""
    q_scale = np.clip(q_scale, 0.01, 655.)
    q_index = int(np.round(q_scale * 100))
    return q_index / 100, q_index


class HemEntropyCoder:
    """EntropyCoder (entropy_models.py:9-51): BufferedRansEncoder +
    RansDecoder over int32 symbols, one headerless stream."""

    def __init__(self):
        self.encoder = BufferedRansEncoder()
        self.decoder = HemRansDecoder()
        self.trace = None

    def reset_encoder(self):
        self.encoder.reset()

    def encode(self, symbols, indexes, table):
        if self.trace is not None:
            self.trace.append(("enc", np.array(symbols, copy=True), np.array(indexes, copy=True)))
        self.encoder.encode_table(symbols, indexes, table)

    def flush_encoder(self):
        return self.encoder.flush()

    def set_stream(self, stream):
        self.decoder.set_stream(stream)

    def decode(self, indexes, table):
        out = self.decoder.decode_table(indexes, table)
        if self.trace is not None:
            self.trace.append(("dec", out.copy(), np.array(indexes, copy=True)))
        return out
