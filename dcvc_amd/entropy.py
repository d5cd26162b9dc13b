"""Host-side entropy model: CDF tables and the per-frame coder session.

Tables are built once at ``update()`` on the host CPU, in fp32 with the same
torch.distributions arithmetic as the reference
(DCVC-DC/src/models/entropy_models.py:124-178 BitEstimator.update,
:228-267 GaussianEncoder.update), quantised by libdcvc_rans's
pmf_to_quantized_cdf, and uploaded once as ``CdfTable`` handles.  They are
computed on the CPU on purpose: the reference's parity target is its CPU
path, and the tables are an input to the bitstream.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from .rans import CdfTable, pmf_to_quantized_cdf, RansEncoder, RansDecoder

GAUSSIAN_TABLES = {  # distribution -> (cdf class, scale_min, scale_max, levels)
    "laplace": (torch.distributions.laplace.Laplace, 0.01, 64.0, 256),
    "gaussian": (torch.distributions.normal.Normal, 0.11, 64.0, 256),
}


def _quantize_rows(pmfs, tails, lengths, max_length):
    cdf = np.zeros((len(lengths), int(max_length) + 2), dtype=np.int32)
    for i, p in enumerate(pmfs):
        n = int(lengths[i])
        prob = torch.cat((p[:n], tails[i]), dim=0)
        q = pmf_to_quantized_cdf(prob.tolist(), 16)
        cdf[i, :len(q)] = q
    return cdf


class ScaleTable:
    """GaussianEncoder: 256 log-spaced scales -> CDF rows; scale -> index."""

    def __init__(self, distribution):
        dist, smin, smax, levels = GAUSSIAN_TABLES[distribution]
        self.log_min = math.log(smin)
        self.log_step = (math.log(smax) - self.log_min) / (levels - 1)
        scales = torch.exp(torch.linspace(math.log(smin), math.log(smax), levels))
        center = torch.zeros_like(scales) + 50
        d = dist(torch.zeros_like(scales), torch.zeros_like(center) + scales)
        for i in range(50, 1, -1):
            p = torch.squeeze(d.cdf(torch.zeros_like(center) + i))
            center = torch.where(p > torch.zeros_like(center) + 0.9999, torch.zeros_like(center) + i, center)
        center = center.int()
        length = 2 * center + 1
        max_length = int(torch.max(length).item())
        x = (torch.arange(max_length) - center[:, None]).float()
        d = dist(torch.zeros_like(x), torch.zeros_like(x) + scales[:, None])
        upper, lower = d.cdf(x + 0.5), d.cdf(x - 0.5)
        cdf = _quantize_rows(upper - lower, 2 * lower[:, :1], length, max_length)
        self.cdf, self.sizes, self.offsets = cdf, (length + 2).int().numpy(), (-center).int().numpy()
        self.table = CdfTable(self.cdf, self.sizes, self.offsets)


def factorized_cdf(params, prefix, x):
    """BitEstimator CDF: sigmoid of 4 Bitparm layers (entropy_models.py:58-77,111-122)."""
    for i in range(1, 5):
        q = f"{prefix}.f{i}"
        x = x * F.softplus(params[q + ".h"]) + params[q + ".b"]
        if i < 4:
            x = x + torch.tanh(x) * torch.tanh(params[q + ".a"])
    return torch.sigmoid(x)


class FactorizedTable:
    """BitEstimator.update: per-channel support search then CDF rows."""

    def __init__(self, state_dict, prefix, channel):
        P = {k: v.detach().float().cpu() for k, v in state_dict.items() if k.startswith(prefix + ".")}
        med = torch.zeros(channel)
        lo, hi = med + 50, med + 50
        for i in range(50, 1, -1):
            p = torch.squeeze(factorized_cdf(P, prefix, (torch.zeros_like(med) - i)[None, :, None, None]))
            lo = torch.where(p < torch.zeros_like(med) + 0.0001, torch.zeros_like(med) + i, lo)
        for i in range(50, 1, -1):
            p = torch.squeeze(factorized_cdf(P, prefix, (torch.zeros_like(med) + i)[None, :, None, None]))
            hi = torch.where(p > torch.zeros_like(med) + 0.9999, torch.zeros_like(med) + i, hi)
        lo, hi = lo.int(), hi.int()
        length = hi + lo + 1
        max_length = length.max()
        x = torch.arange(max_length)[None, :] + (med - lo)[:, None, None]
        lower = factorized_cdf(P, prefix, x - 0.5).squeeze(0)
        upper = factorized_cdf(P, prefix, x + 0.5).squeeze(0)
        pmf = (upper - lower)[:, 0, :]
        tail = lower[:, 0, :1] + (1.0 - upper[:, 0, -1:])
        self.cdf = _quantize_rows(pmf, tail, length, max_length)
        self.sizes, self.offsets = (length + 2).int().numpy(), (-lo).int().numpy()
        self.table = CdfTable(self.cdf, self.sizes, self.offsets)
        self.channel = channel
        # per-channel constants of the Bitparm chain for estimate-mode bits
        # (dcvc_factorized_bits): softplus(h), b, tanh(a) per layer, in fp32
        # with the reference's own torch ops
        cols = []
        for i in range(1, 5):
            q = f"{prefix}.f{i}"
            cols += [F.softplus(P[q + ".h"]).reshape(-1), P[q + ".b"].reshape(-1)]
            if i < 4:
                cols.append(torch.tanh(P[q + ".a"]).reshape(-1))
        self.chain = torch.stack(cols, dim=1).float().contiguous()  # [C][11]
        self._chain_dev = {}

    def chain_on(self, device):
        if device not in self._chain_dev:
            self._chain_dev[device] = self.chain.to(device)
        return self._chain_dev[device]

    def indexes(self, h, w):
        """BitEstimator.build_indexes (entropy_models.py:179-183), NCHW order."""
        return np.repeat(np.arange(self.channel, dtype=np.int16), h * w)


class EntropyCoder:
    """One encoder + one decoder, the reference's EntropyCoder
    (entropy_models.py:9-55): ec_thread / stream_part select the threaded and
    multi-part coder."""

    def __init__(self, ec_thread=False, stream_part=1):
        self.encoder = RansEncoder(ec_thread, stream_part)
        self.decoder = RansDecoder(stream_part)
        self.trace = None  # set to a list to record (side, symbols, indexes)

    def reset(self):
        self.encoder.reset()

    def encode(self, symbols, indexes, table):
        if self.trace is not None:
            self.trace.append(("enc", np.array(symbols, copy=True), np.array(indexes, copy=True)))
        self.encoder.encode_table(symbols, indexes, table)

    def flush(self):
        self.encoder.flush()

    def get_encoded_stream(self):
        return self.encoder.get_encoded_stream().tobytes()

    def set_stream(self, stream):
        self.decoder.set_stream(np.frombuffer(stream, dtype=np.uint8))

    def decode(self, indexes, table):
        out = self.decoder.decode_table(indexes, table)
        if self.trace is not None:
            self.trace.append(("dec", out.copy(), np.array(indexes, copy=True)))
        return out
