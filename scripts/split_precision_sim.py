"""CPU emulation of candidate conv arithmetics against the strict parity bar.

Runs the DCVC-DC oracle twice on the same (teacher-forced) inputs: once in
fp32 (the reference arithmetic) and once with every dense conv computed from
rounded / split operands, then applies tests/parity.py's strict comparison.
This is how the split-operand precision mode was chosen: it
shows, before any kernel is written, which operand formats keep every
differing symbol / index on a rounding tie.

  modes: fp32 | bf16 | bf16x3 | fp16x3 | fp16x3s (fp16 split with power-of-2
  operand scaling) | fp16x3w (weights scaled only) ; --feat-only keeps the latent-rate convs fp32.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as Fn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import dc_oracle as O          # noqa: E402
from oracle import rans_oracle as R        # noqa: E402
from tests.parity import compare_frame     # noqa: E402


def split(t, dt):
    hi = t.to(dt).float()
    lo = (t - hi).to(dt).float()
    return hi, lo


def pow2_scale(t):
    m = float(t.abs().max())
    if m == 0:
        return 1.0
    import math
    return 2.0 ** (14 - math.ceil(math.log2(m)))   # max |t| * s in [2^13, 2^14]


STATS = {"n": 0, "xmax": 0.0, "wmax": 0.0, "xmin_nz": 1e30}


def make_conv(mode, feat_min_hw):
    def conv(P, name, x, stride=1, groups=1):
        w = P[name + ".weight"]
        k = w.shape[-1]
        b = P[name + ".bias"]
        pad = (k - 1) // 2
        latent = x.shape[-1] * x.shape[-2] < feat_min_hw
        if groups != 1 or mode == "fp32" or (latent and FEAT_ONLY):
            return Fn.conv2d(x, w, b, stride=stride, padding=pad, groups=groups)
        STATS["n"] += 1
        STATS["xmax"] = max(STATS["xmax"], float(x.abs().max()))
        STATS["wmax"] = max(STATS["wmax"], float(w.abs().max()))
        c = lambda a, ww: Fn.conv2d(a, ww, None, stride=stride, padding=pad)  # noqa: E731
        if mode == "bf16":
            out = c(x.bfloat16().float(), w.bfloat16().float())
        elif mode in ("bf16x3", "fp16x3", "fp16x3s", "fp16x3w", "bf16x2w", "fp16x2w", "fp16x2x"):
            dt = torch.bfloat16 if mode.startswith("bf16") else torch.float16
            sx = sw = 1.0
            if mode == "fp16x3s":
                sx, sw = pow2_scale(x), pow2_scale(w)
            elif mode == "fp16x3w":       # static per-layer weight scale only
                sw = pow2_scale(w)
            xh, xl = split(x * sx, dt)
            wh, wl = split(w * sw, dt)
            if mode in ("bf16x2w", "fp16x2w"):     # activations hi only, weights split
                out = c(xh, wh) + c(xh, wl)
            elif mode == "fp16x2x":               # weights hi only, activations split
                out = c(xh, wh) + c(xl, wh)
            else:
                out = c(xh, wh) + (c(xh, wl) + c(xl, wh))
            out = out * (1.0 / (sx * sw))
        else:
            raise ValueError(mode)
        return out + b.view(1, -1, 1, 1)
    return conv


FEAT_ONLY = False


def run(mode, frames, i_sd, p_sd, q, feat_min_hw):
    torch.set_num_threads(8)
    orig = O.conv
    oi = O.IntraOracle(i_sd, R.pmf_to_quantized_cdf)
    op = O.DMCOracle(p_sd, R.pmf_to_quantized_cdf)
    rows = []
    dpb = None
    emu = make_conv(mode, feat_min_hw)
    with torch.no_grad():
        for t, (x, xp) in enumerate(frames):
            fidx = t % 4
            res = {}
            for m in ("ref", "emu"):
                O.conv = orig if m == "ref" else emu
                tap = {}
                try:
                    if t == 0:
                        calls, xh = oi.compress(xp, False, q, tap=tap, recon=True)
                        nd = {"ref_frame": xh, "ref_feature": None, "ref_mv_feature": None, "ref_y": None,
                              "ref_mv_y": None}
                    else:
                        calls, nd = op.compress(xp, dpb, False, q, fidx, tap=tap, recon=True)
                finally:
                    O.conv = orig
                res[m] = (calls, tap, nd)
            calls, tap, nd = res["ref"]
            ecalls = [(s.clamp(-30000, 30000).to(torch.int16).numpy(), ix.to(torch.int16).numpy())
                      for _, s, ix in res["emu"][0]]
            st = compare_frame(ecalls, calls, tap)
            h, w = x.shape[-2:]
            ref = nd["ref_frame"][..., :h, :w].clamp(0, 1)
            em = res["emu"][2]["ref_frame"][..., :h, :w].clamp(0, 1)
            ps = lambda a: float(-10 * torch.log10(torch.mean((a - x) ** 2)))  # noqa: E731
            first_d = None if st["first_flip"] is None else max(st["first_flip"]["tie_dist"])
            rows.append({"t": t, "symbols": st["symbols"], "dsym": st["sym_diff"], "didx": st["idx_diff"],
                         "first_flip_dist": first_d, "max_tie": st["max_tie_dist"],
                         "unexplained": len(st["unexplained"]), "dpsnr": ps(em) - ps(ref)})
            dpb = nd
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="bf16,bf16x3,fp16x3,fp16x3s")
    ap.add_argument("--case", default="golden_A", choices=["golden_A", "golden_B", "c3small"])
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--feat-only", action="store_true")
    a = ap.parse_args()
    global FEAT_ONLY
    FEAT_ONLY = a.feat_only
    if a.case == "c3small":
        from tests.test_oracle_c3small import C3Small
        c = C3Small()
        frames = [(x, x) for x in c.frames()][:a.frames]
        i_sd, p_sd, q = c.i_sd, c.p_sd, 0
    else:
        from tests.dc_fixtures import DCGolden
        g = DCGolden()
        tag = a.case[-1]
        frames = [g.frame_tensor(tag, t) for t in range(min(a.frames, g.meta[tag]["frames"]))]
        i_sd, p_sd, q = g.i_state_dict(), g.p_state_dict(), g.meta[tag]["q_index"]
    hw = frames[0][1].shape[-1] * frames[0][1].shape[-2]
    out = {}
    for m in a.modes.split(","):
        STATS.update(n=0, xmax=0.0, wmax=0.0)
        rows = run(m, frames, i_sd, p_sd, q, hw // 64)
        out[m] = rows
        print(m, json.dumps(rows), json.dumps(STATS), flush=True)


if __name__ == "__main__":
    main()
