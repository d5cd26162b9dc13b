"""Repeat single kernels on fixed inputs and count runs whose output bits
differ from the first run (co-running divergence study).

    python scripts/determinism_stress.py [--iters 400] [--ops warp8,copy,...]

Run it alone (control) and next to a codec process (bench.py) on the same
GPU.  Prints one JSON line per op: {"op", "iters", "mismatches"}.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bits_sum(t):
    t = t.contiguous()
    v = t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)
    return v.long().sum()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--ops", default="warp8,warp_f32,copy,conv3p,torch_gather,torch_add")
    ap.add_argument("--fresh", action="store_true",
                    help="produce each op's input afresh (clone into newly allocated memory) right before the op, "
                         "as in the codec's producer -> consumer chains")
    a = ap.parse_args()
    args_fresh = a.fresh
    from dcvc_amd import hip as K
    from dcvc_amd.layers import Grids
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H, W = 1088, 1920
    grids = Grids(dev)(H, W)
    flow = K.from_nchw(torch.randn(1, 2, H, W, device=dev) * 3, K.F32)
    x = K.from_nchw(torch.randn(1, 48, H, W, device=dev), K.BF16)
    x32 = K.from_nchw(torch.randn(1, 8, H, W, device=dev), K.F32)
    aux = K.zeros(H, W, 56, K.BF16, dev)
    cw = K.ConvW(torch.randn(48, 48, 3, 3) / 20, torch.randn(48) * 0.1, 1, K.BF16, dev)
    idx = torch.randint(0, H * W, (H * W,), device=dev)
    tx = torch.randn(H * W, 48, device=dev)

    mv = K.from_nchw(torch.randn(1, 2, H, W, device=dev) * 3, K.F32)
    tmv = torch.randn(1, 2, H, W, device=dev)

    def fresh(a):
        if not args_fresh:
            return a
        if isinstance(a, K.Act):
            return K.Act(a.buf.clone(), a.coff, a.C)
        return a.clone()

    def run(op):
        if op == "warp8":
            return K.flow_warp(fresh(x), fresh(flow), grids, y=aux.ch(0, 48)).t()
        if op == "warp_f32":
            return K.flow_warp(fresh(x32), fresh(flow), grids).t()
        if op == "copy":
            return K.copy(fresh(x), aux.ch(8, 48)).t()
        if op == "conv3p":
            return K.conv(cw, fresh(x)).t()
        if op == "resize":
            return K.resize2x(fresh(mv), False, 0.5).t()
        if op == "torch_gather":
            return fresh(tx).index_select(0, idx)
        if op == "torch_add":
            return fresh(tx) * 1.5 + 0.25
        if op == "torch_interp":
            return torch.nn.functional.interpolate(fresh(tmv), scale_factor=0.5, mode="bilinear",
                                                   align_corners=False)
        raise ValueError(op)

    for op in a.ops.split(","):
        ref = bits_sum(run(op))
        sums = torch.empty(a.iters, dtype=torch.long, device=dev)
        for i in range(a.iters):
            sums[i] = bits_sum(run(op))
        torch.cuda.synchronize()
        mism = int((sums != ref).sum())
        print(json.dumps({"op": op, "iters": a.iters, "mismatches": mism, "pid": os.getpid()}), flush=True)


if __name__ == "__main__":
    main()
