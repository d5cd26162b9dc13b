"""Debug aid for the co-running divergence: one DC 1080p
sequence per process, run as two processes on one GPU (see corun_pair.sh).
Per P-frame it records bit checksums (device-side sums of the raw bits, no
host sync) of what the encoder and the decoder must agree on: the inputs and
outputs of the mv prior, mv decoder, motion compensation, residual prior and
every quadtree step (spatial-prior params, CDF indexes).  At the first frame
whose stream fails to decode, or whose checksums differ, it prints the
encoder/decoder comparison in call order and exits 3.

    python scripts/corun_debug.py [--frames 24] [--detail]

--detail also checksums every kernel wrapper's output (conv, dwconv, copy,
warp, ...) between the first differing method's inputs and outputs.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def csum(a):
    t = a.buf if hasattr(a, "buf") else a
    if hasattr(a, "buf"):
        t = a.t()
    t = t.contiguous()
    if t.is_floating_point():
        t = t + 0  # -0.0 -> +0.0: round() gives -0 where the decoder's symbols give +0, the same value
    b = t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)
    return b.long().sum()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--detail", action="store_true")
    ap.add_argument("--precision", default="fast")
    args = ap.parse_args()
    import bench
    from dcvc_amd import hip as K
    from dcvc_amd.dc import DMC, IntraNoAR
    from dcvc_amd.dc import common as C
    from dcvc_amd.layers import Precision
    from dcvc_amd.harness import FrameStage
    from dcvc_amd.synth import moving_pattern
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    isd, psd = bench.make_weights(None, 0, dev, "dc")
    prec = {"fast": Precision.fast, "split": Precision.split, "parity": Precision.parity}[args.precision]()
    h, w = 1080, 1920
    log = {"cur": None}

    def rec(name, v):
        if log["cur"] is not None and v is not None:
            log["cur"].append((name, csum(v)))

    inet = IntraNoAR(precision=prec, stream_part=8, device=dev).load_state_dict(isd)
    pnet = DMC(precision=prec, stream_part=8, device=dev).load_state_dict(psd)
    inet.update(force=True)
    pnet.update(force=True)

    def wrap_method(obj, m, ins=()):
        f = getattr(obj, m)

        def wrapped(*a, **kw):
            for j in ins:
                v = a[j]
                if isinstance(v, dict):
                    for k in sorted(v):
                        if v[k] is not None:
                            rec(f"{m} in[{j}].{k}", v[k])
                else:
                    rec(f"{m} in[{j}]", v)
            out = f(*a, **kw)
            outs = tuple(out) if isinstance(out, tuple) or hasattr(out, "__iter__") and not hasattr(out, "buf") \
                and not isinstance(out, (dict, torch.Tensor)) else (out,)
            for j, o in enumerate(outs):
                rec(f"{m} out[{j}]", o)
            return out
        setattr(obj, m, wrapped)

    wrap_method(pnet, "_mv_prior_params", ins=(0, 1))
    wrap_method(pnet, "_mv_decoder", ins=(0,))
    wrap_method(pnet, "_motion_compensation", ins=(0, 1))
    mc = pnet._motion_compensation

    def mc_flag(*a, **kw):
        log["in_mc"] = True
        try:
            return mc(*a, **kw)
        finally:
            log["in_mc"] = False
    pnet._motion_compensation = mc_flag
    wrap_method(pnet, "_res_prior_params", ins=(0, 1, 2))
    for pr, tag in ((pnet.mv_prior, "mv"), (pnet.y_prior, "y")):
        f = pr.step_params

        def sp(buf, k, _f=f, _t=tag):
            rec(f"{_t}.step{k} buf", buf)
            out = _f(buf, k)
            rec(f"{_t}.step{k} params", out)
            return out
        pr.step_params = sp
    for name in ("qt_encode_step", "qt_indexes_step"):
        f = getattr(K, name)

        def q(*a, _f=f, _n=name):
            out = _f(*a)
            k, idx, prm = (a[3], a[7], a[1]) if _n == "qt_encode_step" else (a[2], a[3], a[0])
            rec(f"qt step{k} C{prm.C} indexes", idx)
            return out
        setattr(K, name, q)
    if args.detail:
        for name in ("conv", "dwconv3x3", "copy", "flow_warp", "offset_diversity", "resize2x", "pad_replicate",
                     "fill", "depthconv_block"):
            f = getattr(K, name)

            def kw_(*a, _f=f, _n=name, **kw):
                if _n in ("flow_warp", "resize2x") and log.get("in_mc"):
                    s0 = log.get("seq", 0) + 1
                    out = _f(*a, **kw)
                    y = out
                    kw2 = dict(kw)
                    kw2["y"] = K.empty(y.H, y.W, y.C, y.dtype, y.buf.device)   # NaN under DCVC_POISON=nan
                    _f(*a, **kw2)
                    log.setdefault("reruns", []).append((s0, _n, y.t().clone(), kw2["y"].t(), a))
                else:
                    out = _f(*a, **kw)
                if out is not None and log.get("in_mc"):
                    kn = K.lib().dcvc_last_kernel().decode() if _n in ("conv", "depthconv_block") else _n
                    log["seq"] = log.get("seq", 0) + 1
                    rec(f"  mc#{log['seq']:03d} {_n} {kn}", out if hasattr(out, "buf") else a[1])
                return out
            setattr(K, name, kw_)

    stage = FrameStage(h, w, 16, False, False, args.frames, dev)
    dpb = None
    out_dir = f"/dev/shm/corun_dbg_{os.getpid()}"
    os.makedirs(out_dir, exist_ok=True)
    for i in range(args.frames):
        src = torch.from_numpy(moving_pattern(h, w, i, seed=1 + os.getpid() % 7)).to(dev)
        x = stage.load(src)
        path = os.path.join(out_dir, f"{i}.bin")
        if i == 0:
            r = inet.encode_decode(x, False, 0, path, pic_width=w, pic_height=h)
            dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_mv_feature": None, "ref_y": None,
                   "ref_mv_y": None}
            continue
        log["cur"] = enc_log = []
        log["seq"] = 0
        enc = pnet.compress(x, dpb, False, 0, i % 4)
        log["cur"] = dec_log = []
        log["seq"] = 0
        err = None
        try:
            dec = pnet.decompress(dpb, enc["bit_stream"], h, w, False, 0, i % 4)
        except Exception as e:  # noqa: BLE001
            dec, err = None, e
        log["cur"] = None
        torch.cuda.synchronize()
        e = {}
        for n, c in enc_log:
            e.setdefault(n, []).append(int(c))
        d = {}
        for n, c in dec_log:
            d.setdefault(n, []).append(int(c))
        diff = [n for n in d if n in e and e[n][:len(d[n])] != d[n]]
        for s0, nm, y1, y2, args_ in log.pop("reruns", []):
            d = (y1 != y2)
            if bool(d.any()):
                pos = torch.nonzero(d.any(-1))
                print(f"pid {os.getpid()} frame {i} {nm} mc#{s0}: {int(pos.shape[0])} pixels differ between two "
                      f"runs on the same inputs; nan in run1 {int(torch.isnan(y1.float()).sum())}, in run2 "
                      f"{int(torch.isnan(y2.float()).sum())}; pixels {pos[:8].tolist()}", flush=True)
                ref = None
                if nm == "flow_warp":
                    import numpy as np
                    x, fl, grid = args_[0], args_[1], args_[2]
                    X = x.t().float().cpu().numpy()
                    F = fl.t().float().cpu().numpy()
                    gx, gy = grid[0].cpu().numpy(), grid[1].cpu().numpy()
                    Hh, Ww = X.shape[:2]
                    P = pos.cpu().numpy()
                    ref = []
                    for py, px in P[:200]:
                        fx, fy = F[py, px]
                        ix = min(Ww - 1, max(0.0, (gx[px] + fx / ((Ww - 1) / 2) + 1) * (Ww - 1) / 2))
                        iy = min(Hh - 1, max(0.0, (gy[py] + fy / ((Hh - 1) / 2) + 1) * (Hh - 1) / 2))
                        x0, y0 = int(np.floor(ix)), int(np.floor(iy))
                        x1, y1_ = min(x0 + 1, Ww - 1), min(y0 + 1, Hh - 1)
                        wx, wy = ix - x0, iy - y0
                        ref.append(X[y0, x0] * (1 - wx) * (1 - wy) + X[y0, x1] * wx * (1 - wy)
                                   + X[y1_, x0] * (1 - wx) * wy + X[y1_, x1] * wx * wy)
                    ref = np.stack(ref)
                    e1 = np.abs(y1.float().cpu().numpy()[P[:200, 0], P[:200, 1]] - ref).max(-1)
                    e2 = np.abs(y2.float().cpu().numpy()[P[:200, 0], P[:200, 1]] - ref).max(-1)
                    print(f"   vs CPU recompute (first {len(ref)} differing pixels): run1 wrong at "
                          f"{int((e1 > 0.01).sum())}, run2 wrong at {int((e2 > 0.01).sum())}; max err run1 "
                          f"{e1.max():.3g} run2 {e2.max():.3g}")
                for p0 in pos[:3].tolist():
                    print("   run1", [round(v, 4) for v in y1[p0[0], p0[1]].float().tolist()[:12]])
                    print("   run2", [round(v, 4) for v in y2[p0[0], p0[1]].float().tolist()[:12]])
        if err is not None or diff:
            print(f"pid {os.getpid()} frame {i}: err={err} first differing keys={diff[:6]}", flush=True)
            seen = set()
            for n, _ in dec_log:
                if n in seen or n not in e:
                    continue
                seen.add(n)
                print(f"   {'DIFF' if e[n][:len(d[n])] != d[n] else 'same'} {n}: enc={e[n][:4]} dec={d[n][:4]}",
                      flush=True)
            sys.exit(3)
        dpb = dec["dpb"]
    print(f"pid {os.getpid()}: {args.frames} frames, encoder and decoder agree", flush=True)


if __name__ == "__main__":
    main()
