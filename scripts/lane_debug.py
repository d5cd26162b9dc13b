"""Debug aid for concurrent GOP lanes: run two DC lanes on separate streams /
threads and compare, for the first P-frame, bit-level checksums of the
tensors the encoder and decoder must agree on (mv_hat, contexts, prior
params).  Prints the first disagreement.

    python scripts/lane_debug.py [--lanes 2] [--frames 3]
"""
import argparse
import os
import sys
import threading

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def csum(a):
    t = a.buf if hasattr(a, "buf") else a
    b = t.contiguous().view(torch.int16) if t.element_size() == 2 else t.contiguous().view(torch.int32)
    return b.long().sum()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=2)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--detail", action="store_true", help="checksum every kernel wrapper output")
    args = ap.parse_args()
    import bench
    from dcvc_amd import hip as K
    from dcvc_amd.dc import DMC, IntraNoAR
    from dcvc_amd.layers import Precision
    from dcvc_amd.harness import FrameStage
    from dcvc_amd.synth import moving_pattern
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    isd, psd = bench.make_weights(None, 0, dev, "dc")
    prec = Precision.fast(latent_compute=K.BF16)
    h, w = 1080, 1920
    tl = threading.local()

    def rec(name, out):
        log = getattr(tl, "log", None)
        if log is not None:
            log.append((name, csum(out)))
        return out

    class Lane:
        def __init__(self, l):
            self.l = l
            self.inet = IntraNoAR(precision=prec, stream_part=8, device=dev).load_state_dict(isd)
            self.pnet = DMC(precision=prec, stream_part=8, device=dev).load_state_dict(psd)
            self.inet.update(force=True)
            self.pnet.update(force=True)
            self.stage = FrameStage(h, w, 16, False, False, args.frames, dev)
            self.frames = [torch.from_numpy(moving_pattern(h, w, t + 32 * l)).to(dev) for t in range(args.frames)]
            self.stream = torch.cuda.Stream(dev)
            self.logs = []
            p = self.pnet
            for m in ("_mv_decoder", "_motion_compensation", "_res_prior_params", "_mv_prior_params"):
                f = getattr(p, m)

                def wrapped(*a, _f=f, _m=m, **kw):
                    tl.in_mc = _m == "_motion_compensation"
                    out = _f(*a, **kw)
                    tl.in_mc = False
                    outs = out if isinstance(out, tuple) else tuple(out) if type(out).__name__ == "Contexts" else (out,)
                    for j, o in enumerate(outs):
                        rec(f"{_m}[{j}]", o)
                    return out
                setattr(p, m, wrapped)
        def run(self):
            with torch.cuda.device(dev), torch.cuda.stream(self.stream):
                dpb = None
                for i in range(args.frames):
                    x = self.stage.load(self.frames[i])
                    path = f"/dev/shm/lanedbg_{os.getpid()}_{self.l}_{i}.bin"
                    if i == 0:
                        r = self.inet.encode_decode(x, False, 0, path, pic_width=w, pic_height=h)
                        dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_mv_feature": None,
                               "ref_y": None, "ref_mv_y": None}
                        continue
                    tl.log = []
                    p = self.pnet
                    enc = p.compress(x, dpb, False, 0, i % 4)
                    enc_log = tl.log
                    tl.log = []
                    try:
                        dec = p.decompress(dpb, enc["bit_stream"], h, w, False, 0, i % 4)
                        err = None
                    except Exception as e:  # noqa: BLE001
                        dec, err = None, e
                    dec_log = tl.log
                    tl.log = None
                    self.logs.append((i, enc_log, dec_log, err))
                    if dec is None:
                        return
                    dpb = dec["dpb"]
                    os.remove(path) if os.path.exists(path) else None

    if args.detail:
        # checksum every kernel wrapper's inputs and output inside motion
        # compensation (thread-local flag), to find the first divergent launch
        for name in ("conv", "flow_warp", "offset_diversity", "resize2x", "copy", "depthconv_block",
                     "dwconv3x3", "pool2x2", "add"):
            f = getattr(K, name)

            def kw_(*a, _f=f, _n=name, **kw):
                ins = [csum(v) for v in list(a) + list(kw.values()) if isinstance(v, K.Act)]
                out = _f(*a, **kw)
                if getattr(tl, "in_mc", False) and out is not None:
                    kn = K.lib().dcvc_last_kernel().decode() if _n in ("conv", "depthconv_block") else _n
                    rec(f"{_n} {kn} ins={len(ins)}", out)
                    for j, c in enumerate(ins):
                        tl.log.append((f"  in{j} of {_n}", c))
                return out
            setattr(K, name, kw_)
    lanes = [Lane(l) for l in range(args.lanes)]
    torch.cuda.synchronize()
    th = [threading.Thread(target=ln.run) for ln in lanes]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    for ln in lanes:
        for i, el, dl, err in ln.logs:
            print(f"lane {ln.l} frame {i} err={err}")
            enc = {}
            for n, c in el:
                enc.setdefault(n, []).append(int(c))
            dcc = {}
            for n, c in dl:
                dcc.setdefault(n, []).append(int(c))
            for n in dcc:
                if n in enc and not n.startswith("conv ") and not n.startswith("  in") and "_" in n[:2]:
                    pass
                if n in enc and n.startswith("_"):
                    same = enc[n] == dcc[n]
                    print(f"   {n}: {'same' if same else 'DIFF'} enc={enc[n][:4]} dec={dcc[n][:4]}")
            if args.detail:
                e_mc = [(n, int(c)) for n, c in el if not n.startswith("_")]
                d_mc = [(n, int(c)) for n, c in dl if not n.startswith("_")]
                for j, (a, b) in enumerate(zip(e_mc, d_mc)):
                    if a != b:
                        print(f"   first divergence at launch {j}: enc {a} dec {b}")
                        for k in range(max(0, j - 3), min(len(e_mc), j + 4)):
                            print(f"      {k}: {e_mc[k]} | {d_mc[k] if k < len(d_mc) else None}")
                        break


if __name__ == "__main__":
    main()
