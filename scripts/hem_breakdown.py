"""Where a DCVC-HEM 1080p P-frame's wall time goes (box diagnostic).

Wraps the HEM entropy coder's encode / flush / decode calls with timers and
reports, per P-frame: total encode_decode wall, coder encode (+flush), coder
decode, and the rest (GPU + host glue).  Same weights and frames as bench.py
--model hem.

    python scripts/hem_breakdown.py [--frames 6]
"""
import argparse
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=6)
    ap.add_argument("--cprofile", default="", help="write a cProfile of the P-frames to this path")
    args = ap.parse_args()
    import bench
    from dcvc_amd import hip as K
    from dcvc_amd.hem import DMC, IntraNoAR
    from dcvc_amd.hem import common as C
    from dcvc_amd.layers import Precision
    from dcvc_amd.synth import moving_pattern

    acc = {"enc": 0.0, "flush": 0.0, "dec": 0.0, "n_enc": 0, "n_dec": 0}

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            acc[name] += time.perf_counter() - t
            return r
        return w
    C.HemEntropyCoder.encode = timed("enc", C.HemEntropyCoder.encode)
    C.HemEntropyCoder.flush_encoder = timed("flush", C.HemEntropyCoder.flush_encoder)
    C.HemEntropyCoder.decode = timed("dec", C.HemEntropyCoder.decode)

    dev = torch.device("cuda", 0)
    isd, psd = bench.make_weights(None, 0, dev, "hem")
    prec = Precision.fast(latent_compute=K.BF16)
    inet = IntraNoAR(precision=prec, device=dev).load_state_dict(isd)
    pnet = DMC(precision=prec, device=dev).load_state_dict(psd)
    inet.update(force=True)
    pnet.update(force=True)
    qi, qmv, qy = bench.hem_q(isd, psd, 0)
    h, w = 1080, 1920
    x = K.empty(1088, 1920, 3, K.F32, dev)
    frames = [torch.from_numpy(moving_pattern(h, w, t, seed=1)).to(dev) for t in range(args.frames)]
    dpb = None
    prof = None
    with tempfile.TemporaryDirectory(dir="/dev/shm") as td:
        for i in range(args.frames):
            if i == 2 and args.cprofile:
                import cProfile
                prof = cProfile.Profile()
                prof.enable()
            K.frame_to_nhwc(frames[i], h, w, x, zero_pad=True)
            torch.cuda.synchronize()
            for k in ("enc", "flush", "dec"):
                acc[k] = 0.0
            t = time.perf_counter()
            path = os.path.join(td, f"{i}.bin")
            if i == 0:
                r = inet.encode_decode(x, qi, path, pic_width=w, pic_height=h)
                dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_y": None, "ref_mv_y": None}
            else:
                r = pnet.encode_decode(x, dpb, path, pic_width=w, pic_height=h, mv_y_q_scale=qmv, y_q_scale=qy)
                dpb = r["dpb"]
            torch.cuda.synchronize()
            tot = time.perf_counter() - t
            print(f"frame {i} {'I' if i == 0 else 'P'}: total {tot * 1e3:.1f} ms  enc {acc['enc'] * 1e3:.1f}  "
                  f"flush {acc['flush'] * 1e3:.1f}  dec {acc['dec'] * 1e3:.1f}  "
                  f"rest {(tot - acc['enc'] - acc['flush'] - acc['dec']) * 1e3:.1f}  bits {r['bit']}", flush=True)
    if prof is not None:
        prof.disable()
        import pstats
        with open(args.cprofile, "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(45)


if __name__ == "__main__":
    main()
