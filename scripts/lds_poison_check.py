"""Uninitialised-LDS detector: before every kernel wrapper call, fill the
LDS of all CUs with NaN bytes (dcvc_debug_poison_lds); after it, check the
output for NaN.  The first kernel whose NaN-free inputs give a NaN output
reads LDS it never wrote (its result then depends on whatever a previous or
concurrent kernel left in LDS).

    python scripts/lds_poison_check.py [--model dc|hem] [--frames 2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="dc")
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--vgpr", action="store_true", help="also poison VGPRs before every launch")
    args = ap.parse_args()
    import bench
    from dcvc_amd import hip as K
    from dcvc_amd.layers import Precision
    from dcvc_amd.harness import FrameStage
    from dcvc_amd.synth import moving_pattern
    dev = torch.device("cuda", 0)
    found = []

    def nan(t):
        b = t.t() if isinstance(t, K.Act) else t
        return bool(torch.isnan(b.float()).any())

    for name in ("conv", "flow_warp", "offset_diversity", "resize2x", "depthconv_block", "dwconv3x3",
                 "pool2x2", "add", "copy", "se_scale", "se_apply", "channel_div"):
        if not hasattr(K, name):
            continue
        f = getattr(K, name)

        def wrap(*a, _f=f, _n=name, **kw):
            ins = [v for v in list(a) + list(kw.values()) if isinstance(v, K.Act)]
            K.check(K.lib().dcvc_debug_poison_lds(160 * 1024, 256 * 2, K.stream()), "poison")
            if args.vgpr:
                K.check(K.lib().dcvc_debug_poison_vgpr(256 * 4 * 4, K.stream()), "poison_vgpr")
            out = _f(*a, **kw)
            tgt = out if isinstance(out, K.Act) else (kw.get("y") if isinstance(kw.get("y"), K.Act) else None)
            if tgt is not None and not found and nan(tgt) and not any(nan(v) for v in ins if v is not tgt):
                kn = K.lib().dcvc_last_kernel().decode()
                found.append((_n, kn, [(v.H, v.W, v.C, v.dtype) for v in ins]))
                print("NaN from", _n, kn, found[-1][2], flush=True)
            return out
        setattr(K, name, wrap)

    isd, psd = bench.make_weights(None, 0, dev, args.model)
    prec = Precision.fast(latent_compute=K.BF16)
    hem = args.model == "hem"
    if hem:
        from dcvc_amd.hem import DMC, IntraNoAR
        qi, qmv, qy = bench.hem_q(isd, psd, 0)
    else:
        from dcvc_amd.dc import DMC, IntraNoAR
    inet = IntraNoAR(precision=prec, device=dev).load_state_dict(isd)
    pnet = DMC(precision=prec, device=dev).load_state_dict(psd)
    inet.update(force=True)
    pnet.update(force=True)
    h, w = args.h, args.w
    stage = FrameStage(h, w, 64 if hem else 16, False, hem, args.frames, dev)
    dpb = None
    for i in range(args.frames):
        x = stage.load(torch.from_numpy(moving_pattern(h, w, i)).to(dev))
        path = f"/dev/shm/poison_{os.getpid()}_{i}.bin"
        try:
            if hem:
                if i == 0:
                    r = inet.encode_decode(x, qi, path, pic_width=w, pic_height=h)
                    dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_y": None, "ref_mv_y": None}
                else:
                    dpb = pnet.encode_decode(x, dpb, path, pic_width=w, pic_height=h, mv_y_q_scale=qmv,
                                             y_q_scale=qy)["dpb"]
            else:
                if i == 0:
                    r = inet.encode_decode(x, False, 0, path, pic_width=w, pic_height=h)
                    dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_mv_feature": None, "ref_y": None,
                           "ref_mv_y": None}
                else:
                    dpb = pnet.encode_decode(x, dpb, False, 0, path, pic_width=w, pic_height=h,
                                             frame_idx=i % 4)["dpb"]
        except Exception as e:  # noqa: BLE001
            print(f"frame {i}: {e}", flush=True)
            break
        finally:
            if os.path.exists(path):
                os.remove(path)
        print(f"frame {i} done, found={found}", flush=True)
        if found:
            break


if __name__ == "__main__":
    main()
