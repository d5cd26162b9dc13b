"""Out-of-bounds store detector: run a few DC (or HEM) frames with every
activation allocated with a 4 KiB canary tail (dcvc_amd.hip.CANARY) and
report allocations whose tail was written.

    python scripts/canary_check.py [--model dc|hem] [--frames 3] [--h 1080 --w 1920]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="dc")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--w", type=int, default=1920)
    args = ap.parse_args()
    import bench
    from dcvc_amd import hip as K
    from dcvc_amd.layers import Precision
    from dcvc_amd.harness import FrameStage
    from dcvc_amd.synth import moving_pattern
    K.CANARY = []
    dev = torch.device("cuda", 0)
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
        path = f"/dev/shm/canary_{os.getpid()}_{i}.bin"
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
                dpb = pnet.encode_decode(x, dpb, False, 0, path, pic_width=w, pic_height=h, frame_idx=i % 4)["dpb"]
        os.remove(path)
        torch.cuda.synchronize()
        bad = K.check_canaries()
        print(f"frame {i}: {len(K.CANARY)} allocations, {len(bad)} overwritten tails", flush=True)
        for shape, first, where in bad[:10]:
            print(f"  shape {shape} first bad byte +{first}\n{where}", flush=True)
        if bad:
            sys.exit(1)


if __name__ == "__main__":
    main()
