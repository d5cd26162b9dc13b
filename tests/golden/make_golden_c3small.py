"""Fixture for the survey's C3-small recipe, made by
running the REFERENCE in this container (never on the GPU box).

Recipe: torch.manual_seed(0); IntraNoAR() then DMC() (default PyTorch init);
load_state_dict(own state_dict()) on both (builds DMC's fine q tables,
DCVC-DC/src/models/video_model.py:325-341); update(force=True); frames = 4
draws of torch.rand(1, 3, 256, 256) from Generator().manual_seed(1);
write mode, q_in_ckpt=False, q_index=0, frame_idx = t % 4, GOP 4 (I P P P).
The survey recorded the per-frame bits 194128 / 46968 / 41048 / 38200.

The reference's rANS module cannot be built here (rans64.h is absent,
SURVEY.md §8(c)), so a recorder stands at its EntropyCoder boundary
(make_golden_dc.Recorder) and the recorded calls are coded with the oracle's
C restatement of the coder (oracle/rans_oracle.c): bits = (stream + header) * 8.
It also checks that oracle/torch_init.py's replay of the default init equals
the reference's state dicts tensor for tensor, so the tests can rebuild the
weights without the reference.

    python tests/golden/make_golden_c3small.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden_dc import load_reference, Recorder, digest, psnr  # noqa: E402
from oracle.torch_init import default_init_state_dicts  # noqa: E402
from oracle import rans_oracle as R  # noqa: E402

SURVEY_BITS = [194128, 46968, 41048, 38200]


def main():
    torch.set_num_threads(8)
    DMC, IntraNoAR = load_reference()
    torch.manual_seed(0)
    inet = IntraNoAR()
    pnet = DMC()
    inet.load_state_dict(inet.state_dict())
    pnet.load_state_dict(pnet.state_dict())
    inet.eval()
    pnet.eval()
    spec = json.load(open(os.path.join(REPO, "dcvc_amd", "data", "dc_param_spec.json")))
    i_sd, p_sd = default_init_state_dicts(spec["intra"], spec["inter"], seed=0)
    for ours, net in ((i_sd, inet), (p_sd, pnet)):
        ref = net.state_dict()
        assert list(ref) == list(ours), "spec order differs from the reference state_dict"
        for k, v in ref.items():
            assert torch.equal(v, ours[k]), f"default-init replay differs at {k}"
    rec_i, rec_p = Recorder([]), Recorder([])
    inet.gaussian_encoder.update(force=True, entropy_coder=rec_i)
    inet.bit_estimator_z.update(force=True, entropy_coder=rec_i)
    pnet.gaussian_encoder.update(force=True, entropy_coder=rec_p)
    pnet.bit_estimator_z.update(force=True, entropy_coder=rec_p)
    pnet.bit_estimator_z_mv.update(force=True, entropy_coder=rec_p)
    inet.entropy_coder, pnet.entropy_coder = rec_i, rec_p
    rec_i.tables = [("i_y", inet.gaussian_encoder._quantized_cdf), ("i_z", inet.bit_estimator_z._quantized_cdf)]
    rec_p.tables = [("p_y", pnet.gaussian_encoder._quantized_cdf), ("p_z", pnet.bit_estimator_z._quantized_cdf),
                    ("p_mvz", pnet.bit_estimator_z_mv._quantized_cdf)]
    tabs = {}
    for name, obj in (("i_y", inet.gaussian_encoder), ("i_z", inet.bit_estimator_z),
                      ("p_y", pnet.gaussian_encoder), ("p_z", pnet.bit_estimator_z),
                      ("p_mvz", pnet.bit_estimator_z_mv)):
        c, l, o = obj.get_cdf_info()
        tabs[name] = (np.asarray(c), np.asarray(l).reshape(-1), np.asarray(o).reshape(-1))
    g = torch.Generator().manual_seed(1)
    frames = [torch.rand(1, 3, 256, 256, generator=g) for _ in range(4)]
    out, meta = {}, {"h": 256, "w": 256, "frames": 4, "q_index": 0, "survey_bits": SURVEY_BITS, "write": []}
    dpb = None
    with torch.no_grad():
        for t, x in enumerate(frames):
            meta.setdefault("frame_sha256", []).append(digest(x))
            if t == 0:
                rec_i.reset()
                inet.compress(x, False, 0)
                calls = rec_i.calls
                rec_i.set_stream(b"")
                xh = inet.decompress(b"", 256, 256, False, 0)["x_hat"]
                dpb = {"ref_frame": xh, "ref_feature": None, "ref_mv_feature": None, "ref_y": None, "ref_mv_y": None}
            else:
                rec_p.reset()
                pnet.compress(x, dpb, False, 0, t % 4)
                calls = rec_p.calls
                rec_p.set_stream(b"")
                dpb = pnet.decompress(dpb, b"", 256, 256, False, 0, t % 4)["dpb"]
            stream = R.DCStream().encode([(s, i, tabs[name]) for name, s, i in calls])
            bits = (len(stream) + (13 if t == 0 else 6)) * 8
            recon = dpb["ref_frame"].clamp_(0, 1)
            meta["write"].append({"t": t, "calls": [c[0] for c in calls], "bits": bits, "psnr": psnr(recon, x),
                                  "recon_sha256": digest(recon)})
            for j, (name, s, i) in enumerate(calls):
                out[f"w{t}_c{j}_sym"] = s
                out[f"w{t}_c{j}_idx"] = i
            print(t, bits, SURVEY_BITS[t], "ok" if bits == SURVEY_BITS[t] else "DIFFERS")
    np.savez_compressed(os.path.join(HERE, "c3small_golden.npz"), **out)
    with open(os.path.join(HERE, "c3small_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
