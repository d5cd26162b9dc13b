"""Generate the DCVC-HEM golden fixtures by running the REFERENCE in this container.

Run (only where /root/reference exists; the GPU box never runs this):
    python tests/golden/make_golden_hem.py

What it records (tests/golden/hem_golden.npz / .json + dcvc_amd/data/hem_param_spec.json):
  * the reference models' parameter spec (name, shape) — data, not code;
  * CDF tables built by the reference's own GaussianEncoder.update /
    BitEstimator.update (DCVC-HEM/src/entropy_models/entropy_models.py), with
    the PMF->CDF quantizer compiled from the reference's own ops.cpp
    (oracle/_ref, Makefile target `ref`; HEM's ops.cpp is byte-identical to DC's);
  * write mode: the exact (symbols, indexes, table) sequence the reference's
    compress() hands its entropy coder (video_model.py:310-318,
    image_model.py:150-154) and digests of what decompress() rebuilds;
  * estimate mode: the float bit counts of encode_decode(output_path=None).

Shims (the reference is otherwise run as is):
  * `pytorch_msssim` is not installed; it is only used for the MS-SSIM
    metric (common_model.py:9,30), so a stub module whose MS_SSIM returns
    zeros is registered;
  * the rANS module (MLCodec_rans) cannot be built (ryg_rans' rans64.h is
    not on disk), so a recorder takes the EntropyCoder's place: encode calls
    are recorded with the reference's own int32 conversion
    (entropy_models.py:185-187, 272-274) and decode calls are answered by
    replaying the recorded symbols (lossless coding).
"""
import hashlib
import importlib.machinery
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/DCVC-HEM"
HEM_GAIN = 1.6
sys.path.insert(0, REPO)

from dcvc_amd.weights import synthetic_state_dict  # noqa: E402
from dcvc_amd.synth import moving_pattern, to_float  # noqa: E402


def load_reference():
    stub = types.ModuleType("pytorch_msssim")

    class MS_SSIM(torch.nn.Module):
        def __init__(self, *a, **k):
            super().__init__()

        def forward(self, x, y):
            return torch.zeros(x.shape[0])

    stub.MS_SSIM = MS_SSIM
    stub.ms_ssim = lambda *a, **k: torch.zeros(1)
    sys.modules["pytorch_msssim"] = stub
    sys.path.insert(0, REF)
    import sysconfig
    ext = sysconfig.get_config_var("EXT_SUFFIX")
    so = os.path.join(REPO, "oracle", "_ref", "MLCodec_CXX" + ext)
    if not os.path.exists(so):
        raise SystemExit("build oracle/_ref first: make ref")
    import src.entropy_models  # noqa: F401
    loader = importlib.machinery.ExtensionFileLoader("src.entropy_models.MLCodec_CXX", so)
    spec = importlib.util.spec_from_file_location("src.entropy_models.MLCodec_CXX", so, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules["src.entropy_models.MLCodec_CXX"] = mod
    from src.models.video_model import DMC
    from src.models.image_model import IntraNoAR
    return DMC, IntraNoAR


class Recorder:
    """Stands at the reference's EntropyCoder boundary (entropy_models.py:9-51)."""

    def __init__(self):
        self.tables = []
        self.calls = []
        self.pos = 0
        self.mismatch = 0

    def _table(self, cdf):
        for name, c in self.tables:
            if c is cdf:
                return name
        raise KeyError("unknown cdf table")

    def reset_encoder(self):
        self.calls = []

    def encode_with_indexes(self, symbols, indexes, cdf, cdf_length, offset):
        self.calls.append((self._table(cdf), np.asarray(symbols, dtype=np.int32).copy(),
                           np.asarray(indexes, dtype=np.int32).copy()))

    def flush_encoder(self):
        return b""

    def set_stream(self, stream):
        self.pos = 0

    def decode_stream(self, indexes, cdf, cdf_length, offset):
        name, s, i = self.calls[self.pos]
        self.pos += 1
        if name != self._table(cdf) or not np.array_equal(np.asarray(indexes, dtype=np.int32), i):
            self.mismatch += 1
        return torch.Tensor(s.astype(np.float32)).reshape(1, -1, 1, 1)


def digest(t):
    a = t.detach().float().cpu().contiguous().numpy()
    return hashlib.sha256(a.tobytes()).hexdigest()


def psnr(a, b):
    mse = torch.mean((a - b) ** 2)
    return (20 * torch.log10(1 / torch.sqrt(mse))).item()


def pad64(x):
    h, w = x.shape[2:]
    return torch.nn.functional.pad(x, (0, (64 - w % 64) % 64, 0, (64 - h % 64) % 64), mode="constant", value=0)


def run_sequence(DMC, IntraNoAR, i_sd, p_sd, h, w, nframes, q, seed, out, tag, frames=None, write_frames=None):
    """q = (i_frame_q_scale, p_frame_mv_y_q_scale, p_frame_y_q_scale), the
    harness's args (test_video.py:126-141).  frames: optional list of float
    (1, 3, h, w) frames (else the moving pattern of `seed`); write_frames:
    how many frames write mode codes (default all)."""
    inet = IntraNoAR()
    inet.load_state_dict(i_sd)
    inet.eval()
    pnet = DMC()
    pnet.load_state_dict(p_sd)
    pnet.eval()
    rec_i, rec_p = Recorder(), Recorder()
    inet.gaussian_encoder.update(force=True, entropy_coder=rec_i)
    inet.bit_estimator_z.update(force=True, entropy_coder=rec_i)
    pnet.gaussian_encoder.update(force=True, entropy_coder=rec_p)
    pnet.bit_estimator_z.update(force=True, entropy_coder=rec_p)
    pnet.bit_estimator_z_mv.update(force=True, entropy_coder=rec_p)
    inet.entropy_coder = rec_i
    pnet.entropy_coder = rec_p
    objs = (("i_y", inet.gaussian_encoder), ("i_z", inet.bit_estimator_z),
            ("p_y", pnet.gaussian_encoder), ("p_z", pnet.bit_estimator_z), ("p_mvz", pnet.bit_estimator_z_mv))
    rec_i.tables = [(n, o.cdf_helper._quantized_cdf) for n, o in objs[:2]]
    rec_p.tables = [(n, o.cdf_helper._quantized_cdf) for n, o in objs[2:]]
    for name, obj in objs:
        c, l, o = obj.cdf_helper.get_cdf_info()
        out[f"table_{name}_cdf"] = c
        out[f"table_{name}_len"] = l
        out[f"table_{name}_off"] = o
    qi, qmv, qy = q
    meta = {"h": h, "w": w, "frames": nframes, "q": list(q), "seed": seed, "write": [], "est": []}
    if frames is None:
        frames = []
        for t in range(nframes):
            u8 = moving_pattern(h, w, t, seed=seed)
            out[f"{tag}_frame{t}"] = u8
            frames.append(torch.from_numpy(to_float(u8)).unsqueeze(0))
    else:
        meta["frame_sha256"] = [digest(x) for x in frames]
    with torch.no_grad():
        dpb = None
        for t in range(nframes if write_frames is None else write_frames):
            x = frames[t]
            xp = pad64(x)
            if t == 0:
                qs, qidx = round(qi * 100) / 100, round(qi * 100)
                inet.compress(xp, qs)
                calls = rec_i.calls
                rec_i.set_stream(b"")
                xh = inet.decompress(b"", h, w, qidx / 100)["x_hat"]
                mism = rec_i.mismatch
                dpb = {"ref_frame": xh, "ref_feature": None, "ref_y": None, "ref_mv_y": None}
            else:
                mvq, yq = round(qmv * 100) / 100, round(qy * 100) / 100
                pnet.compress(xp, dpb, mvq, yq)
                calls = rec_p.calls
                rec_p.set_stream(b"")
                dpb = pnet.decompress(dpb, b"", h, w, round(qmv * 100) / 100, round(qy * 100) / 100)["dpb"]
                mism = rec_p.mismatch
            recon = dpb["ref_frame"].clamp_(0, 1)
            entry = {"t": t, "calls": [c[0] for c in calls], "decode_index_mismatch": mism,
                     "recon_sha256": digest(recon), "psnr": psnr(recon[:, :, :h, :w], x),
                     "sym_absmax": int(max(np.abs(c[1]).max() for c in calls))}
            for k in ("ref_feature", "ref_y", "ref_mv_y"):
                if dpb.get(k) is not None:
                    entry[k + "_sha256"] = digest(dpb[k])
            for j, (name, s, i) in enumerate(calls):
                out[f"{tag}_w{t}_c{j}_sym"] = s
                out[f"{tag}_w{t}_c{j}_idx"] = i.astype(np.int16)
            meta["write"].append(entry)
        dpb = None
        for t in range(nframes):
            x = frames[t]
            xp = pad64(x)
            if t == 0:
                r = inet.encode_decode(xp, qi, None, pic_height=h, pic_width=w)
                dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_y": None, "ref_mv_y": None}
            else:
                r = pnet.encode_decode(xp, dpb, None, pic_height=h, pic_width=w, mv_y_q_scale=qmv, y_q_scale=qy)
                dpb = r["dpb"]
            recon = dpb["ref_frame"].clamp_(0, 1)
            e = {"t": t, "bit": float(r["bit"]), "recon_sha256": digest(recon),
                 "psnr": psnr(recon[:, :, :h, :w], x)}
            for k in ("bit_y", "bit_z", "bit_mv_y", "bit_mv_z"):
                if k in r:
                    e[k] = float(r[k])
            meta["est"].append(e)
    return meta


def main():
    DMC, IntraNoAR = load_reference()
    torch.manual_seed(0)
    i_spec = [(k, list(v.shape)) for k, v in IntraNoAR().state_dict().items()]
    p_spec = [(k, list(v.shape)) for k, v in DMC().state_dict().items()]
    with open(os.path.join(REPO, "dcvc_amd", "data", "hem_param_spec.json"), "w") as f:
        json.dump({"intra": i_spec, "inter": p_spec}, f)
    # gain 2: latents that exercise the coder (symbols beyond 0/+-1) without
    # the blow-up of the reference's xavier(gain sqrt 2) init over P-frames
    i_sd = synthetic_state_dict(i_spec, seed=10, gain=HEM_GAIN)
    p_sd = synthetic_state_dict(p_spec, seed=11, gain=HEM_GAIN)
    out, meta = {}, {}
    meta["A"] = run_sequence(DMC, IntraNoAR, i_sd, p_sd, 128, 192, 3, (1.08, 1.10, 0.96), 1, out, "A")
    meta["B"] = run_sequence(DMC, IntraNoAR, i_sd, p_sd, 100, 150, 3, (0.73, 1.01, 0.71), 2, out, "B")
    # config C1 (BASELINE.json configs[0]): 4 random 256x256 frames, IP=4
    # (I P P P), estimate mode on all four, write mode on I, P1, P2 (the survey's
    # recipe); q scales = rate 0 of the weights' ladders
    g = torch.Generator().manual_seed(1)
    c1_frames = [torch.rand(1, 3, 256, 256, generator=g) for _ in range(4)]
    c1_q = (float(i_sd["q_scale"].reshape(-1)[0]), float(p_sd["mv_y_q_scale"].reshape(-1)[0]),
            float(p_sd["y_q_scale"].reshape(-1)[0]))
    meta["C1"] = run_sequence(DMC, IntraNoAR, i_sd, p_sd, 256, 256, 4, c1_q, 1, out, "C1",
                              frames=c1_frames, write_frames=3)
    np.savez_compressed(os.path.join(HERE, "hem_golden.npz"), **out)
    with open(os.path.join(HERE, "hem_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps({k: [(e["t"], round(e["psnr"], 4), e["sym_absmax"], e["calls"]) for e in v["write"]]
                      for k, v in meta.items()}))
    print(json.dumps({k: [(e["t"], e["bit"]) for e in v["est"]] for k, v in meta.items()}))


if __name__ == "__main__":
    main()
