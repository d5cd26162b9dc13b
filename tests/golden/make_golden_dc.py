"""Generate the DCVC-DC golden fixtures by running the REFERENCE in this container.

Run (only where /root/reference exists; the GPU box never runs this):
    python tests/golden/make_golden_dc.py

What it records (tests/golden/dc_golden.npz + dc_param_spec.json):
  * the reference models' parameter spec (name, shape) — data, not code;
  * CDF tables built by the reference's own GaussianEncoder.update /
    BitEstimator.update (DCVC-DC/src/models/entropy_models.py:124-178,228-267),
    with the PMF->CDF quantizer compiled from the reference's own ops.cpp
    (oracle/_ref, see Makefile target `ref`);
  * write mode: the exact (symbols, indexes, table) sequence the reference's
    compress() hands to its entropy coder (video_model.py:455-466,
    image_model.py:214-220), and a digest of the dpb / reconstruction its
    decompress() produces;
  * estimate mode: the float bit counts and reconstruction digests of
    encode_decode(output_path=None).

The reference's rANS module (MLCodec_rans) cannot be built here (ryg_rans'
rans64.h is not on disk), so its place at the EntropyCoder boundary is taken
by a recorder: encode calls are recorded with the reference's own int16
conversion (entropy_models.py:37-40) and decode calls are answered by
replaying the recorded symbols (lossless coding) — no coder of ours runs.
"""
import importlib.machinery
import importlib.util
import json
import os
import sys
import hashlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/DCVC-DC"
sys.path.insert(0, REPO)

from dcvc_amd.weights import synthetic_state_dict  # noqa: E402
from dcvc_amd.synth import moving_pattern, to_float  # noqa: E402


def load_reference():
    sys.path.insert(0, REF)
    import sysconfig
    ext = sysconfig.get_config_var("EXT_SUFFIX")
    so = os.path.join(REPO, "oracle", "_ref", "MLCodec_CXX" + ext)
    if not os.path.exists(so):
        raise SystemExit("build oracle/_ref first: make ref")
    import src.models  # noqa: F401
    loader = importlib.machinery.ExtensionFileLoader("src.models.MLCodec_CXX", so)
    spec = importlib.util.spec_from_file_location("src.models.MLCodec_CXX", so, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules["src.models.MLCodec_CXX"] = mod
    from src.models.video_model import DMC
    from src.models.image_model import IntraNoAR
    return DMC, IntraNoAR


class Recorder:
    """Stands at the reference's EntropyCoder boundary (entropy_models.py:9-55)."""

    def __init__(self, tables):
        self.tables = tables  # list of (name, cdf ndarray) for identification
        self.calls = []
        self.pos = 0
        self.mismatch = 0

    def _table(self, cdf):
        for name, c in self.tables:
            if c is cdf:
                return name
        raise KeyError("unknown cdf table")

    def reset(self):
        self.calls = []

    def encode_with_indexes(self, symbols, indexes, cdf, cdf_length, offset):
        s = symbols.clamp(-30000, 30000).to(torch.int16).cpu().numpy()
        i = indexes.to(torch.int16).cpu().numpy()
        self.calls.append((self._table(cdf), s, i))

    def flush(self):
        pass

    def get_encoded_stream(self):
        return b""

    def set_stream(self, stream):
        self.pos = 0

    def decode_stream(self, indexes, cdf, cdf_length, offset):
        name, s, i = self.calls[self.pos]
        self.pos += 1
        got = indexes.to(torch.int16).cpu().numpy()
        if name != self._table(cdf) or not np.array_equal(got, i):
            self.mismatch += 1
        return torch.Tensor(s)


def digest(t):
    a = t.detach().float().cpu().contiguous().numpy()
    return hashlib.sha256(a.tobytes()).hexdigest()


def psnr(a, b):
    mse = torch.mean((a - b) ** 2)
    return (20 * torch.log10(1 / torch.sqrt(mse))).item()


def run_sequence(DMC, IntraNoAR, i_sd, p_sd, h, w, nframes, q_index, seed, out, tag):
    torch.manual_seed(0)
    inet = IntraNoAR()
    inet.load_state_dict(i_sd)
    inet.eval()
    pnet = DMC()
    pnet.load_state_dict(p_sd)
    pnet.eval()
    i_tables = [("i_y", None), ("i_z", None)]
    rec_i = Recorder([])
    rec_p = Recorder([])
    inet.gaussian_encoder.update(force=True, entropy_coder=rec_i)
    inet.bit_estimator_z.update(force=True, entropy_coder=rec_i)
    pnet.gaussian_encoder.update(force=True, entropy_coder=rec_p)
    pnet.bit_estimator_z.update(force=True, entropy_coder=rec_p)
    pnet.bit_estimator_z_mv.update(force=True, entropy_coder=rec_p)
    inet.entropy_coder = rec_i
    pnet.entropy_coder = rec_p
    rec_i.tables = [("i_y", inet.gaussian_encoder._quantized_cdf),
                    ("i_z", inet.bit_estimator_z._quantized_cdf)]
    rec_p.tables = [("p_y", pnet.gaussian_encoder._quantized_cdf),
                    ("p_z", pnet.bit_estimator_z._quantized_cdf),
                    ("p_mvz", pnet.bit_estimator_z_mv._quantized_cdf)]
    del i_tables
    for name, obj in (("i_y", inet.gaussian_encoder), ("i_z", inet.bit_estimator_z),
                      ("p_y", pnet.gaussian_encoder), ("p_z", pnet.bit_estimator_z),
                      ("p_mvz", pnet.bit_estimator_z_mv)):
        c, l, o = obj.get_cdf_info()
        out[f"table_{name}_cdf"] = c
        out[f"table_{name}_len"] = l
        out[f"table_{name}_off"] = o
    meta = {"h": h, "w": w, "frames": nframes, "q_index": q_index, "seed": seed, "write": [], "est": []}
    pad_b = (16 - h % 16) % 16
    pad_r = (16 - w % 16) % 16
    with torch.no_grad():
        # ---- write mode (compress -> recorded coder -> decompress), gop = nframes
        dpb = None
        for t in range(nframes):
            u8 = moving_pattern(h, w, t, seed=seed)
            out[f"{tag}_frame{t}"] = u8
            x = torch.from_numpy(to_float(u8)).unsqueeze(0)
            xp = torch.nn.functional.pad(x, (0, pad_r, 0, pad_b), mode="replicate")
            H, W = xp.shape[2:]
            if t == 0:
                enc = inet.compress(xp, False, q_index)
                calls = rec_i.calls
                rec_i.set_stream(b"")
                xh = inet.decompress(b"", h, w, False, q_index)["x_hat"]
                mism = rec_i.mismatch
                dpb = {"ref_frame": xh, "ref_feature": None, "ref_mv_feature": None,
                       "ref_y": None, "ref_mv_y": None}
                del enc
            else:
                pnet.compress(xp, dpb, False, q_index, t % 4)
                calls = rec_p.calls
                rec_p.set_stream(b"")
                dpb = pnet.decompress(dpb, b"", h, w, False, q_index, t % 4)["dpb"]
                mism = rec_p.mismatch
            recon = dpb["ref_frame"].clamp_(0, 1)
            xr = recon[:, :, :h, :w]
            entry = {"t": t, "calls": [c[0] for c in calls], "decode_index_mismatch": mism,
                     "recon_sha256": digest(recon), "psnr": psnr(xr, x)}
            for k in ("ref_feature", "ref_mv_feature", "ref_y", "ref_mv_y"):
                if dpb.get(k) is not None:
                    entry[k + "_sha256"] = digest(dpb[k])
            for j, (name, s, i) in enumerate(calls):
                out[f"{tag}_w{t}_c{j}_sym"] = s
                out[f"{tag}_w{t}_c{j}_idx"] = i
            meta["write"].append(entry)
        # ---- estimate mode (float bits)
        dpb = None
        for t in range(nframes):
            x = torch.from_numpy(to_float(out[f"{tag}_frame{t}"])).unsqueeze(0)
            xp = torch.nn.functional.pad(x, (0, pad_r, 0, pad_b), mode="replicate")
            if t == 0:
                r = inet.encode_decode(xp, False, q_index, None, pic_height=h, pic_width=w)
                dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_mv_feature": None,
                       "ref_y": None, "ref_mv_y": None}
                bit = r["bit"]
            else:
                r = pnet.encode_decode(xp, dpb, False, q_index, None, pic_height=h, pic_width=w,
                                       frame_idx=t % 4)
                dpb = r["dpb"]
                bit = r["bit"]
            recon = dpb["ref_frame"].clamp_(0, 1)
            meta["est"].append({"t": t, "bit": float(bit), "recon_sha256": digest(recon),
                                "psnr": psnr(recon[:, :, :h, :w], x)})
    return meta


def main():
    DMC, IntraNoAR = load_reference()
    torch.manual_seed(0)
    i_spec = [(k, list(v.shape)) for k, v in IntraNoAR().state_dict().items()]
    p_spec = [(k, list(v.shape)) for k, v in DMC().state_dict().items()]
    with open(os.path.join(REPO, "dcvc_amd", "data", "dc_param_spec.json"), "w") as f:
        json.dump({"intra": i_spec, "inter": p_spec}, f)
    i_sd = synthetic_state_dict(i_spec, seed=0)
    p_sd = synthetic_state_dict(p_spec, seed=1)
    out = {}
    meta = {}
    meta["A"] = run_sequence(DMC, IntraNoAR, i_sd, p_sd, 176, 240, 4, 0, 1, out, "A")
    meta["B"] = run_sequence(DMC, IntraNoAR, i_sd, p_sd, 100, 130, 3, 40, 2, out, "B")
    np.savez_compressed(os.path.join(HERE, "dc_golden.npz"), **out)
    with open(os.path.join(HERE, "dc_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps({k: [(e["t"], e["psnr"], e["calls"][:2]) for e in v["write"]] for k, v in meta.items()}))
    print(json.dumps({k: [(e["t"], e["bit"]) for e in v["est"]] for k, v in meta.items()}))


if __name__ == "__main__":
    main()
