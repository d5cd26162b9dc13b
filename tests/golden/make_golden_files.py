"""Golden bitstream-header bytes and decoded-frame writer outputs, recorded by
running the reference's own Python modules in this container:

  * DCVC-DC/src/utils/stream_helper.py encode_i / encode_p (:94-139) and
    DCVC-HEM/src/utils/stream_helper.py encode_i / encode_p (:102-143): the
    whole file bytes for fixed headers and payloads (hex, they are short);
  * DCVC-DC/src/utils/video_writer.py PNGWriter / YUVWriter (:26-111) driven
    as DCVC-DC/test_video.py:166-221 drives them (clamp_, crop, and for the
    YUV path ycbcr444_to_420 of src/transforms/functional.py), and
    DCVC-HEM/test_video.py's save_torch_image (:68-71): sha256 of every file
    written and of the decoded PNG pixels.

The frames are regenerated from the seeds stored in the fixture, so the
fixture holds only seeds, sizes, bytes and digests.

    python tests/golden/make_golden_files.py
"""
import hashlib
import importlib.util
import json
import os
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "files_golden.json")

# (tag, h, w, frames, seed): the codec's padded frame is (h + 16) x (w + 16)
WRITER_CASES = [("rgb_a", 18, 22, 2, 5), ("rgb_b", 31, 40, 1, 6), ("yuv_a", 18, 22, 2, 7), ("yuv_b", 32, 46, 1, 8)]
DC_I = [(1080, 1920, 0, 0, 7), (100, 130, 1, 40, 33), (2160, 3840, 1, 63, 0)]
DC_P = [(0, 0, 1, 5), (1, 21, 3, 1000), (0, 63, 0, 0)]
HEM_I = [(1088, 1920, 0, 9), (256, 256, 3, 250)]
HEM_P = [(0, 0, 5), (3, 2, 77)]


def frame(seed, h, w):
    """A padded 3 x (h + 16) x (w + 16) float32 recon, mostly in [0, 1] with
    values outside it (clamp_) and exact rint ties (k + 0.5) / 255."""
    g = np.random.Generator(np.random.PCG64(seed))
    f = g.uniform(-0.05, 1.05, size=(3, h + 16, w + 16)).astype(np.float32)
    ties = (g.integers(0, 255, size=(3, h + 16, w + 16)).astype(np.float32) + np.float32(0.5)) / np.float32(255)
    m = g.random(size=f.shape) < 0.1
    f[m] = ties[m]
    return f


def payload(seed, n):
    return bytes(np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size=n, dtype=np.uint8))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def main():
    import torch
    from PIL import Image
    sys.path.insert(0, os.path.join(REF, "DCVC-DC"))
    from src.utils import video_writer as vw          # noqa: E402 (reference, by path)
    from src.transforms.functional import ycbcr444_to_420   # noqa: E402
    sh_dc = load(os.path.join(REF, "DCVC-DC/src/utils/stream_helper.py"), "ref_sh_dc")
    sh_hem = load(os.path.join(REF, "DCVC-HEM/src/utils/stream_helper.py"), "ref_sh_hem")
    out = {"source": "reference stream_helper.py (DC, HEM), video_writer.py, test_video.py writer call sites",
           "dc_i": [], "dc_p": [], "hem_i": [], "hem_p": [], "writers": []}
    with tempfile.TemporaryDirectory() as td:
        f = os.path.join(td, "s.bin")
        for h, w, qc, qi, n in DC_I:
            sh_dc.encode_i(h, w, qc, qi, payload(n + 1, n), f)
            out["dc_i"].append({"args": [h, w, qc, qi], "payload": [n + 1, n], "hex": open(f, "rb").read().hex()})
        for qc, qi, fi, n in DC_P:
            sh_dc.encode_p(payload(n + 2, n), qc, qi, fi, f)
            out["dc_p"].append({"args": [qc, qi, fi], "payload": [n + 2, n], "hex": open(f, "rb").read().hex()})
        for h, w, qi, n in HEM_I:
            sh_hem.encode_i(h, w, qi, payload(n + 3, n), f)
            out["hem_i"].append({"args": [h, w, qi], "payload": [n + 3, n], "hex": open(f, "rb").read().hex()})
        for mq, yq, n in HEM_P:
            sh_hem.encode_p(payload(n + 4, n), mq, yq, f)
            out["hem_p"].append({"args": [mq, yq], "payload": [n + 4, n], "hex": open(f, "rb").read().hex()})

        for tag, h, w, nfr, seed in WRITER_CASES:
            yuv = tag.startswith("yuv")
            d = os.path.join(td, tag)
            dh = os.path.join(td, tag + "_hem")
            os.makedirs(d)
            os.makedirs(dh)
            writer = vw.YUVWriter(d, w, h) if yuv else vw.PNGWriter(d, w, h)
            for t in range(nfr):
                rec = torch.from_numpy(frame(seed + t, h, w)).unsqueeze(0).clamp_(0, 1)
                x_hat = rec[:, :, :h, :w]                     # F.pad with the negative padding: the crop
                if yuv:
                    y_rec, uv_rec = ycbcr444_to_420(x_hat.squeeze(0).cpu().numpy())
                    writer.write_one_frame(y=y_rec, uv=uv_rec, src_format="420")
                else:
                    writer.write_one_frame(rgb=x_hat.squeeze(0).cpu().numpy(), src_format="rgb")
                    # DCVC-HEM/test_video.py:68-71 save_torch_image
                    img = x_hat.squeeze(0).permute(1, 2, 0).detach().cpu().numpy()
                    img = np.clip(np.rint(img * 255), 0, 255).astype(np.uint8)
                    Image.fromarray(img).save(os.path.join(dh, f"{t}.png"))
            writer.close()
            files = {}
            for root in (d, dh):
                for name in sorted(os.listdir(root)):
                    p = os.path.join(root, name)
                    rec = {"sha256": sha(open(p, "rb").read()), "bytes": os.path.getsize(p)}
                    if name.endswith(".png"):
                        rec["pixels_sha256"] = sha(np.asarray(Image.open(p)).tobytes())
                    files[("hem/" if root == dh else "") + name] = rec
            out["writers"].append({"tag": tag, "h": h, "w": w, "frames": nfr, "seed": seed, "files": files})
    with open(OUT, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps({k: len(v) for k, v in out.items() if isinstance(v, list)}))


if __name__ == "__main__":
    main()
