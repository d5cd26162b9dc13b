"""Bitstream headers and decoded-frame files against bytes the reference's own
code wrote (tests/golden/files_golden.json, recorded by
tests/golden/make_golden_files.py from DCVC-DC/src/utils/stream_helper.py
:94-139, DCVC-HEM/src/utils/stream_helper.py:102-143,
DCVC-DC/src/utils/video_writer.py:26-111 and DCVC-HEM/test_video.py:68-71)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from tests.golden.make_golden_files import frame, payload

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "files_golden.json")


@pytest.fixture(scope="module")
def gold():
    with open(GOLDEN) as f:
        return json.load(f)


def test_dc_headers_byte_identical(gold, tmp_path):
    from dcvc_amd import stream_helper as sh
    f = str(tmp_path / "s.bin")
    for e in gold["dc_i"]:
        h, w, qc, qi = e["args"]
        data = payload(*e["payload"])
        sh.encode_i(h, w, qc, qi, data, f)
        assert open(f, "rb").read().hex() == e["hex"]
        assert sh.decode_i(f) == (h, w, bool(qc), qi, data)
    for e in gold["dc_p"]:
        qc, qi, fi = e["args"]
        data = payload(*e["payload"])
        sh.encode_p(data, qc, qi, fi, f)
        assert open(f, "rb").read().hex() == e["hex"]
        assert sh.decode_p(f) == (bool(qc), qi, fi, data)


def test_hem_headers_byte_identical(gold, tmp_path):
    from dcvc_amd.hem import stream_helper as sh
    f = str(tmp_path / "s.bin")
    for e in gold["hem_i"]:
        h, w, qi = e["args"]
        data = payload(*e["payload"])
        sh.encode_i(h, w, qi, data, f)
        assert open(f, "rb").read().hex() == e["hex"]
        assert sh.decode_i(f) == (h, w, qi, data)
    for e in gold["hem_p"]:
        mq, yq = e["args"]
        data = payload(*e["payload"])
        sh.encode_p(data, mq, yq, f)
        assert open(f, "rb").read().hex() == e["hex"]
        assert sh.decode_p(f) == (mq, yq, data)


@pytest.mark.gpu
def test_recon_writers_byte_identical_to_reference(gold, tmp_path):
    """ReconWriter (GPU quantisation, background writer thread) on the padded,
    clamped recon the harness hands it: every PNG / out.yuv file equals the
    file the reference's writers produced for the same frame."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from PIL import Image
    from dcvc_amd import hip as K
    from dcvc_amd.harness import ReconWriter
    dev = torch.device("cuda", 0)
    for case in gold["writers"]:
        tag, h, w = case["tag"], case["h"], case["w"]
        yuv = tag.startswith("yuv")
        d = tmp_path / tag
        kinds = [("yuv", "420", d)] if yuv else [("png", "rgb", d), ("hem_png", "rgb", tmp_path / (tag + "_hem"))]
        for kind, fmt, path in kinds:
            with ReconWriter(str(path), h, w, kind, fmt, dev) as wr:
                for t in range(case["frames"]):
                    rec = torch.from_numpy(frame(case["seed"] + t, h, w)).clamp_(0, 1)   # test_video.py:167 clamp_
                    wr.write(K.Act(rec.permute(1, 2, 0).contiguous().to(dev)), t)
        for name, want in case["files"].items():
            p = (tmp_path / (tag + "_hem") / name[4:]) if name.startswith("hem/") else d / name
            data = p.read_bytes()
            if name.endswith(".png"):
                got_px = hashlib.sha256(np.asarray(Image.open(p)).tobytes()).hexdigest()
                assert got_px == want["pixels_sha256"], (tag, name)
            assert hashlib.sha256(data).hexdigest() == want["sha256"], (tag, name, len(data), want["bytes"])
