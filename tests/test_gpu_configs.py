"""BASELINE.json configurations at full size on the GPU, in the bench's
precision (Precision.split(): fp32 feature maps and latents, every conv on
split-fp16 MFMA) and in the bf16 Precision.fast() kept for comparison: config
C2 (DCVC-HEM 1920x1080, zero pad to 1088), C3 (DCVC-DC RGB 1920x1080,
replicate pad) and C4 (DCVC-DC YUV420 3840x2160, coded as YCbCr 4:4:4), each
an I-frame and two P-frames through encode_decode(..., output_path) as
bench.py runs them (in split precision encode_decode also checks the fp16
range guard, dcvc_split_range_flag).

Size-independent properties checked per frame: the decoder reads back exactly
the symbols and CDF indexes the encoder wrote (lossless round trip through the
file), bits equal the file size, and the reconstruction and its PSNR (the
harness's in-place clamp + squared-error kernels) are finite.  Oracle parity at full
size is tests/test_gpu_parity_strict.py (C3, C2, and the C4 path at 1080p).
"""
import math
import os
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


CONFIGS = {"C2": ("hem", False, 1080, 1920), "C3": ("dc", False, 1080, 1920), "C4": ("dc", True, 2160, 3840)}


@pytest.mark.parametrize("prec", ["split", "fast"])
@pytest.mark.parametrize("cfg", ["C3", "C2", "C4"])
def test_full_size_lossless(cfg, prec):
    import bench
    from dcvc_amd.harness import FrameStage, psnr_rgb, psnr_yuv
    from dcvc_amd.layers import Precision
    from dcvc_amd.synth import moving_pattern, moving_pattern_yuv420
    model, yuv, h, w = CONFIGS[cfg]
    dev = torch.device("cuda", 0)
    isd, psd = bench.make_weights(None, 0, dev, model)
    hem = model == "hem"
    if hem:
        from dcvc_amd.hem import DMC, IntraNoAR
        qi, qmv, qy = bench.hem_q(isd, psd, 0)
    else:
        from dcvc_amd.dc import DMC, IntraNoAR
    inet = IntraNoAR(precision=getattr(Precision, prec)()).load_state_dict(isd)
    pnet = DMC(precision=getattr(Precision, prec)()).load_state_dict(psd)
    inet.update(force=True)
    pnet.update(force=True)
    stage = FrameStage(h, w, 64 if hem else 16, yuv, zero_pad=hem, frame_num=3, device=dev)
    dpb, out = None, []
    with tempfile.TemporaryDirectory() as td:
        for t in range(3):
            if yuv:
                src = tuple(torch.from_numpy(a).to(dev) for a in moving_pattern_yuv420(h, w, t, seed=1))
            else:
                src = torch.from_numpy(moving_pattern(h, w, t, seed=1)).to(dev)
            x = stage.load(src)
            path = os.path.join(td, f"{t}.bin")
            net = inet if t == 0 else pnet
            net.entropy_coder.trace = []
            if hem:
                if t == 0:
                    r = inet.encode_decode(x, qi, path, pic_width=w, pic_height=h)
                    dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_y": None, "ref_mv_y": None}
                else:
                    r = pnet.encode_decode(x, dpb, path, pic_width=w, pic_height=h, mv_y_q_scale=qmv, y_q_scale=qy)
                    dpb = r["dpb"]
            elif t == 0:
                r = inet.encode_decode(x, False, 0, path, pic_width=w, pic_height=h)
                dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_mv_feature": None, "ref_y": None,
                       "ref_mv_y": None}
            else:
                r = pnet.encode_decode(x, dpb, False, 0, path, pic_width=w, pic_height=h, frame_idx=t % 4)
                dpb = r["dpb"]
            tr = net.entropy_coder.trace
            net.entropy_coder.trace = None
            enc = [e for e in tr if e[0] == "enc"]
            dec = [e for e in tr if e[0] == "dec"]
            assert len(enc) == len(dec) > 0
            nsym = 0
            for (_, se, ie), (_, sd, id_) in zip(enc, dec):
                np.testing.assert_array_equal(ie.reshape(-1), id_.reshape(-1), err_msg=f"{cfg} t={t} indexes")
                np.testing.assert_array_equal(se.reshape(-1), sd.reshape(-1), err_msg=f"{cfg} t={t} symbols")
                nsym += se.size
            assert r["bit"] == os.path.getsize(path) * 8
            stage.distortion(dpb["ref_frame"], src, t)
            rec = dpb["ref_frame"]
            assert bool(torch.isfinite(rec).all())
            out.append((r["bit"], nsym))
    sums = stage.sums()
    for t in range(3):
        p = psnr_yuv(sums[t], h, w)[3] if yuv else psnr_rgb(sums[t], h, w)
        assert math.isfinite(p) and p > 0, (cfg, t, p)
    print(cfg, [(b, n) for b, n in out])
