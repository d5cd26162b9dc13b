"""run_test harness (DCVC-DC/test_video.py:71-237): YUV420 input conversion,
in-place clamp, per-plane distortion and the JSON log.

CPU tests pin the numpy restatement (oracle/harness_oracle.py) to the
reference's own dependency (scipy.ndimage.zoom, numpy means) and check the
log arithmetic.  GPU tests check the HIP kernels against that restatement
(bit-exact input conversion, fp64 sums to 1e-12) and one YUV420 sequence of
DCVC-DC through ``run_test`` against the CPU oracle codec (config C4's path at
a small size; PSNR formula of test_video.py:171-181)."""
import os
import tempfile

import numpy as np
import pytest
import scipy.ndimage
import torch

from oracle import harness_oracle as HO


# --------------------------------------------------------------------- CPU
@pytest.mark.parametrize("n", [1, 2, 3, 17, 50, 65, 68, 540, 1080, 1920])
def test_zoom_index_matches_scipy(n):
    src = np.arange(n, dtype=np.float64).reshape(1, n)
    z = scipy.ndimage.zoom(src, (1, 2), order=0)
    np.testing.assert_array_equal(z[0].astype(np.int64), HO.zoom_index(2 * n, n))


def test_yuv_input_matches_reference_pipeline():
    g = np.random.default_rng(3)
    h, w = 38, 54
    y = g.integers(0, 256, (h, w), dtype=np.uint8)
    uv = g.integers(0, 256, (2, h // 2, w // 2), dtype=np.uint8)
    # test_video.py:110-112 + functional.py:61-72 + F.pad(replicate), :128-132
    yf = y.astype(np.float32)[None] / 255
    uvf = uv.astype(np.float32) / 255
    ref = np.concatenate((yf, scipy.ndimage.zoom(uvf, (1, 2, 2), order=0)), axis=0)
    ref = torch.nn.functional.pad(torch.from_numpy(ref)[None], (0, 10, 0, 10), mode="replicate")[0]
    ours = HO.yuv_u8_to_input(y, uv, h + 10, w + 10)
    np.testing.assert_array_equal(ours, ref.permute(1, 2, 0).numpy())


def test_chroma_mean_order():
    """dcvc_frame_sse sums each 2x2 chroma block as (x00 + x01) + (x10 + x11),
    the order numpy's float32 mean over axes (-1, -3) uses."""
    g = np.random.default_rng(0)
    a = g.random((1, 64, 2, 96, 2)).astype(np.float32)
    m = np.mean(a, axis=(-1, -3))
    s = (a[:, :, 0, :, 0] + a[:, :, 0, :, 1]) + (a[:, :, 1, :, 0] + a[:, :, 1, :, 1])
    np.testing.assert_array_equal(m, s / np.float32(4))


def test_psnr_formulas():
    from dcvc_amd.harness import psnr_rgb, psnr_yuv, calc_psnr_from_sse
    g = np.random.default_rng(1)
    h, w = 20, 30
    a = torch.from_numpy(g.random((1, 3, h, w)).astype(np.float32))
    b = torch.from_numpy(g.random((1, 3, h, w)).astype(np.float32))
    d = (a - b).numpy().astype(np.float32)
    sse = np.array([np.sum((d[0, c].astype(np.float64)) ** 2) for c in range(3)])
    assert abs(psnr_rgb(sse, h, w) - HO.psnr_torch(a, b)) < 1e-5
    assert calc_psnr_from_sse(0.0, 10) == 999.9
    x = g.random((3, h, w)).astype(np.float32)
    yu8 = g.integers(0, 256, (h, w), dtype=np.uint8)
    uvu8 = g.integers(0, 256, (2, h // 2, w // 2), dtype=np.uint8)
    ours = psnr_yuv(HO.yuv_sse(x, yu8, uvu8), h, w)
    np.testing.assert_allclose(ours, HO.yuv_distortion(x, yu8, uvu8), rtol=0, atol=1e-9)


def test_generate_log_json_fields():
    from dcvc_amd.harness import generate_log_json, generate_log_json_hem
    types, bits, ps = [0, 1, 1, 0], [100, 40, 60, 120], [30.0, 29.0, 28.0, 31.0]
    log = generate_log_json(4, 10, 1.5, types, bits, ps, [0.0] * 4)
    assert log["i_frame_num"] == 2 and log["p_frame_num"] == 2
    assert log["ave_i_frame_bpp"] == 220 / 2 / 10
    assert log["ave_p_frame_bpp"] == 100 / 20
    assert log["ave_all_frame_bpp"] == 320 / 40
    assert log["ave_all_frame_psnr"] == sum(ps) / 4
    assert "frame_bpp" not in log
    yl = generate_log_json(4, 10, 1.5, types, bits, ps, [0.0] * 4, ps, ps, ps, [0.0] * 4, [0.0] * 4, [0.0] * 4)
    assert yl["ave_p_frame_psnr_u"] == 28.5 and yl["ave_all_frame_psnr_v"] == sum(ps) / 4
    hl = generate_log_json_hem(4, types, bits, ps, [0.0] * 4, 10, 1.5)
    assert hl["frame_type"] == types and hl["frame_bpp"] == [10.0, 4.0, 6.0, 12.0]
    assert "ave_i_frame_psnr_y" not in hl


def test_yuv_reader_roundtrip(tmp_path):
    from dcvc_amd.harness import YUVReader
    g = np.random.default_rng(2)
    h, w = 6, 8
    frames = [(g.integers(0, 256, (h, w), dtype=np.uint8), g.integers(0, 256, (2, h // 2, w // 2), dtype=np.uint8))
              for _ in range(3)]
    p = tmp_path / "seq.yuv"
    with open(p, "wb") as f:
        for y, uv in frames:
            f.write(y.tobytes())
            f.write(uv.tobytes())
    r = YUVReader(str(p)[:-4], w, h, skip_frame=1)   # the reader appends .yuv
    for y, uv in frames[1:]:
        ry, ruv = r.read_one_frame()
        np.testing.assert_array_equal(ry, y)
        np.testing.assert_array_equal(ruv, uv)
    assert r.read_one_frame() == (None, None)
    r.close()


# --------------------------------------------------------------------- GPU
gpu = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@gpu
@pytest.mark.parametrize("shape", [(38, 54, 48, 64), (100, 130, 112, 144), (2160, 3840, 2160, 3840)])
def test_yuv420_to_nhwc_bit_exact(shape):
    _need_gpu()
    from dcvc_amd import hip as K
    h, w, H, W = shape
    g = np.random.default_rng(h)
    y = g.integers(0, 256, (h, w), dtype=np.uint8)
    uv = g.integers(0, 256, (2, h // 2, w // 2), dtype=np.uint8)
    out = K.empty(H, W, 3, K.F32)
    K.yuv420_to_nhwc(torch.from_numpy(y).cuda(), torch.from_numpy(uv).cuda(), h, w, out)
    np.testing.assert_array_equal(out.t().cpu().numpy(), HO.yuv_u8_to_input(y, uv, H, W))


@gpu
@pytest.mark.parametrize("yuv", [False, True])
@pytest.mark.parametrize("shape", [(38, 54, 48, 64), (1080, 1920, 1088, 1920)])
def test_frame_sse_and_inplace_clamp(yuv, shape):
    _need_gpu()
    from dcvc_amd import hip as K
    h, w, H, W = shape
    g = np.random.default_rng(w)
    xh = torch.from_numpy((g.random((H, W, 3)) * 1.4 - 0.2).astype(np.float32)).cuda()
    x_act = K.Act(xh.clone())
    clamped = xh.clamp(0, 1).cpu().numpy()
    ws = K.frame_sse_workspace(xh.device)
    out = torch.zeros(3, dtype=torch.float64, device=xh.device)
    crop = clamped[:h, :w].transpose(2, 0, 1)
    if yuv:
        y = g.integers(0, 256, (h, w), dtype=np.uint8)
        uv = g.integers(0, 256, (2, h // 2, w // 2), dtype=np.uint8)
        K.frame_sse(x_act, torch.from_numpy(y).cuda(), h, w, ws, out, uv_u8=torch.from_numpy(uv).cuda())
        ref = HO.yuv_sse(np.ascontiguousarray(crop), y, uv)
    else:
        src = g.integers(0, 256, (3, h, w), dtype=np.uint8)
        K.frame_sse(x_act, torch.from_numpy(src).cuda(), h, w, ws, out)
        d = crop - src.astype(np.float32) / np.float32(255)
        ref = np.array([np.sum((d[c] * d[c]).astype(np.float64)) for c in range(3)])
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-12)
    # recon_frame.clamp_(0, 1) acted on the whole padded buffer
    np.testing.assert_array_equal(x_act.t().cpu().numpy(), clamped)


def _oracle_sequence(i, p, xps, h, w, q):
    """test_video.py's loop with the oracle codec and the C oracle coder."""
    from oracle import rans_oracle as R
    from tests.test_oracle_dc import oracle_tables, KIND
    tabs = oracle_tables(i, p)
    dpb, out = None, []
    for t, xp in enumerate(xps):
        pre = "i_" if t == 0 else "p_"
        with torch.no_grad():
            calls = i.compress(xp, False, q) if t == 0 else p.compress(xp, dpb, False, q, t % 4)
            coder_calls = [(s.clamp(-30000, 30000).to(torch.int16).numpy(), ix.to(torch.int16).numpy(),
                            tabs[pre + KIND[k]]) for k, s, ix in calls]
            enc = R.DCStream()
            stream = enc.encode(coder_calls)
            decoded = enc.decode(stream)
            pos = [0]

            def decoder(kind, idx):
                n = idx.numel()
                v = decoded[pos[0]:pos[0] + n]
                pos[0] += n
                return v

            if t == 0:
                xh = i.decompress(decoder, h, w, False, q)
                dpb = {"ref_frame": xh, "ref_feature": None, "ref_mv_feature": None, "ref_y": None, "ref_mv_y": None}
            else:
                dpb = p.decompress(dpb, decoder, h, w, False, q, t % 4)
        dpb["ref_frame"].clamp_(0, 1)
        out.append(((len(stream) + (13 if t == 0 else 6)) * 8, dpb["ref_frame"][0, :, :h, :w].numpy()))
    return out


@gpu
@pytest.mark.parametrize("prec", ["split", "parity"])
def test_run_test_yuv420_matches_oracle(dc_golden, prec):
    """A YUV420 sequence (the C4 path at 100x130) through run_test in the
    bench's split precision and in fp32: bits and PSNR_y/u/v against the
    oracle codec on the same 4:4:4 input, within the parity tolerance of
    tests/test_gpu_model_dc.py."""
    _need_gpu()
    from dcvc_amd.dc import DMC, IntraNoAR
    from dcvc_amd.harness import run_test, ArrayReader
    from dcvc_amd.layers import Precision
    from dcvc_amd.synth import moving_pattern_yuv420
    from oracle import dc_oracle as O
    from oracle import rans_oracle as R
    from tests.test_gpu_model_dc import PARITY_TOL
    h, w, n, q = 100, 130, 3, 0
    frames = [moving_pattern_yuv420(h, w, t, seed=5) for t in range(n)]
    inet = IntraNoAR(precision=getattr(Precision, prec)()).load_state_dict(dc_golden.i_state_dict())
    pnet = DMC(precision=getattr(Precision, prec)()).load_state_dict(dc_golden.p_state_dict())
    inet.update(force=True)
    pnet.update(force=True)
    with tempfile.TemporaryDirectory() as td:
        log = run_test(pnet, inet, {"frame_num": n, "gop_size": 32, "write_stream": True, "bin_folder": td,
                                    "src_reader": ArrayReader(frames), "src_type": "yuv420",
                                    "src_height": h, "src_width": w, "dist_in_yuv420": True,
                                    "q_in_ckpt": False, "i_frame_q_index": q, "verbose": 1})
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    io = O.IntraOracle(dc_golden.i_state_dict(), R.pmf_to_quantized_cdf)
    po = O.DMCOracle(dc_golden.p_state_dict(), R.pmf_to_quantized_cdf)
    H, W = 112, 144
    xps = [torch.from_numpy(HO.yuv_u8_to_input(y, uv, H, W)).permute(2, 0, 1)[None].contiguous() for y, uv in frames]
    ref = _oracle_sequence(io, po, xps, h, w, q)
    for t, (bits, rec) in enumerate(ref):
        py, pu, pv, p = HO.yuv_distortion(rec, *frames[t])
        assert abs(log["frame_bpp"][t] * h * w - bits) / bits <= PARITY_TOL["bits_rel"], (t, log["frame_bpp"][t], bits)
        assert abs(log["frame_psnr_y"][t] - py) <= PARITY_TOL["psnr_db"], t
        assert abs(log["frame_psnr_u"][t] - pu) <= PARITY_TOL["psnr_db"], t
        assert abs(log["frame_psnr_v"][t] - pv) <= PARITY_TOL["psnr_db"], t
        assert abs(log["frame_psnr"][t] - p) <= PARITY_TOL["psnr_db"], t
    assert log["i_frame_num"] == 1 and log["p_frame_num"] == n - 1


# ------------------------------------------------------------------ MS-SSIM
def _golden_msssim():
    import importlib.util
    import json
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    spec = importlib.util.spec_from_file_location("make_golden_msssim", os.path.join(here, "make_golden_msssim.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    with open(os.path.join(here, "msssim_golden.json")) as f:
        return m.planes, json.load(f)["cases"]


def test_down2_reflect_matches_scipy():
    import scipy.ndimage as nd
    g = np.random.default_rng(4)
    for h, w in ((5, 7), (6, 8), (11, 10)):
        a = g.random((h, w))
        ref = nd.convolve(a, np.ones((2, 2)) / 4.0, mode="reflect")[::2, ::2]
        np.testing.assert_allclose(HO.down2_reflect(a), ref, rtol=0, atol=1e-15)


def test_msssim_oracle_matches_reference_fixtures():
    """oracle calc_msssim vs the reference's own calc_msssim outputs
    (tests/golden/make_golden_msssim.py imported metrics.py)."""
    planes, cases = _golden_msssim()
    for c in cases[:4]:
        src, rec = planes(c["seed"], c["h"], c["w"])
        assert abs(HO.calc_msssim(src, rec) - c["msssim"]) < 1e-12, c
        assert abs(HO.calc_psnr(src, rec, data_range=1) - c["psnr"]) < 1e-9, c


def _gpu_msssim(a, b):
    """calc_msssim of two host planes through dcvc_ssim_level / dcvc_down2_f64."""
    from dcvc_amd import hip as K
    from dcvc_amd.harness import MsSsim
    dev = torch.device("cuda", 0)
    h, w = a.shape
    x, y = np.mgrid[-5:6, -5:6]
    g = np.exp(-((x ** 2 + y ** 2) / (2.0 * 1.5 ** 2)))
    win = torch.from_numpy(g / g.sum()).to(dev)
    ws = torch.empty(int(K.lib().dcvc_ssim_workspace()) // 8, dtype=torch.float64, device=dev)
    L = 5 if h >= 176 and w >= 176 else 4
    out = torch.zeros((L, 2), dtype=torch.float64, device=dev)
    ta = torch.from_numpy(a.astype(np.float64).reshape(-1)).to(dev)
    tb = torch.from_numpy(b.astype(np.float64).reshape(-1)).to(dev)
    for k in range(L):
        K.ssim_level(ta, tb, h, w, win, ws, out[k])
        if k < L - 1:
            nh, nw = (h + 1) // 2, (w + 1) // 2
            na = torch.empty(nh * nw, dtype=torch.float64, device=dev)
            nb = torch.empty(nh * nw, dtype=torch.float64, device=dev)
            K.down2_f64(ta, h, w, na)
            K.down2_f64(tb, h, w, nb)
            ta, tb, h, w = na, nb, nh, nw
    o = out.cpu().numpy()
    wgt = MsSsim.W5 if L == 5 else MsSsim.W4
    return float(np.prod(o[:L - 1, 1] ** wgt[:L - 1]) * o[L - 1, 0] ** wgt[L - 1])


@gpu
def test_gpu_msssim_matches_reference_fixtures():
    """The GPU level chain against the reference's calc_msssim outputs (fp64;
    the reference filters with fftconvolve, the GPU sums directly: agreement
    to 1e-10)."""
    _need_gpu()
    planes, cases = _golden_msssim()
    for c in cases:
        src, rec = planes(c["seed"], c["h"], c["w"])
        assert abs(_gpu_msssim(src, rec) - c["msssim"]) < 1e-10, c


@gpu
def test_run_test_yuv420_msssim():
    """run_test(calc_ssim=True) on a YUV420 sequence: MS-SSIM of Y/U/V from
    the GPU against the oracle's calc_msssim of the same recon planes."""
    _need_gpu()
    from dcvc_amd import hip as K
    from dcvc_amd.harness import MsSsim, FrameStage
    from dcvc_amd.synth import moving_pattern_yuv420
    h, w = 200, 256
    y, uv = moving_pattern_yuv420(h, w, 0, seed=9)
    g = np.random.default_rng(9)
    H, W = 208, 256
    xh = torch.from_numpy((HO.yuv_u8_to_input(y, uv, H, W) + g.normal(0, 0.04, (H, W, 3))).astype(np.float32)).cuda()
    act = K.Act(xh)
    ms = MsSsim(h, w, 1, xh.device)
    ms.run(act, torch.from_numpy(y).cuda(), torch.from_numpy(uv).cuda(), 0)
    got = ms.values(1)[0]
    crop = np.clip(xh.cpu().numpy()[:h, :w].transpose(2, 0, 1), 0, 1)
    y_rec, uv_rec = HO.ycbcr444_to_420(np.ascontiguousarray(crop))
    ref = [HO.calc_msssim(y.astype(np.float32) / 255, y_rec[0]),
           HO.calc_msssim(uv[0].astype(np.float32) / 255, uv_rec[0]),
           HO.calc_msssim(uv[1].astype(np.float32) / 255, uv_rec[1])]
    np.testing.assert_allclose(got[:3], ref, rtol=0, atol=1e-10)
    assert abs(got[3] - (6 * ref[0] + ref[1] + ref[2]) / 8) < 1e-10


def test_avgpool2_padding_semantics():
    """avg_pool2d(kernel 2, padding = size % 2, count_include_pad) as the
    GPU kernel restates it: zero rows/columns on both sides of odd sizes."""
    import torch.nn.functional as F
    x = torch.arange(35, dtype=torch.float64).reshape(1, 1, 5, 7)
    got = F.avg_pool2d(x, kernel_size=2, padding=[1, 1])
    p = F.pad(x, (1, 1, 1, 1))
    ref = (p[..., 0:-1:2, 0:-1:2] + p[..., 0:-1:2, 1::2] + p[..., 1::2, 0:-1:2] + p[..., 1::2, 1::2]) / 4
    assert torch.equal(got, ref[..., :got.shape[2], :got.shape[3]])


@gpu
@pytest.mark.parametrize("h,w", [(256, 256), (181, 243), (1080, 1920)])
def test_gpu_rgb_msssim_matches_restatement(h, w):
    """MsSsimRGB (fp64 GPU) vs the fp32 torch restatement of pytorch_msssim
    (parity unpinned: the package is absent); agreement to 1e-5."""
    _need_gpu()
    from dcvc_amd import hip as K
    from dcvc_amd.harness import MsSsimRGB
    g = np.random.default_rng(h)
    src = g.integers(0, 256, (3, h, w), dtype=np.uint8)
    rec = np.clip(src.astype(np.float32) / 255 + g.normal(0, 0.05, (3, h, w)).astype(np.float32), 0, 1)
    xh = torch.from_numpy(np.ascontiguousarray(rec.transpose(1, 2, 0))).cuda()
    ms = MsSsimRGB(h, w, 1, xh.device)
    ms.run(K.Act(xh), torch.from_numpy(src).cuda(), 0)
    got = ms.values(1)[0]
    ref = HO.ms_ssim_torch(torch.from_numpy(rec)[None], torch.from_numpy(src.astype(np.float32) / 255)[None])
    assert abs(got - ref) < 1e-5, (got, ref)


# ------------------------------------------------------- decoded-frame writers
@gpu
@pytest.mark.parametrize("kind,fmt", [("png", "rgb"), ("yuv", "420"), ("hem_png", "rgb"), ("yuv", "rgb"),
                                      ("png", "420")])
def test_recon_writers_match_reference_formulas(tmp_path, kind, fmt):
    """--save_decoded_frame: what ReconWriter stores for a decoded frame (values
    outside [0, 1] included, padded buffer cropped) equals the reference's
    writers applied to the same frame (video_writer.py:26-111 restated in
    oracle/harness_oracle.py; the 4:2:0 cases through ycbcr444_to_420)."""
    _need_gpu()
    from PIL import Image
    from dcvc_amd import hip as K
    from dcvc_amd.harness import ReconWriter
    h, w, H, W = 38, 54, 48, 64
    g = torch.Generator().manual_seed(3)
    frames = [torch.rand(H, W, 3, generator=g) * 1.2 - 0.1 for _ in range(2)]
    wr = ReconWriter(str(tmp_path / "rec"), h, w, kind, fmt, torch.device("cuda", 0))
    for t, f in enumerate(frames):
        wr.write(K.Act(f.cuda().contiguous()), t)
    wr.close()
    for t, f in enumerate(frames):
        crop = f[:h, :w].permute(2, 0, 1).numpy()
        if kind in ("png", "hem_png"):
            name = f"im{t + 1:05d}.png" if kind == "png" else f"{t}.png"
            got = np.asarray(Image.open(tmp_path / "rec" / name))
            if fmt == "rgb":
                np.testing.assert_array_equal(got, HO.png_writer_u8(crop))
            else:
                # 4:2:0 frame into PNGWriter: ycbcr420_to_rgb(order=1) of y_rec, uv_rec
                y, uv = HO.ycbcr444_to_420(crop)
                uvz = scipy.ndimage.zoom(uv, (1, 2, 2), order=1)
                r = y + (2 - 2 * 0.2126) * (uvz[1:2] - 0.5)
                b = y + (2 - 2 * 0.0722) * (uvz[0:1] - 0.5)
                gg = (y - 0.2126 * r - 0.0722 * b) / 0.7152
                np.testing.assert_array_equal(got, HO.png_writer_u8(np.clip(np.concatenate((r, gg, b)), 0, 1)))
        else:
            data = (tmp_path / "rec" / "out.yuv").read_bytes()
            n = h * w * 3 // 2
            frame = data[t * n:(t + 1) * n]
            if fmt == "420":
                y, uv = HO.ycbcr444_to_420(crop)
            else:
                kr, kg, kb = 0.2126, 0.7152, 0.0722
                r, gg, b = crop[0:1], crop[1:2], crop[2:3]
                y = kr * r + kg * gg + kb * b
                cb = 0.5 * (b - y) / (1 - kb) + 0.5
                cr = 0.5 * (r - y) / (1 - kr) + 0.5
                uv = np.concatenate(HO.ycbcr444_to_420(np.concatenate((y, cb, cr)))[1:], 0)
                y = np.clip(y, 0, 1)
            assert frame == HO.yuv_writer_bytes(y, uv)


@gpu
def test_run_test_saves_decoded_frames(dc_golden, tmp_path):
    """run_test with save_decoded_frame (test_video.py:84-88, 210-221): one
    PNG per frame, named from 1, in a folder renamed after the averages."""
    _need_gpu()
    from dcvc_amd.dc import DMC, IntraNoAR
    from dcvc_amd.harness import run_test, ArrayReader
    from dcvc_amd.layers import Precision
    from dcvc_amd.synth import moving_pattern
    h, w, n = 100, 130, 3
    inet = IntraNoAR(precision=Precision.fast()).load_state_dict(dc_golden.i_state_dict())
    pnet = DMC(precision=Precision.fast()).load_state_dict(dc_golden.p_state_dict())
    inet.update(force=True)
    pnet.update(force=True)
    rec = tmp_path / "dec" / "seq" / "0"
    log = run_test(pnet, inet, {"frame_num": n, "gop_size": 32, "write_stream": True, "bin_folder": str(tmp_path),
                                "src_reader": ArrayReader([moving_pattern(h, w, t, seed=3) for t in range(n)]),
                                "src_type": "png", "src_height": h, "src_width": w, "q_in_ckpt": False,
                                "i_frame_q_index": 0, "save_decoded_frame": True, "recon_path": str(rec),
                                "rate_idx": 0, "verbose": 1})
    folders = [d for d in os.listdir(tmp_path / "dec" / "seq") if d.startswith("0_")]
    assert len(folders) == 1 and not rec.exists()
    avg_bpp = sum(b * h * w for b in log["frame_bpp"]) / n / h / w
    assert folders[0] == f"0_{avg_bpp:.4f}_{log['ave_all_frame_psnr']:.4f}"
    assert sorted(os.listdir(tmp_path / "dec" / "seq" / folders[0])) == [f"im{i:05d}.png" for i in range(1, n + 1)]
