"""The test harness around the codecs: ``run_test`` of DCVC-DC/test_video.py:
71-237 (RGB and YUV420 sources, I/P schedule, DPB aliasing, in-place clamp,
crop, PSNR, the JSON log of src/utils/common.py:44-140) and of
DCVC-HEM/test_video.py:80-172, with the per-frame tensor work on the GPU.

Source frames cross to the GPU as uint8 (a quarter of the reference's fp32
upload).  ``FrameStage`` turns them into the padded NHWC codec input
(``dcvc_frame_to_nhwc`` / ``dcvc_yuv420_to_nhwc``) and computes each frame's
distortion with ``dcvc_frame_sse``, which also performs
``recon_frame.clamp_(0, 1)`` on the DPB frame in place.  The squared-error
sums stay on the device until the end of the sequence (one transfer), and the
PSNR formulas are evaluated on the host exactly as the reference writes them.

MS-SSIM: for YUV420 sources ``calc_ssim`` runs the reference's per-plane
``calc_msssim`` (src/utils/metrics.py:39-62) on the GPU in fp64 (``MsSsim``,
msssim.hip), pinned to the reference's outputs.  RGB MS-SSIM is
``pytorch_msssim.ms_ssim`` in the reference (DC and HEM), a package absent
from this image: ``MsSsimRGB`` follows its published algorithm on the GPU and
the log carries ``msssim_unpinned``.
"""
import contextlib
import os
import time

import numpy as np
import torch

from . import hip as K
from .stream_helper import get_padding_size


# ----------------------------------------------------------------- readers
class YUVReader:
    """Raw 8-bit YUV420 file reader (DCVC-DC/src/utils/video_reader.py:
    121-161).  ``read_one_frame`` returns uint8 ``(y (h, w), uv (2, h/2,
    w/2))``, or ``(None, None)`` at the end of the file; the reference's
    float conversion (x / 255) happens on the GPU."""

    def __init__(self, src_path, width, height, src_format="420", skip_frame=0):
        if src_format != "420":
            raise ValueError("only 420 sources are supported (video_reader.py:127)")
        if not src_path.endswith(".yuv"):
            src_path = src_path + ".yuv"
        self.src_path, self.width, self.height = src_path, width, height
        self.y_size = width * height
        self.uv_size = width * height // 2
        self.eof = False
        self.file = open(src_path, "rb")  # noqa: SIM115 (closed in close())
        for _ in range(skip_frame):
            if not self._read():
                break

    def _read(self):
        y = self.file.read(self.y_size)
        uv = self.file.read(self.uv_size)
        if len(y) < self.y_size or len(uv) < self.uv_size:
            self.eof = True
            return None
        return y, uv

    def read_one_frame(self, dst_format="420"):
        if dst_format != "420":
            raise ValueError("YUVReader hands over 420 planes; RGB sources use PNGReader")
        if self.eof:
            return None, None
        r = self._read()
        if r is None:
            return None, None
        y = np.frombuffer(r[0], dtype=np.uint8).reshape(self.height, self.width)
        uv = np.frombuffer(r[1], dtype=np.uint8).reshape(2, self.height // 2, self.width // 2)
        return y, uv

    def close(self):
        self.file.close()


class PNGReader:
    """Folder of im1.png / im00001.png frames (video_reader.py:44-80);
    returns uint8 CHW RGB, or None at the end."""

    def __init__(self, src_path, width, height, start_num=1):
        pngs = os.listdir(src_path)
        if "im1.png" in pngs:
            self.padding = 1
        elif "im00001.png" in pngs:
            self.padding = 5
        else:
            raise ValueError("unknown image naming convention; please specify")
        self.src_path, self.width, self.height = src_path, width, height
        self.current_frame_index = start_num
        self.eof = False

    def read_one_frame(self, dst_format="rgb"):
        from PIL import Image
        if dst_format != "rgb":
            raise ValueError("PNGReader hands over RGB frames")
        if self.eof:
            return None
        p = os.path.join(self.src_path, f"im{str(self.current_frame_index).zfill(self.padding)}.png")
        if not os.path.exists(p):
            self.eof = True
            return None
        rgb = np.asarray(Image.open(p).convert("RGB")).transpose(2, 0, 1)
        if rgb.shape[1:] != (self.height, self.width):
            raise ValueError(f"{p}: {rgb.shape[1:]} != {(self.height, self.width)}")
        self.current_frame_index += 1
        return np.ascontiguousarray(rgb)

    def close(self):
        self.current_frame_index = 1


class ArrayReader:
    """In-memory frames (synthetic sequences, tests): uint8 CHW RGB arrays,
    or (y, uv) uint8 plane pairs for YUV420."""

    def __init__(self, frames):
        self.frames = list(frames)
        self.i = 0

    def read_one_frame(self, dst_format="rgb"):
        if self.i >= len(self.frames):
            return (None, None) if dst_format == "420" else None
        f = self.frames[self.i]
        self.i += 1
        return f

    def close(self):
        pass


# ----------------------------------------------------------- device staging
class FrameStage:
    """Device side of one sequence: uint8 source upload, padded NHWC codec
    input, and the per-frame squared-error sums (frame_num x 3, fp64)."""

    def __init__(self, h, w, align, yuv420, zero_pad, frame_num, device):
        self.h, self.w, self.yuv, self.zero_pad = h, w, yuv420, zero_pad
        _, pr, _, pb = get_padding_size(h, w, align)
        self.H, self.W = h + pb, w + pr
        self.dev = device
        self.x = K.empty(self.H, self.W, 3, K.F32, device)
        self.ws = K.frame_sse_workspace(device)
        self.sse = torch.zeros((max(frame_num, 1), 3), dtype=torch.float64, device=device)

    def upload(self, frame):
        """Host uint8 frame (CHW RGB, or (y, uv)) -> device tensors."""
        if self.yuv:
            y, uv = frame
            return K.upload(y, self.dev, "frame_y"), K.upload(uv, self.dev, "frame_uv")
        return K.upload(frame, self.dev, "frame")

    def load(self, dframe):
        """Device uint8 frame -> padded NHWC fp32 codec input (test_video.py:
        108-132: ycbcr420_to_444(order=0) for YUV, x / 255, F.pad)."""
        if self.yuv:
            K.yuv420_to_nhwc(dframe[0], dframe[1], self.h, self.w, self.x)
        else:
            K.frame_to_nhwc(dframe, self.h, self.w, self.x, zero_pad=self.zero_pad)
        return self.x

    def distortion(self, recon, dframe, slot):
        """recon_frame.clamp_(0, 1), crop, and the squared-error sums of the
        frame into row ``slot`` (test_video.py:169-195)."""
        from .dc.video_model import as_act
        r = as_act(recon)
        if self.yuv:
            K.frame_sse(r, dframe[0], self.h, self.w, self.ws, self.sse[slot], uv_u8=dframe[1])
        else:
            K.frame_sse(r, dframe, self.h, self.w, self.ws, self.sse[slot])

    def sums(self):
        return self.sse.cpu().numpy()


class MsSsim:
    """calc_msssim (DCVC-DC/src/utils/metrics.py:39-62) of the three planes of
    a YUV420 frame, test_video.py:182-185: per level, the means of the ssim
    and cs maps on the GPU (dcvc_ssim_level), the 2x2 reflect downsample
    (dcvc_down2_f64); the weighted product on the host."""

    W5 = np.array([0.0448, 0.2856, 0.3001, 0.2363, 0.1333])
    W4 = np.array([0.0517, 0.3295, 0.3462, 0.2726])

    def __init__(self, h, w, frame_num, device):
        if min(h // 2, w // 2) < 88:
            raise ValueError("calc_msssim needs planes of at least 88 x 88 (metrics.py:49-50)")
        self.h, self.w, self.dev = h, w, device
        n = h * w + 2 * (h // 2) * (w // 2)
        self.src = torch.empty(n, dtype=torch.float64, device=device)
        self.rec = torch.empty(n, dtype=torch.float64, device=device)
        x, y = np.mgrid[-5:6, -5:6]                         # fspecial_gauss(11, 1.5), metrics.py:9-12
        g = np.exp(-((x ** 2 + y ** 2) / (2.0 * 1.5 ** 2)))
        self.win = torch.from_numpy(g / g.sum()).to(device)
        self.ws = torch.empty(int(K.lib().dcvc_ssim_workspace()) // 8, dtype=torch.float64, device=device)
        self.out = torch.zeros((max(frame_num, 1), 3, 5, 2), dtype=torch.float64, device=device)
        self.planes = []                                    # (offset, ph, pw, levels, level buffers)
        off = 0
        for ph, pw in ((h, w), (h // 2, w // 2), (h // 2, w // 2)):
            L = 5 if ph >= 176 and pw >= 176 else 4
            bufs, sh, sw = [], ph, pw
            for _ in range(L - 1):
                sh, sw = (sh + 1) // 2, (sw + 1) // 2
                bufs.append((torch.empty(sh * sw, dtype=torch.float64, device=device),
                             torch.empty(sh * sw, dtype=torch.float64, device=device), sh, sw))
            self.planes.append((off, ph, pw, L, bufs))
            off += ph * pw

    def run(self, x_hat, y_u8, uv_u8, slot):
        K.yuv_planes_f64(x_hat, y_u8, uv_u8, self.h, self.w, self.src, self.rec)
        for p, (off, ph, pw, L, bufs) in enumerate(self.planes):
            a, b, sh, sw = self.src[off:off + ph * pw], self.rec[off:off + ph * pw], ph, pw
            for k in range(L):
                K.ssim_level(a, b, sh, sw, self.win, self.ws, self.out[slot, p, k])
                if k < L - 1:
                    na, nb, nh, nw = bufs[k]
                    K.down2_f64(a, sh, sw, na)
                    K.down2_f64(b, sh, sw, nb)
                    a, b, sh, sw = na, nb, nh, nw

    def values(self, n):
        """(msssim_y, msssim_u, msssim_v, (6 y + u + v) / 8) per frame."""
        o = self.out[:n].cpu().numpy()
        res = []
        for f in range(n):
            v = []
            for p, (_, _, _, L, _) in enumerate(self.planes):
                wgt = self.W5 if L == 5 else self.W4
                mssim, mcs = o[f, p, :L, 0], o[f, p, :L, 1]
                v.append(float(np.prod(mcs[0:L - 1] ** wgt[0:L - 1]) * (mssim[L - 1] ** wgt[L - 1])))
            res.append((v[0], v[1], v[2], (6 * v[0] + v[1] + v[2]) / 8))
        return res


class MsSsimRGB:
    """pytorch_msssim.ms_ssim(x_hat, x, data_range=1) as DCVC-DC/test_video.py:188
    and DCVC-HEM/test_video.py:153 call it, on the GPU in fp64.  The package is
    not installed here, so this follows its published algorithm (5 levels,
    weights W5, Gaussian 11 / 1.5 'valid' statistics (dcvc_ssim_level), relu on
    cs and ssim, F.avg_pool2d(2, padding=size % 2) between levels
    (dcvc_avgpool2_f64), mean over the 3 channels); parity unpinned."""

    def __init__(self, h, w, frame_num, device):
        if min(h, w) <= 160:
            raise ValueError("ms_ssim needs the smaller side > (11 - 1) * 2**4")
        self.h, self.w = h, w
        n = 3 * h * w
        self.src = torch.empty(n, dtype=torch.float64, device=device)
        self.rec = torch.empty(n, dtype=torch.float64, device=device)
        x = np.arange(11, dtype=np.float64) - 5
        g = np.exp(-(x ** 2) / (2 * 1.5 ** 2))
        g /= g.sum()
        self.win = torch.from_numpy(np.outer(g, g)).to(device)
        self.ws = torch.empty(int(K.lib().dcvc_ssim_workspace()) // 8, dtype=torch.float64, device=device)
        self.out = torch.zeros((max(frame_num, 1), 3, 5, 2), dtype=torch.float64, device=device)
        self.bufs, sh, sw = [], h, w
        for _ in range(4):
            sh, sw = (sh + 2 * (sh % 2) - 2) // 2 + 1, (sw + 2 * (sw % 2) - 2) // 2 + 1
            self.bufs.append([torch.empty(sh * sw, dtype=torch.float64, device=device) for _ in range(6)] + [sh, sw])

    def run(self, x_hat, src_u8, slot):
        K.rgb_planes_f64(x_hat, src_u8, self.h, self.w, self.src, self.rec)
        n = self.h * self.w
        for c in range(3):
            a, b, sh, sw = self.src[c * n:(c + 1) * n], self.rec[c * n:(c + 1) * n], self.h, self.w
            for k in range(5):
                K.ssim_level(a, b, sh, sw, self.win, self.ws, self.out[slot, c, k])
                if k < 4:
                    bufs = self.bufs[k]
                    na, nb, nh, nw = bufs[2 * c], bufs[2 * c + 1], bufs[6], bufs[7]
                    K.avgpool2_f64(a, sh, sw, na)
                    K.avgpool2_f64(b, sh, sw, nb)
                    a, b, sh, sw = na, nb, nh, nw

    def values(self, n):
        o = self.out[:n].cpu().numpy()
        res = []
        for f in range(n):
            per = []
            for c in range(3):
                mcs = np.maximum(o[f, c, :4, 1], 0.0)
                ssim = max(o[f, c, 4, 0], 0.0)
                per.append(float(np.prod(np.append(mcs, ssim) ** MsSsim.W5)))
            res.append(float(np.mean(per)))
        return res


class ReconWriter:
    """--save_decoded_frame: PNGWriter (im00001.png, ...) and YUVWriter
    (out.yuv) of DCVC-DC/src/utils/video_writer.py:26-111 as test_video.py:
    84-88, 210-221 drives them, and DCVC-HEM's save_torch_image
    ({frame_idx}.png, DCVC-HEM/test_video.py:68-71, 161-163).

    The decoded frame is quantised on the GPU (dcvc_recon_to_u8: the crop,
    clip(rint(v * 255)), and for YUV the ycbcr444_to_420 chroma means), copied
    once to pinned memory, and written by one background thread in frame order
    so file encoding overlaps the next frame.  kind: "png" | "yuv" | "hem_png";
    src_format "rgb" | "420" (what the codec's frames hold, dist_in_yuv420).
    The reference's cross cases (a 4:2:0 frame into PNGWriter, an RGB frame into
    YUVWriter) convert on the host with its own formulas
    (functional.py:16-58)."""

    def __init__(self, path, h, w, kind, src_format, device):
        from concurrent.futures import ThreadPoolExecutor
        os.makedirs(path, exist_ok=True)
        self.path, self.h, self.w, self.kind, self.fmt = path, h, w, kind, src_format
        self.yuv_out = kind == "yuv"
        quant_yuv = src_format == "420"
        self.quant_yuv = quant_yuv
        self.n = h * w + 2 * (h // 2) * (w // 2) if quant_yuv else 3 * h * w
        self.dev_buf = torch.empty(self.n, dtype=torch.uint8, device=device)
        self.pool = ThreadPoolExecutor(1)
        self.jobs = []
        self.index = 1                              # PNGWriter.current_frame_index starts at 1
        self.file = open(os.path.join(path, "out.yuv"), "wb") if self.yuv_out else None

    def write(self, recon, frame_idx):
        from .dc.video_model import as_act
        x = as_act(recon)
        if (self.fmt == "rgb") == self.yuv_out:
            # the cross cases: the float frame to the host, the reference's conversion there
            f = x.t()[:self.h, :self.w].float().permute(2, 0, 1).cpu().numpy()
            if self.yuv_out:
                self.jobs.append(self.pool.submit(self._yuv_from_rgb, f))
            else:
                name = f"im{str(self.index).zfill(5)}.png"
                self.index += 1
                self.jobs.append(self.pool.submit(self._png_from_444, f, name))
            return
        K.recon_to_u8(x, self.h, self.w, self.quant_yuv, self.dev_buf)
        host = torch.empty(self.n, dtype=torch.uint8, pin_memory=True)
        host.copy_(self.dev_buf, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        name = (f"im{str(self.index).zfill(5)}.png" if self.kind == "png" else f"{frame_idx}.png")
        self.index += 1
        self.jobs.append(self.pool.submit(self._emit, host, ev, name))

    def _emit(self, host, ev, name):
        ev.synchronize()
        a = host.numpy()
        h, w = self.h, self.w
        if self.yuv_out:
            self.file.write(a.tobytes())            # Y plane then U, V planes (YUVWriter)
            return
        from PIL import Image
        Image.fromarray(a.reshape(h, w, 3)).save(os.path.join(self.path, name))

    def _png_from_444(self, yuv, name):
        # 4:2:0 frame into PNGWriter: ycbcr444_to_420 (y_rec, uv_rec as test_video.py:170-171 forms them),
        # then ycbcr420_to_rgb(order=1) and the PNG quantisation (functional.py:42-58, video_writer.py:34-45)
        import scipy.ndimage
        from PIL import Image
        h, w = self.h, self.w
        y = np.clip(yuv[0:1], 0.0, 1.0)
        u = np.mean(np.reshape(yuv[1:2], (1, h // 2, 2, w // 2, 2)), axis=(-1, -3))
        v = np.mean(np.reshape(yuv[2:3], (1, h // 2, 2, w // 2, 2)), axis=(-1, -3))
        uv = scipy.ndimage.zoom(np.clip(np.concatenate((u, v), axis=0), 0.0, 1.0), (1, 2, 2), order=1)
        kr, kg, kb = 0.2126, 0.7152, 0.0722
        r = y + (2 - 2 * kr) * (uv[1:2] - 0.5)
        b = y + (2 - 2 * kb) * (uv[0:1] - 0.5)
        g = (y - kr * r - kb * b) / kg
        rgb = np.clip(np.concatenate((r, g, b), 0), 0.0, 1.0).transpose(1, 2, 0)
        Image.fromarray(np.clip(np.rint(rgb * 255), 0, 255).astype(np.uint8)).save(os.path.join(self.path, name))

    def _yuv_from_rgb(self, rgb):
        r, g, b = np.split(rgb, 3, axis=0)
        kr, kg, kb = 0.2126, 0.7152, 0.0722
        y = kr * r + kg * g + kb * b
        cb = 0.5 * (b - y) / (1 - kb) + 0.5
        cr = 0.5 * (r - y) / (1 - kr) + 0.5
        h, w = self.h, self.w
        cb = np.mean(np.reshape(cb, (1, h // 2, 2, w // 2, 2)), axis=(-1, -3))
        cr = np.mean(np.reshape(cr, (1, h // 2, 2, w // 2, 2)), axis=(-1, -3))
        uv = np.clip(np.concatenate((cb, cr), axis=0), 0.0, 1.0)
        y = np.clip(y, 0.0, 1.0)
        self.file.write(np.clip(np.rint(y * 255), 0, 255).astype(np.uint8).tobytes())
        self.file.write(np.clip(np.rint(uv * 255), 0, 255).astype(np.uint8).tobytes())

    def close(self):
        """Drain the writer thread and close out.yuv (idempotent)."""
        try:
            for j in self.jobs:
                j.result()
        finally:
            self.jobs = []
            self.pool.shutdown()
            if self.file is not None:
                self.file.close()
                self.file = None

    # run_test holds the writer in a `with`: on an exception mid-sequence the
    # queued frames are still written and the file closed
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def psnr_rgb(sse3, h, w):
    """PSNR() of test_video.py:65-68: mse = mean((x_hat - x)^2) as an fp32
    tensor, psnr = 20 * log10(1 / sqrt(mse)) in fp32."""
    mse = torch.tensor(float(np.sum(sse3)) / (3.0 * h * w), dtype=torch.float32)
    return (20 * torch.log10(1 / torch.sqrt(mse))).item()


def calc_psnr_from_sse(sse, n, data_range=1.0):
    """calc_psnr (src/utils/metrics.py:81-92) from an fp64 squared-error sum."""
    mse = sse / n
    if mse > 1e-10:
        return 10 * np.log10(data_range * data_range / mse)
    return 999.9


def psnr_yuv(sse3, h, w):
    """(psnr_y, psnr_u, psnr_v, (6 y + u + v) / 8), test_video.py:177-181."""
    py = calc_psnr_from_sse(sse3[0], h * w)
    pu = calc_psnr_from_sse(sse3[1], (h // 2) * (w // 2))
    pv = calc_psnr_from_sse(sse3[2], (h // 2) * (w // 2))
    return py, pu, pv, (6 * py + pu + pv) / 8


# ---------------------------------------------------------------- run_test
def generate_log_json(frame_num, frame_pixel_num, test_time, frame_types, bits, psnrs, ssims,
                      psnrs_y=None, psnrs_u=None, psnrs_v=None, ssims_y=None, ssims_u=None, ssims_v=None,
                      verbose=False):
    """DCVC-DC/src/utils/common.py:44-140 (same keys and averages)."""
    yuv = psnrs_y is not None
    acc = {k: {"bits": 0, "psnr": 0, "ssim": 0, "y": 0, "u": 0, "v": 0, "sy": 0, "su": 0, "sv": 0, "n": 0}
           for k in (0, 1)}
    for i in range(frame_num):
        a = acc[0 if frame_types[i] == 0 else 1]
        a["bits"] += bits[i]
        a["psnr"] += psnrs[i]
        a["ssim"] += ssims[i]
        a["n"] += 1
        if yuv:
            for key, src in (("y", psnrs_y), ("u", psnrs_u), ("v", psnrs_v),
                             ("sy", ssims_y), ("su", ssims_u), ("sv", ssims_v)):
                a[key] += src[i]
    ai, ap = acc[0], acc[1]
    log = {"frame_pixel_num": frame_pixel_num, "i_frame_num": ai["n"], "p_frame_num": ap["n"],
           "ave_i_frame_bpp": ai["bits"] / ai["n"] / frame_pixel_num,
           "ave_i_frame_psnr": ai["psnr"] / ai["n"], "ave_i_frame_msssim": ai["ssim"] / ai["n"]}
    if yuv:
        for c in "yuv":
            log[f"ave_i_frame_psnr_{c}"] = ai[c] / ai["n"]
        for c in "yuv":
            log[f"ave_i_frame_msssim_{c}"] = ai["s" + c] / ai["n"]
    if verbose:
        log["frame_bpp"] = list(np.array(bits) / frame_pixel_num)
        log["frame_psnr"] = psnrs
        log["frame_msssim"] = ssims
        log["frame_type"] = frame_types
        if yuv:
            log.update(frame_psnr_y=psnrs_y, frame_psnr_u=psnrs_u, frame_psnr_v=psnrs_v,
                       frame_msssim_y=ssims_y, frame_msssim_u=ssims_u, frame_msssim_v=ssims_v)
    log["test_time"] = test_time
    if ap["n"] > 0:
        log["ave_p_frame_bpp"] = ap["bits"] / (ap["n"] * frame_pixel_num)
        log["ave_p_frame_psnr"] = ap["psnr"] / ap["n"]
        log["ave_p_frame_msssim"] = ap["ssim"] / ap["n"]
        if yuv:
            for c in "yuv":
                log[f"ave_p_frame_psnr_{c}"] = ap[c] / ap["n"]
            for c in "yuv":
                log[f"ave_p_frame_msssim_{c}"] = ap["s" + c] / ap["n"]
    else:
        log["ave_p_frame_bpp"] = 0
        log["ave_p_frame_psnr"] = 0
        log["ave_p_frame_msssim"] = 0
        if yuv:
            for c in "yuv":
                log[f"ave_p_frame_psnr_{c}"] = 0
            for c in "yuv":
                log[f"ave_p_frame_msssim_{c}"] = 0
    log["ave_all_frame_bpp"] = (ai["bits"] + ap["bits"]) / (frame_num * frame_pixel_num)
    log["ave_all_frame_psnr"] = (ai["psnr"] + ap["psnr"]) / frame_num
    log["ave_all_frame_msssim"] = (ai["ssim"] + ap["ssim"]) / frame_num
    if yuv:
        for c in "yuv":
            log[f"ave_all_frame_psnr_{c}"] = (ai[c] + ap[c]) / frame_num
        for c in "yuv":
            log[f"ave_all_frame_msssim_{c}"] = (ai["s" + c] + ap["s" + c]) / frame_num
    return log


def _reader(args, yuv):
    if "src_reader" in args:
        return args["src_reader"]
    if args["src_type"] == "yuv420":
        return YUVReader(args["src_path"], args["src_width"], args["src_height"])
    if args["src_type"] == "png":
        return PNGReader(args.get("src_path", args.get("img_path")), args["src_width"], args["src_height"])
    raise ValueError(f"unknown src_type {args['src_type']!r}")


def run_test(p_frame_net, i_frame_net, args):
    """DCVC-DC/test_video.py:71-237 on the GPU codecs.  ``args`` takes the
    reference's keys (frame_num, gop_size, write_stream, bin_folder,
    src_type 'png' | 'yuv420', src_path, src_width, src_height,
    dist_in_yuv420, q_in_ckpt, i_frame_q_index, verbose, calc_ssim) plus an
    optional ``src_reader`` (an ArrayReader) in place of a file source.
    YUV420 sources are coded as YCbCr 4:4:4 (``dist_in_yuv420``), as the
    reference's yuv420 checkpoints expect."""
    frame_num, gop_size = args["frame_num"], args["gop_size"]
    write_stream = bool(args.get("write_stream", False))
    verbose = args.get("verbose", 0)
    yuv = bool(args.get("dist_in_yuv420", False))
    if yuv and args.get("src_type", "yuv420") != "yuv420" and "src_reader" not in args:
        raise ValueError("dist_in_yuv420 needs a yuv420 source")
    device = i_frame_net.dev
    reader = _reader(args, yuv)
    h, w = args["src_height"], args["src_width"]
    stage = FrameStage(h, w, 16, yuv, zero_pad=False, frame_num=frame_num, device=device)
    writer = None
    if args.get("save_decoded_frame"):   # test_video.py:84-88
        writer = ReconWriter(args["recon_path"], h, w, "png" if args.get("src_type", "yuv420") == "png" else "yuv",
                             "420" if yuv else "rgb", device)
    ms = None
    if args.get("calc_ssim"):
        ms = MsSsim(h, w, frame_num, device) if yuv else MsSsimRGB(h, w, frame_num, device)
    frame_types, bits = [], []
    start_time = time.time()
    p_frame_number = 0
    enc_t = dec_t = 0.0
    dpb = None
    with torch.no_grad(), (writer if writer is not None else contextlib.nullcontext()):
        for frame_idx in range(frame_num):
            frame = reader.read_one_frame(dst_format="420" if yuv else "rgb")
            if frame is None or (yuv and frame[0] is None):
                raise ValueError(f"source ended at frame {frame_idx} of {frame_num}")
            dframe = stage.upload(frame)
            x = stage.load(dframe)
            bin_path = os.path.join(args["bin_folder"], f"{frame_idx}.bin") if write_stream else None
            if frame_idx % gop_size == 0:
                result = i_frame_net.encode_decode(x, args["q_in_ckpt"], args["i_frame_q_index"], bin_path,
                                                   pic_height=h, pic_width=w)
                dpb = {"ref_frame": result["x_hat"], "ref_feature": None, "ref_mv_feature": None,
                       "ref_y": None, "ref_mv_y": None}
                recon = result["x_hat"]
                frame_types.append(0)
            else:
                # test_video.py:152-155 passes i_frame_q_index to the P codec too
                result = p_frame_net.encode_decode(x, dpb, args["q_in_ckpt"], args["i_frame_q_index"], bin_path,
                                                   pic_height=h, pic_width=w, frame_idx=frame_idx % 4)
                dpb = result["dpb"]
                recon = dpb["ref_frame"]
                frame_types.append(1)
                p_frame_number += 1
                enc_t += result["encoding_time"]
                dec_t += result["decoding_time"]
            bits.append(result["bit"])
            stage.distortion(recon, dframe, frame_idx)
            if ms is not None:
                from .dc.video_model import as_act
                if yuv:
                    ms.run(as_act(recon), dframe[0], dframe[1], frame_idx)
                else:
                    ms.run(as_act(recon), dframe, frame_idx)
            if writer is not None:
                writer.write(recon, frame_idx)
            if verbose >= 2:
                print(f"frame {frame_idx}, bits: {bits[-1]:.3f}", flush=True)
    sse = stage.sums()
    test_time = time.time() - start_time
    if verbose >= 1 and p_frame_number > 0:
        print(f"encoding/decoding {p_frame_number} P frames, "
              f"average encoding time {enc_t / p_frame_number * 1000:.0f} ms, "
              f"average decoding time {dec_t / p_frame_number * 1000:.0f} ms.")
    zeros = [0.0] * frame_num
    if yuv:
        per = [psnr_yuv(sse[i], h, w) for i in range(frame_num)]
        mv = ms.values(frame_num) if ms is not None else [(0.0, 0.0, 0.0, 0.0)] * frame_num
        log = generate_log_json(frame_num, h * w, test_time, frame_types, bits, [p[3] for p in per],
                                [m[3] for m in mv], [p[0] for p in per], [p[1] for p in per], [p[2] for p in per],
                                [m[0] for m in mv], [m[1] for m in mv], [m[2] for m in mv], verbose=verbose >= 1)
    else:
        psnrs = [psnr_rgb(sse[i], h, w) for i in range(frame_num)]
        mv = ms.values(frame_num) if ms is not None else zeros
        log = generate_log_json(frame_num, h * w, test_time, frame_types, bits, psnrs, mv,
                                verbose=verbose >= 1)
    if args.get("calc_ssim") and not yuv:
        log["msssim_unpinned"] = True   # pytorch_msssim's algorithm, package absent (MsSsimRGB)
    if writer is not None:
        # test_video.py:217-221: the recon folder is renamed after the rate point's averages
        avg_bpp = sum(bits) / len(bits) / w / h
        avg_psnr = log["ave_all_frame_psnr"]
        folder = f"{args.get('rate_idx', 0)}_{avg_bpp:.4f}_{avg_psnr:.4f}"
        os.rename(args["recon_path"], args["recon_path"] + f"/../{folder}")
    return log


def generate_log_json_hem(frame_num, frame_types, bits, psnrs, ssims, frame_pixel_num, test_time):
    """DCVC-HEM/src/utils/common.py:63-104."""
    log = generate_log_json(frame_num, frame_pixel_num, test_time, frame_types, bits, psnrs, ssims, verbose=True)
    keep = ("frame_pixel_num", "i_frame_num", "p_frame_num", "ave_i_frame_bpp", "ave_i_frame_psnr",
            "ave_i_frame_msssim", "frame_bpp", "frame_psnr", "frame_msssim", "frame_type", "test_time",
            "ave_p_frame_bpp", "ave_p_frame_psnr", "ave_p_frame_msssim", "ave_all_frame_bpp",
            "ave_all_frame_psnr", "ave_all_frame_msssim")
    return {k: log[k] for k in keep if k in log}


def run_test_hem(video_net, i_frame_net, args, device=None):
    """DCVC-HEM/test_video.py:80-172: PNG (or in-memory) RGB source, zero
    padding to a multiple of 64, q scales from ``args`` (i_frame_q_scale,
    p_frame_mv_y_q_scale, p_frame_y_q_scale)."""
    frame_num, gop_size = args["frame_num"], args["gop_size"]
    write_stream = bool(args.get("write_stream", False))
    device = device if device is not None else i_frame_net.dev
    reader = _reader({**args, "src_type": args.get("src_type", "png")}, False)
    h, w = args["src_height"], args["src_width"]
    stage = FrameStage(h, w, 64, False, zero_pad=True, frame_num=frame_num, device=device)
    ms = MsSsimRGB(h, w, frame_num, device) if min(h, w) > 160 else None  # HEM always reports ms_ssim (:150)
    writer = None
    if args.get("save_decoded_frame"):   # DCVC-HEM/test_video.py:161-163, 204-209
        writer = ReconWriter(args["decoded_frame_folder"], h, w, "hem_png", "rgb", device)
    frame_types, bits = [], []
    start_time = time.time()
    dpb = None
    with torch.no_grad(), (writer if writer is not None else contextlib.nullcontext()):
        for frame_idx in range(frame_num):
            frame = reader.read_one_frame(dst_format="rgb")
            if frame is None:
                raise ValueError(f"source ended at frame {frame_idx} of {frame_num}")
            dframe = stage.upload(frame)
            x = stage.load(dframe)
            bin_path = os.path.join(args["bin_folder"], f"{frame_idx}.bin") if write_stream else None
            if frame_idx % gop_size == 0:
                result = i_frame_net.encode_decode(x, args["i_frame_q_scale"], bin_path, pic_height=h, pic_width=w)
                dpb = {"ref_frame": result["x_hat"], "ref_feature": None, "ref_y": None, "ref_mv_y": None}
                recon = result["x_hat"]
                frame_types.append(0)
            else:
                result = video_net.encode_decode(x, dpb, bin_path, pic_height=h, pic_width=w,
                                                 mv_y_q_scale=args["p_frame_mv_y_q_scale"],
                                                 y_q_scale=args["p_frame_y_q_scale"])
                dpb = result["dpb"]
                recon = dpb["ref_frame"]
                frame_types.append(1)
            bits.append(result["bit"])
            stage.distortion(recon, dframe, frame_idx)
            if ms is not None:
                from .dc.video_model import as_act
                ms.run(as_act(recon), dframe, frame_idx)
            if writer is not None:
                writer.write(recon, frame_idx)
    sse = stage.sums()
    psnrs = [psnr_rgb(sse[i], h, w) for i in range(frame_num)]
    mv = ms.values(frame_num) if ms is not None else [0.0] * frame_num
    log = generate_log_json_hem(frame_num, frame_types, bits, psnrs, mv, h * w, time.time() - start_time)
    log["msssim_unpinned"] = True   # pytorch_msssim's algorithm, package absent (MsSsimRGB)
    return log
