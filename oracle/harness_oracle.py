"""run_test frame handling, CPU restatement — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module, as the checker.  The product path never imports it.

numpy restatement of what DCVC-DC/test_video.py:108-195 does to a frame
around the codec (paths relative to /root/reference/DCVC-DC):

* ``ycbcr420_to_444`` with order=0 (src/transforms/functional.py:61-72):
  ``scipy.ndimage.zoom(uv, (1, 2, 2), order=0)``, restated as the index map
  ``round(i * (n - 1) / (2n - 1))``; tests pin the map against scipy itself.
* ``np_image_to_tensor`` + ``F.pad(replicate)`` (test_video.py:56-62, 128-132).
* ``ycbcr444_to_420`` (functional.py:75-95): float32 2x2 means, clip.
* ``calc_psnr`` (src/utils/metrics.py:81-92) and ``PSNR`` (test_video.py:65-68).
"""
import numpy as np
import torch


def zoom_index(n_out, n_in):
    """Nearest-neighbour source index of scipy.ndimage.zoom (order=0,
    grid_mode=False) along one axis."""
    if n_in <= 1:
        return np.zeros(n_out, dtype=np.int64)
    z = (n_in - 1) / (n_out - 1)
    return np.floor(np.arange(n_out, dtype=np.float64) * z + 0.5).astype(np.int64)


def ycbcr420_to_444_nearest(y, uv):
    """y (1, h, w) float32, uv (2, h/2, w/2) float32 -> (3, h, w) float32."""
    _, h, w = y.shape
    ri = zoom_index(h, uv.shape[1])
    ci = zoom_index(w, uv.shape[2])
    up = uv[:, ri][:, :, ci]
    return np.concatenate((y, up), axis=0)


def yuv_u8_to_input(y_u8, uv_u8, H, W):
    """uint8 planes -> (H, W, 3) float32 NHWC codec input, replicate-padded."""
    y = y_u8.astype(np.float32)[None] / 255
    uv = uv_u8.astype(np.float32) / 255
    yuv = ycbcr420_to_444_nearest(y, uv)
    h, w = yuv.shape[1:]
    yuv = np.pad(yuv, ((0, 0), (0, H - h), (0, W - w)), mode="edge")
    return np.ascontiguousarray(yuv.transpose(1, 2, 0))


def ycbcr444_to_420(yuv):
    """functional.py:75-95 (float32 in, float32 out)."""
    c, h, w = yuv.shape
    y, u, v = np.split(yuv, 3, axis=0)
    u = np.mean(np.reshape(u, (1, h // 2, 2, w // 2, 2)), axis=(-1, -3))
    v = np.mean(np.reshape(v, (1, h // 2, 2, w // 2, 2)), axis=(-1, -3))
    uv = np.concatenate((u, v), axis=0)
    return np.clip(y, 0., 1.), np.clip(uv, 0., 1.)


def png_writer_u8(rgb):
    """PNGWriter.write_one_frame / HEM save_torch_image (video_writer.py:34-45,
    DCVC-HEM/test_video.py:68-71): 3 x h x w float32 -> h x w x 3 uint8."""
    return np.clip(np.rint(rgb.transpose(1, 2, 0) * 255), 0, 255).astype(np.uint8)


def yuv_writer_bytes(y, uv):
    """YUVWriter.write_one_frame with src_format '420' (video_writer.py:100-108)."""
    y = np.clip(np.rint(y * 255), 0, 255).astype(np.uint8)
    uv = np.clip(np.rint(uv * 255), 0, 255).astype(np.uint8)
    return y.tobytes() + uv.tobytes()


def calc_psnr(img1, img2, data_range=255):
    """metrics.py:81-92."""
    img1 = img1.astype(np.float64)
    img2 = img2.astype(np.float64)
    mse = np.mean(np.square(img1 - img2))
    if mse > 1e-10:
        return 10 * np.log10(data_range * data_range / mse)
    return 999.9


def psnr_torch(a, b):
    """test_video.py:65-68 on fp32 torch tensors."""
    mse = torch.mean((a - b) ** 2)
    return (20 * torch.log10(1 / torch.sqrt(mse))).item()


def yuv_distortion(x_hat_chw, y_u8, uv_u8):
    """(psnr_y, psnr_u, psnr_v, psnr) of a cropped, clamped 444 recon."""
    y = y_u8.astype(np.float32) / 255
    uv = uv_u8.astype(np.float32) / 255
    y_rec, uv_rec = ycbcr444_to_420(x_hat_chw)
    py = calc_psnr(y, y_rec[0], data_range=1)
    pu = calc_psnr(uv[0], uv_rec[0], data_range=1)
    pv = calc_psnr(uv[1], uv_rec[1], data_range=1)
    return py, pu, pv, (6 * py + pu + pv) / 8


def yuv_sse(x_hat_chw, y_u8, uv_u8):
    """Per-plane fp64 squared-error sums behind yuv_distortion."""
    y = y_u8.astype(np.float32) / 255
    uv = uv_u8.astype(np.float32) / 255
    y_rec, uv_rec = ycbcr444_to_420(x_hat_chw)
    d = [y_rec[0].astype(np.float64) - y, uv_rec[0].astype(np.float64) - uv[0],
         uv_rec[1].astype(np.float64) - uv[1]]
    return np.array([np.sum(np.square(e)) for e in d])



# --------------------------------------------------------------- MS-SSIM
def fspecial_gauss(size=11, sigma=1.5):
    """metrics.py:9-12."""
    x, y = np.mgrid[-size // 2 + 1:size // 2 + 1, -size // 2 + 1:size // 2 + 1]
    g = np.exp(-((x ** 2 + y ** 2) / (2.0 * sigma ** 2)))
    return g / g.sum()


def _filter_valid(win, img):
    """fftconvolve(window, img, 'valid') restated as the direct 'valid'
    correlation with the flipped window (same linear map)."""
    k = win[::-1, ::-1]
    h, w = img.shape
    out = np.zeros((h - 10, w - 10))
    for ky in range(11):
        for kx in range(11):
            out += k[ky, kx] * img[ky:ky + h - 10, kx:kx + w - 10]
    return out


def calc_ssim(img1, img2, data_range=1.0):
    """metrics.py:15-36 (means of the ssim and cs maps)."""
    img1 = img1.astype(np.float64)
    img2 = img2.astype(np.float64)
    win = fspecial_gauss(11, 1.5)
    C1, C2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    mu1, mu2 = _filter_valid(win, img1), _filter_valid(win, img2)
    m1s, m2s, m12 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    s1 = _filter_valid(win, img1 * img1) - m1s
    s2 = _filter_valid(win, img2 * img2) - m2s
    s12 = _filter_valid(win, img1 * img2) - m12
    ssim = ((2 * m12 + C1) * (2 * s12 + C2)) / ((m1s + m2s + C1) * (s1 + s2 + C2))
    cs = (2.0 * s12 + C2) / (s1 + s2 + C2)
    return ssim.mean(), cs.mean()


def down2_reflect(im):
    """ndimage.convolve(im, ones((2,2))/4, mode='reflect')[::2, ::2]
    (metrics.py:54-59): 2x2 means, the row/column past an odd edge reflecting
    to the edge."""
    h, w = im.shape
    p = np.pad(im, ((0, h % 2), (0, w % 2)), mode="edge")
    return ((p[0::2, 0::2] + p[0::2, 1::2]) + p[1::2, 0::2] + p[1::2, 1::2]) * 0.25


def calc_msssim(img1, img2, data_range=1.0):
    """metrics.py:39-62."""
    level, weight = 5, np.array([0.0448, 0.2856, 0.3001, 0.2363, 0.1333])
    h, w = img1.shape
    if h < 176 or w < 176:
        level, weight = 4, np.array([0.0517, 0.3295, 0.3462, 0.2726])
    assert h >= 88 and w >= 88
    im1, im2 = img1.astype(np.float64), img2.astype(np.float64)
    mssim, mcs = [], []
    for _ in range(level):
        s, c = calc_ssim(im1, im2, data_range)
        mssim.append(s)
        mcs.append(c)
        im1, im2 = down2_reflect(im1), down2_reflect(im2)
    mssim, mcs = np.array(mssim), np.array(mcs)
    return np.prod(mcs[0:level - 1] ** weight[0:level - 1]) * (mssim[level - 1] ** weight[level - 1])


def ms_ssim_torch(X, Y, data_range=1.0):
    """pytorch_msssim.ms_ssim (size_average=True, win 11 / 1.5, K (0.01, 0.03),
    default weights) restated from its published algorithm in fp32 torch —
    the package is not installed, so this restatement is parity unpinned.
    X, Y: (N, C, H, W) float tensors."""
    import torch.nn.functional as F
    coords = torch.arange(11, dtype=torch.float) - 5
    g = torch.exp(-(coords ** 2) / (2 * 1.5 ** 2))
    g = (g / g.sum()).reshape(1, 1, 1, 11)
    C = X.shape[1]
    wh, wv = g.repeat(C, 1, 1, 1), g.transpose(2, 3).repeat(C, 1, 1, 1)

    def filt(x):
        return F.conv2d(F.conv2d(x, wv, groups=C), wh, groups=C)

    def ssim(x, y):
        C1, C2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
        mu1, mu2 = filt(x), filt(y)
        m1s, m2s, m12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
        s1, s2, s12 = filt(x * x) - m1s, filt(y * y) - m2s, filt(x * y) - m12
        cs_map = (2 * s12 + C2) / (s1 + s2 + C2)
        ssim_map = ((2 * m12 + C1) / (m1s + m2s + C1)) * cs_map
        return torch.flatten(ssim_map, 2).mean(-1), torch.flatten(cs_map, 2).mean(-1)

    weights = torch.tensor([0.0448, 0.2856, 0.3001, 0.2363, 0.1333])
    mcs = []
    for i in range(5):
        s, cs = ssim(X, Y)
        if i < 4:
            mcs.append(torch.relu(cs))
            pad = [d % 2 for d in X.shape[2:]]
            X = F.avg_pool2d(X, kernel_size=2, padding=pad)
            Y = F.avg_pool2d(Y, kernel_size=2, padding=pad)
    s = torch.relu(s)
    v = torch.prod(torch.stack(mcs + [s], dim=0) ** weights.view(-1, 1, 1), dim=0)
    return v.mean().item()
