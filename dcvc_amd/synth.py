"""Synthetic frames (no datasets offline).

``moving_pattern`` is the throughput input of SURVEY §8d: a smooth sum of
sinusoids translating 2 px/frame plus noise, so motion estimation and the
warps see coherent motion.  Frames are produced as uint8 (what a PNG source
hands over), so the same (seed, t) gives the same bytes on every host.
"""
import numpy as np


def moving_pattern(h, w, t, seed=1, speed=2):
    g = np.random.Generator(np.random.PCG64([seed, 7]))
    fx = g.uniform(2.0, 9.0, size=(3, 4))
    fy = g.uniform(2.0, 9.0, size=(3, 4))
    ph = g.uniform(0, 2 * np.pi, size=(3, 4))
    yy = np.arange(h, dtype=np.float64)[:, None] / h
    xx = (np.arange(w, dtype=np.float64)[None, :] + speed * t) / w
    img = np.empty((3, h, w), dtype=np.float64)
    for c in range(3):
        acc = np.zeros((h, w))
        for k in range(4):
            acc += np.sin(2 * np.pi * (fx[c, k] * xx + fy[c, k] * yy) + ph[c, k])
        img[c] = 0.5 + 0.12 * acc
    noise = np.random.Generator(np.random.PCG64([seed, 1000 + t])).normal(0, 0.02, size=img.shape)
    return np.clip(np.round((img + noise) * 255.0), 0, 255).astype(np.uint8)


def uniform_frame(h, w, t, seed=1):
    """Uniform random RGB frame (the parity input of SURVEY §8d)."""
    g = np.random.Generator(np.random.PCG64([seed, 2000 + t]))
    return g.integers(0, 256, size=(3, h, w), dtype=np.uint8)


def to_float(frame_u8):
    """uint8 CHW -> float32 [0, 1], as PNGReader does (x / 255)."""
    return frame_u8.astype(np.float32) / np.float32(255.0)


def moving_pattern_yuv420(h, w, t, seed=1, speed=2):
    """The moving pattern as an 8-bit YUV420 source (config C4): BT.709
    rgb_to_ycbcr420 (DCVC-DC/src/transforms/functional.py:16-39) rounded to
    uint8, i.e. what a .yuv file of the sequence holds.  Returns (y (h, w),
    uv (2, h/2, w/2))."""
    rgb = moving_pattern(h, w, t, seed=seed, speed=speed).astype(np.float32) / 255
    r, g, b = rgb[0:1], rgb[1:2], rgb[2:3]
    kr, kg, kb = 0.2126, 0.7152, 0.0722
    y = kr * r + kg * g + kb * b
    cb = 0.5 * (b - y) / (1 - kb) + 0.5
    cr = 0.5 * (r - y) / (1 - kr) + 0.5
    cb = np.mean(np.reshape(cb, (1, h // 2, 2, w // 2, 2)), axis=(-1, -3))
    cr = np.mean(np.reshape(cr, (1, h // 2, 2, w // 2, 2)), axis=(-1, -3))
    uv = np.clip(np.concatenate((cb, cr), axis=0), 0, 1)
    y = np.clip(y, 0, 1)
    return np.round(y[0] * 255).astype(np.uint8), np.round(uv * 255).astype(np.uint8)
