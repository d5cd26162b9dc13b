"""Deterministic synthetic weights in the reference's state_dict format.

Pretrained checkpoints are unavailable offline, so every test, fixture and
benchmark uses weights generated here from (parameter name, shape) and a seed.
Each tensor has its own PCG64 stream seeded by (seed, crc32(name)), so the
values do not depend on construction order, device or library version.

Distributions follow the reference's defaults: conv weights/biases uniform in
±gain/sqrt(fan_in) (PyTorch's Conv2d init), Bitparm h/b/a ~ N(0, 0.01)
(DCVC-DC/src/models/entropy_models.py:60-69), q_basic = 1; q_scale anchors
are a decreasing ladder so the 64-entry fine q tables are non-trivial.
"""
import json
import zlib

import numpy as np
import torch

Q_SCALE_ANCHORS = {
    "enc": (1.6, 1.2, 0.9, 0.65),
    "dec": (1.3, 1.1, 0.95, 0.8),
}


def _rng(seed, name):
    return np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(name.encode())]))


def synth_tensor(name, shape, seed=0, gain=1.0):
    g = _rng(seed, name)
    shape = tuple(int(s) for s in shape)
    leaf = name.rsplit(".", 1)[-1]
    if "q_scale" in name:
        anchors = Q_SCALE_ANCHORS["enc" if name.endswith("enc") else "dec"]
        v = np.array(anchors[: shape[0]], dtype=np.float32).reshape(shape)
    elif "q_basic" in name:
        v = np.ones(shape, dtype=np.float32)
    elif ".f" in name and leaf in ("h", "b", "a") and "bit_estimator" in name:
        v = g.normal(0.0, 0.01, size=shape).astype(np.float32)
    elif leaf == "weight" and len(shape) == 4:
        fan_in = shape[1] * shape[2] * shape[3]
        b = gain / np.sqrt(fan_in)
        v = g.uniform(-b, b, size=shape).astype(np.float32)
    elif leaf == "bias":
        # bias bound uses the owning conv's fan_in; recover it from the name's
        # weight shape when given via `fan_in_hint`, else 1/sqrt(shape[0])
        b = 1.0 / np.sqrt(max(1, shape[0]))
        v = g.uniform(-b, b, size=shape).astype(np.float32)
    else:
        v = g.normal(0.0, 0.02, size=shape).astype(np.float32)
    return torch.from_numpy(v)


def synthetic_state_dict(spec, seed=0, gain=1.0):
    """spec: iterable of (name, shape).  Biases use 1/sqrt(fan_in) of their
    conv weight when the weight is in the spec."""
    spec = [(n, tuple(s)) for n, s in spec]
    shapes = dict(spec)
    sd = {}
    for name, shape in spec:
        t = synth_tensor(name, shape, seed, gain)
        if name.endswith(".bias"):
            w = shapes.get(name[: -len("bias")] + "weight")
            if w is not None and len(w) == 4:
                fan_in = w[1] * w[2] * w[3]
                b = 1.0 / np.sqrt(fan_in)
                g = _rng(seed, name)
                t = torch.from_numpy(g.uniform(-b, b, size=shape).astype(np.float32))
        sd[name] = t
    return sd


def load_spec(path):
    with open(path) as f:
        d = json.load(f)
    return [(n, tuple(s)) for n, s in d]
