"""Access to the committed DCVC-DC golden fixtures (tests/golden/, made by
tests/golden/make_golden_dc.py from the reference) and oracle drivers that
replay the reference harness (DCVC-DC/test_video.py:108-167) on them."""
import hashlib
import json
import os

import numpy as np
import torch

from dcvc_amd.weights import synthetic_state_dict
from dcvc_amd.synth import to_float

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def digest(t):
    a = t.detach().float().cpu().contiguous().numpy()
    return hashlib.sha256(a.tobytes()).hexdigest()


class DCGolden:
    def __init__(self):
        with open(os.path.join(os.path.dirname(GOLDEN), "..", "dcvc_amd", "data", "dc_param_spec.json")) as f:
            spec = json.load(f)
        self.i_spec = [(n, tuple(s)) for n, s in spec["intra"]]
        self.p_spec = [(n, tuple(s)) for n, s in spec["inter"]]
        with open(os.path.join(GOLDEN, "dc_golden.json")) as f:
            self.meta = json.load(f)
        self.npz = np.load(os.path.join(GOLDEN, "dc_golden.npz"))

    def i_state_dict(self):
        return synthetic_state_dict(self.i_spec, seed=0)

    def p_state_dict(self):
        return synthetic_state_dict(self.p_spec, seed=1)

    def table(self, name):
        z = self.npz
        return z[f"table_{name}_cdf"], z[f"table_{name}_len"], z[f"table_{name}_off"]

    def frame(self, tag, t):
        return self.npz[f"{tag}_frame{t}"]

    def frame_tensor(self, tag, t):
        """Padded float frame as the harness builds it (replicate to x16)."""
        u8 = self.frame(tag, t)
        x = torch.from_numpy(to_float(u8)).unsqueeze(0)
        h, w = u8.shape[1:]
        xp = torch.nn.functional.pad(x, (0, (16 - w % 16) % 16, 0, (16 - h % 16) % 16), mode="replicate")
        return x, xp

    def calls(self, tag, t):
        e = self.meta[tag]["write"][t]
        return [(name, self.npz[f"{tag}_w{t}_c{j}_sym"], self.npz[f"{tag}_w{t}_c{j}_idx"])
                for j, name in enumerate(e["calls"])]
