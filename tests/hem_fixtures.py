"""Access to the committed DCVC-HEM golden fixtures (tests/golden/, made by
tests/golden/make_golden_hem.py from the reference)."""
import json
import os

import numpy as np
import torch

from dcvc_amd.weights import synthetic_state_dict
from dcvc_amd.synth import to_float

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
HEM_GAIN = 1.6  # make_golden_hem.py


class HEMGolden:
    def __init__(self):
        with open(os.path.join(os.path.dirname(GOLDEN), "..", "dcvc_amd", "data", "hem_param_spec.json")) as f:
            spec = json.load(f)
        self.i_spec = [(n, tuple(s)) for n, s in spec["intra"]]
        self.p_spec = [(n, tuple(s)) for n, s in spec["inter"]]
        with open(os.path.join(GOLDEN, "hem_golden.json")) as f:
            self.meta = json.load(f)
        self.npz = np.load(os.path.join(GOLDEN, "hem_golden.npz"))

    def i_state_dict(self):
        return synthetic_state_dict(self.i_spec, seed=10, gain=HEM_GAIN)

    def p_state_dict(self):
        return synthetic_state_dict(self.p_spec, seed=11, gain=HEM_GAIN)

    def table(self, name):
        z = self.npz
        return z[f"table_{name}_cdf"], z[f"table_{name}_len"], z[f"table_{name}_off"]

    def frame_tensor(self, tag, t):
        """Frame padded with zeros to a multiple of 64 (HEM test_video.py:113-119).
        Config C1's frames are torch.rand draws (make_golden_hem.py), rebuilt here."""
        if "frame_sha256" in self.meta[tag]:
            g = torch.Generator().manual_seed(1)
            x = [torch.rand(1, 3, self.meta[tag]["h"], self.meta[tag]["w"], generator=g) for _ in range(t + 1)][t]
        else:
            x = torch.from_numpy(to_float(self.npz[f"{tag}_frame{t}"])).unsqueeze(0)
        h, w = x.shape[2:]
        xp = torch.nn.functional.pad(x, (0, (64 - w % 64) % 64, 0, (64 - h % 64) % 64), mode="constant", value=0)
        return x, xp

    def write_frames(self, tag):
        return len(self.meta[tag]["write"])

    def calls(self, tag, t):
        e = self.meta[tag]["write"][t]
        return [(name, self.npz[f"{tag}_w{t}_c{j}_sym"], self.npz[f"{tag}_w{t}_c{j}_idx"])
                for j, name in enumerate(e["calls"])]

    def q(self, tag):
        """(i q_scale, mv_y q_scale, y q_scale) as the harness passes them and
        as get_rounded_q turns them into stream q indexes."""
        qi, qmv, qy = self.meta[tag]["q"]
        return qi, qmv, qy
