"""PyTorch default initialisation of the DCVC-DC models, replayed from their
(name, shape) spec — test infrastructure only (see oracle/__init__.py).

SURVEY.md §8(c) records a configuration of the reference run with its own
default init: ``torch.manual_seed(0)``, then ``IntraNoAR()``, then ``DMC()``
(DCVC-DC/src/models/image_model.py:61-105, video_model.py:235-323).  Their
random parameters are every ``nn.Conv2d`` (``reset_parameters``:
``kaiming_uniform_(weight, a=sqrt(5))`` then ``uniform_(bias, +-1/sqrt(fan_in))``)
and the ``Bitparm`` tensors h, b, a (``normal_(0, 0.01)``,
DCVC-DC/src/models/entropy_models.py:58-69); q_basic / q_scale start at one.
Construction draws them from the global CPU generator in module-registration
order, which for these models is the state_dict order of the parameters that
consume random numbers, so replaying the same torch.nn.init calls in spec
order on the same generator reproduces the tensors bit for bit
(tests/golden/make_golden_c3small.py checks this against the reference).
"""
import math

import torch


def _draw(name, shape):
    leaf = name.rsplit(".", 1)[-1]
    if "q_basic" in name or "q_scale" in name:
        return torch.ones(shape)
    if "bit_estimator" in name and leaf in ("h", "b", "a"):
        return torch.nn.init.normal_(torch.empty(shape), 0, 0.01)
    if leaf == "weight" and len(shape) == 4:
        return torch.nn.init.kaiming_uniform_(torch.empty(shape), a=math.sqrt(5))
    raise ValueError(f"no default-init rule for {name} {shape}")


def default_init_state_dicts(i_spec, p_spec, seed=0):
    """(IntraNoAR state_dict, DMC state_dict) after torch.manual_seed(seed),
    IntraNoAR(), DMC() — the generator state is saved and restored around it."""
    saved = torch.random.get_rng_state()
    torch.manual_seed(seed)
    try:
        out = []
        for spec in (i_spec, p_spec):
            sd = {}
            shapes = dict((n, tuple(s)) for n, s in spec)
            for name, shape in spec:
                shape = tuple(shape)
                if name.endswith(".bias") and len(shapes.get(name[:-4] + "weight", ())) == 4:
                    w = shapes[name[:-4] + "weight"]
                    bound = 1 / math.sqrt(w[1] * w[2] * w[3])
                    sd[name] = torch.nn.init.uniform_(torch.empty(shape), -bound, bound)
                else:
                    sd[name] = _draw(name, shape)
            out.append(sd)
        return out[0], out[1]
    finally:
        torch.random.set_rng_state(saved)
