"""CPU check of the product's layer graph against the reference's parameter
set: building DMC / IntraNoAR consumes every key of a reference-format
state_dict (load_state_dict(strict=True) semantics) with the right shapes.
Packing is stubbed so no GPU is needed."""
import json
import os

import pytest
import torch

from dcvc_amd import hip as K
from dcvc_amd.weights import synthetic_state_dict

SPEC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dcvc_amd", "data",
                    "dc_param_spec.json")


class StubConvW:
    def __init__(self, weight, bias, stride=1, compute=K.BF16, device=None):
        self.cout, self.cin, self.kh, self.kw = weight.shape
        self.stride, self.compute = stride, compute


@pytest.fixture
def stub(monkeypatch):
    monkeypatch.setattr(K, "ConvW", StubConvW)


def _sd(kind):
    spec = json.load(open(SPEC))[kind]
    return synthetic_state_dict([(n, tuple(s)) for n, s in spec], seed=0)


def test_dmc_consumes_reference_state_dict(stub):
    from dcvc_amd.dc import DMC
    m = DMC(device=torch.device("cpu")).load_state_dict(_sd("inter"))
    assert m.ce_c4.cout == 128 and m.optic_flow.levels[0][0].kh == 7


def test_intra_consumes_reference_state_dict(stub):
    from dcvc_amd.dc import IntraNoAR
    m = IntraNoAR(device=torch.device("cpu")).load_state_dict(_sd("intra"))
    assert m.e2c.cout == 256


def test_strict_rejects_unknown_key(stub):
    from dcvc_amd.dc import DMC
    sd = _sd("inter")
    sd["not_a_layer.weight"] = torch.zeros(1)
    with pytest.raises(RuntimeError):
        DMC(device=torch.device("cpu")).load_state_dict(sd)


def _hem_sd(kind):
    spec = json.load(open(SPEC.replace("dc_param_spec", "hem_param_spec")))[kind]
    return synthetic_state_dict([(n, tuple(s)) for n, s in spec], seed=0)


def test_hem_dmc_consumes_reference_state_dict(stub):
    from dcvc_amd.hem import DMC
    m = DMC(device=torch.device("cpu")).load_state_dict(_hem_sd("inter"))
    assert m.ce_c4.cout == 96 and m.y_fusion.c0.cin == 480 and m.y_prior.spatial.c4.cout == 192


def test_hem_intra_consumes_reference_state_dict(stub):
    from dcvc_amd.hem import IntraNoAR
    m = IntraNoAR(device=torch.device("cpu")).load_state_dict(_hem_sd("intra"))
    assert m.enc.last.cout == 192 and m.prior.spatial.c0.cin == 768
