"""The DCVC-HEM CPU oracle against the reference's own behaviour, recorded in
tests/golden/hem_golden.* by make_golden_hem.py: CDF tables, every coder
call of write mode (symbols and CDF indexes, bit-exact), the decoder's dpb
(sha256 of the fp32 tensors) and estimate-mode bit counts."""
import os

import numpy as np
import pytest
import torch

from oracle import hem_oracle as O
from oracle import rans_oracle as R
from tests.dc_fixtures import digest
from tests.hem_fixtures import HEMGolden


@pytest.fixture(scope="module")
def hem_golden():
    return HEMGolden()


@pytest.fixture(scope="module")
def oracles(hem_golden):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    return (O.IntraOracle(hem_golden.i_state_dict(), R.pmf_to_quantized_cdf),
            O.DMCOracle(hem_golden.p_state_dict(), R.pmf_to_quantized_cdf))


def test_cdf_tables_match_reference(hem_golden, oracles):
    i, p = oracles
    for name, tab in (("i_y", i.tab_y), ("i_z", i.tab_z), ("p_y", p.tab_y), ("p_z", p.tab_z), ("p_mvz", p.tab_mvz)):
        c, l, o = hem_golden.table(name)
        np.testing.assert_array_equal(tab[0], c)
        np.testing.assert_array_equal(tab[1], l)
        np.testing.assert_array_equal(tab[2], o)


def _indexes(oracle, kind, sym, scales):
    if scales is None:
        C, h, w = sym.shape[1:]
        return O.channel_indexes(C, h, w)
    return O.build_indexes(scales, oracle.tab_y[3], oracle.tab_y[4]).reshape(-1)


@pytest.mark.parametrize("tag", ["A", "B", "C1"])
def test_write_mode_matches_reference(hem_golden, oracles, tag):
    i, p = oracles
    meta = hem_golden.meta[tag]
    qi, qmv, qy = hem_golden.q(tag)
    h, w = meta["h"], meta["w"]
    dpb = None
    with torch.no_grad():
        for t in range(hem_golden.write_frames(tag)):
            _, xp = hem_golden.frame_tensor(tag, t)
            ref_calls = hem_golden.calls(tag, t)
            if t == 0:
                calls = i.compress(xp, round(qi * 100) / 100)
            else:
                calls = p.compress(xp, dpb, round(qmv * 100) / 100, round(qy * 100) / 100)
            assert [c[0] for c in calls] == [c[0] for c in ref_calls]
            net = i if t == 0 else p
            for (kind, sym, scales), (_, rs, ri) in zip(calls, ref_calls):
                np.testing.assert_array_equal(sym.reshape(-1).int().numpy(), rs)
                np.testing.assert_array_equal(_indexes(net, kind, sym, scales).numpy().astype(np.int16), ri)
            pos = [0]

            def decoder(kind, idx):
                name, s, ri = ref_calls[pos[0]]
                pos[0] += 1
                assert name == kind
                np.testing.assert_array_equal(idx.numpy().astype(np.int16), ri)
                return torch.from_numpy(s.astype(np.int64))
            if t == 0:
                xh = i.decompress(decoder, h, w, round(qi * 100) / 100)
                dpb = {"ref_frame": xh, "ref_feature": None, "ref_y": None, "ref_mv_y": None}
            else:
                dpb = p.decompress(dpb, decoder, h, w, round(qmv * 100) / 100, round(qy * 100) / 100)
            e = meta["write"][t]
            assert digest(dpb["ref_frame"]) == e["recon_sha256"], f"{tag} t={t}"
            for k in ("ref_feature", "ref_y", "ref_mv_y"):
                if k + "_sha256" in e:
                    assert digest(dpb[k]) == e[k + "_sha256"], f"{tag} t={t} {k}"


def test_c1_frames(hem_golden):
    for t in range(hem_golden.meta["C1"]["frames"]):
        x, _ = hem_golden.frame_tensor("C1", t)
        assert digest(x) == hem_golden.meta["C1"]["frame_sha256"][t]


@pytest.mark.parametrize("tag", ["A", "B", "C1"])
def test_estimate_mode_matches_reference(hem_golden, oracles, tag):
    i, p = oracles
    meta = hem_golden.meta[tag]
    qi, qmv, qy = hem_golden.q(tag)
    dpb = None
    with torch.no_grad():
        for t in range(meta["frames"]):
            _, xp = hem_golden.frame_tensor(tag, t)
            if t == 0:
                bit, xh = i.forward(xp, qi)
                dpb = {"ref_frame": xh, "ref_feature": None, "ref_y": None, "ref_mv_y": None}
            else:
                bit, dpb = p.forward_one_frame(xp, dpb, qmv, qy)
            dpb["ref_frame"].clamp_(0, 1)
            e = meta["est"][t]
            assert bit == e["bit"], f"{tag} t={t}"
            assert digest(dpb["ref_frame"]) == e["recon_sha256"], f"{tag} t={t}"
