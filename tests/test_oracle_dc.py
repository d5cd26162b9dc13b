"""Pin the CPU oracle (oracle/) to the reference's own outputs (tests/golden/).

The oracle is a functional fp32 restatement of DCVC-DC; on the CPU it must
reproduce the reference bit for bit: CDF tables, every symbol/index the
reference hands its entropy coder, the decoded dpb, and estimate-mode bits.
"""
import numpy as np
import pytest
import torch

from oracle import dc_oracle as O
from oracle import rans_oracle as R
from tests.dc_fixtures import digest


@pytest.fixture(scope="module")
def oracles(dc_golden):
    torch.set_num_threads(8)
    i = O.IntraOracle(dc_golden.i_state_dict(), R.pmf_to_quantized_cdf)
    p = O.DMCOracle(dc_golden.p_state_dict(), R.pmf_to_quantized_cdf)
    return i, p


def test_cdf_tables_match_reference(dc_golden, oracles):
    i, p = oracles
    ours = {"i_y": (i.y_cdf, i.y_sizes, i.y_offsets), "i_z": i.z_tab,
            "p_y": (p.y_cdf, p.y_sizes, p.y_offsets), "p_z": p.z_tab, "p_mvz": p.mvz_tab}
    for name, (c, l, o) in ours.items():
        rc, rl, ro = dc_golden.table(name)
        np.testing.assert_array_equal(c, rc, err_msg=name)
        np.testing.assert_array_equal(l.reshape(-1), rl.reshape(-1), err_msg=name)
        np.testing.assert_array_equal(o.reshape(-1), ro.reshape(-1), err_msg=name)


def oracle_tables(i, p):
    return {"i_y": (i.y_cdf, i.y_sizes, i.y_offsets), "i_z": i.z_tab,
            "p_y": (p.y_cdf, p.y_sizes, p.y_offsets), "p_z": p.z_tab, "p_mvz": p.mvz_tab}


KIND = {"y": "y", "z": "z", "mvz": "mvz"}


def run_oracle_write(dc_golden, oracles, tag):
    """Replay test_video.py's I/P loop in write mode with the oracle models and
    the oracle C coder; yield per frame (calls, stream, dpb)."""
    i, p = oracles
    tabs = oracle_tables(i, p)
    meta = dc_golden.meta[tag]
    h, w, q = meta["h"], meta["w"], meta["q_index"]
    dpb = None
    for t in range(meta["frames"]):
        x, xp = dc_golden.frame_tensor(tag, t)
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
                dpb = {"ref_frame": xh, "ref_feature": None, "ref_mv_feature": None,
                       "ref_y": None, "ref_mv_y": None}
            else:
                dpb = p.decompress(dpb, decoder, h, w, False, q, t % 4)
        dpb["ref_frame"].clamp_(0, 1)
        yield t, calls, coder_calls, stream, dpb


@pytest.mark.parametrize("tag", ["A", "B"])
def test_write_mode_matches_reference(dc_golden, oracles, tag):
    for t, calls, coder_calls, stream, dpb in run_oracle_write(dc_golden, oracles, tag):
        ref = dc_golden.calls(tag, t)
        assert [k for k, _, _ in calls] == [n[2:] for n, _, _ in ref]
        for (s, ix, _), (name, rs, ri) in zip(coder_calls, ref):
            np.testing.assert_array_equal(s.reshape(-1), rs.reshape(-1), err_msg=f"{tag} t={t} {name} symbols")
            np.testing.assert_array_equal(ix.reshape(-1), ri.reshape(-1), err_msg=f"{tag} t={t} {name} indexes")
        e = dc_golden.meta[tag]["write"][t]
        assert e["decode_index_mismatch"] == 0
        assert digest(dpb["ref_frame"]) == e["recon_sha256"], f"{tag} t={t} recon"
        for k in ("ref_feature", "ref_mv_feature", "ref_y", "ref_mv_y"):
            if k + "_sha256" in e:
                assert digest(dpb[k]) == e[k + "_sha256"], f"{tag} t={t} {k}"


@pytest.mark.parametrize("tag", ["A", "B"])
def test_estimate_mode_matches_reference(dc_golden, oracles, tag):
    i, p = oracles
    meta = dc_golden.meta[tag]
    q = meta["q_index"]
    dpb = None
    with torch.no_grad():
        for t in range(meta["frames"]):
            x, xp = dc_golden.frame_tensor(tag, t)
            if t == 0:
                bit, xh = i.forward(xp, False, q)
                dpb = {"ref_frame": xh, "ref_feature": None, "ref_mv_feature": None,
                       "ref_y": None, "ref_mv_y": None}
            else:
                bit, dpb = p.forward_one_frame(xp, dpb, False, q, t % 4)
            dpb["ref_frame"].clamp_(0, 1)
            e = meta["est"][t]
            assert bit == e["bit"], f"{tag} t={t}"
            assert digest(dpb["ref_frame"]) == e["recon_sha256"], f"{tag} t={t}"
