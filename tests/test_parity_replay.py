"""The parity bar's replay (tests/parity.py, oracle.dc_oracle.Forcer) on the CPU.

After a product symbol flips at a rounding tie, the strict tests make the
oracle code the frame again with the product's symbols forced at its ties, so
the rest of the frame is checked element by element instead of being counted
as a cascade.  These tests pin the instrumentation itself: forcing the
oracle's own symbols changes nothing; a forced symbol lands in the coder call
it belongs to and every later quadtree step and call runs on the changed
y_hat; compare_forced accepts a consistent replay and flags a non-tie
difference.
"""
import pytest
import torch

from oracle import dc_oracle as O
from oracle import hem_oracle as H
from oracle import rans_oracle as R
from tests.parity import compare_forced


@pytest.fixture(scope="module")
def dc(dc_golden):
    torch.set_num_threads(8)
    return (O.IntraOracle(dc_golden.i_state_dict(), R.pmf_to_quantized_cdf),
            O.DMCOracle(dc_golden.p_state_dict(), R.pmf_to_quantized_cdf))


def _as_prod(calls):
    return [(s.clamp(-30000, 30000).to(torch.int16).numpy().reshape(-1), i.to(torch.int16).numpy().reshape(-1))
            for _, s, i in calls]


def _p_frame(dc_golden, dc):
    i, p = dc
    meta = dc_golden.meta["B"]
    _, x0 = dc_golden.frame_tensor("B", 0)
    _, x1 = dc_golden.frame_tensor("B", 1)
    with torch.no_grad():
        _, xh = i.compress(x0, False, meta["q_index"], recon=True)
    dpb = {"ref_frame": xh, "ref_feature": None, "ref_mv_feature": None, "ref_y": None, "ref_mv_y": None}
    return x1, dpb, meta["q_index"]


def test_forcing_own_symbols_is_identity(dc_golden, dc):
    x1, dpb, q = _p_frame(dc_golden, dc)
    _, p = dc
    with torch.no_grad():
        tap = {}
        calls, d0 = p.compress(x1, dpb, False, q, 1, tap=tap, recon=True)
        fr = O.Forcer([s for s, _ in _as_prod(calls)], 1e-3)
        tap_f = {}
        calls_f, d1 = p.compress(x1, dpb, False, q, 1, tap=tap_f, recon=True, force=fr)
    assert fr.forced == 0
    for (_, a, ia), (_, b, ib) in zip(calls, calls_f):
        assert torch.equal(a, b) and torch.equal(ia, ib)
    assert torch.equal(d0["ref_frame"], d1["ref_frame"])
    sf = compare_forced(_as_prod(calls), calls_f, tap_f, fr.forced)
    assert sf["identical"] and not sf["unexplained"]


def test_forced_symbol_propagates(dc_golden, dc):
    """A product that codes one mv_y symbol of quadtree step 0 differently: with
    a tie window wide enough to admit it, the replay takes that symbol, and the
    later steps (which read y_hat) change with it exactly as the product's
    would; compare_forced then accepts the replay."""
    x1, dpb, q = _p_frame(dc_golden, dc)
    _, p = dc
    with torch.no_grad():
        tap = {}
        calls = p.compress(x1, dpb, False, q, 1, tap=tap)
        prod = _as_prod(calls)
        # flip the mv_y step-0 symbol (call 2) whose pre-rounding value is nearest a tie
        pre = tap["pre"][2].reshape(-1).double()
        nz = torch.nonzero(pre.abs() > 0).reshape(-1)
        a = pre[nz].abs()
        k = int(nz[torch.argmin((a - torch.floor(a) - 0.5).abs())])
        s = prod[2][0].copy()
        s[k] += 1 if pre[k] > s[k] else -1
        prod[2] = (s, prod[2][1])
        # only call 2 replayed (the tie window 0.5 admits any difference)
        fr = O.Forcer([sy if c == 2 else None for c, (sy, _) in enumerate(prod)], 0.5)
        tap_f = {}
        calls_f = p.compress(x1, dpb, False, q, 1, tap=tap_f, force=fr)
    assert fr.forced == 1
    assert int(calls_f[2][1].reshape(-1)[k]) == int(s[k])
    # steps 1..3 of mv_y read y_hat: the replay's later calls are its own,
    # computed on the changed y_hat; a product that followed the same y_hat
    # codes exactly them
    follow = [(c[1].clamp(-30000, 30000).to(torch.int16).numpy().reshape(-1),
               c[2].to(torch.int16).numpy().reshape(-1)) for c in calls_f]
    sf = compare_forced(follow, calls_f, tap_f, fr.forced)
    assert sf["identical"] and not sf["unexplained"], sf


def test_compare_forced_flags_non_tie(dc_golden, dc):
    x1, dpb, q = _p_frame(dc_golden, dc)
    _, p = dc
    with torch.no_grad():
        tap = {}
        calls = p.compress(x1, dpb, False, q, 1, tap=tap)
    prod = _as_prod(calls)
    s = prod[6][0].copy()
    pre = tap["pre"][6].reshape(-1).double()
    a = pre.abs()
    k = int(torch.argmax(-(a - torch.floor(a) - 0.5).abs() + (a > 0).double() * 10))   # far from a tie
    s[k] += 3
    prod[6] = (s, prod[6][1])
    sf = compare_forced(prod, calls, tap, 0)
    assert sf["unexplained"] and sf["unexplained"][0]["what"] == "symbol (replay)"


def test_hem_forcing_own_symbols_is_identity():
    from tests.hem_fixtures import HEMGolden
    g = HEMGolden()
    torch.set_num_threads(8)
    oi = H.IntraOracle(g.i_state_dict(), R.pmf_to_quantized_cdf)
    qi = round(g.q("B")[0] * 100) / 100
    _, x0 = g.frame_tensor("B", 0)
    with torch.no_grad():
        calls, xh = oi.compress(x0, qi, recon=True)
        fr = O.Forcer([s.reshape(-1).int().numpy() for _, s, _ in calls], 1e-3)
        calls_f, xh_f = oi.compress(x0, qi, recon=True, force=fr)
    assert fr.forced == 0
    assert torch.equal(xh, xh_f)
    for (_, a, _), (_, b, _) in zip(calls, calls_f):
        assert torch.equal(a, b)
