"""Strict per-frame parity between the HIP product and the CPU oracle.

The reference computes every symbol as round(y - means) and every CDF index
as int((log(scale) - log_min) / step) of fp32 network outputs.  Both are
discontinuous: a value within float rounding error of a half-integer (symbol)
or of an integer (index) lands on either side depending on the order in
which a convolution sums its products.  The reference itself is not stable
under that: the same model on the same input run with 1 and with 8 CPU threads
changes a CDF index and the estimated bits.  So "bit-exact" is
checked here as:

  * every coder call the product makes equals the oracle's, symbol for symbol
    and index for index, EXCEPT at elements whose oracle pre-rounding /
    pre-truncation value lies within TIE_EPS of the discontinuity (a tie);
  * the first symbol that differs, in the order the codec computes them
    (mv_z, mv_y quadtree steps, z, y quadtree steps), must be such a tie.  A
    changed symbol changes y_hat, which every later step and call of the frame
    reads, so differences after it are a consequence (a "cascade");
  * the cascade is then checked element by element, not excused: the oracle
    codes the frame again with the product's symbols replayed at its own
    rounding ties (oracle.dc_oracle.Forcer), so it runs every later step on the
    product's y_hat.  In that replay every symbol must equal the product's and
    every index must equal it or sit on a tie of the replay's own values
    (compare_forced), and the product's reconstruction must lie within PSNR_DB
    of the replay's, which is the oracle's decode of the product's stream;
  * a frame whose calls all agree has identical bits (the coder is
    deterministic) and its reconstruction within PSNR_DB of the oracle's.
"""
import numpy as np

TIE_EPS = 1e-3        # distance of an oracle value to the rounding discontinuity (largest seen: 4.5e-4)
PSNR_DB = 1e-4        # BASELINE.json: PSNR delta < 1e-4 dB


def _np(t):
    return t.detach().reshape(-1).cpu().numpy() if hasattr(t, "detach") else np.asarray(t).reshape(-1)


def sym_tie_distance(pre):
    """|distance of pre to the nearest half-integer| (round() flips there)."""
    a = np.abs(pre.astype(np.float64))
    return np.abs(a - np.floor(a) - 0.5)


def idx_tie_distance(v):
    """distance of the pre-truncation index to the nearest integer."""
    v = v.astype(np.float64)
    return np.abs(v - np.round(v))


def compare_frame(prod_calls, oracle_calls, tap):
    """prod_calls: [(symbols, indexes)] in stream order (the product's encoder
    trace); oracle_calls: [(kind, symbols, indexes)] in stream order; tap: the
    oracle's compress(tap=...) dict.  Returns a stats dict."""
    assert len(prod_calls) == len(oracle_calls), (len(prod_calls), len(oracle_calls))
    out = {"calls": [], "symbols": 0, "sym_diff": 0, "idx_diff": 0, "first_flip": None,
           "unexplained": [], "cascade_sym": 0, "cascade_idx": 0, "max_tie_dist": 0.0}
    flipped = False
    for c in tap["order"]:
        ps, pi = (np.asarray(a).reshape(-1) for a in prod_calls[c])
        kind, os_, oi = oracle_calls[c]
        os_ = np.clip(_np(os_), -30000, 30000).astype(np.int64)
        oi = _np(oi).astype(np.int64)
        ds = np.nonzero(ps.astype(np.int64) != os_)[0]
        di = np.nonzero(pi.astype(np.int64) != oi)[0]
        out["symbols"] += ps.size
        out["sym_diff"] += int(ds.size)
        out["idx_diff"] += int(di.size)
        rec = {"call": c, "kind": kind, "n": int(ps.size), "sym_diff": int(ds.size), "idx_diff": int(di.size)}
        if flipped:
            out["cascade_sym"] += int(ds.size)
            out["cascade_idx"] += int(di.size)
        else:
            if di.size:
                d = idx_tie_distance(_np(tap["idx_f"][c])[di]) if tap["idx_f"][c] is not None else np.full(di.size, 1.0)
                rec["idx_tie_max"] = float(d.max())
                out["max_tie_dist"] = max(out["max_tie_dist"], float(d.max()))
                bad = di[d >= TIE_EPS]
                if bad.size:
                    out["unexplained"].append({"call": c, "what": "index", "pos": bad[:8].tolist(),
                                               "dist": d[d >= TIE_EPS][:8].tolist()})
            if ds.size:
                d = sym_tie_distance(_np(tap["pre"][c])[ds])
                rec["sym_tie_max"] = float(d.max())
                out["max_tie_dist"] = max(out["max_tie_dist"], float(d.max()))
                bad = ds[d >= TIE_EPS]
                if bad.size:
                    out["unexplained"].append({"call": c, "what": "symbol", "pos": bad[:8].tolist(),
                                               "dist": d[d >= TIE_EPS][:8].tolist()})
                out["first_flip"] = {"call": c, "kind": kind, "count": int(ds.size), "tie_dist": d[:8].tolist()}
                flipped = True
        out["calls"].append(rec)
    out["identical"] = out["sym_diff"] == 0 and out["idx_diff"] == 0
    return out


def compare_forced(prod_calls, oracle_calls, tap, forced):
    """The replay (module docstring): oracle_calls / tap from the oracle coding
    the frame with the product's symbols forced at ties (``forced`` of them).
    Every symbol must now agree; every differing index must be a tie of the
    replay's own pre-truncation values."""
    out = {"forced": int(forced), "sym_diff": 0, "idx_diff": 0, "unexplained": [], "max_tie_dist": 0.0}
    for c in tap["order"]:
        ps, pi = (np.asarray(a).reshape(-1) for a in prod_calls[c])
        kind, os_, oi = oracle_calls[c]
        os_ = np.clip(_np(os_), -30000, 30000).astype(np.int64)
        oi = _np(oi).astype(np.int64)
        ds = np.nonzero(ps.astype(np.int64) != os_)[0]
        di = np.nonzero(pi.astype(np.int64) != oi)[0]
        out["sym_diff"] += int(ds.size)
        out["idx_diff"] += int(di.size)
        if ds.size:
            d = sym_tie_distance(_np(tap["pre"][c])[ds])
            out["unexplained"].append({"call": c, "what": "symbol (replay)", "pos": ds[:8].tolist(),
                                       "dist": d[:8].tolist()})
        if di.size:
            d = idx_tie_distance(_np(tap["idx_f"][c])[di]) if tap["idx_f"][c] is not None else np.full(di.size, 1.0)
            out["max_tie_dist"] = max(out["max_tie_dist"], float(d.max()))
            bad = di[d >= TIE_EPS]
            if bad.size:
                out["unexplained"].append({"call": c, "what": "index (replay)", "pos": bad[:8].tolist(),
                                           "dist": d[d >= TIE_EPS][:8].tolist()})
    out["identical"] = out["sym_diff"] == 0 and out["idx_diff"] == 0
    return out


def check_forced(sf, bits, bits_replay, psnr, psnr_replay, name=""):
    """The replay's bar (compare_forced's dict)."""
    msg = (f"{name} replay: forced={sf['forced']} dsym={sf['sym_diff']} didx={sf['idx_diff']}, "
           f"bits {bits} vs replay {bits_replay}, dPSNR={psnr - psnr_replay:.3g} dB, unexplained={sf['unexplained']}")
    assert not sf["unexplained"], msg
    if sf["identical"]:
        assert bits == bits_replay, msg
    if "bits_replay_tied" in sf:
        # symbols all agree: the replay coded with the product's decisions at
        # its index ties is the product's stream
        assert bits == sf["bits_replay_tied"], msg + f", replay with the product's tie indexes {sf['bits_replay_tied']}"
    assert abs(psnr - psnr_replay) < PSNR_DB, msg
    return msg


def check_frame(st, bits, bits_oracle, psnr, psnr_oracle, name=""):
    """The strict bar (module docstring).  st: compare_frame's dict."""
    msg = (f"{name}: dsym={st['sym_diff']} didx={st['idx_diff']} of {st['symbols']} symbols, "
           f"bits {bits} vs oracle {bits_oracle} (d={bits - bits_oracle}), "
           f"dPSNR={psnr - psnr_oracle:.3g} dB, first_flip={st['first_flip']}, unexplained={st['unexplained']}")
    assert not st["unexplained"], msg
    if st["identical"]:
        assert bits == bits_oracle, msg
    if st["sym_diff"] == 0:
        assert abs(psnr - psnr_oracle) < PSNR_DB, msg
    return msg
