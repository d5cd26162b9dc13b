"""End-to-end DCVC-HEM parity on the GPU: the product (dcvc_amd.hem, HIP
kernels) against the reference's coder inputs (tests/golden/hem_golden.*,
recorded from the reference and reproduced bit-exactly by the CPU oracle,
tests/test_oracle_hem.py) in write mode, and against the reference's
estimate-mode bit counts.

Write mode, per frame: lossless self-consistency (decoder symbols/indexes ==
encoder symbols/indexes, bit-exact), symbol/index agreement with the
reference, stream size against the same coder run on the reference's
symbols, and reconstruction PSNR against the oracle's decoder.  As for DC,
float convs on MFMA sum in a different order than the CPU, so agreement is
statistical with the tolerances of tests/test_gpu_model_dc.py.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from tests.hem_fixtures import HEMGolden
from tests.test_gpu_model_dc import PARITY_TOL, FAST_TOL, psnr, _dump

pytestmark = pytest.mark.gpu

# bf16 features move more HEM symbols across rounding boundaries than DC's
# (HEM's latents are wider: |y_q| up to ~8 here vs 0/+-1 for DC's random
# weights), so the per-symbol agreement bound is looser; bits and PSNR bounds
# are FAST_TOL's.  Parity mode (fp32) is held to PARITY_TOL and measures 0
# differing symbols on these fixtures.
HEM_FAST_TOL = dict(FAST_TOL, sym_frac=0.1)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def hem_golden():
    return HEMGolden()


def _stream_bits(calls, tables, header):
    """Size of the HEM stream the product coder writes for these calls, in bits
    (the coder itself is pinned byte-exact by tests/test_rans.py)."""
    from dcvc_amd.rans import BufferedRansEncoder
    enc = BufferedRansEncoder()
    for name, s, i in calls:
        c, l, o = tables[name]
        enc.encode_with_indexes(s.astype(np.int32), i.astype(np.int32), c, l, o)
    return (len(enc.flush()) + header) * 8


@pytest.fixture(scope="module")
def oracle_runs(hem_golden):
    from oracle import hem_oracle as O
    from oracle import rans_oracle as R
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    i = O.IntraOracle(hem_golden.i_state_dict(), R.pmf_to_quantized_cdf)
    p = O.DMCOracle(hem_golden.p_state_dict(), R.pmf_to_quantized_cdf)
    tables = {n: hem_golden.table(n) for n in ("i_y", "i_z", "p_y", "p_z", "p_mvz")}
    runs = {}
    with torch.no_grad():
        for tag in ("A", "B", "C1"):
            meta = hem_golden.meta[tag]
            qi, qmv, qy = hem_golden.q(tag)
            h, w = meta["h"], meta["w"]
            frames, dpb = [], None
            for t in range(hem_golden.write_frames(tag)):
                x, _ = hem_golden.frame_tensor(tag, t)
                calls = hem_golden.calls(tag, t)
                pos = [0]

                def decoder(kind, idx):
                    s = calls[pos[0]][1]
                    pos[0] += 1
                    return torch.from_numpy(s.astype(np.int64))
                if t == 0:
                    xh = i.decompress(decoder, h, w, round(qi * 100) / 100)
                    dpb = {"ref_frame": xh, "ref_feature": None, "ref_y": None, "ref_mv_y": None}
                else:
                    dpb = p.decompress(dpb, decoder, h, w, round(qmv * 100) / 100, round(qy * 100) / 100)
                rec = dpb["ref_frame"][:, :, :h, :w]
                frames.append({"syms": [c[1] for c in calls], "idx": [c[2] for c in calls],
                               "bits": _stream_bits(calls, tables, 14 if t == 0 else 8), "psnr": psnr(rec, x)})
            runs[tag] = frames
    return runs


def run_product(g, tag, prec, estimate=False):
    from dcvc_amd.hem import DMC, IntraNoAR
    meta = g.meta[tag]
    h, w = meta["h"], meta["w"]
    qi, qmv, qy = g.q(tag)
    inet = IntraNoAR(precision=prec).load_state_dict(g.i_state_dict())
    pnet = DMC(precision=prec).load_state_dict(g.p_state_dict())
    inet.update(force=True)
    pnet.update(force=True)
    out, dpb = [], None
    with tempfile.TemporaryDirectory() as td:
        for t in range(meta["frames"] if estimate else g.write_frames(tag)):
            x, xp = g.frame_tensor(tag, t)
            xp = xp.cuda()
            net = inet if t == 0 else pnet
            net.entropy_coder.trace = []
            path = None if estimate else os.path.join(td, f"{t}.bin")
            if t == 0:
                r = inet.encode_decode(xp, qi, path, pic_width=w, pic_height=h)
                dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_y": None, "ref_mv_y": None}
            else:
                r = pnet.encode_decode(xp, dpb, path, pic_width=w, pic_height=h, mv_y_q_scale=qmv, y_q_scale=qy)
                dpb = r["dpb"]
            tr = net.entropy_coder.trace
            recon = dpb["ref_frame"].clamp_(0, 1)     # test_video.py:148-150
            rec = recon[:, :, :h, :w].cpu()
            out.append({"enc": [e for e in tr if e[0] == "enc"], "dec": [e for e in tr if e[0] == "dec"],
                        "bits": r["bit"], "psnr": psnr(rec, x)})
    return out


def compare(prod, orc):
    stats = []
    for t, (a, b) in enumerate(zip(prod, orc)):
        assert len(a["enc"]) == len(a["dec"]) == len(b["syms"])
        for (_, s_e, i_e), (_, s_d, i_d) in zip(a["enc"], a["dec"]):
            np.testing.assert_array_equal(i_e.reshape(-1), i_d.reshape(-1))
            np.testing.assert_array_equal(s_e.reshape(-1), s_d.reshape(-1))
        n = sum(s.size for s in b["syms"])
        ds = sum(int((e[1].reshape(-1) != s.reshape(-1)).sum()) for e, s in zip(a["enc"], b["syms"]))
        di = sum(int((e[2].reshape(-1) != s.reshape(-1)).sum()) for e, s in zip(a["enc"], b["idx"]))
        stats.append({"t": t, "symbols": n, "sym_diff": ds, "idx_diff": di, "bits": a["bits"],
                      "bits_oracle": b["bits"], "psnr": a["psnr"], "psnr_oracle": b["psnr"]})
    return stats


def check(stats, tol):
    for s in stats:
        assert s["sym_diff"] / s["symbols"] <= tol["sym_frac"], s
        assert abs(s["bits"] - s["bits_oracle"]) / s["bits_oracle"] <= tol["bits_rel"], s
        assert abs(s["psnr"] - s["psnr_oracle"]) <= tol["psnr_db"], s


# C1's random frames and wider latents move HEM symbols across rounding ties
# more often; a tie flipped in one frame changes that frame's y_hat and with it
# every later frame of a free-running sequence, so C1 parity is checked per
# frame on the reference's own dpb (teacher-forced) in
# tests/test_gpu_parity_strict.py; free-running C1 runs in fast mode here.
@pytest.mark.parametrize("mode,tag", [("parity", "A"), ("parity", "B"), ("fast", "A"), ("fast", "B"),
                                      ("fast", "C1")])
def test_hem_write_mode_vs_reference(hem_golden, oracle_runs, tag, mode):
    from dcvc_amd.layers import Precision
    prec = Precision.parity() if mode == "parity" else Precision.fast()
    stats = compare(run_product(hem_golden, tag, prec), oracle_runs[tag])
    _dump(f"hem_{mode}_{tag}", stats)
    check(stats, PARITY_TOL if mode == "parity" else HEM_FAST_TOL)


@pytest.mark.parametrize("mode,tag", [("parity", "A"), ("parity", "B"), ("fast", "A"), ("fast", "B"),
                                      ("fast", "C1")])
def test_hem_estimate_mode_vs_reference(hem_golden, tag, mode):
    from dcvc_amd.layers import Precision
    prec = Precision.parity() if mode == "parity" else Precision.fast()
    tol = PARITY_TOL if mode == "parity" else HEM_FAST_TOL
    prod = run_product(hem_golden, tag, prec, estimate=True)
    stats = [{"t": t, "bit": a["bits"], "bit_ref": e["bit"], "psnr": a["psnr"], "psnr_ref": e["psnr"]}
             for t, (a, e) in enumerate(zip(prod, hem_golden.meta[tag]["est"]))]
    _dump(f"hem_estimate_{mode}_{tag}", stats)
    for s in stats:
        assert abs(s["bit"] - s["bit_ref"]) / s["bit_ref"] <= tol["bits_rel"], s
        assert abs(s["psnr"] - s["psnr_ref"]) <= tol["psnr_db"], s
