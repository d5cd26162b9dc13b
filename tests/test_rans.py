"""Host rANS coder (libdcvc_rans) parity: known-answer vectors from the
reference's ops.cpp, byte-exact streams against the C oracle, lossless round
trips (DC multi-part with header, HEM headerless int32), and the reference's
real coder inputs from the golden fixtures."""
import os

import numpy as np
import pytest

from dcvc_amd import rans as P
from oracle import rans_oracle as R
from tests.dc_fixtures import GOLDEN


def kat():
    z = np.load(os.path.join(GOLDEN, "coder_golden.npz"))
    n = len([k for k in z.files if k.startswith("pmf")])
    return [(z[f"pmf{k}"], z[f"cdf{k}"]) for k in range(n)]


def test_pmf_to_quantized_cdf_matches_reference_ops_cpp():
    for pmf, cdf in kat():
        assert P.pmf_to_quantized_cdf(pmf.tolist(), 16) == cdf.tolist()
        assert R.pmf_to_quantized_cdf(pmf, 16) == cdf.tolist()


def test_pmf_to_quantized_cdf_rejects_all_zero():
    with pytest.raises(Exception):
        P.pmf_to_quantized_cdf([0.0, 0.0, 0.0], 16)


def laplace_table(scales=(0.05, 0.3, 1.0, 4.0, 20.0)):
    """A small laplace table built like GaussianEncoder.update, quantised by
    the product quantizer (already pinned above)."""
    rows, sizes, offs = [], [], []
    for s in scales:
        c = 2
        while c < 50 and 0.5 * np.exp(-c / s) > 1e-4:
            c += 1
        x = np.arange(-c, c + 1, dtype=np.float64)
        cdf = lambda v: np.where(v < 0, 0.5 * np.exp(v / s), 1 - 0.5 * np.exp(-v / s))  # noqa: E731
        pmf = (cdf(x + 0.5) - cdf(x - 0.5)).astype(np.float32)
        tail = np.float32(2 * cdf(-c - 0.5))
        q = P.pmf_to_quantized_cdf(np.concatenate([pmf, [tail]]).tolist(), 16)
        rows.append(q)
        sizes.append(len(pmf) + 2)
        offs.append(-c)
    w = max(len(r) for r in rows)
    m = np.zeros((len(rows), w), dtype=np.int32)
    for i, r in enumerate(rows):
        m[i, :len(r)] = r
    return m, np.array(sizes, np.int32), np.array(offs, np.int32)


def symbols(n, ntab, seed, wide=False, negative_idx=False):
    g = np.random.Generator(np.random.PCG64(seed))
    idx = g.integers(0, ntab, size=n).astype(np.int16)
    s = np.round(g.laplace(0, 2.0 if not wide else 300.0, size=n)).astype(np.int16)
    if wide:  # far escapes through the bypass path
        s[::97] = g.integers(-30000, 30000, size=s[::97].size)
    if negative_idx:
        idx[::11] = -1
    return s, idx


@pytest.mark.parametrize("parts", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("mt", [False, True])
def test_dc_stream_byte_exact_vs_oracle_and_roundtrip(parts, mt):
    tab = laplace_table()
    calls = []
    for k, n in enumerate([0, 1, 777, 4096, 12345]):
        s, i = symbols(n, tab[0].shape[0], 10 + k, wide=(k == 3), negative_idx=(k == 4))
        calls.append((s, i))
    enc = P.RansEncoder(mt, parts)
    ct = P.CdfTable(*tab)
    for s, i in calls:
        enc.encode_table(s, i, ct)
    enc.flush()
    stream = enc.get_encoded_stream()
    o = R.DCStream(parts)
    ostream = o.encode([(s, i, tab) for s, i in calls])
    assert stream.tobytes() == ostream
    dec = P.RansDecoder(parts)
    dec.set_stream(stream)
    for s, i in calls:
        out = dec.decode_table(i, ct)
        exp = np.where(i >= 0, s, 0)
        np.testing.assert_array_equal(out, exp)
    # reference-signature entry points (tables passed per call) agree too
    enc2 = P.RansEncoder(False, parts)
    for s, i in calls:
        enc2.encode_with_indexes(s, i, *tab)
    enc2.flush()
    assert enc2.get_encoded_stream().tobytes() == ostream
    enc.reset()
    enc.encode_table(calls[2][0], calls[2][1], ct)
    enc.flush()
    assert len(enc.get_encoded_stream()) > 0


def test_dc_header_bytes():
    tab = laplace_table()
    s, i = symbols(1000, 5, 3)
    e = P.RansEncoder(False, 1)
    e.encode_with_indexes(s, i, *tab)
    e.flush()
    b = e.get_encoded_stream()
    assert b[0] == 0x01 and (len(b) - 1) % 4 == 0  # 1 part, 2-byte sizes flag
    e = P.RansEncoder(False, 3)
    e.encode_with_indexes(s, i, *tab)
    e.flush()
    b = e.get_encoded_stream()
    assert b[0] == ((3 - 1) << 4) + 1


def test_hem_stream_byte_exact_vs_oracle_and_roundtrip():
    tab = laplace_table()
    g = np.random.Generator(np.random.PCG64(5))
    n = 20000
    idx = g.integers(0, 5, size=n).astype(np.int32)
    s = np.round(g.laplace(0, 3.0, size=n)).astype(np.int32)
    s[::53] = g.integers(-(1 << 20), 1 << 20, size=s[::53].size)  # beyond int16
    e = P.BufferedRansEncoder()
    e.encode_with_indexes(s, idx, *tab)
    stream = e.flush()
    assert stream == R.hem_encode(s, idx, *tab)
    d = P.HemRansDecoder()
    d.set_stream(stream)
    np.testing.assert_array_equal(d.decode_stream(idx, *tab), s)
    np.testing.assert_array_equal(R.hem_decode(stream, idx, *tab), s)


def test_hem_rejects_unencodable_symbol_instead_of_hanging():
    tab = laplace_table()
    e = P.BufferedRansEncoder()
    with pytest.raises(P.NativeError if hasattr(P, "NativeError") else Exception):
        e.encode_with_indexes(np.array([1 << 29], np.int32), np.array([0], np.int32), *tab)


def test_bad_index_and_truncated_stream_are_errors():
    tab = laplace_table()
    e = P.RansEncoder(False, 1)
    with pytest.raises(Exception):
        e.encode_with_indexes(np.array([0], np.int16), np.array([7], np.int16), *tab)
    s, i = symbols(5000, 5, 9)
    e.encode_with_indexes(s, i, *tab)
    e.flush()
    b = e.get_encoded_stream()
    d = P.RansDecoder(1)
    d.set_stream(b[: 1 + 8])
    with pytest.raises(Exception):
        d.decode_stream(i, *tab)


def test_reference_coder_inputs_roundtrip_byte_exact(dc_golden):
    """The reference's own symbols/indexes/CDF tables (golden fixtures) through
    the product coder and the oracle coder: identical bytes, lossless."""
    for tag in ("A", "B"):
        for t in range(dc_golden.meta[tag]["frames"]):
            calls = dc_golden.calls(tag, t)
            enc = P.RansEncoder(False, 1)
            tabs = {}
            for name, s, i in calls:
                tabs.setdefault(name, P.CdfTable(*dc_golden.table(name)))
                enc.encode_table(s, i, tabs[name])
            enc.flush()
            stream = enc.get_encoded_stream().tobytes()
            o = R.DCStream(1)
            assert stream == o.encode([(s, i, dc_golden.table(n)) for n, s, i in calls])
            dec = P.RansDecoder(1)
            dec.set_stream(stream)
            for name, s, i in calls:
                np.testing.assert_array_equal(dec.decode_table(i, tabs[name]), s.reshape(-1))


def _nthreads():
    return len(os.listdir("/proc/self/task"))


def test_shared_pool_concurrent_coders_byte_exact():
    """All coders of a process share one worker pool (dcvc_rans_set_threads /
    dcvc_rans_threads): creating many multi-part coders adds no threads, and
    six host threads coding 8-part streams at once (GOP lanes x I/P codecs)
    each get the oracle's bytes and a lossless decode."""
    import threading
    from dcvc_amd._native import rans_lib
    L = rans_lib()
    workers = L.dcvc_rans_threads()
    assert 0 <= workers <= 64
    assert L.dcvc_rans_set_threads(workers) == 0
    assert L.dcvc_rans_set_threads(workers + 1) == -5   # running pool: DCVC_EBUSY
    tab = laplace_table()
    ct = P.CdfTable(*tab)
    jobs = []
    for k in range(6):
        s, i = symbols(20000 + 977 * k, tab[0].shape[0], 100 + k, wide=(k % 3 == 0))
        jobs.append((s, i, R.DCStream(8).encode([(s, i, tab)])))
    # (counted after the oracle's encodes, whose native library may start a
    # thread team of its own; <=: a thread another test left may end meanwhile)
    base = _nthreads()
    coders = [(P.RansEncoder(True, 8), P.RansDecoder(8)) for _ in range(12)]
    assert _nthreads() <= base, "coders must not start threads of their own"
    errors = []

    def lane(k):
        enc, dec = coders[k]
        s, i, want = jobs[k]
        try:
            for _ in range(8):
                enc.reset()
                enc.encode_table(s, i, ct)
                enc.flush()
                got = enc.get_encoded_stream()
                assert got.tobytes() == want
                dec.set_stream(got)
                np.testing.assert_array_equal(dec.decode_table(i, ct), np.where(i >= 0, s, 0))
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))
    th = [threading.Thread(target=lane, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    # (a joined Python thread can still be listed in /proc for a moment)
    import time
    for _ in range(100):
        if _nthreads() <= base:
            break
        time.sleep(0.01)
    assert _nthreads() <= base
