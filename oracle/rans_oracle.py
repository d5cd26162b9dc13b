"""ctypes face of oracle/rans_oracle.c — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py)."""
import ctypes
import os

import numpy as np

_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "liboracle_rans.so")
_L = ctypes.CDLL(_SO)
_P = ctypes.c_void_p
_L.oracle_pmf_to_quantized_cdf.argtypes = [_P, ctypes.c_int, ctypes.c_int, _P]
_L.oracle_dc_encode.restype = ctypes.c_int64
_L.oracle_dc_encode.argtypes = [ctypes.c_int, _P, _P, _P, _P, ctypes.c_int, _P, _P, ctypes.c_int, _P,
                                ctypes.c_int64]
_L.oracle_dc_decode.argtypes = [_P, ctypes.c_int64, ctypes.c_int, _P, _P, _P, ctypes.c_int, _P, _P,
                                ctypes.c_int, _P]
_L.oracle_hem_encode.restype = ctypes.c_int64
_L.oracle_hem_encode.argtypes = [ctypes.c_int64, _P, _P, _P, ctypes.c_int, _P, _P, _P, ctypes.c_int64]
_L.oracle_hem_decode.argtypes = [_P, ctypes.c_int64, ctypes.c_int64, _P, _P, ctypes.c_int, _P, _P, _P]


def _a(x, dt):
    return np.ascontiguousarray(np.asarray(x), dtype=dt)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def pmf_to_quantized_cdf(pmf, precision=16):
    p = _a(pmf, np.float32)
    out = np.zeros(p.size + 1, dtype=np.uint32)
    if _L.oracle_pmf_to_quantized_cdf(_p(p), p.size, precision, _p(out)) != 0:
        raise ValueError("pmf_to_quantized_cdf failed")
    return out.tolist()


class DCStream:
    """Encode a list of calls, each with its own table (encoded through one
    coder state, exactly as the reference's single RansEncoder would)."""

    def __init__(self, parts=1):
        self.parts = parts

    def encode(self, calls):
        # merge tables: stack every distinct table into one matrix and offset indexes
        tabs, key = [], {}
        for _, _, t in calls:
            if id(t[0]) not in key:
                key[id(t[0])] = sum(x[0].shape[0] for x in tabs)
                tabs.append(t)
        stride = max(t[0].shape[1] for t in tabs)
        cdfs = np.zeros((sum(t[0].shape[0] for t in tabs), stride), dtype=np.int32)
        r = 0
        for t in tabs:
            cdfs[r:r + t[0].shape[0], :t[0].shape[1]] = t[0]
            r += t[0].shape[0]
        sizes = _a(np.concatenate([np.asarray(t[1]).reshape(-1) for t in tabs]), np.int32)
        offs = _a(np.concatenate([np.asarray(t[2]).reshape(-1) for t in tabs]), np.int32)
        syms = _a(np.concatenate([np.asarray(s).reshape(-1) for s, _, _ in calls]), np.int16)
        idxs = []
        for s, i, t in calls:
            i = np.asarray(i).reshape(-1).astype(np.int32)
            i = np.where(i >= 0, i + key[id(t[0])], i)
            idxs.append(i)
        idxs = _a(np.concatenate(idxs), np.int16)
        lens = _a([np.asarray(s).size for s, _, _ in calls], np.int64)
        cap = syms.size * 16 + 4096
        buf = np.zeros(cap, dtype=np.uint8)
        n = _L.oracle_dc_encode(len(calls), _p(lens), _p(syms), _p(idxs), _p(cdfs), stride, _p(sizes),
                                _p(offs), self.parts, _p(buf), cap)
        if n < 0:
            raise ValueError("oracle encode failed")
        self._ctx = (lens, idxs, cdfs, stride, sizes, offs)
        return buf[:n].tobytes()

    def decode(self, stream):
        lens, idxs, cdfs, stride, sizes, offs = self._ctx
        b = _a(np.frombuffer(stream, dtype=np.uint8), np.uint8)
        out = np.zeros(idxs.size, dtype=np.int16)
        if _L.oracle_dc_decode(_p(b), b.size, lens.size, _p(lens), _p(idxs), _p(cdfs), stride, _p(sizes),
                               _p(offs), self.parts, _p(out)) != 0:
            raise ValueError("oracle decode failed")
        return out


def hem_encode(symbols, indexes, cdfs, sizes, offsets):
    s, i = _a(symbols, np.int32).reshape(-1), _a(indexes, np.int32).reshape(-1)
    c = _a(cdfs, np.int32)
    sz, of = _a(sizes, np.int32).reshape(-1), _a(offsets, np.int32).reshape(-1)
    cap = s.size * 16 + 4096
    buf = np.zeros(cap, dtype=np.uint8)
    n = _L.oracle_hem_encode(s.size, _p(s), _p(i), _p(c), c.shape[1], _p(sz), _p(of), _p(buf), cap)
    if n < 0:
        raise ValueError("oracle encode failed")
    return buf[:n].tobytes()


def hem_decode(stream, indexes, cdfs, sizes, offsets):
    i = _a(indexes, np.int32).reshape(-1)
    c = _a(cdfs, np.int32)
    sz, of = _a(sizes, np.int32).reshape(-1), _a(offsets, np.int32).reshape(-1)
    b = _a(np.frombuffer(stream, dtype=np.uint8), np.uint8)
    out = np.zeros(i.size, dtype=np.int32)
    _L.oracle_hem_decode(_p(b), b.size, i.size, _p(i), _p(c), c.shape[1], _p(sz), _p(of), _p(out))
    return out
