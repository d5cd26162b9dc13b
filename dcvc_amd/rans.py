"""Python face of libdcvc_rans, mirroring the reference's pybind11 modules.

DC (``MLCodec_rans`` of DCVC-DC, DCVC-DC/src/cpp/py_rans/py_rans.cpp:227-243):
    RansEncoder(multiThread, streamPart).encode_with_indexes / flush /
    get_encoded_stream / reset;  RansDecoder(streamPart).set_stream /
    decode_stream.
HEM (``MLCodec_rans`` of DCVC-HEM, DCVC-HEM/src/cpp/rans/rans_interface.cpp:246-261):
    BufferedRansEncoder().encode_with_indexes / flush -> bytes / reset;
    HemRansDecoder().set_stream(bytes) / decode_stream.
``MLCodec_CXX.pmf_to_quantized_cdf`` (DCVC-DC/src/cpp/ops/ops.cpp:84-91) is
``pmf_to_quantized_cdf``.

Argument meaning and output types follow the reference.  Where the reference
has undefined behaviour (out-of-range indexes, HEM symbols beyond 2^27 from
their offset) a ``NativeError`` is raised instead.  ``CdfTable`` is the
upload-once fast path used by the codec models.
"""
import ctypes

import numpy as np

from ._native import rans_lib, check, ptr

_L = rans_lib()


def pmf_to_quantized_cdf(pmf, precision=16):
    p = np.ascontiguousarray(np.asarray(pmf, dtype=np.float32))
    out = np.zeros(p.size + 1, dtype=np.uint32)
    check(_L.dcvc_pmf_to_quantized_cdf(ptr(p, ctypes.c_float), p.size, precision,
                                       ptr(out, ctypes.c_uint32)), "pmf_to_quantized_cdf")
    return out.tolist()


def _i32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


class CdfTable:
    """A [cdf_num, stride] int32 CDF matrix + sizes + offsets, uploaded once."""

    def __init__(self, cdfs, cdf_sizes, offsets):
        cdfs = _i32(cdfs)
        if cdfs.ndim != 2:
            raise ValueError("cdfs must be 2-D")
        self.cdfs = cdfs
        self.sizes = _i32(cdf_sizes).reshape(-1)
        self.offsets = _i32(offsets).reshape(-1)
        if self.sizes.size != cdfs.shape[0] or self.offsets.size != cdfs.shape[0]:
            raise ValueError("cdf_sizes/offsets must have one entry per cdf row")
        h = _L.dcvc_cdf_table_create(ptr(cdfs, ctypes.c_int32), cdfs.shape[0], cdfs.shape[1],
                                     ptr(self.sizes, ctypes.c_int32),
                                     ptr(self.offsets, ctypes.c_int32))
        if not h:
            raise ValueError("invalid CDF table")
        self.handle = ctypes.c_void_p(h)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            _L.dcvc_cdf_table_destroy(h)
            self.handle = None


class _Encoder:
    def __init__(self, multithread, parts, with_header):
        h = _L.dcvc_rans_enc_create(int(bool(multithread)), int(parts))
        if not h:
            raise ValueError(f"bad encoder config multithread={multithread} parts={parts}")
        self._h = ctypes.c_void_p(h)
        self._with_header = with_header
        self._keep = []

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _L.dcvc_rans_enc_destroy(h)
            self._h = None

    def encode_table(self, symbols, indexes, table):
        dt = np.int16 if self._with_header else np.int32
        s = np.ascontiguousarray(np.asarray(symbols).reshape(-1), dtype=dt)
        x = np.ascontiguousarray(np.asarray(indexes).reshape(-1), dtype=dt)
        if s.size != x.size:
            raise ValueError("symbols and indexes differ in length")
        self._keep.append(table)  # table must outlive queued work
        if dt is np.int16:
            r = _L.dcvc_rans_enc_encode_table_i16(self._h, ptr(s, ctypes.c_int16),
                                                  ptr(x, ctypes.c_int16), s.size, table.handle)
        else:
            r = _L.dcvc_rans_enc_encode_table_i32(self._h, ptr(s, ctypes.c_int32),
                                                  ptr(x, ctypes.c_int32), s.size, table.handle)
        check(r, "encode_with_indexes")

    def flush(self):
        check(_L.dcvc_rans_enc_flush(self._h), "flush")

    def _stream(self):
        n = check(_L.dcvc_rans_enc_stream_size(self._h, int(self._with_header)), "stream_size")
        out = np.empty(n, dtype=np.uint8)
        check(_L.dcvc_rans_enc_get_stream(self._h, int(self._with_header),
                                          ptr(out, ctypes.c_uint8), n), "get_stream")
        return out

    def reset(self):
        check(_L.dcvc_rans_enc_reset(self._h), "reset")
        self._keep = []


class RansEncoder(_Encoder):
    """DC coder: int16 symbols, multi-part stream with header (py_rans.cpp:11-125)."""

    def __init__(self, multiThread=False, streamPart=1):
        super().__init__(multiThread, streamPart, with_header=True)

    def encode_with_indexes(self, symbols, indexes, cdfs, cdfs_sizes, offsets):
        self.encode_table(symbols, indexes, CdfTable(cdfs, cdfs_sizes, offsets))

    def get_encoded_stream(self):
        return self._stream()


class BufferedRansEncoder(_Encoder):
    """HEM coder: int32 symbols, one headerless stream (rans_interface.cpp:85-174)."""

    def __init__(self):
        super().__init__(False, 1, with_header=False)

    def encode_with_indexes(self, symbols, indexes, cdfs, cdfs_sizes, offsets):
        self.encode_table(symbols, indexes, CdfTable(cdfs, cdfs_sizes, offsets))

    def flush(self):
        super().flush()
        return self._stream().tobytes()


class _Decoder:
    def __init__(self, parts, with_header):
        h = _L.dcvc_rans_dec_create(int(parts))
        if not h:
            raise ValueError(f"bad decoder config parts={parts}")
        self._h = ctypes.c_void_p(h)
        self._with_header = with_header

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _L.dcvc_rans_dec_destroy(h)
            self._h = None

    def set_stream(self, stream):
        if isinstance(stream, (bytes, bytearray, memoryview)):
            stream = np.frombuffer(bytes(stream), dtype=np.uint8)
        b = np.ascontiguousarray(stream, dtype=np.uint8)
        check(_L.dcvc_rans_dec_set_stream(self._h, ptr(b, ctypes.c_uint8), b.size,
                                          int(self._with_header)), "set_stream")

    def decode_table(self, indexes, table):
        if self._with_header:
            x = np.ascontiguousarray(np.asarray(indexes).reshape(-1), dtype=np.int16)
            out = np.empty(x.size, dtype=np.int16)
            r = _L.dcvc_rans_dec_decode_table_i16(self._h, ptr(x, ctypes.c_int16), x.size,
                                                  table.handle, ptr(out, ctypes.c_int16))
        else:
            x = np.ascontiguousarray(np.asarray(indexes).reshape(-1), dtype=np.int32)
            out = np.empty(x.size, dtype=np.int32)
            r = _L.dcvc_rans_dec_decode_table_i32(self._h, ptr(x, ctypes.c_int32), x.size,
                                                  table.handle, ptr(out, ctypes.c_int32))
        check(r, "decode_stream")
        return out

    def decode_stream(self, indexes, cdfs, cdfs_sizes, offsets):
        return self.decode_table(indexes, CdfTable(cdfs, cdfs_sizes, offsets))


class RansDecoder(_Decoder):
    """DC decoder (py_rans.cpp:127-225)."""

    def __init__(self, streamPart=1):
        super().__init__(streamPart, with_header=True)


class HemRansDecoder(_Decoder):
    """HEM decoder (rans_interface.cpp:176-244)."""

    def __init__(self):
        super().__init__(1, with_header=False)
