"""Loader for the native libraries behind the C ABI (include/*.h).

Both libraries live in-tree under ``dcvc_amd/lib`` (built by ``make`` /
``__graft_entry__.build()``).  There is no fallback: if a library is missing
or fails to load, the import error propagates — the product path never
silently degrades to a Python or PyTorch implementation.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")

_c = ctypes
_i16p = _c.POINTER(_c.c_int16)
_i32p = _c.POINTER(_c.c_int32)
_u8p = _c.POINTER(_c.c_uint8)
_u32p = _c.POINTER(_c.c_uint32)
_f32p = _c.POINTER(_c.c_float)
_vp = _c.c_void_p

DCVC_OK = 0
DCVC_EINVAL = -1
DCVC_ERANGE = -2
DCVC_ENOMEM = -3
DCVC_ESTREAM = -4
DCVC_EBUSY = -5

_ERRORS = {
    DCVC_EINVAL: "invalid argument",
    DCVC_ERANGE: "symbol out of codable range",
    DCVC_ENOMEM: "out of memory",
    DCVC_ESTREAM: "malformed stream",
    DCVC_EBUSY: "stream not flushed",
}


class NativeError(RuntimeError):
    pass


def check(status, what):
    if status < 0:
        raise NativeError(f"{what}: {_ERRORS.get(status, status)}")
    return status


def _load(name):
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `make` or __graft_entry__.build()")
    return ctypes.CDLL(path)


# (symbol, restype, argtypes) for libdcvc_rans.so — mirrors include/dcvc_rans.h
RANS_SYMBOLS = [
    ("dcvc_pmf_to_quantized_cdf", _c.c_int, [_f32p, _c.c_int, _c.c_int, _u32p]),
    ("dcvc_cdf_table_create", _vp, [_i32p, _c.c_int, _c.c_int, _i32p, _i32p]),
    ("dcvc_cdf_table_destroy", None, [_vp]),
    ("dcvc_rans_enc_create", _vp, [_c.c_int, _c.c_int]),
    ("dcvc_rans_enc_destroy", None, [_vp]),
    ("dcvc_rans_enc_encode_with_indexes_i16", _c.c_int,
     [_vp, _i16p, _i16p, _c.c_int64, _i32p, _c.c_int, _c.c_int, _i32p, _i32p]),
    ("dcvc_rans_enc_encode_table_i16", _c.c_int, [_vp, _i16p, _i16p, _c.c_int64, _vp]),
    ("dcvc_rans_enc_encode_table_i32", _c.c_int, [_vp, _i32p, _i32p, _c.c_int64, _vp]),
    ("dcvc_rans_enc_flush", _c.c_int, [_vp]),
    ("dcvc_rans_enc_stream_size", _c.c_int64, [_vp, _c.c_int]),
    ("dcvc_rans_enc_get_stream", _c.c_int64, [_vp, _c.c_int, _u8p, _c.c_int64]),
    ("dcvc_rans_enc_reset", _c.c_int, [_vp]),
    ("dcvc_rans_dec_create", _vp, [_c.c_int]),
    ("dcvc_rans_dec_destroy", None, [_vp]),
    ("dcvc_rans_dec_set_stream", _c.c_int, [_vp, _u8p, _c.c_int64, _c.c_int]),
    ("dcvc_rans_dec_decode_with_indexes_i16", _c.c_int,
     [_vp, _i16p, _c.c_int64, _i32p, _c.c_int, _c.c_int, _i32p, _i32p, _i16p]),
    ("dcvc_rans_dec_decode_table_i16", _c.c_int, [_vp, _i16p, _c.c_int64, _vp, _i16p]),
    ("dcvc_rans_dec_decode_table_i32", _c.c_int, [_vp, _i32p, _c.c_int64, _vp, _i32p]),
    ("dcvc_rans_set_threads", _c.c_int, [_c.c_int]),
    ("dcvc_rans_threads", _c.c_int, []),
]


def _bind(lib, table):
    for name, res, args in table:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_rans = None
_hip = None


def rans_lib():
    global _rans
    if _rans is None:
        _rans = _bind(_load("libdcvc_rans.so"), RANS_SYMBOLS)
    return _rans


def hip_lib():
    """libdcvc_hip.so; its symbol table is declared in dcvc_amd/hip.py."""
    global _hip
    if _hip is None:
        from .hip import HIP_SYMBOLS
        # DCVC_HIP_LIB names an alternative build in dcvc_amd/lib (kernel
        # A/B experiments, scripts/conv_microbench.py); default is the product.
        _hip = _bind(_load(os.environ.get("DCVC_HIP_LIB", "libdcvc_hip.so")), HIP_SYMBOLS)
    return _hip


def ptr(arr, ctype):
    """ctypes pointer to a C-contiguous numpy array."""
    return arr.ctypes.data_as(ctypes.POINTER(ctype))
